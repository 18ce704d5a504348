"""Full-row fused GEMM (csrc/rowgemm.hip) against a torch fp32 restatement of
the reference's autocast dataflow (dpvo/net.py:75-93, blocks.py:15-30):
Linear -> fp16 output, glue ops in fp32, LayerNorm in fp32.  Accumulation
order differs from hipBLASLt, so fp16 outputs may differ by an ulp."""
import pytest
import torch
from tests_helpers import same

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("poisoned")]

D = 384


def lin(K, seed):
    g = torch.Generator().manual_seed(seed)
    w = (torch.rand(D, K, generator=g) * 2 - 1) / K ** 0.5
    b = (torch.rand(D, generator=g) * 2 - 1) / K ** 0.5
    return w.cuda(), b.cuda()


def y16(A16, w, b):
    """autocast Linear: fp16 operands, fp32 accumulate, fp16 result."""
    return (A16.float() @ w.half().float().t() + b.half().float()).half()


def close16(got, want, tol=2e-2):
    torch.testing.assert_close(got.float(), want.float(), rtol=tol, atol=tol)


@pytest.mark.parametrize("M", [1, 127, 128, 1000, 20000])
@pytest.mark.parametrize("flags", [0, 1, 2])
def test_linear_activations(M, flags):
    import update_ops as U
    A = torch.randn(M, D, device="cuda").half()
    w, b = lin(D, 1)
    W16, b16 = U.pack_linear(w, b)
    _, out, _ = U.rowgemm(A, W16, b16, flags=flags)
    want = y16(A, w, b)
    if flags == U.RELU:
        want = want.clamp_min(0)
    if flags == U.SIGMOID:
        want = torch.sigmoid(want.float()).half()
    close16(out, want)


def test_padded_k_and_row_gather():
    """K = 882 (the corr features) padded to 896; A rows gathered, idx < 0 -> zeros."""
    import update_ops as U
    M, K = 3000, 882
    buf = torch.zeros(M, 896, device="cuda", dtype=torch.float16)
    buf[:, :K] = torch.randn(M, K, device="cuda").half()
    w, b = lin(K, 2)
    W16, b16 = U.pack_linear(w, b)
    assert W16.shape == (D, 896)
    idx = torch.randint(-1, M, (5000,), device="cuda")
    _, out, _ = U.rowgemm(buf, W16, b16, flags=U.RELU, a_idx=idx)
    rows = torch.where(idx[:, None] >= 0, buf[idx.clamp_min(0), :K], torch.zeros_like(buf[:1, :K]))
    close16(out, y16(rows, w, b).clamp_min(0))


def test_residual_layernorm_and_gather():
    """corr L3: net = LN(net + imap[kk] + Linear(h))  (net.py:78-79)."""
    import update_ops as U
    M = 5000
    A = torch.randn(M, D, device="cuda").half()
    w, b = lin(D, 3)
    W16, b16 = U.pack_linear(w, b)
    net = torch.randn(M, D, device="cuda")
    imap = torch.randn(700, D, device="cuda").half()
    kk = torch.randint(0, 700, (M,), device="cuda")
    g = torch.rand(D, device="cuda") + 0.5
    be = torch.randn(D, device="cuda") * 0.1
    o32, o16, _ = U.rowgemm(A, W16, b16, flags=U.RES | U.LN, res32=net, res16=imap, res16_idx=kk,
                            ln=(g, be, 1e-3), want32=True)
    v = net + imap[kk].float() + y16(A, w, b).float()
    want = torch.nn.functional.layer_norm(v, (D,), g, be, 1e-3)
    torch.testing.assert_close(o32, want, rtol=1e-3, atol=2e-3)
    close16(o16, want.half())


def test_layernorm_relu_fp16_out():
    """corr L2: relu(LN(Linear(h))) -> fp16 (the next Linear's autocast input)."""
    import update_ops as U
    M = 4000
    A = torch.randn(M, D, device="cuda").half()
    w, b = lin(D, 4)
    W16, b16 = U.pack_linear(w, b)
    g = torch.rand(D, device="cuda") + 0.5
    be = torch.randn(D, device="cuda") * 0.1
    _, o16, _ = U.rowgemm(A, W16, b16, flags=U.LN | U.LN_RELU, ln=(g, be, 1e-3))
    want = torch.nn.functional.layer_norm(y16(A, w, b).float(), (D,), g, be, 1e-3).clamp_min(0)
    close16(o16, want.half())


@pytest.mark.parametrize("with_ln", [False, True])
def test_gated_residual_and_heads(with_ln):
    """GatedResidual x + gate(x) * res(x) (blocks.py:26-30), then LN or the d/w heads (net.py:63-72)."""
    import update_ops as U
    M = 3000
    h = torch.randn(M, D, device="cuda").half()
    x = torch.randn(M, D, device="cuda")
    gate = torch.sigmoid(torch.randn(M, D, device="cuda")).half()
    w, b = lin(D, 5)
    W16, b16 = U.pack_linear(w, b)
    r = y16(h, w, b)
    v = x + (gate * r).float()
    if with_ln:
        g = torch.rand(D, device="cuda") + 0.5
        be = torch.randn(D, device="cuda") * 0.1
        o32, o16, _ = U.rowgemm(h, W16, b16, flags=U.GATE | U.LN, res32=x, gate16=gate, ln=(g, be, 1e-3),
                                want32=True)
        want = torch.nn.functional.layer_norm(v, (D,), g, be, 1e-3)
        torch.testing.assert_close(o32, want, rtol=1e-3, atol=2e-3)
    else:
        hw = (torch.randn(4, D, device="cuda") * 0.05).half()
        hb = (torch.randn(4, device="cuda") * 0.1).half()
        o32, _, heads = U.rowgemm(h, W16, b16, flags=U.GATE | U.HEADS, res32=x, gate16=gate, heads=(hw, hb),
                                  want32=True, want16=False)
        torch.testing.assert_close(o32, v, rtol=1e-3, atol=2e-3)
        z = (v.clamp_min(0).half().float() @ hw.float().t() + hb.float()).half()
        want = torch.cat([z[:, :2], torch.sigmoid(z[:, 2:].float()).half()], 1)
        close16(heads, want)


@pytest.mark.parametrize("M", [1, 127, 3000, 40000])
def test_rowgemm_pair_equals_two_launches(M):
    """SoftAgg's f / g in one launch sharing A: bit-identical to two rowgemms."""
    import update_ops as U
    A = torch.randn(M, D, device="cuda").half()
    (wa, ba), (wb, bb) = lin(D, 5), lin(D, 6)
    Wa, ba16 = U.pack_linear(wa, ba)
    Wb, bb16 = U.pack_linear(wb, bb)
    f, g = U.rowgemm_pair(A, Wa, ba16, Wb, bb16)
    assert same(f, U.rowgemm(A, Wa, ba16)[1])
    assert same(g, U.rowgemm(A, Wb, bb16)[1])
    # device row count (the SoftAgg h GEMM's G): rows past it untouched
    Md = torch.tensor([M // 2], dtype=torch.int64, device="cuda")
    f2, g2 = U.rowgemm_pair(A, Wa, ba16, Wb, bb16, M_dev=Md)
    assert same(f2[:M // 2], f[:M // 2]) and same(g2[:M // 2], g[:M // 2])


@pytest.mark.parametrize("M", [1, 127, 3000, 40000])
@pytest.mark.parametrize("flags", [0, 1, 2])
def test_kblocked_w_is_bit_identical(M, flags):
    """W read k-blocked ([K/32][384][32], update_ops.kblock; the SoftAgg
    GEMMs' layout) == the [384][K] kernel bit for bit: single GEMM with a
    padded K, a gathered A with idx < 0 rows, a device row count, and the pair."""
    import update_ops as U
    K = 882
    buf = torch.zeros(M, 896, device="cuda", dtype=torch.float16)
    buf[:, :K] = torch.randn(M, K, device="cuda").half()
    W16, b16 = U.pack_linear(*lin(K, 7))
    idx = torch.randint(-1, M, (M + 37,), device="cuda")
    want = U.rowgemm(buf, W16, b16, flags=flags, a_idx=idx)[1]
    got = U.rowgemm(buf, U.kblock(W16), b16, flags=flags, a_idx=idx)[1]
    assert same(got, want)
    Md = torch.tensor([(M + 1) // 2], dtype=torch.int64, device="cuda")
    out = torch.full_like(want, 7.0)
    U.rowgemm(buf, U.kblock(W16), b16, flags=flags, a_idx=idx, out16=out, M_dev=Md)
    h = (M + 1) // 2
    assert same(out[:h], want[:h]) and bool((out[h:] == 7.0).all())
    A = torch.randn(M, D, device="cuda").half()
    (Wa, ba), (Wb, bb) = U.pack_linear(*lin(D, 8)), U.pack_linear(*lin(D, 9))
    # K = 384 with a device row count: the small-M kernel (the SoftAgg h Linear)
    want = U.rowgemm(A, Wa, ba, flags=flags)[1]
    out = torch.full_like(want, 7.0)
    U.rowgemm(A, U.kblock(Wa), ba, flags=flags, out16=out, M_dev=Md)
    assert same(out[:h], want[:h]) and bool((out[h:] == 7.0).all())
    f, g = U.rowgemm_pair(A, U.kblock(Wa), ba, U.kblock(Wb), bb)
    assert same(f, U.rowgemm(A, Wa, ba)[1]) and same(g, U.rowgemm(A, Wb, bb)[1])
    # the pair with the A tile resident (K = 384) under a device row count, and
    # the ring-streamed pair (K = 896 and K = 64: the tile does not fit, or is
    # shorter than the staging depth)
    f2, g2 = U.rowgemm_pair(A, U.kblock(Wa), ba, U.kblock(Wb), bb, M_dev=Md)
    assert same(f2[:h], f[:h]) and same(g2[:h], g[:h])
    W16b, b16b = U.pack_linear(*lin(K, 10))
    f, g = U.rowgemm_pair(buf, U.kblock(W16), b16, U.kblock(W16b), b16b)
    assert same(f, U.rowgemm(buf, W16, b16)[1]) and same(g, U.rowgemm(buf, W16b, b16b)[1])
    # the resident-A pair at its shortest tiles (K = 128: four k-steps, the
    # prologue's whole staging depth; K = 256), several tiles per block
    for Kr in (128, 256):
        Ar = torch.randn(70001, Kr, device="cuda").half()
        (Wra, bra), (Wrb, brb) = U.pack_linear(*lin(Kr, 13)), U.pack_linear(*lin(Kr, 14))
        f, g = U.rowgemm_pair(Ar, U.kblock(Wra), bra, U.kblock(Wrb), brb)
        assert same(f, U.rowgemm(Ar, Wra, bra)[1]) and same(g, U.rowgemm(Ar, Wrb, brb)[1])
    (W64a, b64a), (W64b, b64b) = U.pack_linear(*lin(64, 11)), U.pack_linear(*lin(64, 12))
    A64 = A[:, :64]
    f, g = U.rowgemm_pair(A64, U.kblock(W64a), b64a, U.kblock(W64b), b64b)
    assert same(f, U.rowgemm(A64, W64a, b64a)[1]) and same(g, U.rowgemm(A64, W64b, b64b)[1])
    with pytest.raises(RuntimeError):
        U.rowgemm(A, U.kblock(Wa), ba, flags=U.RES, res32=torch.zeros(M, D, device="cuda"))


def test_rowadd_ln():
    import update_ops as U
    M = 3000
    a = torch.randn(M, D, device="cuda")
    hk = torch.randn(500, D, device="cuda").half()
    jx = torch.randint(0, 500, (M,), device="cuda")
    g = torch.rand(D, device="cuda") + 0.5
    be = torch.randn(D, device="cuda") * 0.1
    o32, o16 = U.rowadd_ln(a, hk, jx)
    torch.testing.assert_close(o32, a + hk[jx].float())
    o32, o16 = U.rowadd_ln(a, hk, jx, ln=(g, be, 1e-3))
    want = torch.nn.functional.layer_norm(a + hk[jx].float(), (D,), g, be, 1e-3)
    torch.testing.assert_close(o32, want, rtol=1e-4, atol=1e-4)
    close16(o16, want.half())
    # fp16 input with a padded row stride, out-of-range gather rows add nothing
    a16 = torch.randn(M, D + 4, device="cuda").half()[:, :D]
    jx[::7] = -1
    jx[1::7] = 500
    o32, o16 = U.rowadd_ln(a16, hk, jx, ln=(g, be, 1e-3))
    add = torch.where((jx >= 0) & (jx < 500), 1.0, 0.0)[:, None] * hk[jx.clamp(0, 499)].float()
    want = torch.nn.functional.layer_norm(a16.float() + add, (D,), g, be, 1e-3)
    torch.testing.assert_close(o32, want, rtol=1e-4, atol=1e-4)
    assert U.rowadd_ln(a[:0], hk, jx[:0])[0].shape == (0, D)
    # a second gathered addend: bit-identical to two calls (the update
    # operator's net + agg_kk + agg_ij without the fp32 rows in between)
    h2 = torch.randn(300, D, device="cuda").half()
    ix2 = torch.randint(-1, 301, (M,), device="cuda")
    s32, s16 = U.rowadd_ln(a, hk, jx, want16=False)[0], U.rowadd_ln(a, hk, jx, want32=False)[1]
    r32, r16 = U.rowadd_ln(s32, h2, ix2, ln=(g, be, 1e-3))
    c32, c16 = U.rowadd_ln(a, hk, jx, ln=(g, be, 1e-3), c16=h2, c_idx=ix2)
    assert same(c32, r32) and same(c16, r16)
    assert same(s16, U.rowadd_ln(a, hk, jx)[1])


def test_errors():
    import update_ops as U
    A = torch.randn(10, D, device="cuda").half()
    w, b = lin(D, 6)
    W16, b16 = U.pack_linear(w, b)
    with pytest.raises(RuntimeError):
        U.rowgemm(A, W16, b16, flags=U.RES)           # residual missing
    with pytest.raises(RuntimeError):
        U.rowgemm(A, W16, b16, flags=U.RELU | U.LN)   # unsupported combination
    with pytest.raises(RuntimeError):
        U.rowgemm(A.float(), W16, b16)
    # k-blocked W needs K % 64 == 0 (K = 32: one k-step per tile, no barrier
    # between a tile's y-tile reads and the next tile's writes)
    A32 = torch.randn(300, 32, device="cuda").half()
    w32, b32 = lin(32, 7)
    W32, c32 = U.pack_linear(w32, b32)
    with pytest.raises(RuntimeError, match="multiple of 64"):
        U.rowgemm(A32, U.kblock(W32[:, :32].contiguous()), c32)


def test_fused_update_operator_matches_torch_path():
    """Update.forward (net.py:75-93) fused path vs the module's own torch
    composition, same weights and inputs, both under fp16 autocast."""
    from dpvo.net import Update
    from dpvo.synthetic import steady_state_edges
    torch.manual_seed(0)
    upd = Update(3).cuda()
    with torch.no_grad():
        for m in upd.modules():        # livelier than default init so LN/gates see O(1) values
            if isinstance(m, torch.nn.Linear):
                m.weight.mul_(3.0)
    ii, jj, kk = steady_state_edges(40, 16, 13, 22, "cuda")
    E = ii.numel()
    net = torch.randn(1, E, 384, device="cuda")
    inp = torch.randn(1, E, 384, device="cuda").half()
    corr = torch.zeros(E, 896, device="cuda", dtype=torch.float16)
    corr[:, :882] = torch.randn(E, 882, device="cuda").half()
    corr = corr[:, :882][None]
    outs = {}
    for fused in (True, False):
        Update.FUSED = fused
        with torch.no_grad(), torch.autocast("cuda", enabled=True):
            outs[fused] = upd(net, inp, corr, None, ii, jj, kk)
    Update.FUSED = True
    (nf, (df, wf, _)), (nt, (dt, wt, _)) = outs[True], outs[False]
    assert nf.dtype == nt.dtype == torch.float32 and nf.shape == nt.shape == (1, E, 384)
    assert df.dtype == torch.float16 and df.shape == dt.shape == (1, E, 2) and wf.shape == (1, E, 2)
    err = (nf - nt).abs().max().item() / nt.abs().max().item()
    assert err < 2e-2, err
    torch.testing.assert_close(df.float(), dt.float(), rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(wf.float(), wt.float(), rtol=2e-2, atol=2e-2)


def test_fused_update_operator_context_index_is_the_gathered_context():
    """DPVO.update passes the context ring + kk % (M pmem) (dpvo.py:718) and the
    fused operator gathers the rows in its epilogue: identical to passing the
    gathered ctx."""
    from dpvo.net import Update
    from dpvo.synthetic import steady_state_edges
    torch.manual_seed(1)
    upd = Update(3).cuda()
    ii, jj, kk = steady_state_edges(40, 16, 13, 22, "cuda")
    E = ii.numel()
    net = torch.randn(1, E, 384, device="cuda")
    ring = torch.randn(1, 36 * 16, 384, device="cuda").half()
    idx = kk % (36 * 16)
    corr = torch.randn(1, E, 882, device="cuda").half()
    with torch.no_grad(), torch.autocast("cuda", enabled=True):
        a = upd(net, ring[:, idx], corr, None, ii, jj, kk)
        b = upd(net, ring, corr, None, ii, jj, kk, inp_idx=idx)
    assert same(a[0], b[0])
    assert same(a[1][0], b[1][0]) and same(a[1][1], b[1][1])


@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("case", ["corr", "gather_res", "gather_res16", "gate_ln", "gate_heads"])
def test_rowchain_is_two_rowgemms(case, big):
    """dpvo_rowchain (the intermediate kept in LDS) is bit-identical to two
    rowgemm launches with the intermediate in HBM: same MFMA chunk order,
    same fp16 rounding of the intermediate.  big: more 128-row tiles than
    workgroups, so blocks run several tiles and the row pass of one tile is
    interleaved with the next tile's first GEMM (ILV).  gather_res: c1 / c2's
    chain (no res16: the no-addend epilogue); gather_res16: with a gathered
    fp16 addend (the general residual epilogue)."""
    import update_ops as U
    torch.manual_seed(3)
    M = 777 if case.startswith("gather_res") else 1000
    if big:
        M = 70001
    K1 = 896 if case == "corr" else 384
    dev = "cuda"
    A = (torch.randn(max(1200, M), K1, device=dev) * 0.5).half()
    W1, b1 = U.pack_linear(torch.randn(384, K1, device=dev) / K1 ** 0.5, torch.randn(384, device=dev) * 0.1)
    W2, b2 = U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    ln = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    res32 = torch.randn(M, 384, device=dev)
    gate16 = torch.rand(M, 384, device=dev).half()
    heads = (torch.randn(4, 384, device=dev).half() * 0.05, torch.randn(4, device=dev).half())
    a_idx = torch.randint(-1, A.shape[0], (M,), device=dev) if case.startswith("gather_res") else None
    r16 = torch.randn(600, 384, device=dev).half()
    ridx = torch.randint(-1, 600, (M,), device=dev)
    kw = {"corr": dict(flags=U.LN | U.LN_RELU, ln=ln),
          "gather_res": dict(flags=U.RES, res32=res32, want32=True),
          "gather_res16": dict(flags=U.RES, res32=res32, res16=r16, res16_idx=ridx, want32=True),
          "gate_ln": dict(flags=U.GATE | U.LN, res32=res32, gate16=gate16, ln=ln, want32=True),
          "gate_heads": dict(flags=U.GATE | U.HEADS, res32=res32, gate16=gate16, heads=heads, want32=True,
                             want16=False)}[case]
    _, h, _ = U.rowgemm(A, W1, b1, flags=U.RELU, a_idx=a_idx, M=None if a_idx is not None else M)
    ref = U.rowgemm(h, W2, b2, **kw)
    got = U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, a_idx=a_idx, M=None if a_idx is not None else M, **kw)
    for r, g in zip(ref, got):
        assert (r is None) == (g is None)
        if r is not None:
            assert same(r, g)


@pytest.mark.parametrize("flags1,M", [("relu", 2048 * 128 + 77), ("sigmoid", 3000), ("none", 3000)])
def test_rowchain_gather_many_tiles_and_runtime_activation(flags1, M):
    """c1 / c2's gathered chain with more than 8 tiles per 256 workgroups
    (2,049 tiles: the launch then sizes the grid so that each block's row
    sources fit its LDS table), and the first GEMM's activation when it is not
    the compile-time ReLU (read from the flags at run time): both still
    bit-identical to two rowgemm launches."""
    import update_ops as U
    torch.manual_seed(5)
    dev = "cuda"
    f1 = {"relu": U.RELU, "sigmoid": U.SIGMOID, "none": 0}[flags1]
    A = (torch.randn(4096, 384, device=dev) * 0.5).half()
    W1, b1 = U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    W2, b2 = U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    res32 = torch.randn(M, 384, device=dev)
    a_idx = torch.randint(-1, A.shape[0], (M,), device=dev)
    _, h, _ = U.rowgemm(A, W1, b1, flags=f1, a_idx=a_idx)
    ref = U.rowgemm(h, W2, b2, flags=U.RES, res32=res32, want32=True)
    got = U.rowchain(A, W1, b1, W2, b2, flags1=f1, a_idx=a_idx, flags=U.RES, res32=res32, want32=True)
    for r, g in zip(ref, got):
        assert (r is None) == (g is None)
        if r is not None:
            assert same(r, g)


@pytest.mark.parametrize("M", [1, 1000, 50000])
@pytest.mark.parametrize("last", [False, True])
def test_rowchain_gated_is_gate_gemm_plus_chain(M, last):
    """dpvo_rowchain_gated (gate Linear + sigmoid on chip, y stored as
    fp16(gate * y)) is bit-identical to rowgemm(SIGMOID) -> gate16 followed by
    the GATE chain: the GRU's GatedResidual (blocks.py:27-30)."""
    import update_ops as U
    torch.manual_seed(4)
    dev = "cuda"
    A = (torch.randn(M, 384, device=dev) * 0.5).half()
    lin_ = lambda s: U.pack_linear(torch.randn(384, 384, device=dev) / s, torch.randn(384, device=dev) * 0.1)
    (Wg, bg), (W1, b1), (W2, b2) = lin_(20.0), lin_(20.0), lin_(20.0)
    res32 = torch.randn(M, 384, device=dev)
    if last:
        heads = (torch.randn(4, 384, device=dev).half() * 0.05, torch.randn(4, device=dev).half())
        kw = dict(flags=U.GATE | U.HEADS, res32=res32, heads=heads, want32=True, want16=False)
    else:
        ln = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
        kw = dict(flags=U.GATE | U.LN, res32=res32, ln=ln, want32=True)
    _, g16, _ = U.rowgemm(A, Wg, bg, flags=U.SIGMOID)
    ref = U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, gate16=g16, **kw)
    got = U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, gate=(Wg, bg), **kw)
    for r, g in zip(ref, got):
        assert (r is None) == (g is None)
        if r is not None:
            assert same(r, g)
    with pytest.raises(RuntimeError):
        U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, gate16=g16, gate=(Wg, bg), **kw)


@pytest.mark.parametrize("M", [1, 1000, 70001])
def test_rowchain_gated_pre_is_rowadd_then_chain(M):
    """dpvo_rowchain_gated_pre (the residual rows LayerNorm(a + b16[b_idx] +
    c16[c_idx]) formed in the row epilogue) is bit-identical to rowadd_ln
    writing them as out32 followed by dpvo_rowchain_gated with res32 = those
    rows: the first GRU chain after `norm(net + agg_kk + agg_ij)` (net.py:90-92),
    including absent / out-of-range addend indices and rows past M."""
    import update_ops as U
    torch.manual_seed(6)
    dev = "cuda"
    G1, G2 = 700, 300
    a32 = torch.randn(M, 384, device=dev)
    b16 = torch.randn(G1, 384, device=dev).half()
    c16 = torch.randn(G2, 384, device=dev).half()
    bidx = torch.randint(-1, G1 + 5, (M,), device=dev)
    cidx = torch.randint(-1, G2 + 5, (M,), device=dev)
    ln0 = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    ln1 = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    lin_ = lambda s: U.pack_linear(torch.randn(384, 384, device=dev) / s, torch.randn(384, device=dev) * 0.1)
    (Wg, bg), (W1, b1), (W2, b2) = lin_(20.0), lin_(20.0), lin_(20.0)
    r32, r16 = U.rowadd_ln(a32, b16, bidx, ln0, c16=c16, c_idx=cidx)
    _, p16 = U.rowadd_ln(a32, b16, bidx, ln0, c16=c16, c_idx=cidx, want32=False)
    assert same(r16, p16)
    kw = dict(flags=U.GATE | U.LN, ln=ln1, want32=True, gate=(Wg, bg))
    ref = U.rowchain(r16, W1, b1, W2, b2, flags1=U.RELU, res32=r32, **kw)
    got = U.rowchain(p16, W1, b1, W2, b2, flags1=U.RELU, pre=(a32, b16, bidx, c16, cidx, ln0), **kw)
    for r, g in zip(ref, got):
        assert (r is None) == (g is None)
        if r is not None:
            assert same(r, g)
    with pytest.raises(RuntimeError):   # res32 and pre together
        U.rowchain(p16, W1, b1, W2, b2, flags1=U.RELU, res32=r32, pre=(a32, b16, bidx, c16, cidx, ln0), **kw)


@pytest.mark.parametrize("M", [1, 1000, 95424])
@pytest.mark.parametrize("gathered", [False, True])
def test_rowchain3_is_chain_plus_rowgemm(M, gathered):
    """dpvo_rowchain3 (the corr MLP of net.py:54-61 and norm(net + inp + .),
    :78-79, in one launch: both intermediates and the middle LayerNorm on
    chip) is bit-identical to rowchain(LN | LN_RELU) writing fp16 rows
    followed by rowgemm(RES | LN) with the context-row gather."""
    import update_ops as U
    torch.manual_seed(5)
    dev = "cuda"
    A = torch.zeros(M, 896, device=dev, dtype=torch.float16)
    A[:, :882] = (torch.randn(M, 882, device=dev) * 0.7).half()
    W1, b1 = U.pack_linear(torch.randn(384, 882, device=dev) / 30.0, torch.randn(384, device=dev) * 0.1)
    Wm, bm = U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    W3, b3 = U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    lnm = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    ln3 = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    res32 = torch.randn(M, 384, device=dev)
    ring = torch.randn(max(M, 64) + 17, 384, device=dev).half()
    idx = torch.randint(0, ring.shape[0], (M,), device=dev) if gathered else None
    res16 = ring if gathered else ring[:M].contiguous()
    kw = dict(flags=U.RES | U.LN, res32=res32, res16=res16, res16_idx=idx, ln=ln3, want32=True)
    _, h, _ = U.rowchain(A, W1, b1, Wm, bm, flags1=U.RELU, flags=U.LN | U.LN_RELU, ln=lnm)
    ref = U.rowgemm(h, W3, b3, **kw)
    got = U.rowchain(A, W1, b1, W3, b3, flags1=U.RELU, mid=(Wm, bm, lnm), **kw)
    for r, g in zip(ref, got):
        assert (r is None) == (g is None)
        if r is not None:
            assert same(r, g)


def test_update_operator_corr_chain3_is_two_launches():
    """Update.forward's fused path with the three-GEMM corr chain equals the
    two-launch path bit for bit"""
    from dpvo.net import Update
    from dpvo.synthetic import steady_state_edges
    torch.manual_seed(6)
    upd = Update(3).cuda()
    ii, jj, kk = steady_state_edges(40, 16, 13, 22, "cuda")
    E = ii.numel()
    net = torch.randn(1, E, 384, device="cuda")
    inp = torch.randn(1, E, 384, device="cuda").half()
    corr = torch.randn(1, E, 882, device="cuda").half()
    outs = []
    for chain3 in (True, False):
        Update.CORR_CHAIN3 = chain3
        with torch.no_grad(), torch.autocast("cuda", enabled=True):
            outs.append(upd(net, inp, corr, None, ii, jj, kk))
    Update.CORR_CHAIN3 = True
    (a, (da, wa, _)), (b, (db, wb, _)) = outs
    assert same(a, b) and same(da, db) and same(wa, wb)


@pytest.mark.parametrize("M", [1, 300, 20000, 70000, 95424])
def test_rowgemm_pair_pre_equals_rowadd_then_pair(M):
    """dpvo_rowgemm_pair_pre (A rows fp16(a32 + b16[idx]) formed while staged)
    is bit-identical to rowadd_ln(a32, b16, idx, want32=False) feeding
    rowgemm_pair, including out-of-range indices (no addend) and rows past M.
    M = 70000 / 95424 (C3's edge count) give a block several tiles, so the
    addend sources come from the LDS table."""
    import update_ops as U
    g = torch.Generator().manual_seed(M)
    a32 = torch.randn(M, D, generator=g).cuda()
    G = max(M // 20, 1)
    b16 = torch.randn(G + 3, D, generator=g).half().cuda()
    idx = torch.randint(0, G, (M,), generator=g)
    idx[::17] = -1                      # no addend
    idx[5::23] = G + 7                  # beyond b_rows: no addend
    idx = idx.cuda()
    (wf, bf), (wg, bg) = lin(D, 1), lin(D, 2)
    Wf, cf = U.pack_linear(wf, bf)
    Wg, cg = U.pack_linear(wg, bg)
    Wf, Wg = U.kblock(Wf), U.kblock(Wg)
    _, n16 = U.rowadd_ln(a32, b16[:G], idx, want32=False)
    f_ref, g_ref = U.rowgemm_pair(n16, Wf, cf, Wg, cg)
    f, gg = U.rowgemm_pair_pre(a32, b16, idx, Wf, cf, Wg, cg, b_rows=G)
    assert same(f, f_ref) and same(gg, g_ref)
