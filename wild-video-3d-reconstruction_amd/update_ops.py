"""Native glue of the learned update operator (csrc/updateop.hip).

Replaces torch_scatter 2.1.2's ``scatter_softmax`` + ``scatter_sum`` in
SoftAgg (reference dpvo/blocks.py:40-48) and the masked neighbour gather of
Update.forward (dpvo/net.py:82-85).  Inference only (no autograd); the
dpvo.blocks / dpvo.net mirrors call these under ``torch.no_grad`` and keep a
torch composition for training.  Like the other shims there is no CPU path.
"""
import torch

import _dpvo_hot as H


def softagg(f, s, group, groups, eps=1e-12):
    """y[g] = sum_{e: group[e]==g} f[e] * softmax_g(s)[e]  (per channel).

    f, s: [E, D] with unit channel stride and any row stride (two column
    halves of one fused GEMM output work); group: [E] int64 in [0, groups);
    returns y [groups, D] of f's dtype."""
    H.on_gpu(f, s, group)
    if f.dim() != 2 or s.shape != f.shape:
        raise RuntimeError("softagg: f and s must both be [E, D]")
    if f.dtype != s.dtype:
        raise RuntimeError("softagg: f and s must have the same dtype")
    if f.stride(1) != 1 or s.stride(1) != 1:
        raise RuntimeError("softagg: rows must be channel-contiguous")
    E, D = f.shape
    group = H.idx64(group)
    y = H.empty(groups, D, dtype=f.dtype, device=f.device)
    nbytes = H.lib().dpvo_softagg_workspace_bytes(E, groups)
    ws = H.empty(nbytes, dtype=torch.uint8, device=f.device)
    H.check(H.lib().dpvo_softagg_forward(H.dtype_code(f), H.ptr(f), f.stride(0), H.ptr(s), s.stride(0),
                                         H.ptr(group), E, D, groups, float(eps), H.ptr(y), H.ptr(ws), nbytes,
                                         H.stream_of(f)))
    return y


def key_bits_for(bound):
    """radix-sort key width for keys known to lie in [0, bound)."""
    return max(1, (int(bound) - 1).bit_length())


def group_by(key, key_bits=64, radix=False):
    """torch.unique(key, return_inverse=True) without a host sync, plus the
    groups' CSR: -> (gid int64 [E], offs int32 [E+1], perm int32 [E],
    groups int64 [1] on the device).  key_bits <= 32 promises keys in
    [0, 2**key_bits) (fewer radix passes: pass key_bits_for(bound) when the
    caller knows a bound); the default sorts full 64-bit keys.  key_bits <= 22
    runs as a counting sort over 2**key_bits bins unless radix=True (the
    radix-sort path; same outputs)."""
    if not 1 <= int(key_bits) <= 64:
        raise RuntimeError("group_by: key_bits must be 1..64")
    H.on_gpu(key)
    key = H.idx64(key)
    n = key.numel()
    dev = key.device
    gid = H.empty(n, dtype=torch.int64, device=dev)
    offs = H.empty(n + 1, dtype=torch.int32, device=dev)
    perm = H.empty(max(n, 1), dtype=torch.int32, device=dev)
    groups = H.empty(1, dtype=torch.int64, device=dev)
    nbytes = (H.lib().dpvo_group_by_workspace_bytes(n) if radix
              else H.lib().dpvo_group_by_workspace_bytes_for(n, int(key_bits)))
    ws = H.empty(nbytes, dtype=torch.uint8, device=dev)
    H.check(H.lib().dpvo_group_by(H.ptr(key), n, int(key_bits), H.ptr(gid), H.ptr(offs), H.ptr(perm), H.ptr(groups),
                                  H.ptr(ws), nbytes, H.stream_of(key)))
    return gid, offs, perm, groups


def softagg_csr(f, s, offs, perm, groups, max_groups, eps=1e-12, long_groups=False):
    """softagg over group_by's CSR; y [max_groups, D], rows >= groups untouched.
    long_groups: split groups of >= 64 edges over four waves (dpvo_softagg_csr_long)."""
    H.on_gpu(f, s, offs, perm, groups)
    if f.dim() != 2 or s.shape != f.shape or f.dtype != s.dtype or f.stride(1) != 1 or s.stride(1) != 1:
        raise RuntimeError("softagg_csr: f and s must be [E, D] with channel-contiguous rows, same dtype")
    D = f.shape[1]
    y = H.empty(max_groups, D, dtype=f.dtype, device=f.device)
    fn = H.lib().dpvo_softagg_csr_long if long_groups else H.lib().dpvo_softagg_csr
    H.check(fn(H.dtype_code(f), H.ptr(f), f.stride(0), H.ptr(s), s.stride(0), H.ptr(offs), H.ptr(perm), H.ptr(groups),
               int(max_groups), D, float(eps), H.ptr(y), H.stream_of(f)))
    return y


def rowchain(A, W1, b1, W2, b2, flags1=None, flags=0, a_idx=None, M=None, res32=None, res16=None, res16_idx=None,
             gate16=None, ln=None, heads=None, want32=False, want16=True, M_dev=None, gate=None, mid=None,
             pre=None):
    """rowgemm(rowgemm(A, W1, b1, flags1, a_idx).y16, W2, b2, flags, ...) in one
    launch, the 384-wide intermediate kept on chip (dpvo_rowchain).
    gate = (Wg, bg) with GATE in flags: gate16 = rowgemm(A, Wg, bg, SIGMOID)
    computed in the same launch (dpvo_rowchain_gated) instead of passed in.
    mid = (Wm, bm, (ln_g, ln_b, eps)): a middle Linear between the two, its
    output LayerNorm'd and ReLU'd on chip (dpvo_rowchain3; flags must be
    RES | LN): rowgemm(rowchain(A, W1, b1, Wm, bm, LN | LN_RELU).out16, W2, b2,
    flags, ...) in one launch.
    pre = (a32, b16, b_idx, c16, c_idx, (ln_g, ln_b, eps)) with gate and res32
    None: the residual rows are rowadd_ln(a32, b16, b_idx, ln, c16=c16,
    c_idx=c_idx)'s out32, formed in the row epilogue instead of read
    (dpvo_rowchain_gated_pre, bit-identical).
    Weights may be given as [384, Kp] (re-laid out per call) or already
    k-blocked by kblock() (what the kernel reads; the fused Update caches them).
    Returns (out32, out16, head_out) of the last GEMM."""
    H.on_gpu(A, W1, b1, W2, b2)
    if flags1 is None:
        flags1 = RELU
    if any(t.dtype != torch.float16 for t in (A, W1, b1, W2, b2)):
        raise RuntimeError("rowchain: A, weights and biases must be fp16")
    if A.dim() != 2 or A.stride(1) != 1:
        raise RuntimeError("rowchain: A must be [rows, K] row-contiguous")
    for W in (W1, W2):
        if W.dim() == 2 and (W.shape[0] != WIDTH or not W.is_contiguous()):
            raise RuntimeError("rowchain: W must be [384, Kp] contiguous")
    W1, W2 = kblock(W1), kblock(W2)
    if _kb_K(W2) != WIDTH:
        raise RuntimeError("rowchain: W2 must be [384, 384]")
    Kp = _kb_K(W1)
    if A.stride(0) < Kp:
        raise RuntimeError(f"rowchain: A's row stride {A.stride(0)} < padded K {Kp}")
    dev = A.device
    if a_idx is not None:
        a_idx = H.idx64(a_idx)
        M = a_idx.numel()
    elif M is None:
        M = A.shape[0]
    out32 = H.empty(M, WIDTH, dtype=torch.float32, device=dev) if want32 else None
    out16 = H.empty(M, WIDTH, dtype=torch.float16, device=dev) if want16 else None
    head_out = H.empty(M, 4, dtype=torch.float16, device=dev) if heads is not None else None
    if res16_idx is not None:
        res16_idx = H.idx64(res16_idx)
    g1 = RowGemmArgs()
    g1.A, g1.lda, g1.a_idx, g1.a_rows = _p(A), A.stride(0), _p(a_idx), A.shape[0]
    g1.W, g1.K, g1.N, g1.bias, g1.zero_row = _p(W1), Kp, WIDTH, _p(b1), _p(zero_row(dev, Kp))
    g1.M, g1.flags = M, int(flags1)
    if M_dev is not None:
        if M_dev.dtype != torch.int64 or not M_dev.is_cuda:
            raise RuntimeError("rowchain: M_dev must be a device int64 scalar")
        g1.M_dev = M_dev.data_ptr()
    g2 = RowGemmArgs()
    g2.W, g2.K, g2.N, g2.bias = _p(W2), WIDTH, WIDTH, _p(b2)
    g2.res32, g2.ldr = _p(res32), (res32.stride(0) if res32 is not None else 0)
    g2.res16, g2.res16_idx, g2.gate16 = _p(res16), _p(res16_idx), _p(gate16)
    if ln is not None:
        g2.ln_g, g2.ln_b, g2.ln_eps = _p(ln[0]), _p(ln[1]), float(ln[2])
    if heads is not None:
        g2.head_w, g2.head_b, g2.head_out = _p(heads[0]), _p(heads[1]), _p(head_out)
    g2.out32, g2.ldo32 = _p(out32), (out32.stride(0) if out32 is not None else 0)
    g2.out16, g2.ldo16 = _p(out16), (out16.stride(0) if out16 is not None else 0)
    g2.flags = int(flags)
    for t, nm in ((res32, "res32"), (out32, "out32")):
        if t is not None and (t.dtype != torch.float32 or t.stride(1) != 1):
            raise RuntimeError(f"rowchain: {nm} must be fp32 with contiguous rows")
    for t, nm in ((res16, "res16"), (gate16, "gate16")):
        if t is not None and (t.dtype != torch.float16 or not t.is_contiguous() or t.shape[-1] != WIDTH):
            raise RuntimeError(f"rowchain: {nm} must be contiguous fp16 [*, 384]")
    if gate is not None:
        Wg, bg = gate
        H.on_gpu(Wg, bg)
        Wg = kblock(Wg)
        if Wg.dtype != torch.float16 or bg.dtype != torch.float16 or Wg.shape != W1.shape or not Wg.is_contiguous():
            raise RuntimeError("rowchain: gate W must be fp16 contiguous of W1's shape, bias fp16")
        if gate16 is not None:
            raise RuntimeError("rowchain: pass either gate16 or gate, not both")
        gg = RowGemmArgs()
        gg.W, gg.K, gg.N, gg.bias = _p(Wg), Kp, WIDTH, _p(bg)
        if pre is not None:
            a32, pb16, pbi, pc16, pci, pln = pre
            H.on_gpu(a32, pb16, pc16, pln[0], pln[1])
            if res32 is not None or a32.dtype != torch.float32 or a32.dim() != 2 or a32.shape != (M, WIDTH) \
                    or a32.stride(1) != 1:
                raise RuntimeError("rowchain: pre's a32 must be fp32 [M, 384] row-contiguous, res32 None")
            for t in (pb16, pc16):
                if t.dtype != torch.float16 or not t.is_contiguous() or t.shape[-1] != WIDTH:
                    raise RuntimeError("rowchain: pre's b16 / c16 must be contiguous fp16 [*, 384]")
            pbi, pci = H.idx64(pbi), H.idx64(pci)
            pa = RowAddArgs()
            pa.a, pa.a_f16, pa.lda, pa.M = _p(a32), 0, a32.stride(0), M
            pa.b16, pa.b_idx, pa.b_rows = _p(pb16), _p(pbi), pb16.shape[0]
            pa.c16, pa.c_idx, pa.c_rows = _p(pc16), _p(pci), pc16.shape[0]
            pa.ln_g, pa.ln_b, pa.ln_eps = _p(pln[0]), _p(pln[1]), float(pln[2])
            H.check(H.lib().dpvo_rowchain_gated_pre(_ct.byref(gg), _ct.byref(g1), _ct.byref(g2), _ct.byref(pa),
                                                    H.stream_of(A)))
        else:
            H.check(H.lib().dpvo_rowchain_gated(_ct.byref(gg), _ct.byref(g1), _ct.byref(g2), H.stream_of(A)))
    elif mid is not None:
        Wm, bm, lnm = mid
        H.on_gpu(Wm, bm, lnm[0], lnm[1])
        Wm = kblock(Wm)
        if Wm.dtype != torch.float16 or bm.dtype != torch.float16 or _kb_K(Wm) != WIDTH:
            raise RuntimeError("rowchain: the middle W must be a contiguous fp16 [384, 384], bias fp16")
        gm = RowGemmArgs()
        gm.W, gm.K, gm.N, gm.bias = _p(Wm), WIDTH, WIDTH, _p(bm)
        gm.ln_g, gm.ln_b, gm.ln_eps = _p(lnm[0]), _p(lnm[1]), float(lnm[2])
        gm.flags = LN | LN_RELU
        H.check(H.lib().dpvo_rowchain3(_ct.byref(g1), _ct.byref(gm), _ct.byref(g2), H.stream_of(A)))
    else:
        H.check(H.lib().dpvo_rowchain(_ct.byref(g1), _ct.byref(g2), H.stream_of(A)))
    return out32, out16, head_out


def neighbors_csr(jj, offs, perm, groups, max_groups):
    """cuda_ba.neighbors(kk, jj) from the CSR of group_by(kk): -> (ix, jx) int64,
    the previous / next edge of the same patch in (jj, edge) order, -1 at the
    ends (ba.cpp:113-158) -- no radix sort of its own."""
    H.on_gpu(jj, offs, perm, groups)
    jj = H.idx64(jj)
    E = jj.numel()
    ix = H.empty(E, dtype=torch.int64, device=jj.device)
    jx = H.empty(E, dtype=torch.int64, device=jj.device)
    H.check(H.lib().dpvo_neighbors_csr(H.ptr(jj), H.ptr(offs), H.ptr(perm), H.ptr(groups), int(max_groups), E,
                                       H.ptr(ix), H.ptr(jx), H.stream_of(jj)))
    return ix, jx


def window_keys(ii, jj, kk, M, base, ring, frames, flag=None):
    """(kk - M base, (ii - base) * 64 + (jj - base), kk mod ring, jj mod frames)
    as int64 [E] each, in one launch (dpvo_window_keys).  flag: optional int32
    device word set to -2 (if 0) when an edge falls outside the key window."""
    H.on_gpu(ii, jj, kk)
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    E = kk.numel()
    if ii.numel() != E or jj.numel() != E:
        raise RuntimeError("window_keys: ii, jj and kk must have the same length")
    out = H.empty(4, E, dtype=torch.int64, device=kk.device)
    H.check(H.lib().dpvo_window_keys(H.ptr(ii), H.ptr(jj), H.ptr(kk), E, int(M), int(base), int(ring), int(frames),
                                     H.ptr(out[0]), H.ptr(out[1]), H.ptr(out[2]), H.ptr(out[3]), H.ptr(flag),
                                     H.stream_of(kk)))
    return out[0], out[1], out[2], out[3]


def window_group_by(ii, jj, kk, M, base, ring, frames, flag=None, jj_order=False):
    """window_keys + group_by(key_kk, key_bits_for(64 M)) + group_by(key_ij, 12)
    in one memset and four launches (dpvo_window_group_by; same outputs):
    -> (ctx, jslot, kk_groups, ij_groups[, order]), each groups tuple as
    group_by's; jj_order: also the edges grouped by target frame (int32 [E],
    altcorr's visiting order, what cuda_corr.edge_order gives by ring slot)."""
    H.on_gpu(ii, jj, kk)
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    E = kk.numel()
    if ii.numel() != E or jj.numel() != E:
        raise RuntimeError("window_group_by: ii, jj and kk must have the same length")
    bits = key_bits_for(64 * int(M))
    nbytes = H.lib().dpvo_window_group_by_workspace_bytes(E, bits)
    if nbytes == 0:
        raise RuntimeError("window_group_by: 64 M above the counting-sort range")
    dev = kk.device
    slots = H.empty(2, E, dtype=torch.int64, device=dev)
    gid = H.empty(2, E, dtype=torch.int64, device=dev)
    offs = H.empty(2, E + 1, dtype=torch.int32, device=dev)
    perm = H.empty(2, max(E, 1), dtype=torch.int32, device=dev)
    groups = H.empty(2, 1, dtype=torch.int64, device=dev)
    ws = H.empty(nbytes, dtype=torch.uint8, device=dev)
    order = H.empty(max(E, 1), dtype=torch.int32, device=dev) if jj_order else None
    H.check(H.lib().dpvo_window_group_by(
        H.ptr(ii), H.ptr(jj), H.ptr(kk), E, int(M), int(base), int(ring), int(frames), bits, H.ptr(slots[0]),
        H.ptr(slots[1]), H.ptr(flag), H.ptr(gid[0]), H.ptr(offs[0]), H.ptr(perm[0]), H.ptr(groups[0]), H.ptr(gid[1]),
        H.ptr(offs[1]), H.ptr(perm[1]), H.ptr(groups[1]), H.ptr(order), H.ptr(ws), nbytes, H.stream_of(kk)))
    out = (slots[0], slots[1], (gid[0], offs[0], perm[0], groups[0]), (gid[1], offs[1], perm[1], groups[1]))
    return out + (order[:E],) if jj_order else out


def append_edges(ii, jj, kk, ix, n, M, r):
    """DPVO.__call__'s edge append (dpvo.py:756-769,799-800) in one launch:
    -> (ii, jj, kk) int64 = the old edges, then the forward and backward edges
    of the new frame (n = frame count including it, r = PATCH_LIFETIME)."""
    H.on_gpu(ii, jj, kk, ix)
    ii, jj, kk, ix = H.idx64(ii), H.idx64(jj), H.idx64(kk), H.idx64(ix)
    E = kk.numel()
    if ii.numel() != E or jj.numel() != E:
        raise RuntimeError("append_edges: ii, jj and kk must have the same length")
    add = H.lib().dpvo_append_edges_count(int(n), int(M), int(r))
    if add < 0:
        raise RuntimeError("append_edges: n >= 1, M >= 1 and PATCH_LIFETIME >= 1 required")
    out = H.empty(3, E + add, dtype=torch.int64, device=kk.device)
    H.check(H.lib().dpvo_append_edges(H.ptr(ii), H.ptr(jj), H.ptr(kk), E, H.ptr(ix), int(n), int(M), int(r),
                                      H.ptr(out[0]), H.ptr(out[1]), H.ptr(out[2]), H.stream_of(kk)))
    return out[0], out[1], out[2]


def edge_targets(centre, delta, weight):
    """(centre + delta.float(), weight.float()) for [1, E, 2] views (fp32 centre,
    fp16 delta / weight with unit component stride) in one launch."""
    H.on_gpu(centre, delta, weight)
    E = delta.shape[1]
    if (delta.dtype != torch.float16 or weight.dtype != torch.float16 or centre.dtype != torch.float32 or
            delta.shape != (1, E, 2) or weight.shape != (1, E, 2) or centre.shape != (1, E, 2) or
            delta.stride(2) != 1 or weight.stride(2) != 1):
        raise RuntimeError("edge_targets: centre fp32, delta / weight fp16 [1, E, 2] with unit component stride")
    target = H.empty(1, E, 2, dtype=torch.float32, device=delta.device)
    w32 = H.empty(1, E, 2, dtype=torch.float32, device=delta.device)
    H.check(H.lib().dpvo_edge_targets(H.ptr(delta), delta.stride(1), H.ptr(weight), weight.stride(1), H.ptr(centre),
                                      centre.stride(1), centre.stride(2), E, H.ptr(target), H.ptr(w32),
                                      H.stream_of(delta)))
    return target, w32


def gather_rows(x, idx, dtype=None):
    """out[e] = x[idx[e]] if idx[e] >= 0 else 0, cast to ``dtype`` (default x's).
    x: [R, D] with unit channel stride; idx: [n] int64."""
    H.on_gpu(x, idx)
    if x.dim() != 2 or x.stride(1) != 1:
        raise RuntimeError("gather_rows: x must be [R, D] with contiguous rows")
    dtype = dtype or x.dtype
    idx = H.idx64(idx)
    out = H.empty(idx.numel(), x.shape[1], dtype=dtype, device=x.device)
    H.check(H.lib().dpvo_gather_rows(H.dtype_code(x), H.ptr(x), x.stride(0), x.shape[0], H.ptr(idx), idx.numel(),
                                     x.shape[1], H.dtype_code(out), H.ptr(out), H.stream_of(x)))
    return out


# ---------------------------------------------------------------------------
# full-row fused GEMM (csrc/rowgemm.hip)
# ---------------------------------------------------------------------------
import ctypes as _ct  # noqa: E402

RELU, SIGMOID, RES, GATE, LN, LN_RELU, HEADS, WKB = 1, 2, 4, 8, 16, 32, 64, 128
WIDTH = 384


class RowGemmArgs(_ct.Structure):
    _fields_ = [("A", _ct.c_void_p), ("lda", _ct.c_int64), ("a_idx", _ct.c_void_p), ("a_rows", _ct.c_int64),
                ("W", _ct.c_void_p), ("K", _ct.c_int), ("N", _ct.c_int), ("bias", _ct.c_void_p),
                ("zero_row", _ct.c_void_p), ("M", _ct.c_int64),
                ("res32", _ct.c_void_p), ("ldr", _ct.c_int64), ("res16", _ct.c_void_p), ("res16_idx", _ct.c_void_p),
                ("gate16", _ct.c_void_p),
                ("ln_g", _ct.c_void_p), ("ln_b", _ct.c_void_p), ("ln_eps", _ct.c_float),
                ("head_w", _ct.c_void_p), ("head_b", _ct.c_void_p), ("head_out", _ct.c_void_p),
                ("out32", _ct.c_void_p), ("ldo32", _ct.c_int64), ("out16", _ct.c_void_p), ("ldo16", _ct.c_int64),
                ("flags", _ct.c_int), ("M_dev", _ct.c_void_p)]


class RowAddArgs(_ct.Structure):
    _fields_ = [("a", _ct.c_void_p), ("a_f16", _ct.c_int), ("lda", _ct.c_int64), ("M", _ct.c_int64),
                ("b16", _ct.c_void_p), ("b_idx", _ct.c_void_p), ("b_rows", _ct.c_int64),
                ("ln_g", _ct.c_void_p), ("ln_b", _ct.c_void_p), ("ln_eps", _ct.c_float),
                ("out32", _ct.c_void_p), ("out16", _ct.c_void_p),
                ("c16", _ct.c_void_p), ("c_idx", _ct.c_void_p), ("c_rows", _ct.c_int64)]


_ZEROS = {}


def zero_row(device, K):
    z = _ZEROS.get(device)
    if z is None or z.numel() < K:
        z = torch.zeros(max(K, 4096), dtype=torch.float16, device=device)
        _ZEROS[device] = z
    return z


def pack_linear(weight, bias, kpad=64):
    """nn.Linear(K -> 384) parameters as the kernel's operands: fp16 W [384][Kp]
    (zero columns up to a multiple of 64) and fp16 bias -- what autocast casts them to."""
    n, k = weight.shape
    kp = (k + kpad - 1) // kpad * kpad
    w = torch.zeros(n, kp, dtype=torch.float16, device=weight.device)
    w[:, :k] = weight.detach()
    return w.contiguous(), bias.detach().to(torch.float16).contiguous()


def kblock(W16):
    """[384, Kp] fp16 -> the k-blocked layout dpvo_rowchain reads, [Kp / 32, 384, 32]
    contiguous: every 32-wide k stage of all 384 rows is one contiguous 24 KB
    block, so the kernel's stage loads read whole 128-B lines."""
    if W16.dim() == 3:
        return W16
    n, kp = W16.shape
    if n != WIDTH or kp % 32:
        raise RuntimeError("kblock: W must be [384, Kp] with Kp a multiple of 32")
    return W16.view(n, kp // 32, 32).permute(1, 0, 2).contiguous()


def _kb_K(Wkb):
    """(Kp) of a k-blocked weight; validates the layout"""
    if Wkb.dim() != 3 or Wkb.shape[1] != WIDTH or Wkb.shape[2] != 32 or not Wkb.is_contiguous():
        raise RuntimeError("rowchain: weights must be [384, Kp] or k-blocked [Kp / 32, 384, 32] contiguous")
    return Wkb.shape[0] * 32


def _p(t):
    return t.data_ptr() if t is not None else None


def rowgemm(A, W16, b16, flags=0, a_idx=None, M=None, res32=None, res16=None, res16_idx=None, gate16=None, ln=None,
            heads=None, out32=None, out16=None, want32=False, want16=True, M_dev=None):
    """Y = epilogue(A W^T + b) over 384-wide rows (see include/dpvo_hot.h).
    A: fp16 [R, >=Kp] (row-contiguous); a_idx: optional int64 [M] row gather.
    ln = (gamma f32, beta f32, eps); heads = (W fp16 [4,384], b fp16 [4]).
    Returns (out32, out16, head_out)."""
    H.on_gpu(A, W16, b16)
    if A.dtype != torch.float16 or W16.dtype != torch.float16 or b16.dtype != torch.float16:
        raise RuntimeError("rowgemm: A, W and bias must be fp16")
    if W16.dim() == 3:   # k-blocked W (kblock): the plain-GEMM kernel without LDS-DMA (flags 0 / RELU / SIGMOID)
        if flags & ~(RELU | SIGMOID) or want32 or out32 is not None:
            raise RuntimeError("rowgemm: a k-blocked W takes only RELU / SIGMOID and writes out16")
        Kp = _kb_K(W16)
        flags |= WKB
    elif W16.shape[0] != WIDTH or not W16.is_contiguous():
        raise RuntimeError("rowgemm: W must be [384, Kp] contiguous (or k-blocked)")
    else:
        Kp = W16.shape[1]
    if A.dim() != 2 or A.stride(1) != 1:
        raise RuntimeError("rowgemm: A must be [rows, K] row-contiguous")
    if A.stride(0) < Kp:
        raise RuntimeError(f"rowgemm: A's row stride {A.stride(0)} < padded K {Kp}")
    dev = A.device
    if a_idx is not None:
        a_idx = H.idx64(a_idx)
        M = a_idx.numel()
    elif M is None:
        M = A.shape[0]
    if want32 and out32 is None:
        out32 = H.empty(M, WIDTH, dtype=torch.float32, device=dev)
    if want16 and out16 is None:
        out16 = H.empty(M, WIDTH, dtype=torch.float16, device=dev)
    head_out = H.empty(M, 4, dtype=torch.float16, device=dev) if heads is not None else None
    if res16_idx is not None:
        res16_idx = H.idx64(res16_idx)
    a = RowGemmArgs()
    a.A, a.lda, a.a_idx, a.a_rows = _p(A), A.stride(0), _p(a_idx), A.shape[0]
    a.W, a.K, a.N, a.bias, a.zero_row = _p(W16), Kp, WIDTH, _p(b16), _p(zero_row(dev, Kp))
    a.M = M
    a.res32, a.ldr = _p(res32), (res32.stride(0) if res32 is not None else 0)
    a.res16, a.res16_idx, a.gate16 = _p(res16), _p(res16_idx), _p(gate16)
    if ln is not None:
        a.ln_g, a.ln_b, a.ln_eps = _p(ln[0]), _p(ln[1]), float(ln[2])
    if heads is not None:
        a.head_w, a.head_b, a.head_out = _p(heads[0]), _p(heads[1]), _p(head_out)
    a.out32, a.ldo32 = _p(out32), (out32.stride(0) if out32 is not None else 0)
    a.out16, a.ldo16 = _p(out16), (out16.stride(0) if out16 is not None else 0)
    a.flags = int(flags)
    if M_dev is not None:
        if M_dev.dtype != torch.int64 or not M_dev.is_cuda:
            raise RuntimeError("rowgemm: M_dev must be a device int64 scalar")
        a.M_dev = M_dev.data_ptr()
    for t, nm in ((res32, "res32"), (out32, "out32")):
        if t is not None and (t.dtype != torch.float32 or t.stride(1) != 1):
            raise RuntimeError(f"rowgemm: {nm} must be fp32 with contiguous rows")
    for t, nm in ((res16, "res16"), (gate16, "gate16")):
        if t is not None and (t.dtype != torch.float16 or not t.is_contiguous() or t.shape[-1] != WIDTH):
            raise RuntimeError(f"rowgemm: {nm} must be contiguous fp16 [*, 384]")
    H.check(H.lib().dpvo_rowgemm(_ct.byref(a), H.stream_of(A)))
    return out32, out16, head_out


def rowgemm_pair(A, Wa, ba, Wb, bb, M_dev=None):
    """(A Wa^T + ba, A Wb^T + bb) as fp16 [M, 384] each, one launch sharing A
    (dpvo_rowgemm_pair: SoftAgg's f and g)."""
    H.on_gpu(A, Wa, ba, Wb, bb)
    if any(t.dtype != torch.float16 for t in (A, Wa, ba, Wb, bb)):
        raise RuntimeError("rowgemm_pair: A, weights and biases must be fp16")
    if Wa.shape != Wb.shape or not (Wa.is_contiguous() and Wb.is_contiguous()):
        raise RuntimeError("rowgemm_pair: Wa and Wb must be contiguous, of one shape")
    kb = Wa.dim() == 3   # k-blocked (kblock): the plain-GEMM kernel without LDS-DMA
    Kp = _kb_K(Wa) if kb else Wa.shape[1]
    if not kb and Wa.shape[0] != WIDTH:
        raise RuntimeError("rowgemm_pair: Wa and Wb must be [384, Kp] or k-blocked")
    if A.dim() != 2 or A.stride(1) != 1 or A.stride(0) < Kp:
        raise RuntimeError("rowgemm_pair: A must be [rows, >=Kp] row-contiguous")
    M, dev = A.shape[0], A.device
    outs = []
    args = []
    for W, b in ((Wa, ba), (Wb, bb)):
        o = H.empty(M, WIDTH, dtype=torch.float16, device=dev)
        a = RowGemmArgs()
        a.A, a.lda, a.a_idx, a.a_rows = _p(A), A.stride(0), None, M
        a.W, a.K, a.N, a.bias, a.zero_row = _p(W), Kp, WIDTH, _p(b), _p(zero_row(dev, Kp))
        a.M, a.flags = M, WKB if kb else 0
        a.out16, a.ldo16 = _p(o), o.stride(0)
        if M_dev is not None:
            if M_dev.dtype != torch.int64 or not M_dev.is_cuda:
                raise RuntimeError("rowgemm_pair: M_dev must be a device int64 scalar")
            a.M_dev = M_dev.data_ptr()
        outs.append(o)
        args.append(a)
    H.check(H.lib().dpvo_rowgemm_pair(_ct.byref(args[0]), _ct.byref(args[1]), H.stream_of(A)))
    return outs[0], outs[1]


def rowgemm_pair_pre(a32, b16, b_idx, Wa, ba, Wb, bb, b_rows=None):
    """rowgemm_pair(rowadd_ln(a32, b16, b_idx, want32=False)[1], Wa, ba, Wb, bb)
    in one launch (dpvo_rowgemm_pair_pre): the A rows fp16(a32 + b16[b_idx])
    are formed as the GEMM stages them -- the same bits, without the fp16 rows
    in HBM.  Wa / Wb k-blocked [12, 384, 32] (K = 384)."""
    H.on_gpu(a32, b16, b_idx, Wa, ba, Wb, bb)
    if a32.dtype != torch.float32 or a32.dim() != 2 or a32.shape[1] != WIDTH or a32.stride(1) != 1:
        raise RuntimeError("rowgemm_pair_pre: a32 must be fp32 [M, 384] row-contiguous")
    if b16.dtype != torch.float16 or b16.dim() != 2 or b16.shape[1] != WIDTH or not b16.is_contiguous():
        raise RuntimeError("rowgemm_pair_pre: b16 must be fp16 [G, 384] contiguous")
    if b_idx.dtype != torch.int64 or b_idx.numel() < a32.shape[0]:
        raise RuntimeError("rowgemm_pair_pre: b_idx must be int64 with one entry per row")
    if any(t.dtype != torch.float16 for t in (Wa, ba, Wb, bb)) or Wa.dim() != 3 or Wb.shape != Wa.shape:
        raise RuntimeError("rowgemm_pair_pre: k-blocked fp16 weights and fp16 biases")
    Kp = _kb_K(Wa)
    M, dev = a32.shape[0], a32.device
    outs, args = [], []
    for W, b in ((Wa, ba), (Wb, bb)):
        o = H.empty(M, WIDTH, dtype=torch.float16, device=dev)
        a = RowGemmArgs()
        z = _p(zero_row(dev, Kp))
        a.A, a.lda, a.a_idx, a.a_rows = z, Kp, None, M   # (A unused: the rows are pre's)
        a.W, a.K, a.N, a.bias, a.zero_row = _p(W), Kp, WIDTH, _p(b), z
        a.M, a.flags = M, WKB
        a.out16, a.ldo16 = _p(o), o.stride(0)
        outs.append(o)
        args.append(a)
    pre = RowAddArgs()
    pre.a, pre.a_f16, pre.lda, pre.M = _p(a32), 0, a32.stride(0), M
    pre.b16, pre.b_idx, pre.b_rows = _p(b16), _p(b_idx), b16.shape[0] if b_rows is None else b_rows
    H.check(H.lib().dpvo_rowgemm_pair_pre(_ct.byref(args[0]), _ct.byref(args[1]), _ct.byref(pre), H.stream_of(a32)))
    return outs[0], outs[1]


def rowadd_ln(a, b16=None, b_idx=None, ln=None, want32=True, want16=True, c16=None, c_idx=None):
    """v = a (+ b16[b_idx]) (+ c16[c_idx]) [-> LayerNorm] over 384-wide rows ->
    (out32, out16).  The second addend is the next row add, in order: one call
    with c16 is bit-identical to rowadd_ln(a, b16, b_idx)[0] fed to
    rowadd_ln(., c16, c_idx, ln), without the fp32 rows in between."""
    H.on_gpu(a)
    if a.dim() != 2 or a.shape[1] != WIDTH or a.stride(1) != 1 or a.dtype not in (torch.float16, torch.float32):
        raise RuntimeError("rowadd_ln: a must be [M, 384] fp16/fp32 with contiguous rows")
    M, dev = a.shape[0], a.device
    out32 = H.empty(M, WIDTH, dtype=torch.float32, device=dev) if want32 else None
    out16 = H.empty(M, WIDTH, dtype=torch.float16, device=dev) if want16 else None
    if b_idx is not None:
        b_idx = H.idx64(b_idx)
    args = RowAddArgs()
    args.a, args.a_f16, args.lda, args.M = _p(a), int(a.dtype == torch.float16), a.stride(0), M
    if b16 is not None:
        if b16.dtype != torch.float16 or not b16.is_contiguous():
            raise RuntimeError("rowadd_ln: b16 must be contiguous fp16 [*, 384]")
        args.b16, args.b_idx, args.b_rows = _p(b16), _p(b_idx), b16.shape[0]
    if c16 is not None:
        if b16 is None or c16.dtype != torch.float16 or not c16.is_contiguous():
            raise RuntimeError("rowadd_ln: c16 must be contiguous fp16 [*, 384] and follow b16")
        if c_idx is not None:
            c_idx = H.idx64(c_idx)
        args.c16, args.c_idx, args.c_rows = _p(c16), _p(c_idx), c16.shape[0]
    if ln is not None:
        args.ln_g, args.ln_b, args.ln_eps = _p(ln[0]), _p(ln[1]), float(ln[2])
    args.out32, args.out16 = _p(out32), _p(out16)
    H.check(H.lib().dpvo_rowadd_ln(_ct.byref(args), H.stream_of(a)))
    return out32, out16


SCATTER_SUM, SCATTER_MEAN, SCATTER_MAX, SCATTER_SOFTMAX = 0, 1, 2, 3


def scatter_csr(op, src3, index, csr, out, out_rows=0, argmax=None, eps=1e-12):
    """dpvo_scatter_csr: src3 [outer, E, inner] contiguous, index [E] int64,
    csr = group_by(index); out [outer, out_rows, inner] (sum / mean / max,
    written only at keys with members) or shaped like src3 (softmax)."""
    H.on_gpu(src3, index, out)
    gid, offs, perm, groups = csr
    outer, E, inner = src3.shape
    H.check(H.lib().dpvo_scatter_csr(int(op), H.dtype_code(src3), H.ptr(src3), outer, E, inner, H.ptr(index),
                                     H.ptr(offs), H.ptr(perm), H.ptr(groups), E, float(eps), H.ptr(out),
                                     int(out_rows), H.ptr(argmax) if argmax is not None else None,
                                     H.stream_of(src3)))
    return out
