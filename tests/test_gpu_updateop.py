"""Native update-operator glue (csrc/updateop.hip) against the oracle:
SoftAgg's grouped softmax-sum (torch_scatter scatter_softmax + scatter_sum,
reference dpvo/blocks.py:40-48) and the masked neighbour gather
(dpvo/net.py:82-85)."""
import numpy as np
import pytest
import torch

from oracle import oracle
from tests_helpers import same

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("poisoned")]


def _case(E, G, D, dtype, seed, empty=()):
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, G, (E,), generator=g)
    for k in empty:
        labels[labels == k] = (k + 1) % G
    f = torch.randn(E, D, generator=g) * 2
    s = torch.randn(E, D, generator=g) * 3
    return f.to(dtype), s.to(dtype), labels


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.float16, 2e-3), (torch.float64, 2e-5)])
@pytest.mark.parametrize("E,G,D", [(1000, 37, 384), (4096, 5, 256), (333, 333, 130), (64, 1, 2)])
def test_softagg_matches_oracle(dtype, tol, E, G, D):
    import update_ops
    f, s, lab = _case(E, G, D, dtype, seed=E + G + D)
    y = update_ops.softagg(f.cuda(), s.cuda(), lab.cuda(), G).cpu().double().numpy()
    want = oracle.softagg(f.double().numpy(), s.double().numpy(), lab.numpy(), G)
    np.testing.assert_allclose(y, want, rtol=tol, atol=tol)


def test_softagg_large_group_and_empty_groups():
    """A group above the LDS sort cap (arrival order) and groups with no edges (y = 0)."""
    import update_ops
    E, G, D = 5000, 6, 128
    f, s, _ = _case(E, G, D, torch.float32, seed=3)
    lab = torch.zeros(E, dtype=torch.int64)
    lab[:700] = 2
    lab[4000:] = 5          # groups 1, 3, 4 empty; group 0 has 3300 edges > cap
    y = update_ops.softagg(f.cuda(), s.cuda(), lab.cuda(), G).cpu().double().numpy()
    want = oracle.softagg(f.double().numpy(), s.double().numpy(), lab.numpy(), G)
    np.testing.assert_allclose(y, want, rtol=1e-4, atol=1e-5)
    assert (y[[1, 3, 4]] == 0).all()


def test_softagg_strided_halves_and_determinism():
    """f|s as the two halves of one fused [E, 2D] GEMM output; repeated runs are bit-identical."""
    import update_ops
    E, G, D = 20000, 900, 384
    fs = torch.randn(E, 2 * D, device="cuda").half()
    lab = torch.randint(0, G, (E,), device="cuda")
    a = update_ops.softagg(fs[:, :D], fs[:, D:], lab, G)
    b = update_ops.softagg(fs[:, :D], fs[:, D:], lab, G)
    assert same(a, b)
    want = oracle.softagg(fs[:, :D].double().cpu().numpy(), fs[:, D:].double().cpu().numpy(), lab.cpu().numpy(), G)
    np.testing.assert_allclose(a.double().cpu().numpy(), want, rtol=2e-3, atol=2e-3)


def test_softagg_module_native_vs_torch_composition():
    """dpvo.blocks.SoftAgg: the inference (native) path equals the autograd (torch) path."""
    from dpvo.blocks import SoftAgg
    torch.manual_seed(0)
    m = SoftAgg(384).cuda()
    x = torch.randn(1, 3000, 384, device="cuda")
    key = torch.randint(0, 50, (3000,), device="cuda") * 12345 + 7
    with torch.no_grad():
        native = m(x, key)
    xr = x.clone().requires_grad_(True)
    ref = m(xr, key)
    torch.testing.assert_close(native, ref.detach(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float16), (torch.float16, torch.float16),
                                          (torch.float32, torch.float32), (torch.float64, torch.float32)])
def test_gather_rows(in_dt, out_dt):
    import update_ops
    g = torch.Generator().manual_seed(1)
    x = torch.randn(500, 384, generator=g).to(in_dt)
    idx = torch.randint(-1, 500, (2000,), generator=g)
    out = update_ops.gather_rows(x.cuda(), idx.cuda(), dtype=out_dt).cpu()
    want = torch.from_numpy(oracle.gather_rows(x.numpy(), idx.numpy())).to(out_dt)
    assert same(out, want)


def test_errors():
    import update_ops
    x = torch.randn(10, 3, device="cuda")
    with pytest.raises(RuntimeError):
        update_ops.gather_rows(x, torch.zeros(4, dtype=torch.int64, device="cuda"))  # odd D
    with pytest.raises(RuntimeError):
        update_ops.softagg(x.cpu(), x.cpu(), torch.zeros(10, dtype=torch.int64), 1)


@pytest.mark.parametrize("n,hi", [(1, 5), (1000, 40), (95424, 4416 * 5), (5000, 2 ** 31 - 1)])
def test_group_by_matches_torch_unique(n, hi):
    """Device group-by == torch.unique(return_inverse=True); CSR lists each group's edges ascending."""
    import update_ops
    key = torch.randint(0, hi, (n,), device="cuda")
    gid, offs, perm, G = update_ops.group_by(key)
    uniq, inv = torch.unique(key, return_inverse=True)
    assert int(G.item()) == uniq.numel()
    assert same(gid, inv)
    g = int(G.item())
    offs, perm = offs[: g + 1].long().cpu(), perm.long().cpu()
    assert offs[0] == 0 and offs[-1] == n
    inv_c = inv.cpu()
    for k in range(0, g, max(1, g // 50)):
        members = perm[offs[k]: offs[k + 1]]
        assert (members[1:] > members[:-1]).all()
        assert (inv_c[members] == k).all()


@pytest.mark.parametrize("n,bits,distinct", [(1, 1, 1), (1000, 6, 40), (95424, 19, 4416), (95424, 22, 600),
                                             (20000, 12, 8), (5000, 22, 5000)])
def test_group_by_counting_sort_equals_radix(n, bits, distinct):
    """key_bits <= 22 takes the counting-sort path: outputs identical to the
    stable radix-sort path (groups of 1 .. ~7000 members, > 64 and <= 64)."""
    import update_ops
    g = torch.Generator(device="cuda").manual_seed(n + bits)
    vals = torch.randint(0, 2 ** bits, (distinct,), device="cuda", generator=g)
    key = vals[torch.randint(0, distinct, (n,), device="cuda", generator=g)]
    a = update_ops.group_by(key, key_bits=bits)
    b = update_ops.group_by(key, key_bits=bits, radix=True)
    G = int(a[3].item())
    assert same(a[3], b[3]) and same(a[0], b[0]) and same(a[2], b[2])
    assert same(a[1][:G + 1], b[1][:G + 1])   # entries past G are unspecified
    uniq, inv = torch.unique(key, return_inverse=True)
    assert int(a[3].item()) == uniq.numel() and same(a[0], inv)


def test_group_by_counting_sort_runs_of_equal_keys():
    """Runs of equal keys (the tracker's edge blocks): one atomic per run in a
    wave; runs crossing wave and block boundaries, a partial last wave."""
    import update_ops
    g = torch.Generator(device="cuda").manual_seed(9)
    runs = torch.randint(1, 300, (700,), device="cuda", generator=g)
    vals = torch.randint(0, 2 ** 16, (700,), device="cuda", generator=g)
    key = torch.repeat_interleave(vals, runs)[:100001]
    a = update_ops.group_by(key, key_bits=16)
    b = update_ops.group_by(key, key_bits=16, radix=True)
    G = int(a[3].item())
    assert same(a[0], b[0]) and same(a[2], b[2]) and same(a[1][:G + 1], b[1][:G + 1])


def test_group_by_empty():
    import update_ops
    gid, offs, perm, G = update_ops.group_by(torch.zeros(0, dtype=torch.int64, device="cuda"))
    assert int(G.item()) == 0 and gid.numel() == 0
    gid, offs, perm, G = update_ops.group_by(torch.zeros(0, dtype=torch.int64, device="cuda"), key_bits=12)
    assert int(G.item()) == 0 and gid.numel() == 0


def test_softagg_csr_matches_oracle_and_dense_path():
    import update_ops
    E, D = 20000, 384
    fs = torch.randn(E, 2 * D, device="cuda").half()
    key = torch.randint(0, 3000, (E,), device="cuda") * 12345 + 11
    gid, offs, perm, G = update_ops.group_by(key)
    g = int(G.item())
    y = update_ops.softagg_csr(fs[:, :D], fs[:, D:], offs, perm, G, E)[:g]
    want = oracle.softagg(fs[:, :D].double().cpu().numpy(), fs[:, D:].double().cpu().numpy(), gid.cpu().numpy(), g)
    np.testing.assert_allclose(y.double().cpu().numpy(), want, rtol=2e-3, atol=2e-3)
    dense = update_ops.softagg(fs[:, :D], fs[:, D:], gid, g)
    assert same(y, dense)   # same ascending order, same arithmetic


def test_rowgemm_device_row_count():
    """rowgemm with M read on the device: rows past *M_dev are left untouched."""
    import update_ops as U
    A = torch.randn(1000, 384, device="cuda").half()
    W16, b16 = U.pack_linear(torch.randn(384, 384, device="cuda") * 0.05, torch.randn(384, device="cuda") * 0.1)
    out = torch.full((1000, 384), 7.0, device="cuda").half()
    U.rowgemm(A, W16, b16, out16=out, M_dev=torch.tensor([300], device="cuda"))
    _, ref, _ = U.rowgemm(A, W16, b16)
    assert same(out[:300], ref[:300])
    assert (out[300:] == 7.0).all()


def test_edge_targets_equal_torch_composition():
    """update_ops.edge_targets == coords[..., 1, 1] + delta.float(), weight.float()
    (dpvo.py:724-727) bit for bit, on strided head views like the fused operator's."""
    import update_ops
    E = 5000
    g = torch.Generator(device="cpu").manual_seed(0)
    heads = (torch.randn(E, 4, generator=g) * 3).half().cuda()
    coords = (torch.randn(1, E, 2, 3, 3, generator=g) * 100).cuda()
    delta, weight = heads[None, :, :2], heads[None, :, 2:]
    centre = coords[..., 1, 1]
    t, w = update_ops.edge_targets(centre, delta, weight)
    assert same(t, centre + delta.float()) and same(w, weight.float())


@pytest.mark.parametrize("ngroups", [50, 3000])
def test_softagg_csr_long_groups(ngroups):
    """softagg_csr(long_groups=True) (groups >= 64 edges split over four waves,
    states merged in a fixed order): within the fp16 bar of the oracle,
    repeatable bit for bit, and equal to the default kernel for short groups."""
    import update_ops
    E, D = 20000, 384
    fs = torch.randn(E, 2 * D, device="cuda").half()
    key = torch.randint(0, ngroups, (E,), device="cuda") * 12345 + 11
    gid, offs, perm, G = update_ops.group_by(key)
    g = int(G.item())
    y = update_ops.softagg_csr(fs[:, :D], fs[:, D:], offs, perm, G, E, long_groups=True)[:g]
    y2 = update_ops.softagg_csr(fs[:, :D], fs[:, D:], offs, perm, G, E, long_groups=True)[:g]
    assert same(y, y2)
    want = oracle.softagg(fs[:, :D].double().cpu().numpy(), fs[:, D:].double().cpu().numpy(), gid.cpu().numpy(), g)
    np.testing.assert_allclose(y.double().cpu().numpy(), want, rtol=2e-3, atol=2e-3)
    if ngroups == 3000:   # ~7 edges per group: the unsplit arithmetic
        assert same(y, update_ops.softagg_csr(fs[:, :D], fs[:, D:], offs, perm, G, E)[:g])
