"""The drop-in ``torch_scatter`` module (wild-video-3d-reconstruction_amd/
torch_scatter.py over dpvo_scatter_csr) with torch-scatter 2.1.2 semantics,
as the reference calls it: SoftAgg (blocks.py:40-48), the Python BA's
scatter_sum (ba.py:40-56) and loop closure's scatter_max (long_term.py:134).
Checked against the numpy oracle (oracle.softagg) and ATen compositions."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _shim():
    import torch_scatter
    assert os.path.basename(os.path.dirname(torch_scatter.__file__)) == "wild-video-3d-reconstruction_amd"
    return torch_scatter


def test_softagg_through_the_shim_matches_oracle():
    """blocks.py:41-43 verbatim: unique -> scatter_softmax -> scatter_sum (dim=1)"""
    from oracle import oracle
    ts = _shim()
    g = torch.Generator().manual_seed(0)
    E, D = 3000, 384
    key = torch.randint(0, 400, (E,), generator=g) * 7 + 3
    gx, fx = torch.randn(1, E, D, generator=g), torch.randn(1, E, D, generator=g)
    _, jx = torch.unique(key, return_inverse=True)
    G = int(jx.max()) + 1
    w = ts.scatter_softmax(gx.cuda(), jx.cuda(), dim=1)
    y = ts.scatter_sum(fx.cuda() * w, jx.cuda(), dim=1)
    assert y.shape == (1, G, D) and w.shape == (1, E, D)
    ref = oracle.softagg(fx[0].numpy(), gx[0].numpy(), jx.numpy(), G)
    np.testing.assert_allclose(y[0].cpu().numpy(), ref, rtol=2e-5, atol=2e-5)
    # the softmax weights sum to 1 per group and channel
    wsum = torch.zeros(G, D, dtype=torch.float64).index_add_(0, jx, w[0].double().cpu())
    np.testing.assert_allclose(wsum.numpy(), 1.0, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.float16])
def test_scatter_sum_mean(dtype):
    ts = _shim()
    g = torch.Generator().manual_seed(1)
    E = 5000
    src = torch.randn(2, E, 6, 6, generator=g).to(dtype)
    idx = torch.randint(0, 90, (E,), generator=g)
    out = ts.scatter_sum(src.cuda(), idx.cuda(), dim=1, dim_size=100)
    want = torch.zeros(2, 100, 6, 6, dtype=torch.float64).index_add_(1, idx, src.double())
    tol = 5e-2 if dtype == torch.float16 else 1e-4
    np.testing.assert_allclose(out.double().cpu().numpy(), want.numpy(), rtol=tol, atol=tol)
    assert out.dtype == dtype and out.shape == (2, 100, 6, 6)
    cnt = torch.zeros(100, dtype=torch.float64).index_add_(0, idx, torch.ones(E, dtype=torch.float64)).clamp(min=1)
    mean = ts.scatter_mean(src.cuda(), idx.cuda(), dim=1, dim_size=100)
    np.testing.assert_allclose(mean.double().cpu().numpy(), (want / cnt.view(1, -1, 1, 1)).numpy(), rtol=tol, atol=tol)
    # out= accumulates, the default dim_size is index.max() + 1, scatter_add is scatter_sum
    acc = torch.ones(2, 100, 6, 6, dtype=dtype, device="cuda")
    ts.scatter_add(src.cuda(), idx.cuda(), dim=1, out=acc)
    np.testing.assert_allclose(acc.double().cpu().numpy(), want.numpy() + 1, rtol=tol, atol=tol)
    assert ts.scatter_sum(src.cuda(), idx.cuda(), dim=1).shape[1] == int(idx.max()) + 1


def test_ba_py_scatter_pattern():
    """ba.py:40-42 safe_scatter_add_mat: [1, E, 6, 6] blocks into n*m keys"""
    ts = _shim()
    g = torch.Generator().manual_seed(2)
    E, n = 4000, 12
    A = torch.randn(1, E, 6, 6, generator=g)
    ii, jj = torch.randint(0, n, (E,), generator=g), torch.randint(0, n, (E,), generator=g)
    v = (ii >= 0) & (jj >= 0)
    out = ts.scatter_sum(A[:, v].cuda(), (ii[v] * n + jj[v]).cuda(), dim=1, dim_size=n * n)
    want = torch.zeros(1, n * n, 6, 6, dtype=torch.float64).index_add_(1, ii * n + jj, A.double())
    np.testing.assert_allclose(out.double().cpu().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


def test_scatter_max():
    """long_term.py:134: scatter_max(residual, kk)[0]"""
    ts = _shim()
    g = torch.Generator().manual_seed(3)
    E = 2000
    src = torch.randn(E, generator=g)
    idx = torch.randint(0, 300, (E,), generator=g) * 2          # odd rows stay empty
    val, arg = ts.scatter_max(src.cuda(), idx.cuda())
    S = int(idx.max()) + 1
    want = torch.full((S,), -float("inf")).scatter_reduce(0, idx, src, "amax")
    present = torch.zeros(S, dtype=torch.bool)
    present[idx] = True
    want[~present] = 0
    np.testing.assert_array_equal(val.cpu().numpy(), want.numpy())
    a = arg.cpu()
    assert (a[~present] == E).all()
    assert torch.equal(src[a[present]], want[present]) and torch.equal(idx[a[present]], torch.nonzero(present)[:, 0])


def test_group_by_large_groups_counting_sort():
    """a counting-sort group-by (key_bits <= 22) with groups far beyond the
    fix-up kernel's LDS capacity stays ordered and fast"""
    import update_ops as U
    g = torch.Generator().manual_seed(4)
    n = 200_000
    key = torch.where(torch.rand(n, generator=g) < 0.7, torch.zeros(n, dtype=torch.long),
                      torch.randint(0, 1000, (n,), generator=g)).cuda()
    gid, offs, perm, groups = U.group_by(key, key_bits=10)
    torch.cuda.synchronize()
    G = int(groups)
    uniq, inv = torch.unique(key.cpu(), return_inverse=True)
    assert G == uniq.numel() and torch.equal(gid.cpu(), inv)
    o, p = offs[:G + 1].cpu().long(), perm[:n].cpu().long()
    for gg in (0, 1, G - 1):
        members = p[o[gg]:o[gg + 1]]
        assert torch.equal(members, torch.nonzero(inv == gg)[:, 0])


def test_out_of_range_index_raises_like_torch_scatter():
    """torch-scatter 2.1.2 fails on an index outside the output:
    no member is dropped silently."""
    ts = _shim()
    src = torch.randn(10, 4, device="cuda")
    idx = torch.arange(10, device="cuda")
    with pytest.raises(IndexError):
        ts.scatter_sum(src, idx, dim=0, dim_size=5)
    with pytest.raises(IndexError):
        ts.scatter_mean(src, idx, dim=0, out=torch.zeros(9, 4, device="cuda"))
    with pytest.raises(IndexError):
        ts.scatter_max(src, idx - 1, dim=0)
    with pytest.raises(IndexError):
        ts.scatter_softmax(src, idx - 3, dim=0)
    assert ts.scatter_sum(src, idx, dim=0, dim_size=10).shape == (10, 4)
