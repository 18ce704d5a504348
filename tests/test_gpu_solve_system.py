"""cuda_ba.solve_system (loop-closure PGO normal equations, reference
dpvo/fastba/ba.cpp:174-234) against the float64 oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def _pgo_case(n, loops, seed):
    g = np.random.default_rng(seed)
    ii = list(range(n - 1)) + list(g.integers(0, n // 2, loops))
    jj = list(range(1, n)) + list(g.integers(n // 2 + 1, n, loops))
    r = len(ii)
    Ji = g.normal(size=(r, 7, 7)).astype(np.float32)
    Jj = g.normal(size=(r, 7, 7)).astype(np.float32)
    res = g.normal(size=(r, 7)).astype(np.float32) * 0.1
    return Ji, Jj, np.array(ii), np.array(jj), res


@pytest.mark.parametrize("n,loops,freen", [(12, 3, -1), (40, 10, -1), (40, 10, 25), (200, 30, -1)])
def test_solve_system_matches_oracle(n, loops, freen):
    import cuda_ba
    Ji, Jj, ii, jj, res = _pgo_case(n, loops, seed=n + loops)
    ep, lm = 1e-4, 1e-3
    want = oracle.solve_system(Ji, Jj, ii, jj, res, ep, lm, freen)
    t = lambda a: torch.from_numpy(a).cuda()
    got, = cuda_ba.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), ep, lm, freen)
    assert got.shape == (n, 7) and got.device.type == "cuda"
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-4, atol=1e-5)
    if freen >= 0:
        assert (got[freen:] == 0).all()


def test_solve_system_self_edge_raises():
    import cuda_ba
    Ji, Jj, ii, jj, res = _pgo_case(10, 0, seed=1)
    ii[3] = jj[3]
    t = lambda a: torch.from_numpy(a).cuda()
    with pytest.raises(RuntimeError):
        cuda_ba.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), 1e-4, 1e-3, -1)


def test_solve_system_accepts_host_tensors():
    """The reference copies its inputs to the host and returns on res.device
    (ba.cpp:153-234); PGO may hand CPU tensors (optim_utils.py:222-255)."""
    import cuda_ba
    Ji, Jj, ii, jj, res = _pgo_case(30, 6, seed=5)
    want = oracle.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-3, -1)
    t = torch.from_numpy
    got, = cuda_ba.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), 1e-4, 1e-3, -1)
    assert got.device.type == "cpu" and got.shape == (30, 7)
    np.testing.assert_allclose(got.numpy(), want, rtol=1e-4, atol=1e-5)
    # mixed placement: Jacobians on the host, residuals on the GPU -> result on the GPU
    got2, = cuda_ba.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res).cuda(), 1e-4, 1e-3, -1)
    assert got2.device.type == "cuda"
    np.testing.assert_allclose(got2.cpu().numpy(), want, rtol=1e-4, atol=1e-5)
