"""lietorch_backends (SO3 / RxSO3 / SE3 / Sim3) on the GPU vs the oracle,
golden vectors and finite differences (the reference's run_tests.py
strategy, restated)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu
GROUPS = {"SO3": (1, 3, 4), "RxSO3": (2, 4, 5), "SE3": (3, 6, 7), "Sim3": (4, 7, 8)}


def rand_group(gid, K, n, g, scale=0.8):
    return oracle.lie_forward("exp", gid, scale * g.standard_normal((n, K)))


def cu(a, dt=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0", dt)


@pytest.mark.parametrize("name", list(GROUPS))
@pytest.mark.parametrize("dt,tol", [(torch.float64, 1e-10), (torch.float32, 2e-5)])
def test_forward_ops_match_oracle(name, dt, tol):
    import lietorch_backends as LB
    gid, K, N = GROUPS[name]
    g = np.random.default_rng(0)
    n = 1000
    a = 0.9 * g.standard_normal((n, K))
    a[:5] *= 1e-8  # small-angle branches
    if K in (4, 7):
        a[5:10, -1] = 0.0  # sigma = 0 branches of calcW (RxSO3 / Sim3)
        a[10:15, K - 4:K - 1] *= 1e-9  # rotation-free, scaled
    X, Y = rand_group(gid, K, n, g), rand_group(gid, K, n, g)
    X[:7] *= 3.0  # un-normalised quaternions are normalised on load
    p3, p4, t = g.standard_normal((n, 3)), g.standard_normal((n, 4)), g.standard_normal((n, K))
    cases = [("exp", LB.expm, (a,), None), ("log", LB.logm, (X,), None), ("inv", LB.inv, (X,), None),
             ("mul", LB.mul, (X, Y), Y), ("adj", LB.adj, (X, t), t), ("adjT", LB.adjT, (X, t), t),
             ("act", LB.act, (X, p3), p3), ("act4", LB.act4, (X, p4), p4), ("matrix", LB.as_matrix, (X,), None),
             ("projector", LB.projector, (X,), None), ("Jinv", LB.Jinv, (X, t), t)]
    for op, fn, args, Yarg in cases:
        got = fn(gid, *[cu(x, dt) for x in args]).cpu().double().numpy()
        ref = oracle.lie_forward(op, gid, args[0], Yarg)
        np.testing.assert_allclose(got, ref, rtol=tol, atol=tol, err_msg=f"{name}.{op}")


def numeric_jacobian(f, x0, h=1e-6):
    cols = []
    for k in range(len(x0)):
        e = np.zeros_like(x0); e[k] = h
        cols.append((f(x0 + e) - f(x0 - e)) / (2 * h))
    return np.stack(cols, -1)


@pytest.mark.parametrize("name", list(GROUPS))
def test_backward_ops_finite_differences(name):
    """Analytic backward vs central differences of the oracle's forward.  Sim3's
    left Jacobian (sim3.h) is a series cut after X^4/120 -- its 1/720 term
    sits after the statement's semicolon -- and its inverse after X^4/720, so
    for Sim3 exp/log the bar is the reference's own run_tests tol 1e-3 at
    0.2-scale tangents (test_exp_log_grad)."""
    import lietorch_backends as LB
    gid, K, N = GROUPS[name]
    g = np.random.default_rng(1)
    L = lambda op, X, Y=None: oracle.lie_forward(op, gid, X[None] if X.ndim == 1 else X,
                                                 None if Y is None else (Y[None] if Y.ndim == 1 else Y))[0]
    left = lambda d, X: L("mul", L("exp", d), X)                    # X <- Exp(d) X
    glog = lambda Z, Z0: L("log", L("mul", Z, L("inv", Z0)))       # left tangent of a group output
    for trial in range(4):
        X, Y = rand_group(gid, K, 1, g)[0], rand_group(gid, K, 1, g)[0]
        a, t = (0.2 if name == "Sim3" else 0.7) * g.standard_normal(K), g.standard_normal(K)
        if name == "Sim3":
            X = rand_group(gid, K, 1, g, scale=0.2)[0]
        p3, p4 = g.standard_normal(3), g.standard_normal(4)
        z = np.zeros(K)
        checks = {
            "exp": (lambda gk: LB.expm_backward(gid, gk, cu(a[None])),
                    [numeric_jacobian(lambda v: glog(L("exp", v), L("exp", a)), a)], K),
            "log": (lambda gk: LB.logm_backward(gid, gk, cu(X[None])),
                    [numeric_jacobian(lambda d: L("log", left(d, X)), z)], K),
            "inv": (lambda gk: LB.inv_backward(gid, gk, cu(X[None])),
                    [numeric_jacobian(lambda d: glog(L("inv", left(d, X)), L("inv", X)), z)], K),
            "mul": (lambda gk: LB.mul_backward(gid, gk, cu(X[None]), cu(Y[None])),
                    [numeric_jacobian(lambda d: glog(L("mul", left(d, X), Y), L("mul", X, Y)), z),
                     numeric_jacobian(lambda d: glog(L("mul", X, left(d, Y)), L("mul", X, Y)), z)], K),
            "adj": (lambda gk: LB.adj_backward(gid, gk, cu(X[None]), cu(t[None])),
                    [numeric_jacobian(lambda d: L("adj", left(d, X), t), z),
                     numeric_jacobian(lambda v: L("adj", X, v), t)], K),
            "adjT": (lambda gk: LB.adjT_backward(gid, gk, cu(X[None]), cu(t[None])),
                     [numeric_jacobian(lambda d: L("adjT", left(d, X), t), z),
                      numeric_jacobian(lambda v: L("adjT", X, v), t)], K),
            "act": (lambda gk: LB.act_backward(gid, gk, cu(X[None]), cu(p3[None])),
                    [numeric_jacobian(lambda d: L("act", left(d, X), p3), z),
                     numeric_jacobian(lambda v: L("act", X, v), p3)], 3),
            "act4": (lambda gk: LB.act4_backward(gid, gk, cu(X[None]), cu(p4[None])),
                     [numeric_jacobian(lambda d: L("act4", left(d, X), p4), z),
                      numeric_jacobian(lambda v: L("act4", X, v), p4)], 4),
        }
        for op, (bwd, jacs, out_dim) in checks.items():
            group_out = op in ("exp", "inv", "mul")
            m = K if group_out else out_dim
            gv = g.standard_normal(m)
            # a group-valued output carries its K-dim tangent gradient in an N-wide row
            gk = np.zeros(N if group_out else m)
            gk[:m] = gv
            grads = bwd(cu(gk[None]))
            series = name == "Sim3" and op in ("exp", "log")
            for gi, J in zip(grads, jacs):
                got = gi.cpu().numpy()[0][:J.shape[1]]
                np.testing.assert_allclose(got, gv @ J, rtol=1e-3 if series else 1e-5, atol=1e-3 if series else 1e-6,
                                           err_msg=f"{name}.{op}")


def test_errors_match_reference_behaviour():
    import lietorch_backends as LB
    X = torch.zeros(4, 14, device="cuda:0", dtype=torch.float64)[:, ::2]
    with pytest.raises(RuntimeError, match="contiguous"):
        LB.inv(3, X)
    with pytest.raises(RuntimeError, match="GPU"):
        LB.inv(3, torch.zeros(4, 7, dtype=torch.float64))
    with pytest.raises(RuntimeError, match="group"):
        LB.inv(5, torch.zeros(4, 8, device="cuda:0"))


def test_golden_vectors_through_shim():
    import lietorch_backends as LB
    gd = np.load(os.path.join(GOLDEN, "lietorch_ref.npz"))
    for name, (gid, K, N) in GROUPS.items():
        a = gd[f"{name}_a"].reshape(-1, K)
        X = LB.expm(gid, cu(a))
        np.testing.assert_allclose(X.cpu().numpy(), gd[f"{name}_exp"].reshape(-1, N), atol=1e-11)
        np.testing.assert_allclose(LB.logm(gid, X).cpu().numpy(), gd[f"{name}_log"].reshape(-1, K), atol=1e-9)
        np.testing.assert_allclose(LB.act4(gid, X, cu(gd[f"{name}_p4"].reshape(-1, 4))).cpu().numpy(),
                                   gd[f"{name}_act4"].reshape(-1, 4), atol=1e-12)
        np.testing.assert_allclose(LB.adjT(gid, X, cu(gd[f"{name}_t"].reshape(-1, K))).cpu().numpy(),
                                   gd[f"{name}_adjT"].reshape(-1, K), atol=1e-12)


@pytest.mark.parametrize("name", list(GROUPS))
def test_python_surface_groups(name):
    """The reference's Python classes (dpvo.lietorch.SO3/RxSO3/SE3/Sim3) over
    the shim: broadcasting products and actions equal the golden vectors the
    reference's own groups.py produced (tests/golden/make_golden.py)."""
    from dpvo import lietorch as L
    G = getattr(L, name)
    gd = np.load(os.path.join(GOLDEN, "lietorch_ref.npz"))
    X = G.exp(cu(gd[f"{name}_a"]))
    Y = G.exp(cu(gd[f"{name}_b"]))
    np.testing.assert_allclose((X * Y).data.cpu().numpy(), gd[f"{name}_mul"], atol=1e-11)
    np.testing.assert_allclose(X.inv().data.cpu().numpy(), gd[f"{name}_inv"], atol=1e-11)
    np.testing.assert_allclose(X.act(cu(gd[f"{name}_p3"])).cpu().numpy(), gd[f"{name}_act"], atol=1e-11)
    np.testing.assert_allclose(X.matrix().cpu().numpy(), gd[f"{name}_matrix"], atol=1e-11)
    np.testing.assert_allclose(X.adj(cu(gd[f"{name}_t"])).cpu().numpy(), gd[f"{name}_adj"], atol=1e-10)
    np.testing.assert_allclose(X.Jinv(cu(gd[f"{name}_t"])).cpu().numpy(), gd[f"{name}_Jinv"], atol=1e-9)
    Xb = G(cu(gd[f"{name}_Xb"]))
    np.testing.assert_allclose((Xb * X).data.cpu().numpy(), gd[f"{name}_bmul"], atol=1e-11)
    np.testing.assert_allclose(Xb.act(cu(gd[f"{name}_p4"])).cpu().numpy(), gd[f"{name}_bact4"], atol=1e-11)
