"""The CPU oracle against the committed golden vectors (no GPU needed).

These pin the checker before anything is checked with it: every product-path
parity test compares the HIP kernels with this oracle.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def h(a):
    return np.asarray(a).view(np.float16)


# ----------------------------------------------------------------------------
# altcorr: bit-exact against the torch-f16 restatement of the reference kernel
# ----------------------------------------------------------------------------
def test_corr_level1_bitexact():
    g = load("altcorr_ref.npz")
    out = oracle.corr_forward(h(g["gmap"]), h(g["fmap1"]), g["coords"], g["ii"], g["jj"], 3)
    got = out.transpose(0, 1, 3, 2, 4, 5)  # the reference returns the permuted view
    assert np.array_equal(got.view(np.uint16), g["corr_l1"].view(np.uint16))


def test_corr_level2_bitexact():
    g = load("altcorr_ref.npz")
    c = (g["coords"] / np.float32(4)).astype(np.float32)
    out = oracle.corr_forward(h(g["gmap"]), h(g["fmap2"]), c, g["ii"], g["jj"], 3)
    assert np.array_equal(out.transpose(0, 1, 3, 2, 4, 5).view(np.uint16), g["corr_l2"].view(np.uint16))


def test_corr_pyramid_stacked_bitexact():
    g = load("altcorr_ref.npz")
    st = oracle.corr_pyramid(h(g["gmap"]), [h(g["fmap1"]), h(g["fmap2"])], g["coords"], g["ii"], g["jj"])
    assert st.shape == g["corr_stacked"].shape
    assert np.array_equal(st.view(np.uint16), g["corr_stacked"].view(np.uint16))


def test_corr_odd_shapes_bitexact():
    g = load("altcorr_ref.npz")
    out = oracle.corr_forward(h(g["b_gmap"]), h(g["b_fmap"]), g["b_coords"], g["b_ii"], g["b_jj"], 1)
    assert np.array_equal(out.transpose(0, 1, 3, 2, 4, 5).view(np.uint16), g["b_corr"].view(np.uint16))


def test_corr_f16_close_to_f64_accuracy_reference():
    """The fp16 chain is the reference's arithmetic; it stays within fp16
    accumulation error of the exact dot products."""
    g = load("altcorr_ref.npz")
    a = oracle.corr_forward(h(g["gmap"]), h(g["fmap1"]), g["coords"], g["ii"], g["jj"], 3).astype(np.float64)
    b = oracle.corr_forward(h(g["gmap"]), h(g["fmap1"]), g["coords"], g["ii"], g["jj"], 3, mode=oracle.F16_ACC64)
    scale = np.abs(b).max()
    assert np.abs(a - b).max() < 2e-2 * scale


# ----------------------------------------------------------------------------
# lietorch: oracle through a local broadcasting layer vs reference vectors
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("name,group,dim", [("SE3", oracle.SE3, 7), ("SO3", oracle.SO3, 4)])
def test_lie_vectors(name, group, dim):
    g = load("lietorch_ref.npz")
    K = dim - 1
    a = g[f"{name}_a"].reshape(-1, K)
    X = oracle.lie_forward("exp", group, a)
    np.testing.assert_allclose(X, g[f"{name}_exp"].reshape(-1, dim), atol=1e-12)
    Y = oracle.lie_forward("exp", group, g[f"{name}_b"].reshape(-1, K))
    np.testing.assert_allclose(oracle.lie_forward("log", group, X), g[f"{name}_log"].reshape(-1, K), atol=1e-10)
    np.testing.assert_allclose(oracle.lie_forward("inv", group, X), g[f"{name}_inv"].reshape(-1, dim), atol=1e-12)
    np.testing.assert_allclose(oracle.lie_forward("mul", group, X, Y), g[f"{name}_mul"].reshape(-1, dim), atol=1e-12)
    np.testing.assert_allclose(oracle.lie_forward("act", group, X, g[f"{name}_p3"].reshape(-1, 3)),
                               g[f"{name}_act"].reshape(-1, 3), atol=1e-12)
    np.testing.assert_allclose(oracle.lie_forward("act4", group, X, g[f"{name}_p4"].reshape(-1, 4)),
                               g[f"{name}_act4"].reshape(-1, 4), atol=1e-12)
    t = g[f"{name}_t"].reshape(-1, K)
    np.testing.assert_allclose(oracle.lie_forward("adj", group, X, t), g[f"{name}_adj"].reshape(-1, K), atol=1e-12)
    np.testing.assert_allclose(oracle.lie_forward("adjT", group, X, t), g[f"{name}_adjT"].reshape(-1, K), atol=1e-12)
    np.testing.assert_allclose(oracle.lie_forward("Jinv", group, X, t), g[f"{name}_Jinv"].reshape(-1, K), atol=1e-10)


# ----------------------------------------------------------------------------
# projective ops
# ----------------------------------------------------------------------------
def test_transform_vs_reference_python():
    g = load("pops_ref.npz")
    c = oracle.transform(g["poses"], g["patches"], g["intrinsics"], g["ii"], g["jj"], g["kk"])
    np.testing.assert_allclose(c, g["coords"], rtol=1e-5, atol=1e-4)
    cd, v = oracle.transform(g["poses"], g["patches"], g["intrinsics"], g["ii"], g["jj"], g["kk"], depth=True,
                             valid=True)
    np.testing.assert_allclose(cd, g["coords_depth"], rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(v, g["valid"])
    ct = oracle.transform(g["poses"], g["patches"], g["intrinsics"], g["ii"], g["jj"], g["kk"], tonly=True)
    np.testing.assert_allclose(ct, g["coords_tonly"], rtol=1e-5, atol=1e-4)


def test_point_cloud_vs_reference_python():
    g = load("pops_ref.npz")
    pc = g["point_cloud"][0]  # [m,P,P,4]
    ref = pc[:, 1, 1, :3] / pc[:, 1, 1, 3:]
    got = oracle.point_cloud_centre(g["poses"], g["patches"], g["intrinsics"], g["ix"])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_fastba_reproject_matches_transform_when_in_front():
    g = load("pops_ref.npz")
    r = oracle.reproject(g["poses"], g["patches"], g["intrinsics"], g["ii"], g["jj"], g["kk"])[0]
    c = g["coords"][0].transpose(0, 3, 1, 2)  # [E,2,P,P]
    front = g["valid"][0][:, None].repeat(2, 1) > 0
    np.testing.assert_allclose(r[front], c[front], rtol=1e-4, atol=1e-3)


# ----------------------------------------------------------------------------
# fastba: CUDA-path restatement vs the reference's own Python BA
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["window", "full", "structure"])
def test_ba_vs_reference_python_ba(case):
    g = load("ba_python_ref.npz")
    f = lambda k: g[f"{case}_{k}"]
    poses, patches, st = oracle.ba_forward(f("poses"), f("patches"), f("intrinsics"), f("target"), f("weight"),
                                           1e-4, f("ii"), f("jj"), f("kk"), int(f("t0")), int(f("t1")),
                                           int(f("iters")))
    assert st == 0
    ref_p = f("poses_out").reshape(-1, 7)
    ref_d = f("patches_out")[:, 2]
    # unchanged inputs stay unchanged; optimised ones moved and agree
    np.testing.assert_allclose(poses, ref_p, rtol=1e-3, atol=2e-5)
    np.testing.assert_allclose(patches[:, 2], ref_d, rtol=1e-3, atol=2e-5)
    if case != "structure":
        assert np.abs(poses - f("poses")).max() > 1e-4  # the step did something
    assert np.abs(patches[:, 2] - f("patches")[:, 2]).max() > 1e-4


def test_ba_cholesky_failure_reports_minor():
    g = load("ba_python_ref.npz")
    f = lambda k: g[f"window_{k}"]
    w = np.full_like(f("weight"), np.nan)
    _, _, st = oracle.ba_forward(f("poses"), f("patches"), f("intrinsics"), f("target"), w, 1e-4, f("ii"),
                                 f("jj"), f("kk"), int(f("t0")), int(f("t1")), 1)
    assert st >= 1


# ----------------------------------------------------------------------------
# neighbors
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("pre", ["", "r_"])
def test_neighbors(pre):
    g = load("neighbors_ref.npz")
    ix, jx = oracle.neighbors(g[pre + "kk"], g[pre + "jj"])
    np.testing.assert_array_equal(ix, g[pre + "ix"])
    np.testing.assert_array_equal(jx, g[pre + "jx"])


def test_patchify_matches_direct_gather():
    rng = np.random.default_rng(0)
    net = rng.standard_normal((2, 5, 7, 9)).astype(np.float32)
    coords = np.stack([rng.integers(-2, 11, (2, 6)), rng.integers(-2, 9, (2, 6))], -1).astype(np.float32)
    out = oracle.patchify_forward(net, coords, 1)
    for b in range(2):
        for m in range(6):
            x, y = int(coords[b, m, 0]), int(coords[b, m, 1])
            for a in range(4):
                for c in range(4):
                    i, j = y + a - 1, x + c - 1
                    exp = net[b, :, i, j] if (0 <= i < 7 and 0 <= j < 9) else 0
                    np.testing.assert_array_equal(out[b, m, :, a, c], exp)


def test_softagg_oracle_matches_torch_scatter_composition():
    """oracle.softagg vs the scatter_softmax/scatter_sum composition of the
    dpvo.blocks mirror run on CPU torch (both restate torch_scatter 2.1.2)."""
    import torch
    from dpvo.blocks import scatter_softmax, scatter_sum
    g = torch.Generator().manual_seed(0)
    E, G, D = 700, 23, 16
    f = torch.randn(1, E, D, generator=g, dtype=torch.float64)
    s = torch.randn(1, E, D, generator=g, dtype=torch.float64) * 4
    lab = torch.randint(0, G, (E,), generator=g)
    want = scatter_sum(f * scatter_softmax(s, lab, 1, G), lab, 1, G)[0].numpy()
    got = oracle.softagg(f[0].numpy(), s[0].numpy(), lab.numpy(), G)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


def test_solve_system_oracle_normal_equations():
    """oracle.solve_system solves (J^T J + lm diag + ep I) delta = -J^T res -- the
    restatement of ba.cpp:174-234 (Eigen absent: parity unpinned by fixtures)."""
    g = np.random.default_rng(0)
    n, r = 6, 8
    ii = np.array([0, 1, 2, 3, 4, 0, 1, 2])
    jj = np.array([1, 2, 3, 4, 5, 3, 4, 5])
    Ji = g.normal(size=(r, 7, 7))
    Jj = g.normal(size=(r, 7, 7))
    res = g.normal(size=(r, 7))
    d = oracle.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-3, -1).astype(np.float64).reshape(-1)
    J = np.zeros((7 * r, 7 * n))
    for x in range(r):
        J[7 * x:7 * x + 7, 7 * ii[x]:7 * ii[x] + 7] = Ji[x]
        J[7 * x:7 * x + 7, 7 * jj[x]:7 * jj[x] + 7] = Jj[x]
    A = J.T @ J
    A += np.diag(np.diag(A) * 1e-3 + 1e-4)
    np.testing.assert_allclose(A @ d, -J.T @ res.reshape(-1), rtol=1e-4, atol=1e-4)
