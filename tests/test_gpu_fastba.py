"""fastba / neighbors / reproject on the GPU (through the C ABI) vs the oracle.

Bars: BA poses and depths within 1e-3 relative of the oracle (the reference
itself sums with unordered float atomics, so it is not bit-reproducible);
neighbors bit-exact (index work); reproject within fp32 rounding.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu
RTOL = 1e-3


def T(a, d="cuda:0"):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def run_gpu_ba(poses, patches, intr, target, weight, ii, jj, kk, t0, t1, iters):
    import cuda_ba
    p = T(poses)
    q = T(patches)[None]
    cuda_ba.forward(p, q, T(intr), T(target), T(weight), torch.tensor([1e-4], device="cuda:0"), T(ii), T(jj), T(kk),
                    t0, t1, iters)
    return p.cpu().numpy(), q[0].cpu().numpy()


def assert_close_rel(got, ref, rtol=RTOL, floor=1e-5):
    """norm-wise per tensor, and per element where |ref| > floor."""
    assert np.linalg.norm(got - ref) <= rtol * max(np.linalg.norm(ref), floor)
    big = np.abs(ref) > 1e-3
    assert np.all(np.abs(got[big] - ref[big]) <= rtol * np.abs(ref[big]) + floor)


@pytest.mark.parametrize("case", ["window", "full", "structure"])
def test_ba_golden_cases(case):
    g = np.load(os.path.join(GOLDEN, "ba_python_ref.npz"))
    f = lambda k: g[f"{case}_{k}"]
    args = (f("poses"), f("patches"), f("intrinsics"), f("target"), f("weight"), f("ii"), f("jj"), f("kk"),
            int(f("t0")), int(f("t1")), int(f("iters")))
    gp, gq = run_gpu_ba(*args)
    rp, rq, st = oracle.ba_forward(*args[:5], 1e-4, *args[5:])
    assert st == 0
    assert_close_rel(gp, rp)
    assert_close_rel(gq[:, 2], rq[:, 2])
    # and against the reference's own Python BA output
    assert_close_rel(gp, f("poses_out").reshape(-1, 7), rtol=2e-3)


def synth_dpvo_state(seed, n=40, M=16, lifetime=13, removal=22):
    """Tracker-shaped state: random-walk poses, DPVO edge rules."""
    from tests_helpers import dpvo_state
    return dpvo_state(seed, n=n, M=M, lifetime=lifetime, removal=removal)


@pytest.mark.parametrize("seed,iters", [(0, 2), (1, 8)])
def test_ba_dpvo_window(seed, iters):
    st = synth_dpvo_state(seed)
    n = st["n"]
    t0, t1 = n - 10, n
    args = (st["poses"], st["patches"], st["intrinsics"], st["target"], st["weight"], st["ii"], st["jj"], st["kk"],
            t0, t1, iters)
    gp, gq = run_gpu_ba(*args)
    rp, rq, status = oracle.ba_forward(*args[:5], 1e-4, *args[5:])
    assert status == 0
    assert_close_rel(gp, rp)
    assert_close_rel(gq[:, 2], rq[:, 2])
    assert np.abs(gp - st["poses"]).max() > 1e-5  # the window moved


def test_ba_fails_like_reference_on_non_spd():
    import cuda_ba
    g = np.load(os.path.join(GOLDEN, "ba_python_ref.npz"))
    f = lambda k: g[f"window_{k}"]
    w = np.full_like(f("weight"), np.nan)
    p = T(f("poses"))
    with pytest.raises(RuntimeError, match="positive-definite"):
        cuda_ba.forward(p, T(f("patches"))[None], T(f("intrinsics")), T(f("target")), T(w),
                        torch.tensor([1e-4], device="cuda:0"), T(f("ii")), T(f("jj")), T(f("kk")), int(f("t0")),
                        int(f("t1")), 2)


def test_ba_empty_edges_is_noop():
    import cuda_ba
    p = torch.zeros(4, 7, device="cuda:0"); p[:, 6] = 1
    q = torch.rand(1, 8, 3, 3, 3, device="cuda:0")
    q0 = q.clone()
    e = torch.zeros(0, dtype=torch.long, device="cuda:0")
    cuda_ba.forward(p, q, torch.ones(4, 4, device="cuda:0"), torch.zeros(1, 0, 2, device="cuda:0"),
                    torch.zeros(1, 0, 2, device="cuda:0"), torch.tensor([1e-4], device="cuda:0"), e, e, e, 1, 4, 2)
    assert torch.equal(q, q0)


@pytest.mark.parametrize("pre", ["", "r_"])
def test_neighbors_golden(pre):
    import cuda_ba
    g = np.load(os.path.join(GOLDEN, "neighbors_ref.npz"))
    ix, jx = cuda_ba.neighbors(T(g[pre + "kk"]), T(g[pre + "jj"]))
    assert np.array_equal(ix.cpu().numpy(), g[pre + "ix"])
    assert np.array_equal(jx.cpu().numpy(), g[pre + "jx"])


def test_neighbors_large_matches_oracle():
    import cuda_ba
    st = synth_dpvo_state(3, n=60, M=32)
    ix, jx = cuda_ba.neighbors(T(st["kk"]), T(st["jj"]))
    rix, rjx = oracle.neighbors(st["kk"], st["jj"])
    assert np.array_equal(ix.cpu().numpy(), rix)
    assert np.array_equal(jx.cpu().numpy(), rjx)


def _neighbors_csr(kk, jj):
    import update_ops as U
    kk, jj = T(kk), T(jj)
    _, offs, perm, G = U.group_by(kk, key_bits=32)
    ix, jx = U.neighbors_csr(jj, offs, perm, G, kk.numel())
    return ix.cpu().numpy(), jx.cpu().numpy()


@pytest.mark.parametrize("pre", ["", "r_"])
def test_neighbors_csr_golden(pre):
    """The fused update operator's neighbours (over the kk group-by CSR) are the
    reference's fastba.neighbors bit for bit."""
    g = np.load(os.path.join(GOLDEN, "neighbors_ref.npz"))
    ix, jx = _neighbors_csr(g[pre + "kk"], g[pre + "jj"])
    assert np.array_equal(ix, g[pre + "ix"])
    assert np.array_equal(jx, g[pre + "jx"])


def test_neighbors_csr_large_and_big_groups():
    st = synth_dpvo_state(3, n=60, M=32)
    ix, jx = _neighbors_csr(st["kk"], st["jj"])
    rix, rjx = oracle.neighbors(st["kk"], st["jj"])
    assert np.array_equal(ix, rix) and np.array_equal(jx, rjx)
    # groups larger than a wave (> 64 members) and repeated (kk, jj) pairs
    rng = np.random.default_rng(0)
    kk = rng.integers(0, 5, 700)
    jj = rng.integers(0, 40, 700)
    ix, jx = _neighbors_csr(kk, jj)
    rix, rjx = oracle.neighbors(kk, jj)
    assert np.array_equal(ix, rix) and np.array_equal(jx, rjx)


def test_reproject_matches_oracle():
    import cuda_ba
    st = synth_dpvo_state(4)
    out = cuda_ba.reproject(T(st["poses"])[None], T(st["patches"])[None], T(st["intrinsics"])[None], T(st["ii"]),
                            T(st["jj"]), T(st["kk"]))
    ref = oracle.reproject(st["poses"], st["patches"], st["intrinsics"], st["ii"], st["jj"], st["kk"])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-3)


def _ba_run(st, t0, t1, iters, csr=False, deterministic=True):
    import cuda_ba
    import update_ops
    p, q = T(st["poses"]), T(st["patches"])[None]
    kk = T(st["kk"])
    groups = update_ops.group_by(kk)[1:] if csr else None
    old = cuda_ba.DETERMINISTIC
    cuda_ba.DETERMINISTIC = deterministic
    try:
        cuda_ba.forward(p, q, T(st["intrinsics"]), T(st["target"]), T(st["weight"]),
                        torch.tensor([1e-4], device="cuda:0"), T(st["ii"]), T(st["jj"]), kk, t0, t1, iters, csr=groups)
    finally:
        cuda_ba.DETERMINISTIC = old
    return p.cpu().numpy(), q[0].cpu().numpy()


@pytest.mark.parametrize("iters", [2, 8])
def test_ba_bitwise_repeatable(iters):
    """The per-patch path has no float atomics: the same inputs give the same
    bits, whether BA groups kk itself or reuses the caller's group-by."""
    st = synth_dpvo_state(5, n=60, M=96)
    n = st["n"]
    runs = [_ba_run(st, n - 10, n, iters, csr=c) for c in (False, True, False)]
    for p, q in runs[1:]:
        assert np.array_equal(p, runs[0][0]) and np.array_equal(q, runs[0][1])
    # the atomic dense path agrees within the parity bar
    pa, qa = _ba_run(st, n - 10, n, iters, deterministic=False)
    assert_close_rel(runs[0][0], pa)
    assert_close_rel(runs[0][1][:, 2], qa[:, 2])


@pytest.mark.parametrize("M,iters", [(96, 2), (96, 8), (200, 2)])
def test_ba_partial_last_round_matches_oracle(M, iters):
    """Patch counts just past a multiple of the 2,048 resident waves (2,112
    and 4,400 patches: a last round of 64 / 304 patches, most slots of the
    final flush empty) match the oracle, bit-repeatably."""
    st = synth_dpvo_state(5, n=60, M=M)
    G = len(np.unique(st["kk"]))
    assert 0 < G % 2048 <= 512, G
    n = st["n"]
    gp, gq = _ba_run(st, n - 10, n, iters)
    rp, rq, status = oracle.ba_forward(st["poses"], st["patches"], st["intrinsics"], st["target"], st["weight"],
                                       1e-4, st["ii"], st["jj"], st["kk"], n - 10, n, iters)
    assert status == 0
    assert_close_rel(gp, rp)
    assert_close_rel(gq[:, 2], rq[:, 2])
    again = _ba_run(st, n - 10, n, iters)
    assert np.array_equal(again[0], gp) and np.array_equal(again[1], gq)


def test_ba_mixed_frames_and_repeated_targets():
    """Outside DPVO's edge rules: edges of one patch from different frames i,
    and the same (patch, target) pair twice -- the lane-by-lane fallback of
    the per-patch path -- still match the oracle."""
    st = synth_dpvo_state(6, n=30, M=16)
    n = st["n"]
    rng = np.random.default_rng(0)
    E = len(st["ii"])
    ii = st["ii"].copy()
    sel = rng.choice(E, E // 10, replace=False)
    ii[sel] = rng.integers(n - 10, n, len(sel))      # another frame's pose for these edges
    dup = rng.choice(E, E // 10, replace=False)      # repeat some edges
    st = dict(st)
    for key in ("jj", "kk"):
        st[key] = np.concatenate([st[key], st[key][dup]])
    st["ii"] = np.concatenate([ii, ii[dup]])
    st["target"] = np.concatenate([st["target"], st["target"][:, dup]], 1)
    st["weight"] = np.concatenate([st["weight"], st["weight"][:, dup]], 1)
    t0, t1 = n - 10, n
    gp, gq = _ba_run(st, t0, t1, 2)
    rp, rq, status = oracle.ba_forward(st["poses"], st["patches"], st["intrinsics"], st["target"], st["weight"],
                                       1e-4, st["ii"], st["jj"], st["kk"], t0, t1, 2)
    assert status == 0
    assert_close_rel(gp, rp)
    assert_close_rel(gq[:, 2], rq[:, 2])


@pytest.mark.parametrize("window", [1, 12])
def test_ba_window_sizes_of_the_per_patch_path(window):
    """1 pose and the largest per-patch window (12 poses, 72 unknowns: two
    system columns per back-substitution lane)."""
    st = synth_dpvo_state(8, n=40, M=16)
    n = st["n"]
    gp, gq = _ba_run(st, n - window, n, 2)
    rp, rq, status = oracle.ba_forward(st["poses"], st["patches"], st["intrinsics"], st["target"], st["weight"],
                                       1e-4, st["ii"], st["jj"], st["kk"], n - window, n, 2)
    assert status == 0
    assert_close_rel(gp, rp)
    assert_close_rel(gq[:, 2], rq[:, 2])


@pytest.mark.parametrize("window", [10, 11, 12])
def test_ba_workspace_guard_untouched(window):
    """The deterministic path writes nothing past its workspace (the dense rows
    for the wave solver exist only for <= 10 poses; 11-12 poses used to overrun
    them into whatever the allocator placed next)."""
    import _dpvo_hot as H
    st = synth_dpvo_state(8, n=40, M=16)
    n = st["n"]
    p, q = T(st["poses"]), T(st["patches"])[None]
    ii, jj, kk = T(st["ii"]), T(st["jj"]), T(st["kk"])
    E = ii.numel()
    nbytes = H.lib().dpvo_ba_workspace_bytes_ex(E, q.numel() // 27, window, 0)
    guard = 1 << 16
    ws = torch.full((nbytes + guard,), 0xAB, dtype=torch.uint8, device="cuda:0")
    status = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    intr, tgt, wt = T(st["intrinsics"]), T(st["target"]), T(st["weight"])
    lm = torch.tensor([1e-4], device="cuda:0")
    H.check(H.lib().dpvo_ba_forward_csr(
        H.ptr(p), H.ptr(q), q.numel() // 27, 3, H.ptr(intr), H.ptr(tgt), H.ptr(wt), H.ptr(lm), H.ptr(ii), H.ptr(jj),
        H.ptr(kk), E, n - window, n, 2, 0, None, None, None, H.ptr(ws), nbytes, H.ptr(status), H.stream_of(p)))
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert bool((ws[nbytes:] == 0xAB).all())
