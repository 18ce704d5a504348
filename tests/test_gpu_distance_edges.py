"""Distance-based global-BA edges on the device: every pair's
keyframe distance (dpvo.py:383-407) from one keyframe_flow launch, and the edge
list of get_distance_based_edges (dpvo.py:409-429) from one compaction --
against the reference's own pair loop (kept as DPVO._distance_edges_loop),
index for index; then terminate()'s global BA with the default
USE_DISTANCE_EDGES at the C4 size (n = 4096)."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def tracker(n, preset="fast", seed=0):
    from dpvo.synthetic import steady_state_tracker
    return steady_state_tracker(preset, buffer=n + 8, n=n, seed=seed, ENABLE_GLOBAL_BA=True)


def test_keyframe_flow_matches_pair_distances():
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    slam = tracker(24)
    n = slam.n
    D = pops.keyframe_flow(SE3(slam.poses), slam.patches, slam.intrinsics, n, slam.M, beta=0.5)
    assert D.shape == (n, n) and torch.isfinite(D).all()
    assert torch.all(D.diagonal().abs() < 1e-3)          # Gaa: the identity up to rounding
    for i, j in [(0, 2), (0, 23), (5, 9), (11, 12), (17, 3), (22, 21)]:
        ref = slam.compute_keyframe_distance(i, j)
        got = 0.5 * (D[i, j] + D[j, i]).item()
        assert abs(got - ref) <= 1e-5 * max(1.0, abs(ref)), (i, j, got, ref)


@pytest.mark.parametrize("seed,n", [(0, 40), (1, 33)])
def test_distance_edges_equal_reference_loop(seed, n):
    slam = tracker(n, seed=seed)
    ii, jj = slam.get_distance_based_edges()
    ri, rj = slam._distance_edges_loop()
    assert ii.tolist() == ri and jj.tolist() == rj
    extra = len(ri) - (n - 1)
    print(f"n={n}: {extra} distance edges of {(n - 1) * (n - 2) // 2} candidate pairs")
    assert 0 < extra < (n - 1) * (n - 2) // 2   # the threshold separates pairs both ways


def test_distance_edges_empty_and_disabled():
    slam = tracker(8)
    slam.use_distance_edges = False
    ii, jj = slam.get_distance_based_edges()
    assert ii.numel() == 0 and jj.numel() == 0
    slam.use_distance_edges = True
    slam.pg.n = 1
    ii, jj = slam.get_distance_based_edges()
    assert ii.numel() == 0


def test_terminate_global_ba_c4_with_distance_edges():
    """C4: terminate() -> global BA over n = 4096 keyframes (dpvo_2k, M = 192)
    with the default distance edges.  The reference's loop would make 8.4M
    host reads here; this is one launch + one compaction."""
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker("dpvo_2k", buffer=4104, n=4096, seed=2, ENABLE_GLOBAL_BA=True)
    assert slam.use_distance_edges
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ii, jj = slam.get_distance_based_edges()
    torch.cuda.synchronize()
    t_edges = time.perf_counter() - t0
    p0 = slam.pg.poses_[:slam.n].clone()
    t0 = time.perf_counter()
    slam.global_bundle_adjustment()
    torch.cuda.synchronize()
    t_gba = time.perf_counter() - t0
    print(f"C4 distance edges: {ii.numel()} frame pairs ({ii.numel() - 4095} beyond the sequential ones) in "
          f"{t_edges * 1e3:.1f} ms; global BA incl. edges {t_gba * 1e3:.1f} ms")
    poses = slam.pg.poses_[:slam.n]
    assert torch.isfinite(poses).all()
    assert (poses - p0).abs().max() > 0
    assert ii.numel() >= 4095
