"""Output formats (reference dpvo/plot_utils.py:50-105,
dpvo_demo.py:129-135) -- host-only, no GPU.  The reference needs evo and
plyfile (absent), so the checks restate the formats they write: the TUM line
layout including the reference's quaternion-component order, COLMAP's text
model (poses inverted to world->camera), and an ASCII PLY round trip."""
import numpy as np
import pytest

from dpvo import io


def _poses(n, seed=0):
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return np.concatenate([rng.normal(size=(n, 3)), q], 1)


def test_tum_from_tracker_output(tmp_path):
    """dpvo_demo.py:187-196: poses [t, qx, qy, qz, qw] wrapped with
    orientations poses[:, [6, 3, 4, 5]] -> TUM lines ``t x y z qx qy qz qw``."""
    poses, ts = _poses(4, seed=5), np.arange(4) * 1.0
    f = tmp_path / "traj.txt"
    io.save_trajectory_tum_format(io.PoseTrajectory3D.from_dpvo(poses, ts), f)
    got = np.loadtxt(f)
    np.testing.assert_allclose(got[:, 0], ts)
    np.testing.assert_allclose(got[:, 1:], poses)


def test_tum_lines(tmp_path):
    poses, ts = _poses(5), np.arange(5) * 0.2
    f = tmp_path / "traj.txt"
    io.save_trajectory_tum_format((poses, ts), f)
    rows = [list(map(float, line.split())) for line in f.read_text().splitlines()]
    assert len(rows) == 5 and all(len(r) == 8 for r in rows)
    got = np.array(rows)
    np.testing.assert_allclose(got[:, 0], ts)
    np.testing.assert_allclose(got[:, 1:4], poses[:, :3])
    # make_traj passes poses[:, 3:] as "wxyz" and the writer emits [1, 2, 3, 0] of it
    np.testing.assert_allclose(got[:, 4:], poses[:, 3:][:, [1, 2, 3, 0]])


def test_colmap_model_inverts_poses(tmp_path):
    poses = _poses(3, seed=1)
    pts = np.random.default_rng(2).normal(size=(4, 3))
    clr = np.random.default_rng(3).random((4, 3))
    traj = io.PoseTrajectory3D.from_dpvo(poses, np.arange(3))
    # the reference's positional call (dpvo_demo.py:205): nerf_studio_format sits before the intrinsics
    io.save_output_for_COLMAP(tmp_path / "m", np.arange(3), traj, pts, clr, False, 80.0, 81.0, 64.0, 48.0, 384, 512)
    assert (tmp_path / "m" / "cameras.txt").read_text() == "1 PINHOLE 512 384 80.0 81.0 64.0 48.0"
    with pytest.raises(NotImplementedError):
        io.save_output_for_COLMAP(tmp_path / "n", np.arange(3), traj, pts, clr, True, 80.0, 81.0, 64.0, 48.0)
    lines = [line for line in (tmp_path / "m" / "images.txt").read_text().split("\n") if line]
    assert len(lines) == 3
    for line, p in zip(lines, poses):
        v = line.split()
        assert v[0].isdigit() and v[8] == "1" and v[9] == "image"
        qw, qx, qy, qz, x, y, z = map(float, v[1:8])
        T = np.linalg.inv(io._se3_matrix(p))
        np.testing.assert_allclose([x, y, z], T[:3, 3], atol=1e-9)
        R = io._se3_matrix(np.r_[0, 0, 0, qx, qy, qz, qw])[:3, :3]
        np.testing.assert_allclose(R, T[:3, :3], atol=1e-9)
    p3 = (tmp_path / "m" / "points3D.txt").read_text().splitlines()
    assert len(p3) == 4 and p3[0].split()[0] == "1" and p3[0].endswith(" 0.0 0 0 0 0 0 0")
    assert [int(c) for c in p3[1].split()[4:7]] == (clr[1] * 255).astype(np.uint8).tolist()


def test_ply_round_trip(tmp_path):
    rng = np.random.default_rng(4)
    pts = rng.normal(size=(50, 3)).astype(np.float32)
    clr = rng.integers(0, 256, size=(50, 3)).astype(np.uint8)
    f = tmp_path / "pc.ply"
    io.save_ply(f, pts, clr)
    head = f.read_text().split("end_header")[0]
    assert "element vertex 50" in head and "property uchar blue" in head
    p2, c2 = io.load_ply(f)
    np.testing.assert_array_equal(p2, pts)
    np.testing.assert_array_equal(c2, clr)
