"""Output formats of the tracker: TUM trajectory, COLMAP text
model and PLY point cloud, with the reference's conventions and without its
evo / plyfile / loguru dependencies (absent here).

References: save_trajectory_tum_format and save_output_for_COLMAP in
dpvo/plot_utils.py:15-20,50-105; the PLY vertex layout in dpvo_demo.py:129-135.
"""
from pathlib import Path

import numpy as np


class PoseTrajectory3D:
    """The fields of evo's PoseTrajectory3D that the writers read (evo is
    absent here): positions_xyz [n, 3], orientations_quat_wxyz [n, 4],
    timestamps [n] and poses_se3 (4x4 matrices, quaternion normalised)."""

    def __init__(self, positions_xyz=None, orientations_quat_wxyz=None, timestamps=None, poses_se3=None):
        if poses_se3 is not None:
            poses_se3 = [np.asarray(T, dtype=np.float64) for T in poses_se3]
            positions_xyz = np.array([T[:3, 3] for T in poses_se3]).reshape(-1, 3)
            orientations_quat_wxyz = np.array([_quat_wxyz(T[:3, :3]) for T in poses_se3]).reshape(-1, 4)
        self.positions_xyz = np.asarray(positions_xyz, dtype=np.float64).reshape(-1, 3)
        self.orientations_quat_wxyz = np.asarray(orientations_quat_wxyz, dtype=np.float64).reshape(-1, 4)
        self.timestamps = np.asarray(timestamps).reshape(-1)

    @property
    def num_poses(self):
        return len(self.positions_xyz)

    @property
    def poses_se3(self):
        out = []
        for t, (w, x, y, z) in zip(self.positions_xyz, self.orientations_quat_wxyz):
            out.append(_se3_matrix(np.r_[t, x, y, z, w]))
        return out

    @classmethod
    def from_dpvo(cls, poses, tstamps):
        """Tracker output (poses [n, 7] as t, qx, qy, qz, qw) the way
        dpvo_demo.py:187-191 wraps it: orientations = poses[:, [6, 3, 4, 5]]."""
        poses = np.asarray(poses, dtype=np.float64).reshape(-1, 7)
        return cls(poses[:, :3], poses[:, [6, 3, 4, 5]], tstamps)


def make_traj(args):
    """plot_utils.make_traj (:15-20): a (poses, tstamps) tuple is wrapped with
    poses[:, 3:] taken as w, x, y, z as is (the reference does not reorder the
    lietorch x, y, z, w quaternion on this path -- reproduced, so files from
    either implementation compare equal); a trajectory is copied."""
    if isinstance(args, tuple):
        poses, tstamps = args
        poses = np.asarray(poses, dtype=np.float64).reshape(-1, 7)
        return PoseTrajectory3D(poses[:, :3], poses[:, 3:], tstamps)
    assert isinstance(args, PoseTrajectory3D), type(args)
    return PoseTrajectory3D(args.positions_xyz.copy(), args.orientations_quat_wxyz.copy(), args.timestamps.copy())


def save_trajectory_tum_format(traj, filename):
    """One line per pose: ``t x y z`` + orientations_quat_wxyz[[1, 2, 3, 0]]
    (plot_utils.py:50-55).  For a trajectory built by from_dpvo that is
    ``t x y z qx qy qz qw`` (TUM order)."""
    traj = make_traj(traj)
    tostr = lambda a: " ".join(map(str, a))
    with Path(filename).open("w") as f:
        for i in range(traj.num_poses):
            f.write(f"{traj.timestamps[i]} {tostr(traj.positions_xyz[i])} "
                    f"{tostr(traj.orientations_quat_wxyz[i][[1, 2, 3, 0]])}\n")


def _se3_matrix(p):
    """[tx ty tz qx qy qz qw] -> 4x4 (lietorch SE3 convention)."""
    t, (x, y, z, w) = p[:3], p[3:] / np.linalg.norm(p[3:])
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return T


def _quat_wxyz(R):
    """rotation matrix -> unit quaternion (w, x, y, z), w >= 0."""
    tr = np.trace(R)
    if tr > 0:
        s = 2.0 * np.sqrt(tr + 1.0)
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.asarray(q)
    return q if q[0] >= 0 else -q


def save_output_for_COLMAP(name, tstamp, traj, points, colors, nerf_studio_format, fx, fy, cx, cy, H=480, W=640, *,
                           image_names=None):
    """COLMAP text model (plot_utils.py:58-95), same positional signature:
    cameras.txt (one PINHOLE camera), images.txt (the inverted poses,
    world->camera, as IMAGE_ID QW QX QY QZ TX TY TZ 1 NAME plus an empty line)
    and points3D.txt (ID X Y Z R G B 0.0 and an empty track).  traj: a
    PoseTrajectory3D (dpvo_demo.py:205 passes the from_dpvo one) or a (poses,
    tstamps) tuple (make_traj's reading).  colors in [0, 1].  The
    nerf_studio_format branch (:96-113) shells out to `colmap
    model_converter` and nerfstudio, which are not part of this build: True
    raises NotImplementedError.  image_names (keyword) replaces the images/
    directory listing (:66-77)."""
    if nerf_studio_format:
        raise NotImplementedError("nerf_studio_format shells out to colmap / nerfstudio (plot_utils.py:96-113); "
                                  "not part of the MI355X build")
    d = Path(name)
    d.mkdir(parents=True, exist_ok=True)
    traj = make_traj(traj)
    inv = PoseTrajectory3D(poses_se3=[np.linalg.inv(T) for T in traj.poses_se3], timestamps=traj.timestamps)
    lines = []
    for ts, idx, (x, y, z), (qw, qx, qy, qz) in zip(np.asarray(tstamp).reshape(-1), range(1, inv.num_poses + 1),
                                                   inv.positions_xyz, inv.orientations_quat_wxyz):
        img = image_names[int(ts)] if image_names is not None else "image"
        lines.append(f"{idx} {qw} {qx} {qy} {qz} {x} {y} {z} 1 {img}\n\n")
    (d / "images.txt").write_text("".join(lines))
    cols = (np.asarray(colors) * 255).astype(np.uint8).tolist()
    pts = np.asarray(points, dtype=np.float64).tolist()
    (d / "points3D.txt").write_text("".join(f"{i} " + " ".join(map(str, p + c)) + " 0.0 0 0 0 0 0 0\n"
                                            for i, (p, c) in enumerate(zip(pts, cols), start=1)))
    (d / "cameras.txt").write_text(f"1 PINHOLE {W} {H} {fx} {fy} {cx} {cy}")


def save_ply(filename, points, colors):
    """ASCII PLY of the point cloud: vertex (x, y, z float; red, green, blue
    uchar), the element dpvo_demo.py:129-135 builds with plyfile (text=True)."""
    pts = np.asarray(points, dtype=np.float32).reshape(-1, 3)
    cls = np.asarray(colors, dtype=np.uint8).reshape(-1, 3)
    with Path(filename).open("w") as f:
        f.write("ply\nformat ascii 1.0\n")
        f.write(f"element vertex {len(pts)}\n")
        f.write("property float x\nproperty float y\nproperty float z\n")
        f.write("property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
        for (x, y, z), (r, g, b) in zip(pts.tolist(), cls.tolist()):
            f.write(f"{x:.9g} {y:.9g} {z:.9g} {r} {g} {b}\n")


def load_ply(filename):
    """points [n, 3] float32, colors [n, 3] uint8 from save_ply's format."""
    with Path(filename).open() as f:
        n = 0
        for line in f:
            if line.startswith("element vertex"):
                n = int(line.split()[-1])
            if line.strip() == "end_header":
                break
        data = np.loadtxt(f, ndmin=2) if n else np.zeros((0, 6))
    return data[:, :3].astype(np.float32), data[:, 3:6].astype(np.uint8)
