"""Patch-graph state container (reference dpvo/patchgraph.py:13-140).

Layout in HBM (all on the tracker's GPU):
  poses_      [N, 7]  fp32  world->camera [t, q]
  patches_    [N, M, 3, P, P] fp32  (x, y, inverse depth) at 1/RES resolution
  intrinsics_ [N, 4]  fp32  (fx, fy, cx, cy) / RES
  points_     [N*M, 3] fp32, colors_ [N, M, 3] u8, index_ [N, M] i64
  edges ii/jj/kk [E] i64, hidden state net [1, E, DIM] fp16
"""
import numpy as np
import torch

from . import projective_ops as pops
from .lietorch import SE3
from .utils import matrix_to_quaternion


class PatchGraph:
    def __init__(self, cfg, P, DIM, pmem, M, ht_resized, wd_resized, RES, device="cuda", **kwargs):
        self.cfg, self.P, self.pmem, self.DIM = cfg, P, pmem, DIM
        self.n = 0  # frames
        self.m = 0  # patches
        self.M = M
        self.N = cfg.BUFFER_SIZE
        dev = torch.device(device)
        f32 = dict(dtype=torch.float, device=dev)
        self.tstamps_ = np.zeros(self.N, dtype=np.int64)
        self.poses_ = torch.zeros(self.N, 7, **f32)
        self.poses_[:, 6] = 1.0
        self.patches_ = torch.zeros(self.N, M, 3, P, P, **f32)
        self.patches_est_ = torch.zeros(self.N, M, 3, P, P, **f32)
        self.intrinsics_ = torch.zeros(self.N, 4, **f32)
        self.points_ = torch.zeros(self.N * M, 3, **f32)
        self.colors_ = torch.zeros(self.N, M, 3, dtype=torch.uint8, device=dev)
        self.index_ = torch.zeros(self.N, M, dtype=torch.long, device=dev)
        self.index_map_ = torch.zeros(self.N, dtype=torch.long, device=dev)
        self.delta = {}  # relative poses of removed keyframes

        net_kw = {k: v for k, v in kwargs.items() if k in ("dtype",)}
        self.net = torch.zeros(1, 0, DIM, device=dev, **net_kw)
        empty = lambda: torch.zeros(0, dtype=torch.long, device=dev)
        self.ii, self.jj, self.kk = empty(), empty(), empty()
        self.ii_inac, self.jj_inac, self.kk_inac = empty(), empty(), empty()
        self.weight = torch.zeros(1, 0, 2, **f32)
        self.target = torch.zeros(1, 0, 2, **f32)
        self.weight_inac = torch.zeros(1, 0, 2, **f32)
        self.target_inac = torch.zeros(1, 0, 2, **f32)
        self.ht_resized, self.wd_resized, self.RES = ht_resized, wd_resized, RES

    @property
    def poses(self):
        return self.poses_.view(1, self.N, 7)

    @property
    def patches(self):
        return self.patches_.view(1, self.N * self.M, 3, self.P, self.P)

    @property
    def intrinsics(self):
        return self.intrinsics_.view(1, self.N, 4)

    @property
    def ix(self):
        return self.index_.view(-1)

    def edges_loop(self):
        return

    def normalize(self):
        """rescale depths to unit mean and re-anchor poses on frame 0 (patchgraph.py:68-79)."""
        s = self.patches_[:self.n, :, 2].mean()
        self.patches_[:self.n, :, 2] /= s
        self.poses_[:self.n, :3] *= s
        for t, (t0, dP) in self.delta.items():
            self.delta[t] = (t0, dP.scale(s))
        self.poses_[:self.n] = (SE3(self.poses_[:self.n]) * SE3(self.poses_[[0]]).inv()).data
        pops.point_cloud_centre(SE3(self.poses), self.patches[:, :self.m], self.intrinsics, self.ix[:self.m],
                                out=self.points_[:self.m])

    def _prior_patch(self, idx, depth):
        """frame idx's patches with the inverse of the median metric depth
        under each patch's 3x3 (full-resolution) sample points."""
        patch = self.patches_[idx]
        xs = torch.clamp(patch[:, 0].long() * self.RES, 0, depth.shape[1] - 1)
        ys = torch.clamp(patch[:, 1].long() * self.RES, 0, depth.shape[0] - 1)
        med = torch.median(depth[ys, xs].view(patch.shape[0], -1), dim=1).values
        patch[:, 2] = 1 / med.view(-1, 1, 1)
        return patch

    def set_prior_depth(self, idx, depth):
        """initialise frame idx's patch depth from a metric depth map (patchgraph.py:97-110)."""
        if depth is None:
            return
        patch = self._prior_patch(idx, depth)
        self.patches_est_[idx] = patch
        self.patches_[idx] = patch

    def init_from_prior(self, depths, poses, indices, images=None):
        """known depths and camera poses for the frames in `indices`
        (patchgraph.py:112-140): depths, a list of full-resolution metric
        depth maps [H, W]; poses [N, 4, 4] camera->world matrices, stored
        inverted (world->camera) as [t, qx, qy, qz, qw].  As in the reference
        the depth is written through the patches_[idx] view (so patches_ and
        patches_est_ both get it)."""
        depths = torch.stack(list(depths), dim=0)
        dpvo_poses = create_se3_from_mat(torch.as_tensor(poses, device=depths.device, dtype=torch.float)).inv()
        for idx in indices:
            self.patches_est_[idx] = self._prior_patch(idx, depths[idx])
            self.poses_[idx] = dpvo_poses[idx].data


def create_se3_from_mat(mats):
    """[N, 4, 4] -> SE3 with data [t, qx, qy, qz, qw] (patchgraph.py:142-148)."""
    q = matrix_to_quaternion(mats[:, :3, :3])[:, [1, 2, 3, 0]]
    return SE3(torch.cat([mats[:, :3, 3], q], dim=1))
