"""Patchifier and learned update operator (reference dpvo/net.py:28-176).

These are the hot path's callers and stay PyTorch (hipBLASLt GEMMs); their
native pieces -- altcorr.patchify and fastba.neighbors -- run on the HIP
library.  Parameter names follow the reference so dpvo.pth loads unchanged.
Training (VONet.forward, net.py:355-440) is out of scope for this build.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

import update_ops

from . import altcorr, fastba
from .blocks import GatedResidual, GradientClip, SoftAgg
from .extractor import BasicEncoder4
from .utils import coords_grid_with_index

DIM = 384


class Update(nn.Module):
    def __init__(self, p):
        super().__init__()
        mlp = lambda: nn.Sequential(nn.Linear(DIM, DIM), nn.ReLU(inplace=True), nn.Linear(DIM, DIM))
        self.c1, self.c2 = mlp(), mlp()
        self.norm = nn.LayerNorm(DIM, eps=1e-3)
        self.agg_kk = SoftAgg(DIM)
        self.agg_ij = SoftAgg(DIM)
        self.gru = nn.Sequential(nn.LayerNorm(DIM, eps=1e-3), GatedResidual(DIM),
                                 nn.LayerNorm(DIM, eps=1e-3), GatedResidual(DIM))
        self.corr = nn.Sequential(nn.Linear(2 * 49 * p * p, DIM), nn.ReLU(inplace=True), nn.Linear(DIM, DIM),
                                  nn.LayerNorm(DIM, eps=1e-3), nn.ReLU(inplace=True), nn.Linear(DIM, DIM))
        self.d = nn.Sequential(nn.ReLU(inplace=False), nn.Linear(DIM, 2), GradientClip())
        self.w = nn.Sequential(nn.ReLU(inplace=False), nn.Linear(DIM, 2), GradientClip(), nn.Sigmoid())

    def forward(self, net, inp, corr, flow, ii, jj, kk):
        """edge hidden state -> (new state, (delta, weight, None)) (net.py:75-93)."""
        net = self.norm(net + inp + self.corr(corr))
        ix, jx = fastba.neighbors(kk, jj)  # temporal neighbours of the same patch, on the device
        net = net + self.c1(self._neighbour(net, ix))
        net = net + self.c2(self._neighbour(net, jx))
        net = net + self.agg_kk(net, kk)
        net = net + self.agg_ij(net, ii * 12345 + jj)
        net = self.gru(net)
        return net, (self.d(net), self.w(net), None)


    @staticmethod
    def _neighbour(net, ix):
        """mask_ix * net[:, ix] (net.py:82-85).  Inference: one native gather
        that writes zeros for ix < 0 and casts straight to the autocast dtype
        the following Linear would cast to anyway."""
        if torch.is_grad_enabled() and net.requires_grad:
            return (ix >= 0).to(net.dtype).view(1, -1, 1) * net[:, ix]
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else net.dtype
        return update_ops.gather_rows(net[0], ix, dtype=dt)[None]


class Patchifier(nn.Module):
    def __init__(self, patch_size=3):
        super().__init__()
        self.patch_size = patch_size
        self.fnet = BasicEncoder4(output_dim=128, norm_fn="instance")
        self.inet = BasicEncoder4(output_dim=DIM, norm_fn="none")

    def _image_gradient(self, images):
        gray = ((images + 0.5) * (255.0 / 2)).sum(dim=2)
        dx = gray[..., :-1, 1:] - gray[..., :-1, :-1]
        dy = gray[..., 1:, :-1] - gray[..., :-1, :-1]
        return F.avg_pool2d(torch.sqrt(dx ** 2 + dy ** 2), 4, 4)

    def forward(self, images, patches_per_image=80, disps=None, gradient_bias=False, return_color=False, mask=None,
                sp_extractor=None):
        """image [3,H,W] uint8 -> fmap, gmap, imap, patches, index[, colours] (net.py:260-325)."""
        if sp_extractor is not None:
            raise NotImplementedError("SuperPoint keypoints are out of scope")
        images = 2 * (images[None, None] / 255.0) - 0.5
        fmap = self.fnet(images) / 4.0
        imap = self.inet(images) / 4.0
        b, n, c, h, w = fmap.shape
        P, dev = self.patch_size, images.device

        if gradient_bias:
            g = self._image_gradient(images)
            x = torch.randint(1, w - 1, size=[n, 3 * patches_per_image], device=dev)
            y = torch.randint(1, h - 1, size=[n, 3 * patches_per_image], device=dev)
            score = altcorr.patchify(g[0, :, None], torch.stack([x, y], -1).float(), 0).view(n, -1)
            top = torch.argsort(score, dim=1)[:, -patches_per_image:]
            x, y = torch.gather(x, 1, top), torch.gather(y, 1, top)
        elif mask is not None:
            valid = (torch.nonzero(mask, as_tuple=False) / 4).floor()
            valid = valid[(valid[:, 1] < w - 1) & (valid[:, 0] < h - 1)]
            valid = torch.unique(valid, dim=0)
            pick = valid[torch.randperm(valid.shape[0], device=valid.device)[:n * patches_per_image]]
            x, y = pick[:, 1].view(n, -1), pick[:, 0].view(n, -1)
        else:
            x = torch.randint(1, w - 1, size=[n, patches_per_image], device=dev)
            y = torch.randint(1, h - 1, size=[n, patches_per_image], device=dev)

        coords = torch.stack([x, y], dim=-1).float()
        imap = altcorr.patchify(imap[0], coords, 0).view(b, -1, DIM, 1, 1)
        gmap = altcorr.patchify(fmap[0], coords, P // 2).view(b, -1, 128, P, P)
        clr = altcorr.patchify(images[0], 4 * (coords + 0.5), 0).view(b, -1, 3) if return_color else None
        if disps is None:
            disps = torch.ones(b, n, h, w, device=dev)
        grid, _ = coords_grid_with_index(disps, device=fmap.device)
        patches = altcorr.patchify(grid[0], coords, P // 2).view(b, -1, 3, P, P)
        index = torch.arange(n, device=dev).view(n, 1).repeat(1, patches_per_image).reshape(-1)
        if return_color:
            return fmap, gmap, imap, patches, index, clr
        return fmap, gmap, imap, patches, index


class VONet(nn.Module):
    def __init__(self, use_viewer=False):
        super().__init__()
        self.P = 3
        self.patchify = Patchifier(self.P)
        self.update = Update(self.P)
        self.DIM = DIM
        self.RES = 4

    def forward(self, *args, **kwargs):
        raise NotImplementedError("VONet training (net.py:355-440) is out of scope for the MI355X hot-path build")
