"""Seeded synthetic workloads: steady-state tracker injection
and smooth random image streams.  No datasets or checkpoints are available,
so the network has seeded random weights."""
import math

import torch

from . import altcorr
from .config import make_cfg
from .dpvo import DPVO
from .lietorch import SE3
from .net import VONet

TARTAN_CALIB = (320.0, 320.0, 320.0, 240.0)  # calib/tartan.txt


def steady_state_edges(n, M, lifetime, removal, device):
    """Edge set seen by update() at n frames in steady state: the append rules
    of dpvo.py:756-769 for every recent frame, filtered by the removal rule
    (dpvo.py:657) as of the previous keyframe; chronological order."""
    ii, jj, kk = [], [], []
    for t in range(max(1, n - removal - 2), n + 1):
        k_f = torch.arange(M * max(t - lifetime, 0), M * max(t - 1, 0))
        ii.append(k_f // M); jj.append(torch.full_like(k_f, t - 1)); kk.append(k_f)
        kb = torch.arange(M * (t - 1), M * t)
        jb = torch.arange(max(t - lifetime, 0), t)
        k_b = kb.repeat_interleave(len(jb))
        ii.append(k_b // M); jj.append(jb.repeat(len(kb))); kk.append(k_b)
    ii, jj, kk = torch.cat(ii), torch.cat(jj), torch.cat(kk)
    keep = ii >= n - 1 - removal
    return ii[keep].to(device), jj[keep].to(device), kk[keep].to(device)


@torch.no_grad()
def steady_state_tracker(preset="dpvo_2k", buffer=2048, n=None, seed=0, ht=384, wd=512, device="cuda",
                         iterations=None, **overrides):
    """A DPVO instance whose patch graph is in the steady state of a long
    sequence (n = buffer - 8 keyframes by default), ready for update()."""
    torch.manual_seed(seed)
    cfg = make_cfg(preset, BUFFER_SIZE=buffer, **overrides)
    if iterations is not None:
        cfg.BA_ITERATIONS = iterations
    net = VONet()
    slam = DPVO(cfg, net, ht=ht, wd=wd, device=device)
    dev = slam.device
    n = buffer - 8 if n is None else n
    M, P, pmem = slam.M, slam.P, slam.pmem
    h, w = ht // slam.RES, wd // slam.RES
    g = torch.Generator().manual_seed(seed + 1)

    # poses: damped random walk (world->camera)
    xi = torch.cat([0.05 * torch.randn(n, 3, generator=g), 0.01 * torch.randn(n, 3, generator=g)], -1)
    steps = SE3.exp(xi.to(dev))
    poses = torch.zeros(n, 7, device=dev)
    poses[0, 6] = 1
    cur = SE3(poses[0:1])
    for i in range(1, n):
        cur = steps[i:i + 1] * cur
        poses[i] = cur.data[0]
    slam.pg.poses_[:n] = poses

    # patches: random integer centres (net.py:151-152), inverse depth U[0.2, 1]
    g2 = torch.Generator().manual_seed(seed + 2)
    xs = torch.randint(1, w - 1, (n, M), generator=g2).float()
    ys = torch.randint(1, h - 1, (n, M), generator=g2).float()
    d = 0.2 + 0.8 * torch.rand(n, M, generator=g2)
    off = torch.arange(P, dtype=torch.float) - P // 2
    pt = torch.empty(n, M, 3, P, P)
    pt[:, :, 0] = xs[..., None, None] + off.view(1, 1, 1, P)
    pt[:, :, 1] = ys[..., None, None] + off.view(1, 1, P, 1)
    pt[:, :, 2] = d[..., None, None]
    slam.pg.patches_[:n] = pt.to(dev)
    slam.pg.intrinsics_[:n] = torch.tensor(TARTAN_CALIB, device=dev) / slam.RES
    slam.pg.index_[:n + 1] = torch.arange(n + 1, device=dev)[:, None]
    slam.pg.tstamps_[:n] = range(n)

    # feature rings: fp16 N(0, 0.25^2); gmap = 3x3 gather at the patch centres
    g3 = torch.Generator(device=dev).manual_seed(seed + 3)
    for s in range(pmem):
        f = (0.25 * torch.randn(128, h, w, generator=g3, device=dev)).to(slam.fmap1_.dtype)
        slam.fmap1_[0, s] = f
        slam.fmap2_[0, s] = torch.nn.functional.avg_pool2d(f[None].float(), 4, 4)[0].to(slam.fmap2_.dtype)
    for f in range(max(0, n - pmem), n):
        s = f % pmem
        centres = torch.stack([xs[f], ys[f]], -1)[None].to(dev)
        slam.gmap_[s] = altcorr.patchify(slam.fmap1_[0, s][None], centres, P // 2).view(M, 128, P, P)
        slam.imap_[s] = torch.randn(M, slam.DIM, generator=g3, device=dev).to(slam.imap_.dtype)

    # edges and hidden state
    ii, jj, kk = steady_state_edges(n, M, cfg.PATCH_LIFETIME, cfg.REMOVAL_WINDOW, dev)
    slam.pg.ii, slam.pg.jj, slam.pg.kk = ii, jj, kk
    # fp32: after its first update() the reference's edge state is the fp32
    # LayerNorm output (autocast), and appended fp16 zeros promote to it
    slam.pg.net = 0.1 * torch.randn(1, len(ii), slam.DIM, generator=g3, device=dev)
    slam.pg.weight = torch.zeros(1, len(ii), 2, device=dev)
    slam.pg.target = torch.zeros(1, len(ii), 2, device=dev)
    slam.pg.n, slam.pg.m = n, n * M
    slam.counter = n
    slam.tlist = list(range(n))
    slam.is_initialized = True
    return slam


def image_stream(num, ht=384, wd=512, seed=0, device="cuda"):
    """Smooth value-noise textures translating across frames (uint8 [3,H,W])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    base = torch.rand(1, 3, ht // 16 + 4, wd // 16 + 4, generator=g)
    big = torch.nn.functional.interpolate(base, scale_factor=16, mode="bicubic", align_corners=False)
    for t in range(num):
        dx, dy = int(2 * t), int(math.sin(t / 5.0) * 6)
        img = torch.roll(big, shifts=(dy, dx), dims=(2, 3))[0, :, :ht, :wd]
        yield t, (img.clamp(0, 1) * 255).to(torch.uint8).to(device)
