"""Helpers used by the tracker (reference dpvo/utils.py:10-89; the cv2 image
helpers are out of scope)."""
import torch
import torch.nn.functional as F

all_times = []


class Timer:
    """Event-timed region on the current HIP stream (reference utils.py:10-31)."""

    def __init__(self, name, enabled=True):
        self.name, self.enabled = name, enabled
        if enabled:
            self.start = torch.cuda.Event(enable_timing=True)
            self.end = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        if self.enabled:
            self.start.record()

    def __exit__(self, *exc):
        if self.enabled:
            self.end.record()
            torch.cuda.synchronize()
            elapsed = self.start.elapsed_time(self.end)
            all_times.append(elapsed)
            print(self.name, elapsed)


def coords_grid(b, n, h, w, **kwargs):
    x = torch.arange(0, w, dtype=torch.float, **kwargs)
    y = torch.arange(0, h, dtype=torch.float, **kwargs)
    yy, xx = torch.meshgrid(y, x, indexing="ij")
    return torch.stack([xx, yy]).view(1, 1, 2, h, w).repeat(b, n, 1, 1, 1)


def coords_grid_with_index(d, **kwargs):
    """per-pixel (x, y, d) grid and frame index (reference utils.py:41-56)."""
    b, n, h, w = d.shape
    x = torch.arange(0, w, dtype=torch.float, **kwargs)
    y = torch.arange(0, h, dtype=torch.float, **kwargs)
    yy, xx = torch.meshgrid(y, x, indexing="ij")
    coords = torch.stack([xx.expand(b, n, h, w), yy.expand(b, n, h, w), d], dim=2)
    index = torch.arange(0, n, dtype=torch.float, **kwargs).view(1, n, 1, 1, 1).expand(b, n, 1, h, w)
    return coords, index.contiguous()


def patchify(x, patch_size=3):
    b, n, c, h, w = x.shape
    y = F.unfold(x.view(b * n, c, h, w), patch_size).transpose(1, 2)
    return y.reshape(b, -1, c, patch_size, patch_size)


def pyramidify(fmap, lvls=(1,)):
    b, n, c, h, w = fmap.shape
    return [F.avg_pool2d(fmap.view(b * n, c, h, w), l, stride=l).view(b, n, c, h // l, w // l) for l in lvls]


def all_pairs_exclusive(n, **kwargs):
    ii, jj = torch.meshgrid(torch.arange(n, **kwargs), torch.arange(n, **kwargs), indexing="ij")
    k = ii != jj
    return ii[k].reshape(-1), jj[k].reshape(-1)


def set_depth(patches, depth):
    patches[..., 2, :, :] = depth[..., None, None]
    return patches


def flatmeshgrid(*args, **kwargs):
    return (x.reshape(-1) for x in torch.meshgrid(*args, **kwargs))
