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


def matrix_to_quaternion(matrix):
    """rotation matrices [..., 3, 3] -> unit quaternions [..., 4] as (w, x, y,
    z) with w >= 0 (reference utils.py:118-167).  Of the four algebraically
    equal candidates (each divides by one of 4w^2, 4x^2, 4y^2, 4z^2) the one
    with the largest divisor is kept, as the reference does."""
    if matrix.shape[-2:] != (3, 3):
        raise ValueError(f"Invalid rotation matrix shape {tuple(matrix.shape)}.")
    m = matrix.reshape(matrix.shape[:-2] + (9,))
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = m.unbind(-1)
    four_sq = torch.stack([1 + m00 + m11 + m22, 1 + m00 - m11 - m22,
                           1 - m00 + m11 - m22, 1 - m00 - m11 + m22], -1)
    r = torch.sqrt(four_sq.clamp(min=0))  # 2|w|, 2|x|, 2|y|, 2|z|
    # candidate c scaled by r_c: rows (w, x, y, z) * r_c
    cand = torch.stack([
        torch.stack([r[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        torch.stack([m21 - m12, r[..., 1] ** 2, m10 + m01, m02 + m20], -1),
        torch.stack([m02 - m20, m10 + m01, r[..., 2] ** 2, m12 + m21], -1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, r[..., 3] ** 2], -1)], -2)
    cand = cand / (2.0 * r.clamp(min=0.1))[..., None]
    best = r.argmax(-1)
    q = torch.gather(cand, -2, best[..., None, None].expand(best.shape + (1, 4))).squeeze(-2)
    return torch.where(q[..., :1] < 0, -q, q)
