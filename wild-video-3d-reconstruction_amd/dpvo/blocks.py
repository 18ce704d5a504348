"""Update-operator building blocks (reference dpvo/blocks.py:15-118).

SoftAgg's grouped softmax/sum used torch-scatter 2.1.2 in the reference
(absent on ROCm wheels).  Inference runs it as one HIP pass
(update_ops.softagg, csrc/updateop.hip) over a single fused f|g GEMM; with
autograd on (training) it falls back to the torch composition below (native
scatter_reduce / index_add, same eps and max-recentring as
torch_scatter.scatter_softmax).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

import update_ops


def scatter_sum(src, index, dim, dim_size):
    shape = list(src.shape)
    shape[dim] = dim_size
    return torch.zeros(shape, dtype=src.dtype, device=src.device).index_add_(dim, index, src)


def scatter_softmax(src, index, dim, dim_size, eps=1e-12):
    idx = index.view([1] * dim + [-1] + [1] * (src.dim() - dim - 1)).expand_as(src)
    shape = list(src.shape)
    shape[dim] = dim_size
    gmax = torch.full(shape, float("-inf"), dtype=src.dtype, device=src.device)
    gmax = gmax.scatter_reduce(dim, idx, src, reduce="amax", include_self=True)
    ex = (src - gmax.gather(dim, idx)).exp()
    den = scatter_sum(ex, index, dim, dim_size) + eps
    return ex / den.gather(dim, idx)


class GatedResidual(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.gate = nn.Sequential(nn.Linear(dim, dim), nn.Sigmoid())
        self.res = nn.Sequential(nn.Linear(dim, dim), nn.ReLU(inplace=True), nn.Linear(dim, dim))

    def forward(self, x):
        return x + self.gate(x) * self.res(x)


class SoftAgg(nn.Module):
    """Softmax-weighted aggregation over edges sharing a key (blocks.py:31-48)."""

    def __init__(self, dim=512, expand=True):
        super().__init__()
        self.dim, self.expand = dim, expand
        self.f = nn.Linear(dim, dim)
        self.g = nn.Linear(dim, dim)
        self.h = nn.Linear(dim, dim)
        self._fg = None

    def _fused_fg(self):
        """[f; g] weights for one [E, 2D] GEMM, rebuilt when either changes."""
        key = tuple((p.data_ptr(), p._version) for p in (self.f.weight, self.f.bias, self.g.weight, self.g.bias))
        if self._fg is None or self._fg[0] != key:
            w = torch.cat([self.f.weight, self.g.weight], 0)
            b = torch.cat([self.f.bias, self.g.bias], 0)
            self._fg = (key, w, b)
        return self._fg[1], self._fg[2]

    def forward(self, x, ix):
        uniq, jx = torch.unique(ix, return_inverse=True)
        groups = uniq.numel()
        if torch.is_grad_enabled() and x.requires_grad:
            w = scatter_softmax(self.g(x), jx, 1, groups)
            y = scatter_sum(self.f(x) * w, jx, 1, groups)
        else:
            w, b = self._fused_fg()
            fg = F.linear(x[0], w, b)
            D = self.dim
            y = update_ops.softagg(fg[:, :D], fg[:, D:], jx, groups)[None]
        return self.h(y)[:, jx] if self.expand else self.h(y)


class GradClip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        g = torch.where(torch.isnan(g), torch.zeros_like(g), g)
        return g.clamp(min=-0.01, max=0.01)


class GradientClip(nn.Module):
    def forward(self, x):
        return GradClip.apply(x)
