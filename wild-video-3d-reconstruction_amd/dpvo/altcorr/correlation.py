"""altcorr operator surface (reference dpvo/altcorr/correlation.py:4-75) over
the cuda_corr drop-in (csrc/altcorr.hip)."""
import torch

import cuda_corr


class CorrLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, coords, ii, jj, radius, dropout):
        ctx.save_for_backward(fmap1, fmap2, coords, ii, jj)
        ctx.radius, ctx.dropout = radius, dropout
        return cuda_corr.forward(fmap1, fmap2, coords, ii, jj, radius)[0]

    @staticmethod
    def backward(ctx, grad):
        fmap1, fmap2, coords, ii, jj = ctx.saved_tensors
        if ctx.dropout < 1:  # train-time edge dropout (correlation.py:20-25)
            keep = torch.rand(len(ii), device=ii.device) < ctx.dropout
            coords, grad, ii, jj = coords[:, keep], grad[:, keep], ii[keep], jj[keep]
        g1, g2 = cuda_corr.backward(fmap1, fmap2, coords, ii, jj, grad, ctx.radius)
        return g1, g2, None, None, None, None, None


class PatchLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, coords, radius):
        ctx.radius = radius
        ctx.save_for_backward(net, coords)
        return cuda_corr.patchify_forward(net, coords, radius)[0]

    @staticmethod
    def backward(ctx, grad):
        net, coords = ctx.saved_tensors
        return cuda_corr.patchify_backward(net, coords, grad, ctx.radius)[0], None, None


def patchify(net, coords, radius, mode="bilinear"):
    """Gather (2r+2)^2 windows at floor(coords); 'bilinear' then reduces them
    to (2r+1)^2 with the fractional offsets (correlation.py:51-69)."""
    patches = PatchLayer.apply(net, coords, radius)
    if mode != "bilinear":
        return patches
    frac = coords - coords.floor()
    dx, dy = frac[:, :, None, None, None].unbind(dim=-1)
    d = 2 * radius + 1
    return ((1 - dy) * (1 - dx) * patches[..., :d, :d] + (1 - dy) * dx * patches[..., :d, 1:]
            + dy * (1 - dx) * patches[..., 1:, :d] + dy * dx * patches[..., 1:, 1:])


def corr(fmap1, fmap2, coords, ii, jj, radius=1, dropout=1):
    """One pyramid level: [B, E, 2r+1 (x), 2r+1 (y), P, P] (correlation.py:72-73)."""
    return CorrLayer.apply(fmap1, fmap2, coords, ii, jj, radius, dropout)


def corr_pyramid(gmap, pyramid, coords, ii, jj, radius=3, levels=(1, 4), out=None, table=None):
    """All pyramid levels in one fused launch, already in the stacked layout
    DPVO.corr builds with torch.stack(..., -1).view(1, E, -1) (dpvo.py:326-333).
    ``out``: optional [1, E, F] destination view (rows may be wider than F);
    ``table``: gmap packed by cuda_corr.pack (packed per call when None).
    Inference only (no autograd)."""
    return cuda_corr.forward_pyramid(gmap, list(pyramid), coords, ii, jj, radius, list(levels), out=out, table=table)


def corr_pyramid_mfma(table, num_patches, pyramid, coords, ii, jj, levels=(1, 4), out=None, order=None):
    """corr_pyramid's two levels (radius 3, 3x3 patches) on the matrix cores:
    fp32 accumulation of the 128-channel products instead of the reference's
    fp16 chain (more accurate; not bit-identical).  table = cuda_corr.pack_mfma(gmap)."""
    return cuda_corr.forward_pyramid_mfma(table, num_patches, list(pyramid), coords, ii, jj, list(levels), out=out,
                                          order=order)


