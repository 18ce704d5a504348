"""Drop-in replacement for the reference's ``cuda_corr`` extension.

Same module name, functions and argument meaning as
dpvo/altcorr/correlation.cpp:57-62 (imported by dpvo/altcorr/correlation.py:2);
the work runs in libdpvo_hot.so (csrc/altcorr.hip) on the current HIP stream.
"""
import torch

import _dpvo_hot as H


def _check_corr_args(fmap1, fmap2, coords, ii, jj):
    H.on_gpu(fmap1, fmap2, coords, ii, jj)
    if fmap1.dtype != fmap2.dtype:
        raise RuntimeError("fmap1 and fmap2 must have the same dtype")
    if coords.dtype != torch.float32:
        raise RuntimeError("coords must be float32")
    if fmap1.dim() != 5 or fmap2.dim() != 5 or coords.dim() != 5:
        raise RuntimeError("expected fmap1 [B,N1,C,P,P], fmap2 [B,N2,C,H,W], coords [B,E,2,P,P]")


def forward(fmap1, fmap2, coords, ii, jj, radius):
    """correlation.cpp:28-35 -> [corr]; corr is the reference's permuted view
    [B, E, 2r+1 (x), 2r+1 (y), P, P] (correlation_kernel.cu:232)."""
    _check_corr_args(fmap1, fmap2, coords, ii, jj)
    B, E, _, Hh, W = coords.shape
    Do = 2 * radius + 1
    out = H.empty((B, E, Do, Do, Hh, W), dtype=fmap1.dtype, device=fmap1.device)
    ii, jj = H.idx64(ii), H.idx64(jj)
    H.check(H.lib().dpvo_corr_forward(
        H.dtype_code(fmap1), H.ptr(fmap1), H.sizes(fmap1), H.strides(fmap1), H.ptr(fmap2), H.sizes(fmap2),
        H.strides(fmap2), H.ptr(coords), H.sizes(coords), H.strides(coords), H.ptr(ii), H.ptr(jj), int(radius),
        H.ptr(out), H.stream_of(fmap1)))
    return [out.permute(0, 1, 3, 2, 4, 5)]


def pack(fmap1, out=None):
    """Patch features -> the fast path's scalar-operand table (dpvo_corr_pack).
    Re-pack whenever fmap1 (the gmap ring) changes."""
    H.on_gpu(fmap1)
    if fmap1.dtype != torch.float16 or fmap1.dim() != 5:
        raise RuntimeError("pack: fmap1 must be an fp16 [B, N1, C, 3, 3] tensor")
    nbytes = H.lib().dpvo_corr_table_bytes(H.sizes(fmap1))
    if out is None or out.numel() * out.element_size() < nbytes:
        out = H.empty((nbytes + 3) // 4, dtype=torch.int32, device=fmap1.device)
    H.check(H.lib().dpvo_corr_pack(H.ptr(fmap1), H.sizes(fmap1), H.strides(fmap1), H.ptr(out), H.stream_of(fmap1)))
    return out


def forward_pyramid(fmap1, pyramid, coords, ii, jj, radius, scales, out=None, table=None):
    """Fused form of DPVO.corr (dpvo/dpvo.py:326-333): all levels in one
    launch, returned in the stacked layout torch.stack([...], -1).view(B, E, -1).
    ``out`` may be a [B, E, F] view of wider rows (e.g. F = 882 of 896)."""
    for f in pyramid:
        _check_corr_args(fmap1, f, coords, ii, jj)
    B, E, _, Hh, W = coords.shape
    L = len(pyramid)
    Do = 2 * radius + 1
    F = Do * Do * Hh * W * L
    if out is None:
        out = H.empty((B, E, F), dtype=fmap1.dtype, device=fmap1.device)
    elif (out.shape != (B, E, F) or out.dtype != fmap1.dtype or out.stride(2) != 1 or
          (B > 1 and out.stride(0) != E * out.stride(1))):
        raise RuntimeError("forward_pyramid: out must be [B, E, F] with unit feature stride")
    ii, jj = H.idx64(ii), H.idx64(jj)
    ptrs = (H._vp * L)(*[f.data_ptr() for f in pyramid])
    fs = H.i64arr([s for f in pyramid for s in f.shape])
    fst = H.i64arr([s for f in pyramid for s in f.stride()])
    sc = (H._fp * L)(*[float(s) for s in scales])
    H.check(H.lib().dpvo_corr_forward_pyramid_ld(
        H.dtype_code(fmap1), H.ptr(fmap1), H.sizes(fmap1), H.strides(fmap1), L, ptrs, fs, fst, sc, H.ptr(coords),
        H.sizes(coords), H.strides(coords), H.ptr(ii), H.ptr(jj), int(radius), H.ptr(out),
        out.stride(1) if E > 0 else 0, H.ptr(table), H.stream_of(fmap1)))
    return out


def pack_mfma(fmap1, out=None):
    """The gmap ring [1, N1, 128, 3, 3] transposed to [N1, 9, 128] for the
    matrix-core correlation (dpvo_corr_pack_mfma); re-pack when it changes."""
    H.on_gpu(fmap1)
    if fmap1.dtype != torch.float16 or fmap1.dim() != 5 or fmap1.shape[0] != 1 or tuple(fmap1.shape[2:]) != (128, 3, 3):
        raise RuntimeError("pack_mfma: fmap1 must be an fp16 [1, N1, 128, 3, 3] tensor")
    n = fmap1.shape[1] * 9 * 128
    if out is None or out.numel() < n:
        out = H.empty(n, dtype=torch.float16, device=fmap1.device)
    H.check(H.lib().dpvo_corr_pack_mfma(H.ptr(fmap1), H.sizes(fmap1), H.strides(fmap1), H.ptr(out),
                                        H.stream_of(fmap1)))
    return out


def edge_order(jj, num_frames):
    """int32 permutation of the edges grouped by target frame jj (in
    [0, num_frames)): the L2-friendly visiting order of forward_pyramid_mfma."""
    H.on_gpu(jj)
    jj = H.idx64(jj)
    order = H.empty(max(jj.numel(), 1), dtype=torch.int32, device=jj.device)
    nbytes = H.lib().dpvo_edge_order_workspace_bytes(int(num_frames))
    ws = H.empty(nbytes, dtype=torch.uint8, device=jj.device)
    H.check(H.lib().dpvo_edge_order(H.ptr(jj), jj.numel(), int(num_frames), H.ptr(order), H.ptr(ws), nbytes,
                                    H.stream_of(jj)))
    return order[:jj.numel()]


def forward_pyramid_mfma(table, num_patches, pyramid, coords, ii, jj, scales=(1, 4), out=None, order=None):
    """DPVO.corr's two levels on the matrix cores (csrc/corrmfma.hip): the
    stacked [1, E, 882] rows of forward_pyramid (radius 3, 3x3 patches), with
    fp32 accumulation instead of the reference's fp16 chain (not bit-identical;
    see include/dpvo_hot.h).  table = pack_mfma(gmap); order (optional) =
    edge_order(jj, frames): a visiting order only, the output is the same."""
    H.on_gpu(table, coords, ii, jj, *pyramid)
    if len(pyramid) != 2 or any(f.dtype != torch.float16 for f in pyramid):
        raise RuntimeError("forward_pyramid_mfma: two fp16 pyramid levels")
    if coords.dtype != torch.float32 or coords.dim() != 5 or tuple(coords.shape[2:]) != (2, 3, 3):
        raise RuntimeError("forward_pyramid_mfma: coords must be float32 [1, E, 2, 3, 3]")
    E = coords.shape[1]
    if out is None:
        out = H.empty((1, E, 882), dtype=torch.float16, device=coords.device)
    elif out.shape != (1, E, 882) or out.dtype != torch.float16 or out.stride(2) != 1:
        raise RuntimeError("forward_pyramid_mfma: out must be [1, E, 882] fp16 with unit feature stride")
    ii, jj = H.idx64(ii), H.idx64(jj)
    ptrs = (H._vp * 2)(*[f.data_ptr() for f in pyramid])
    fs = H.i64arr([s for f in pyramid for s in f.shape])
    fst = H.i64arr([s for f in pyramid for s in f.stride()])
    sc = (H._fp * 2)(*[float(s) for s in scales])
    if order is not None:
        H.on_gpu(order)
        if order.dtype != torch.int32 or order.numel() != E or not order.is_contiguous():
            raise RuntimeError("forward_pyramid_mfma: order must be a contiguous int32 permutation of the E edges")
    H.check(H.lib().dpvo_corr_pyramid_mfma(
        H.ptr(table), int(num_patches), ptrs, fs, fst, sc, H.ptr(coords), H.sizes(coords), H.strides(coords),
        H.ptr(ii), H.ptr(jj), H.ptr(out), out.stride(1) if E > 0 else 0, H.ptr(order), H.stream_of(coords)))
    return out


def backward(fmap1, fmap2, coords, ii, jj, grad, radius):
    """correlation.cpp:37-45 / correlation_kernel.cu:236-286 -> [fmap1_grad, fmap2_grad]."""
    _check_corr_args(fmap1, fmap2, coords, ii, jj)
    g1 = torch.zeros_like(fmap1).contiguous()
    g2 = torch.zeros_like(fmap2).contiguous()
    f1, f2, c = fmap1.contiguous(), fmap2.contiguous(), coords.contiguous()
    grad = grad.float().contiguous()
    ii, jj = H.idx64(ii), H.idx64(jj)
    H.check(H.lib().dpvo_corr_backward(
        H.dtype_code(f1), H.ptr(f1), H.sizes(f1), H.ptr(f2), H.sizes(f2), H.ptr(c), H.sizes(c), H.ptr(ii), H.ptr(jj),
        H.ptr(grad), int(radius), H.ptr(g1), H.ptr(g2), H.stream_of(f1)))
    return [g1, g2]


def patchify_forward(net, coords, radius):
    """correlation.cpp:47-50 / correlation_kernel.cu:288-308 -> [patches [B,M,C,D,D]]."""
    H.on_gpu(net, coords)
    if coords.dtype != torch.float32:
        raise RuntimeError("coords must be float32")
    B, C = net.shape[0], net.shape[1]
    coords = coords.contiguous()
    M = coords.shape[1]
    D = 2 * radius + 2
    out = H.empty((B, M, C, D, D), dtype=net.dtype, device=net.device)
    H.check(H.lib().dpvo_patchify_forward(H.dtype_code(net), H.ptr(net), H.sizes(net), H.strides(net), H.ptr(coords),
                                          M, int(radius), H.ptr(out), H.stream_of(net)))
    return [out]


def patchify_backward(net, coords, gradient, radius):
    """correlation.cpp:52-55 / correlation_kernel.cu:310-333 -> [net_gradient]."""
    H.on_gpu(net, coords, gradient)
    coords = coords.contiguous()
    grad = gradient.contiguous()
    out = torch.zeros(net.shape, dtype=net.dtype, device=net.device)
    H.check(H.lib().dpvo_patchify_backward(H.dtype_code(net), H.sizes(net), H.ptr(coords), coords.shape[1],
                                           int(radius), H.ptr(grad), H.ptr(out), H.stream_of(net)))
    return [out]
