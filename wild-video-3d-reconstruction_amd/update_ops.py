"""Native glue of the learned update operator (csrc/updateop.hip).

Replaces torch_scatter 2.1.2's ``scatter_softmax`` + ``scatter_sum`` in
SoftAgg (reference dpvo/blocks.py:40-48) and the masked neighbour gather of
Update.forward (dpvo/net.py:82-85).  Inference only (no autograd); the
dpvo.blocks / dpvo.net mirrors call these under ``torch.no_grad`` and keep a
torch composition for training.  Like the other shims there is no CPU path.
"""
import torch

import _dpvo_hot as H


def softagg(f, s, group, groups, eps=1e-12):
    """y[g] = sum_{e: group[e]==g} f[e] * softmax_g(s)[e]  (per channel).

    f, s: [E, D] with unit channel stride and any row stride (two column
    halves of one fused GEMM output work); group: [E] int64 in [0, groups);
    returns y [groups, D] of f's dtype."""
    H.on_gpu(f, s, group)
    if f.dim() != 2 or s.shape != f.shape:
        raise RuntimeError("softagg: f and s must both be [E, D]")
    if f.dtype != s.dtype:
        raise RuntimeError("softagg: f and s must have the same dtype")
    if f.stride(1) != 1 or s.stride(1) != 1:
        raise RuntimeError("softagg: rows must be channel-contiguous")
    E, D = f.shape
    group = H.idx64(group)
    y = torch.empty(groups, D, dtype=f.dtype, device=f.device)
    nbytes = H.lib().dpvo_softagg_workspace_bytes(E, groups)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=f.device)
    H.check(H.lib().dpvo_softagg_forward(H.dtype_code(f), H.ptr(f), f.stride(0), H.ptr(s), s.stride(0),
                                         H.ptr(group), E, D, groups, float(eps), H.ptr(y), H.ptr(ws), nbytes,
                                         H.stream_of(f)))
    return y


def gather_rows(x, idx, dtype=None):
    """out[e] = x[idx[e]] if idx[e] >= 0 else 0, cast to ``dtype`` (default x's).
    x: [R, D] with unit channel stride; idx: [n] int64."""
    H.on_gpu(x, idx)
    if x.dim() != 2 or x.stride(1) != 1:
        raise RuntimeError("gather_rows: x must be [R, D] with contiguous rows")
    dtype = dtype or x.dtype
    idx = H.idx64(idx)
    out = torch.empty(idx.numel(), x.shape[1], dtype=dtype, device=x.device)
    H.check(H.lib().dpvo_gather_rows(H.dtype_code(x), H.ptr(x), x.stride(0), x.shape[0], H.ptr(idx), idx.numel(),
                                     x.shape[1], H.dtype_code(out), H.ptr(out), H.stream_of(x)))
    return out
