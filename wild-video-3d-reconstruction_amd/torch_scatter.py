"""Drop-in ``torch_scatter`` (2.1.2 semantics) over the HIP library.

The reference imports torch_scatter in dpvo/blocks.py:5 (scatter_softmax /
scatter_sum in SoftAgg, :42-43), dpvo/net.py:8-9, dpvo/ba.py:2 (scatter_sum,
:40-56) and dpvo/loop_closure/long_term.py:11 (scatter_max, :134).  There is
no ROCm wheel of torch-scatter; this module, on the path next to the
``cuda_corr`` / ``cuda_ba`` / ``lietorch_backends`` shims, lets the
reference's Python import and run unchanged.  Every reduction is one
``dpvo_scatter_csr`` launch over the device group-by of the index
(csrc/updateop.hip): deterministic (members summed in ascending order), no
atomics.  Like the other shims it refuses CPU tensors.

Supported: a 1-D index along ``dim`` (the form every reference call uses), or
an index shaped like ``src`` that is constant off ``dim`` (size 1 there).
Not differentiable (inference surface, as the reference's tracker uses it).
"""
import torch

import _dpvo_hot as H
import update_ops as U

__version__ = "2.1.2"

__all__ = ["scatter", "scatter_sum", "scatter_add", "scatter_mean", "scatter_max", "scatter_softmax"]


def _prep(src, index, dim):
    if not torch.is_floating_point(src):
        raise ValueError("torch_scatter (HIP): src must be a floating point tensor")
    H.on_gpu(src, index)
    dim = dim % src.dim() if src.dim() else 0
    if index.dim() != 1:
        if index.dim() != src.dim() or any(s != 1 for d, s in enumerate(index.shape) if d != dim):
            raise RuntimeError("torch_scatter (HIP): index must be 1-D along dim (or broadcast to it)")
        index = index.reshape(-1)
    E = src.shape[dim]
    if index.numel() != E:
        raise RuntimeError(f"torch_scatter (HIP): index has {index.numel()} entries, src has {E} along dim {dim}")
    outer = 1
    for s in src.shape[:dim]:
        outer *= s
    inner = 1
    for s in src.shape[dim + 1:]:
        inner *= s
    src3 = src.contiguous().view(outer, E, inner)
    index = H.idx64(index)
    return dim, src3, index, outer, E, inner


def _out_shape(src, dim, dim_size):
    shape = list(src.shape)
    shape[dim] = dim_size
    return shape


def _dim_size(index, dim_size):
    if dim_size is not None:
        return int(dim_size)
    return int(index.max().item()) + 1 if index.numel() else 0


def _check_range(index, dim_size=None):
    """torch_scatter 2.1.2 fails on an index outside [0, dim_size) (an
    index-out-of-bounds error); the CSR kernel would skip such members
    silently, so the range is checked first.  One host read: this module is
    the compatibility surface, the tracker's SoftAgg does not come through it."""
    if index.numel() == 0:
        return
    lo, hi = torch.stack([index.min(), index.max()]).tolist()
    if lo < 0 or (dim_size is not None and hi >= dim_size):
        raise IndexError(f"torch_scatter (HIP): index out of range (min {lo}, max {hi}) for an output of "
                         f"{dim_size if dim_size is not None else 'inferred'} rows")


def _reduce(op, src, index, dim, out, dim_size):
    dim, src3, index, outer, E, inner = _prep(src, index, dim)
    if out is None:
        dim_size = _dim_size(index, dim_size)
        out = torch.zeros(_out_shape(src, dim, dim_size), dtype=src.dtype, device=src.device)
    else:
        H.on_gpu(out)
        if out.dtype != src.dtype or not out.is_contiguous():
            raise RuntimeError("torch_scatter (HIP): out must be contiguous and of src's dtype")
        dim_size = out.shape[dim]
    _check_range(index, dim_size)
    if E:
        U.scatter_csr(op, src3, index, U.group_by(index), out, out_rows=dim_size)
    return out


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(U.SCATTER_SUM, src, index, dim, out, dim_size)


scatter_add = scatter_sum


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(U.SCATTER_MEAN, src, index, dim, out, dim_size)


def scatter_max(src, index, dim=-1, out=None, dim_size=None):
    """(max, argmax): empty rows 0 and argmax = src.size(dim), as torch_scatter."""
    if out is not None:
        raise NotImplementedError("torch_scatter (HIP): scatter_max with out= is not supported")
    dim, src3, index, outer, E, inner = _prep(src, index, dim)
    dim_size = _dim_size(index, dim_size)
    shape = _out_shape(src, dim, dim_size)
    out = torch.zeros(shape, dtype=src.dtype, device=src.device)
    arg = torch.full(shape, E, dtype=torch.int64, device=src.device)
    _check_range(index, dim_size)
    if E:
        U.scatter_csr(U.SCATTER_MAX, src3, index, U.group_by(index), out, out_rows=dim_size, argmax=arg)
    return out, arg


def scatter_softmax(src, index, dim=-1, eps=1e-12, dim_size=None):
    dim, src3, index, outer, E, inner = _prep(src, index, dim)
    out = H.empty(src3.shape, dtype=src3.dtype, device=src3.device)
    _check_range(index)
    if E:
        U.scatter_csr(U.SCATTER_SOFTMAX, src3, index, U.group_by(index), out, eps=eps)
    return out.view(src.shape)


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    if reduce in ("sum", "add"):
        return scatter_sum(src, index, dim, out, dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim, out, dim_size)
    if reduce == "max":
        return scatter_max(src, index, dim, out, dim_size)[0]
    raise NotImplementedError(f"torch_scatter (HIP): reduce={reduce!r}")
