"""Drop-in replacement for the reference's ``lietorch_backends`` extension.

Same 19 functions, argument order (group_id first) and output shapes as
dpvo/lietorch/src/lietorch.cpp:286-316 (imported by
dpvo/lietorch/group_ops.py:1).  group_id: 1 = SO3, 2 = RxSO3, 3 = SE3,
4 = Sim3 (dispatch.h:16-31).
Inputs must be contiguous (lietorch.cpp:7 CHECK_CONTIGUOUS) float32/float64
GPU tensors; the math runs in libdpvo_hot.so (csrc/lietorch.hip).
"""
import torch

import _dpvo_hot as H

EXP, LOG, INV, MUL, ADJ, ADJT, ACT, ACT4, MATRIX, PROJECTOR, JINV = range(11)
_DIMS = {1: (3, 4), 2: (4, 5), 3: (6, 7), 4: (7, 8)}  # group -> (K manifold dim, N embedding dim)


def _contig(name, t):
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _dims(group_id):
    if group_id not in _DIMS:
        raise RuntimeError(f"unknown group id {group_id}: 1 = SO3, 2 = RxSO3, 3 = SE3, 4 = Sim3")
    return _DIMS[group_id]


def _fwd(op, group_id, X, Y, out):
    H.on_gpu(X, Y)
    _contig("X", X)
    if Y is not None:
        _contig("Y", Y)
        if Y.dtype != X.dtype:
            raise RuntimeError("operands must share a dtype")
    H.check(H.lib().dpvo_lie_forward(op, group_id, H.dtype_code(X), H.ptr(X), H.ptr(Y), H.ptr(out), X.shape[0],
                                     H.stream_of(X)))
    return out


def _bwd(op, group_id, grad, X, Y, dX, dY):
    H.on_gpu(grad, X, Y)
    _contig("grad", grad)
    _contig("X", X)
    if Y is not None:
        _contig("Y", Y)
    H.check(H.lib().dpvo_lie_backward(op, group_id, H.dtype_code(X), H.ptr(grad), H.ptr(X), H.ptr(Y), H.ptr(dX),
                                      H.ptr(dY), X.shape[0], H.stream_of(X)))


def _new(X, *shape):
    return torch.zeros(shape, dtype=X.dtype, device=X.device)


# ---- unary / binary forward ops (lietorch.cpp:18-283) ----
def expm(group_id, a):
    K, N = _dims(group_id)
    return _fwd(EXP, group_id, a, None, _new(a, a.shape[0], N))


def logm(group_id, X):
    K, N = _dims(group_id)
    return _fwd(LOG, group_id, X, None, _new(X, X.shape[0], K))


def inv(group_id, X):
    _dims(group_id)
    return _fwd(INV, group_id, X, None, torch.zeros_like(X))


def mul(group_id, X, Y):
    _dims(group_id)
    return _fwd(MUL, group_id, X, Y, torch.zeros_like(X))


def adj(group_id, X, a):
    _dims(group_id)
    return _fwd(ADJ, group_id, X, a, torch.zeros_like(a))


def adjT(group_id, X, a):
    _dims(group_id)
    return _fwd(ADJT, group_id, X, a, torch.zeros_like(a))


def act(group_id, X, p):
    _dims(group_id)
    return _fwd(ACT, group_id, X, p, torch.zeros_like(p))


def act4(group_id, X, p):
    _dims(group_id)
    return _fwd(ACT4, group_id, X, p, torch.zeros_like(p))


def as_matrix(group_id, X):
    _dims(group_id)
    return _fwd(MATRIX, group_id, X, None, _new(X, X.shape[0], 4, 4))


def projector(group_id, X):
    K, N = _dims(group_id)
    return _fwd(PROJECTOR, group_id, X, None, _new(X, X.shape[0], N, N))


def Jinv(group_id, X, a):
    _dims(group_id)
    return _fwd(JINV, group_id, X, a, torch.zeros_like(a))


# ---- backward ops (lietorch_gpu.cu:313-601 output conventions) ----
def expm_backward(group_id, grad, a):
    _dims(group_id)
    da = torch.zeros_like(a)
    _bwd(EXP, group_id, grad, a, None, da, None)
    return [da]


def logm_backward(group_id, grad, X):
    _dims(group_id)
    dX = torch.zeros_like(X)
    _bwd(LOG, group_id, grad, X, None, dX, None)
    return [dX]


def inv_backward(group_id, grad, X):
    _dims(group_id)
    dX = torch.zeros_like(X)
    _bwd(INV, group_id, grad, X, None, dX, None)
    return [dX]


def mul_backward(group_id, grad, X, Y):
    _dims(group_id)
    dX, dY = torch.zeros_like(X), torch.zeros_like(Y)
    _bwd(MUL, group_id, grad, X, Y, dX, dY)
    return [dX, dY]


def adj_backward(group_id, grad, X, a):
    _dims(group_id)
    dX, da = torch.zeros_like(X), torch.zeros_like(a)
    _bwd(ADJ, group_id, grad, X, a, dX, da)
    return [dX, da]


def adjT_backward(group_id, grad, X, a):
    _dims(group_id)
    dX, da = torch.zeros_like(X), torch.zeros_like(a)
    _bwd(ADJT, group_id, grad, X, a, dX, da)
    return [dX, da]


def act_backward(group_id, grad, X, p):
    _dims(group_id)
    dX, dp = torch.zeros_like(X), torch.zeros_like(p)
    _bwd(ACT, group_id, grad, X, p, dX, dp)
    return [dX, dp]


def act4_backward(group_id, grad, X, p):
    _dims(group_id)
    dX, dp = torch.zeros_like(X), torch.zeros_like(p)
    _bwd(ACT4, group_id, grad, X, p, dX, dp)
    return [dX, dp]
