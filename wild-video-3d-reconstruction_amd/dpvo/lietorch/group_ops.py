"""Autograd wrappers over lietorch_backends (reference
dpvo/lietorch/group_ops.py:7-101)."""
import torch

import lietorch_backends


class GroupOp(torch.autograd.Function):
    """forward_op(group_id, *inputs) / backward_op(group_id, grad, *inputs)."""
    forward_op = None
    backward_op = None

    @classmethod
    def forward(cls, ctx, group_id, *inputs):
        ctx.group_id = group_id
        ctx.save_for_backward(*inputs)
        return cls.forward_op(group_id, *inputs)

    @classmethod
    def backward(cls, ctx, grad):
        if cls.backward_op is None:
            raise RuntimeError(f"Backward operation not implemented for {cls}")
        grads = cls.backward_op(ctx.group_id, grad.contiguous(), *ctx.saved_tensors)
        return (None,) + tuple(grads)


def _op(name, fwd, bwd=None):
    return type(name, (GroupOp,), {"forward_op": staticmethod(fwd),
                                   "backward_op": staticmethod(bwd) if bwd else None})


B = lietorch_backends
Exp = _op("Exp", B.expm, B.expm_backward)
Log = _op("Log", B.logm, B.logm_backward)
Inv = _op("Inv", B.inv, B.inv_backward)
Mul = _op("Mul", B.mul, B.mul_backward)
Adj = _op("Adj", B.adj, B.adj_backward)
AdjT = _op("AdjT", B.adjT, B.adjT_backward)
Act3 = _op("Act3", B.act, B.act_backward)
Act4 = _op("Act4", B.act4, B.act4_backward)
Jinv = _op("Jinv", B.Jinv)
ToMatrix = _op("ToMatrix", B.as_matrix)


class FromVec(torch.autograd.Function):
    """vector -> group element; gradient through the projector pseudo-inverse."""

    @staticmethod
    def forward(ctx, group_id, *inputs):
        ctx.group_id = group_id
        ctx.save_for_backward(*inputs)
        return inputs[0]

    @staticmethod
    def backward(ctx, grad):
        J = lietorch_backends.projector(ctx.group_id, *ctx.saved_tensors)
        return None, torch.matmul(grad.unsqueeze(-2), torch.linalg.pinv(J)).squeeze(-2)


class ToVec(torch.autograd.Function):
    """group element -> vector; gradient through the projector."""

    @staticmethod
    def forward(ctx, group_id, *inputs):
        ctx.group_id = group_id
        ctx.save_for_backward(*inputs)
        return inputs[0]

    @staticmethod
    def backward(ctx, grad):
        J = lietorch_backends.projector(ctx.group_id, *ctx.saved_tensors)
        return None, torch.matmul(grad.unsqueeze(-2), J).squeeze(-2)
