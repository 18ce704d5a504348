"""Operand broadcasting for the group operators (reference
dpvo/lietorch/broadcasting.py:9-31): leading dims are broadcast, the
trailing (group / tangent / point) dim is kept, and the result is flattened to
the contiguous [n, dim] layout the backend takes."""
import torch


def check_broadcastable(x, y):
    assert x.dim() == y.dim(), "operands must have the same number of dimensions"
    for n, m in zip(x.shape[:-1], y.shape[:-1]):
        assert n == m or n == 1 or m == 1, "leading dimensions are not broadcastable"


def broadcast_inputs(x, y):
    if y is None:
        return (x.reshape(-1, x.shape[-1]).contiguous(),), tuple(x.shape[:-1])
    check_broadcastable(x, y)
    lead = tuple(max(n, m) for n, m in zip(x.shape[:-1], y.shape[:-1]))
    xb = x.expand(lead + x.shape[-1:]).reshape(-1, x.shape[-1]).contiguous()
    yb = y.expand(lead + y.shape[-1:]).reshape(-1, y.shape[-1]).contiguous()
    return (xb, yb), lead
