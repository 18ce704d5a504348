"""Lie-group objects over a flat data tensor (reference
dpvo/lietorch/groups.py).  SE3 data = [tx, ty, tz, qx, qy, qz, qw].

Group arithmetic goes through lietorch_backends (csrc/lietorch.hip via the C
ABI); this layer only handles shapes, broadcasting and autograd plumbing.
"""
import numpy as np
import torch

from .broadcasting import broadcast_inputs
from .group_ops import Act3, Act4, Adj, AdjT, Exp, FromVec, Inv, Jinv, Log, Mul, ToMatrix, ToVec


class LieGroupParameter(torch.Tensor):
    """Tangent-space parameter wrapping a group element (groups.py:9-48)."""

    from torch._C import _disabled_torch_function_impl
    __torch_function__ = _disabled_torch_function_impl

    def __new__(cls, group, requires_grad=True):
        data = torch.zeros(group.tangent_shape, device=group.data.device, dtype=group.data.dtype,
                           requires_grad=True)
        return torch.Tensor._make_subclass(cls, data, requires_grad)

    def __init__(self, group):
        self.group = group

    def retr(self):
        return self.group.retr(self)

    def log(self):
        return self.retr().log()

    def inv(self):
        return self.retr().inv()

    def adj(self, a):
        return self.retr().adj(a)

    def __mul__(self, other):
        left = self.retr()
        return left * (other.retr() if isinstance(other, LieGroupParameter) else other)

    def add_(self, update, alpha):
        self.group = self.group.exp(alpha * update) * self.group

    def __getitem__(self, index):
        return self.retr().__getitem__(index)


class LieGroup:
    group_name = None
    group_id = None
    manifold_dim = None
    embedded_dim = None
    id_elem = None

    def __init__(self, data):
        self.data = data

    def __repr__(self):
        return "{}: size={}, device={}, dtype={}".format(self.group_name, self.shape, self.device, self.dtype)

    # ---- shape / device ----
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def tangent_shape(self):
        return self.data.shape[:-1] + (self.manifold_dim,)

    # ---- constructors ----
    @classmethod
    def Identity(cls, *batch_shape, **kwargs):
        if isinstance(batch_shape[0], (tuple, list)):
            batch_shape = tuple(batch_shape[0])
        data = cls.id_elem.reshape(1, -1)
        if "device" in kwargs:
            data = data.to(kwargs["device"])
        if "dtype" in kwargs:
            data = data.type(kwargs["dtype"])
        return cls(data.repeat(int(np.prod(batch_shape)), 1)).view(batch_shape)

    @classmethod
    def IdentityLike(cls, G):
        return cls.Identity(G.shape, device=G.data.device, dtype=G.data.dtype)

    @classmethod
    def InitFromVec(cls, data):
        return cls(cls.apply_op(FromVec, data))

    @classmethod
    def Random(cls, *batch_shape, sigma=1.0, **kwargs):
        if isinstance(batch_shape[0], (tuple, list)):
            batch_shape = tuple(batch_shape[0])
        return cls.exp(sigma * torch.randn(batch_shape + (cls.manifold_dim,), **kwargs))

    @classmethod
    def apply_op(cls, op, x, y=None):
        inputs, out_shape = broadcast_inputs(x, y)
        out = op.apply(cls.group_id, *inputs)
        return out.view(out_shape + (-1,))

    # ---- operators ----
    @classmethod
    def exp(cls, x):
        return cls(cls.apply_op(Exp, x))

    def quaternion(self):
        return self.data[..., -4:] if self.group_name in ("SO3", "SE3") else self.data[..., 3:7]

    def log(self):
        return self.apply_op(Log, self.data)

    def inv(self):
        return self.__class__(self.apply_op(Inv, self.data))

    def mul(self, other):
        return self.__class__(self.apply_op(Mul, self.data, other.data))

    def retr(self, a):
        """Exp(a) * X"""
        return self.__class__(self.apply_op(Mul, self.__class__.apply_op(Exp, a), self.data))

    def adj(self, a):
        return self.apply_op(Adj, self.data, a)

    def adjT(self, a):
        return self.apply_op(AdjT, self.data, a)

    def Jinv(self, a):
        return self.apply_op(Jinv, self.data, a)

    def act(self, p):
        if p.shape[-1] == 3:
            return self.apply_op(Act3, self.data, p)
        if p.shape[-1] == 4:
            return self.apply_op(Act4, self.data, p)
        raise ValueError("points must have 3 or 4 coordinates")

    def matrix(self):
        I = torch.eye(4, dtype=self.dtype, device=self.device)
        I = I.view([1] * (self.data.dim() - 1) + [4, 4])
        return self.__class__(self.data[..., None, :]).act(I).transpose(-1, -2)

    def translation(self):
        p = torch.as_tensor([0.0, 0.0, 0.0, 1.0], dtype=self.dtype, device=self.device)
        return self.apply_op(Act4, self.data, p.view([1] * (self.data.dim() - 1) + [4]))

    def vec(self):
        return self.apply_op(ToVec, self.data)

    # ---- tensor-like plumbing ----
    def detach(self):
        return self.__class__(self.data.detach())

    def view(self, dims):
        return self.__class__(self.data.view(tuple(dims) + (self.embedded_dim,)))

    def __mul__(self, other):
        if isinstance(other, LieGroup):
            return self.mul(other)
        if isinstance(other, torch.Tensor):
            return self.act(other)
        return NotImplemented

    def __getitem__(self, index):
        return self.__class__(self.data[index])

    def __setitem__(self, index, item):
        self.data[index] = item.data

    def to(self, *args, **kwargs):
        return self.__class__(self.data.to(*args, **kwargs))

    def cpu(self):
        return self.__class__(self.data.cpu())

    def cuda(self):
        return self.__class__(self.data.cuda())

    def float(self, device=None):
        return self.__class__(self.data.float())

    def double(self, device=None):
        return self.__class__(self.data.double())

    def unbind(self, dim=0):
        return [self.__class__(x) for x in self.data.unbind(dim=dim)]


class SO3(LieGroup):
    group_name, group_id, manifold_dim, embedded_dim = "SO3", 1, 3, 4
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 1.0])

    def __init__(self, data):
        if isinstance(data, SE3):
            data = data.data[..., 3:7]
        super().__init__(data)


class RxSO3(LieGroup):
    group_name, group_id, manifold_dim, embedded_dim = "RxSO3", 2, 4, 5
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 1.0, 1.0])

    def __init__(self, data):
        if isinstance(data, Sim3):
            data = data.data[..., 3:8]
        super().__init__(data)


class SE3(LieGroup):
    group_name, group_id, manifold_dim, embedded_dim = "SE3", 3, 6, 7
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0])

    def __init__(self, data):
        if isinstance(data, SO3):
            data = torch.cat([torch.zeros_like(data.data[..., :3]), data.data], -1)
        super().__init__(data)

    def scale(self, s):
        t, q = self.data.split([3, 4], -1)
        return SE3(torch.cat([t * s.unsqueeze(-1), q], dim=-1))


class Sim3(LieGroup):
    group_name, group_id, manifold_dim, embedded_dim = "Sim3", 4, 7, 8
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 1.0])

    def __init__(self, data):
        if isinstance(data, SO3):
            data = torch.cat([torch.zeros_like(data.data[..., :3]), data.data,
                              torch.ones_like(data.data[..., :1])], -1)
        elif isinstance(data, SE3):
            data = torch.cat([data.data, torch.ones_like(data.data[..., :1])], -1)
        elif isinstance(data, Sim3):
            data = data.data
        super().__init__(data)


def cat(group_list, dim):
    return group_list[0].__class__(torch.cat([X.data for X in group_list], dim=dim))


def stack(group_list, dim):
    return group_list[0].__class__(torch.stack([X.data for X in group_list], dim=dim))
