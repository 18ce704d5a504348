"""Projective geometry of the patch graph (reference dpvo/projective_ops.py).

transform / point_cloud / flow_mag keep the reference's signatures and
semantics.  The inference forms (batch 1, no autograd, no Jacobians) run as
one fused HIP kernel each (csrc/geometry.hip): the reference composes ~30
launches and materialises E*P*P broadcast pose copies.  The differentiable /
Jacobian forms compose the lietorch operators exactly as the reference does.
"""
import torch

import _dpvo_hot as H

from .lietorch import SE3

MIN_DEPTH = 0.2
TF_DEPTH, TF_TONLY, TF_CHW = 1, 2, 4


def extract_intrinsics(intrinsics):
    return intrinsics[..., None, None, :].unbind(dim=-1)


def coords_grid(ht, wd, **kwargs):
    y, x = torch.meshgrid(torch.arange(ht).to(**kwargs).float(), torch.arange(wd).to(**kwargs).float(),
                          indexing="ij")
    return torch.stack([x, y], dim=-1)


def iproj(patches, intrinsics):
    """pixel patches (x, y, inverse depth) -> homogeneous rays [X, Y, 1, d]."""
    x, y, d = patches.unbind(dim=2)
    fx, fy, cx, cy = intrinsics[..., None, None].unbind(dim=2)
    return torch.stack([(x - cx) / fx, (y - cy) / fy, torch.ones_like(d), d], dim=-1)


def proj(X, intrinsics, depth=False):
    """homogeneous points -> pixels, depth clamped to >= 0.1."""
    X, Y, Z, W = X.unbind(dim=-1)
    fx, fy, cx, cy = intrinsics[..., None, None].unbind(dim=2)
    d = 1.0 / Z.clamp(min=0.1)
    x = fx * (d * X) + cx
    y = fy * (d * Y) + cy
    return torch.stack([x, y, d], dim=-1) if depth else torch.stack([x, y], dim=-1)


def _fusable(poses, patches, intrinsics):
    data = poses.data
    return (data.is_cuda and data.dim() == 3 and data.shape[0] == 1 and patches.shape[0] == 1
            and intrinsics.shape[0] == 1 and data.dtype == patches.dtype == intrinsics.dtype == torch.float32
            and not (torch.is_grad_enabled() and (data.requires_grad or patches.requires_grad)))


def transform_fused(poses, patches, intrinsics, ii, jj, kk, depth=False, valid=False, tonly=False, chw=False):
    """One launch: coords [1, E, P, P, 2|3] (or [1, E, 2|3, P, P] with chw)."""
    data = poses.data.contiguous()
    patches, intrinsics = patches.contiguous(), intrinsics.contiguous()
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    E, P = ii.numel(), patches.shape[-1]
    od = 3 if depth else 2
    shape = (1, E, od, P, P) if chw else (1, E, P, P, od)
    out = H.empty(shape, dtype=torch.float32, device=data.device)
    v = H.empty((1, E, P, P), dtype=torch.float32, device=data.device) if valid else None
    flags = (TF_DEPTH if depth else 0) | (TF_TONLY if tonly else 0) | (TF_CHW if chw else 0)
    H.check(H.lib().dpvo_transform(H.ptr(data), H.ptr(patches), P, H.ptr(intrinsics), H.ptr(ii), H.ptr(jj),
                                   H.ptr(kk), E, flags, H.ptr(out), H.ptr(v), H.stream_of(data)))
    return (out, v) if valid else out


def pose_extrapolate(poses_, n, s):
    """poses_[n] = Exp(s Log(poses_[n-1] poses_[n-2]^-1)) poses_[n-1] in place
    (the DAMPED_LINEAR motion model, dpvo.py:816-825; poses_ [N, 7] fp32)."""
    H.on_gpu(poses_)
    if poses_.dtype != torch.float32 or not poses_.is_contiguous() or poses_.shape[-1] != 7 or n >= poses_.shape[0]:
        raise RuntimeError("pose_extrapolate: contiguous fp32 [N, 7] poses with n < N required")
    H.check(H.lib().dpvo_pose_extrapolate(H.ptr(poses_), int(n), float(s), H.stream_of(poses_)))


def pose_relative(a, b):
    """SE3 a * b^-1 for two fp32 [7] pose rows, one launch (dpvo.py:613)."""
    H.on_gpu(a, b)
    a, b = a.contiguous().float(), b.contiguous().float()
    out = H.empty(7, dtype=torch.float32, device=a.device)
    H.check(H.lib().dpvo_pose_relative(H.ptr(a), H.ptr(b), H.ptr(out), H.stream_of(a)))
    return SE3(out)


def motion_mag_pair(poses, patches, intrinsics, ii, jj, kk, i, j, beta=0.5):
    """[mean flow_mag over the (i -> j) edges, same for (j -> i)] as a 2-float
    device tensor, one launch and no host sync (dpvo.py:507-514 + :609;
    NaN for a direction without edges, as torch's mean of an empty tensor)."""
    data = poses.data.contiguous()
    patches, intrinsics = patches.contiguous(), intrinsics.contiguous()
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    out = H.empty(2, dtype=torch.float32, device=data.device)
    nb = H.lib().dpvo_motion_mag_workspace_bytes(ii.numel())
    ws = H.empty(nb, dtype=torch.uint8, device=data.device)
    H.check(H.lib().dpvo_motion_mag_ws(H.ptr(data), H.ptr(patches), patches.shape[-1], H.ptr(intrinsics), H.ptr(ii),
                                       H.ptr(jj), H.ptr(kk), ii.numel(), int(i), int(j), float(beta), H.ptr(out),
                                       H.ptr(ws), nb, H.stream_of(data)))
    return out


def keyframe_masks(ii, jj, kk, ix, k, M, n, RW, mm, ba_fail, pose_k):
    """keyframe()'s device work for both outcomes (dpvo.py:605-658) in two
    launches: masks bool [3, E] (old_keep, old_d, rm_d), idx int64 [3, E]
    (ii, jj, kk after the drop's shift) and vals float64 [7] (mm[0], mm[1],
    ba_fail, any(isnan(pose_k)), the three masks' counts) -- see
    dpvo_keyframe_masks in include/dpvo_hot.h."""
    ii, jj, kk, ix = H.idx64(ii), H.idx64(jj), H.idx64(kk), H.idx64(ix)
    H.on_gpu(ii, jj, kk, ix, mm, ba_fail, pose_k)
    if mm.dtype != torch.float32 or ba_fail.dtype != torch.int32 or pose_k.dtype != torch.float32:
        raise RuntimeError("keyframe_masks: mm / pose_k float32, ba_fail int32")
    E, dev = ii.numel(), ii.device
    masks = H.empty(3, E, dtype=torch.bool, device=dev)
    idx = H.empty(3, E, dtype=torch.int64, device=dev)
    vals = H.empty(7, dtype=torch.float64, device=dev)
    nb = H.lib().dpvo_keyframe_masks_workspace_bytes(E)
    ws = H.empty(nb, dtype=torch.uint8, device=dev)
    H.check(H.lib().dpvo_keyframe_masks(H.ptr(ii), H.ptr(jj), H.ptr(kk), E, H.ptr(ix), ix.numel(), int(k), int(M),
                                        int(n), int(RW), H.ptr(mm.contiguous()), H.ptr(ba_fail),
                                        H.ptr(pose_k.contiguous()), H.ptr(masks), H.ptr(idx), H.ptr(vals), H.ptr(ws),
                                        nb, H.stream_of(ii)))
    return masks, idx, vals


def _dense(t):
    """every element of t's storage span used exactly once (any dim order)"""
    expect = 1
    for stride, size in sorted((st, sz) for sz, st in zip(t.shape, t.stride()) if sz != 1):
        if stride != expect:
            return False
        expect *= size
    return True


def frame_shift(buffers, k, n):
    """Move frames k+1 .. n-1 of every buffer down by one slot in one launch
    (a keyframe drop, dpvo.py:626-639).  buffers: (tensor, slot_dim, ring)
    with frame f in slot (f % ring if ring else f) along slot_dim; each slot
    must be one dense block of memory (the dim's stride = the slot's numel)."""
    if n - 1 <= k or not buffers:
        return
    bases, sizes, rings = [], [], []
    for t, d, ring in buffers:
        H.on_gpu(t)
        slot = t.select(d, 0)
        if t.stride(d) != slot.numel() or any(t.shape[i] != 1 for i in range(d)) or not _dense(t):
            raise RuntimeError("frame_shift: each slot must be one dense block")
        bases.append(t.data_ptr())
        sizes.append(t.stride(d) * t.element_size())
        rings.append(int(ring or 0))
    import ctypes
    ns = len(bases)
    H.check(H.lib().dpvo_frame_shift((ctypes.c_void_p * ns)(*bases), (ctypes.c_int64 * ns)(*sizes),
                                     (ctypes.c_int64 * ns)(*rings), ns, int(k), int(n), H.stream_of(buffers[0][0])))
    for t, _, _ in buffers:   # written in place: caches keyed on the version counter see it
        torch.autograd.graph.increment_version(t)


def keyframe_flow(poses, patches, intrinsics, n, M, beta=0.5):
    """[n, n] device matrix: dist[a, b] = mean flow_mag of frame a's M patches
    into frame b (projective_ops.py:111-121) -- every pair of
    compute_keyframe_distance (dpvo.py:383-407) in one launch; the reference's
    pair distance is 0.5 (dist[i, j] + dist[j, i])."""
    data = poses.data.contiguous()
    patches, intrinsics = patches.contiguous(), intrinsics.contiguous()
    P = patches.shape[-1]
    out = H.empty(n, n, dtype=torch.float32, device=data.device)
    H.check(H.lib().dpvo_keyframe_flow(H.ptr(data), H.ptr(patches), P, H.ptr(intrinsics), int(n), int(M), float(beta),
                                       H.ptr(out), H.stream_of(data)))
    return out


def transform(poses, patches, intrinsics, ii, jj, kk, depth=False, valid=False, jacobian=False, tonly=False):
    """Reproject patch kk from frame ii into frame jj (poses are world->camera)."""
    if not jacobian and _fusable(poses, patches, intrinsics):
        return transform_fused(poses, patches, intrinsics, ii, jj, kk, depth=depth, valid=valid, tonly=tonly)

    X0 = iproj(patches[:, kk], intrinsics[:, ii])
    Gij = poses[:, jj] * poses[:, ii].inv()
    if tonly:
        Gij.data[..., 3:] = torch.as_tensor([0, 0, 0, 1], device=Gij.device, dtype=Gij.dtype)
    X1 = Gij[:, :, None, None] * X0
    x1 = proj(X1, intrinsics[:, jj], depth)

    if jacobian:
        p = X1.shape[2]
        X, Y, Z, Hh = X1[..., p // 2, p // 2, :].unbind(dim=-1)
        o = torch.zeros_like(Hh)
        fx, fy, cx, cy = intrinsics[:, jj].unbind(dim=-1)
        d = torch.where(Z.abs() > MIN_DEPTH, 1.0 / Z, torch.zeros_like(Z))
        # d(X1)/d(xi_j) for a left perturbation of Gij, and d(pixel)/d(X1)
        Ja = torch.stack([Hh, o, o, o, Z, -Y,
                          o, Hh, o, -Z, o, X,
                          o, o, Hh, Y, -X, o,
                          o, o, o, o, o, o], dim=-1).view(1, len(ii), 4, 6)
        Jp = torch.stack([fx * d, o, -fx * X * d * d, o,
                          o, fy * d, -fy * Y * d * d, o], dim=-1).view(1, len(ii), 2, 4)
        Jj = torch.matmul(Jp, Ja)
        Ji = -Gij[:, :, None].adjT(Jj)
        Jz = torch.matmul(Jp, Gij.matrix()[..., :, 3:])
        return x1, (Z > MIN_DEPTH).float(), (Ji, Jj, Jz)

    if valid:
        return x1, (X1[..., 2] > MIN_DEPTH).float()
    return x1


def point_cloud(poses, patches, intrinsics, ix):
    """World points of every patch pixel: [1, m, P, P, 4] (X, Y, Z, d)."""
    if _fusable(poses, patches, intrinsics):
        data = poses.data.contiguous()
        patches, intrinsics = patches.contiguous(), intrinsics.contiguous()
        ix = H.idx64(ix)
        m, P = ix.numel(), patches.shape[-1]
        out = H.empty((1, m, P, P, 4), dtype=torch.float32, device=data.device)
        H.check(H.lib().dpvo_point_cloud(H.ptr(data), H.ptr(patches), P, H.ptr(intrinsics), H.ptr(ix), m, 0,
                                         H.ptr(out), H.stream_of(data)))
        return out
    return poses[:, ix, None, None].inv() * iproj(patches, intrinsics[:, ix])


def point_cloud_centre(poses, patches, intrinsics, ix, out=None):
    """Centre pixel of point_cloud divided by w -- what DPVO.update stores in
    pg.points_ (dpvo.py:747-749) -- in one launch, written into `out` [m, 3]."""
    data = poses.data.contiguous()
    patches, intrinsics = patches.contiguous(), intrinsics.contiguous()
    ix = H.idx64(ix)
    m, P = ix.numel(), patches.shape[-1]
    if out is None:
        out = H.empty((m, 3), dtype=torch.float32, device=data.device)
    H.check(H.lib().dpvo_point_cloud(H.ptr(data), H.ptr(patches), P, H.ptr(intrinsics), H.ptr(ix), m, 1,
                                     H.ptr(out), H.stream_of(data)))
    return out


def flow_mag(poses, patches, intrinsics, ii, jj, kk, beta=0.3):
    """Mean-able flow magnitude mixing full and translation-only motion."""
    coords0 = transform(poses, patches, intrinsics, ii, ii, kk)
    coords1 = transform(poses, patches, intrinsics, ii, jj, kk, tonly=False)
    coords2 = transform(poses, patches, intrinsics, ii, jj, kk, tonly=True)
    flow1 = (coords1 - coords0).norm(dim=-1)
    flow2 = (coords2 - coords0).norm(dim=-1)
    return beta * flow1 + (1 - beta) * flow2
