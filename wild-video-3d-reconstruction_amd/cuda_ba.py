"""Drop-in replacement for the reference's ``cuda_ba`` extension.

Same module name, functions and argument meaning as dpvo/fastba/ba.cpp:236-241
(imported by dpvo/fastba/ba.py:2); the work runs in libdpvo_hot.so
(csrc/fastba.hip) on the current HIP stream.

``CHECK_CHOLESKY`` (default True) keeps the reference's behaviour of raising
when the Schur system is not positive definite (torch::linalg::cholesky in
ba_cuda.cu:521 raises); it costs one device->host read of a status word per
call.  Set it to False for fully asynchronous / graph-captured use; the
status is then left in ``last_status`` (a device tensor).  A caller may
instead pass ``status=`` (a device int32 tensor): the call then never reads
it, and the caller raises later (DPVO.update does, at keyframe()'s host read).

Windows of up to 12 optimised poses (DPVO's sliding window) take the
deterministic per-patch path: no float atomics, bitwise repeatable.  It
groups the edges by kk on the device, or reuses a caller's grouping
(``csr=(offs, perm, groups)`` from update_ops.group_by(kk), which
DPVO.update already computes for the update operator).  ``DETERMINISTIC =
False`` selects the atomic dense path instead (A/B tests).

Windows of more than 64 optimised poses (the global BA of dpvo.py:436-505)
take the sparse path automatically: per-edge Schur entries and a tiled band
Cholesky instead of the dense E / S (see include/dpvo_hot.h).  ``SPARSE =
True`` forces it for any window (used by the parity tests).
"""
import torch

import _dpvo_hot as H

CHECK_CHOLESKY = True
SPARSE = False
DETERMINISTIC = True
last_status = None


def raise_for_status(s):
    """the reference's error for a BA status word (0: no error)."""
    s = int(s)
    if s > 0:
        raise RuntimeError(
            "linalg.cholesky: The factorization could not be completed because the input is not positive-"
            f"definite (the leading minor of order {s} is not positive-definite).")
    if s == -2:
        raise RuntimeError("DPVO.update: an edge lies outside the 64-frame key window "
                           "(REMOVAL_WINDOW / PATCH_LIFETIME invariant; set cfg.WINDOW_IJ_KEY = False)")
    if s < 0:
        raise RuntimeError("cuda_ba.forward: patch index out of range")


def forward(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, iterations, csr=None,
            status=None, keep_status=False):
    """ba.cpp:31-43 -> ba_cuda.cu:422-540.  Updates poses and patches in place; returns [].
    csr (optional, not in the reference): (offs int32 [E+1], perm int32 [E],
    groups int64 [1]) of update_ops.group_by(kk) for these edges.
    status (optional, not in the reference): a device int32 [1] the call's
    status word is written to instead of being read here -- no host
    synchronisation; the caller checks it later (raise_for_status).
    keep_status (with status=): the word is not cleared first; if it already
    holds a failure (DPVO.update's window-key check) the call leaves poses and
    patches untouched (deterministic sliding-window path, DPVO_BA_KEEP_STATUS)."""
    global last_status
    H.on_gpu(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk)
    for name, t in (("poses", poses), ("patches", patches), ("intrinsics", intrinsics), ("target", target),
                    ("weight", weight)):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name} must be float32")
        if not t.is_contiguous():
            raise RuntimeError(f"{name} must be contiguous (the reference views it, ba_cuda.cu:446-451)")
    P = patches.shape[3] if patches.dim() == 5 else patches.shape[-1]
    num_patches = patches.numel() // (3 * P * P)
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    lmbda = lmbda.to(device=poses.device, dtype=torch.float32).contiguous()
    E = ii.numel()
    N = int(t1) - int(t0)
    flags = (1 if SPARSE else 0) | (0 if DETERMINISTIC else 2) | (4 if keep_status and status is not None else 0)
    nbytes = H.lib().dpvo_ba_workspace_bytes_ex(E, num_patches, max(N, 0), flags)
    ws = H.empty(nbytes, dtype=torch.uint8, device=poses.device)
    deferred = status is not None
    if deferred:
        if status.dtype != torch.int32 or status.numel() < 1 or status.device != poses.device:
            raise RuntimeError("status must be a device int32 tensor of at least one element")
    else:
        status = torch.zeros(1, dtype=torch.int32, device=poses.device)
    offs = perm = groups = None
    if csr is not None:
        offs, perm, groups = csr
        H.on_gpu(offs, perm, groups)
        if (offs.dtype != torch.int32 or perm.dtype != torch.int32 or groups.dtype != torch.int64 or
                offs.numel() < E + 1 or perm.numel() < E):
            raise RuntimeError("csr must be update_ops.group_by(kk)'s (offs int32 [E+1], perm int32 [E], groups int64)")
    H.check(H.lib().dpvo_ba_forward_csr(
        H.ptr(poses), H.ptr(patches), num_patches, P, H.ptr(intrinsics), H.ptr(target), H.ptr(weight), H.ptr(lmbda),
        H.ptr(ii), H.ptr(jj), H.ptr(kk), E, int(t0), int(t1), int(iterations), flags, H.ptr(offs), H.ptr(perm),
        H.ptr(groups), H.ptr(ws), nbytes, H.ptr(status), H.stream_of(poses)))
    last_status = status
    if CHECK_CHOLESKY and not deferred:
        raise_for_status(status.item())
    return []


def neighbors(ii, jj):
    """ba.cpp:113-158, GPU-resident: -> [ix, jx] (int64)."""
    H.on_gpu(ii, jj)
    ii, jj = H.idx64(ii), H.idx64(jj)
    E = ii.numel()
    ix = H.empty(E, dtype=torch.int64, device=ii.device)
    jx = H.empty(E, dtype=torch.int64, device=ii.device)
    if E:
        nbytes = H.lib().dpvo_neighbors_workspace_bytes(E)
        ws = H.empty(nbytes, dtype=torch.uint8, device=ii.device)
        H.check(H.lib().dpvo_neighbors(H.ptr(ii), H.ptr(jj), E, H.ptr(ix), H.ptr(jx), H.ptr(ws), nbytes,
                                       H.stream_of(ii)))
    return [ix, jx]


def reproject(poses, patches, intrinsics, ii, jj, kk):
    """ba.cpp:53-61 / ba_cuda.cu:543-575 -> coords [1, E, 2, P, P]."""
    H.on_gpu(poses, patches, intrinsics, ii, jj, kk)
    poses, patches, intrinsics = poses.contiguous(), patches.contiguous(), intrinsics.contiguous()
    P = patches.shape[-1]
    ii, jj, kk = H.idx64(ii), H.idx64(jj), H.idx64(kk)
    E = ii.numel()
    out = H.empty((E, 2, P, P), dtype=torch.float32, device=poses.device)
    H.check(H.lib().dpvo_reproject(H.ptr(poses), H.ptr(patches), P, H.ptr(intrinsics), H.ptr(ii), H.ptr(jj),
                                   H.ptr(kk), E, H.ptr(out), H.stream_of(poses)))
    return out.view(1, E, 2, P, P)


def solve_system(J_Ginv_i, J_Ginv_j, ii, jj, res, ep, lm, freen):
    """ba.cpp:174-234 (loop-closure PGO): -> [delta [n, 7]] on res.device.

    A = J^T J, b = -J^T res (fp64) are assembled on the device
    (dpvo_solve_system_assemble); the reference's Eigen SimplicialCholesky is a
    dense fp64 Cholesky here (rocSOLVER via torch.linalg).  freen >= 0 solves
    only the top-left 7*freen block (the rest of delta is zero), like the
    reference.  An edge with ii == jj raises (the reference calls exit(1)).

    Like the reference (which copies every input to the host itself), the
    inputs may live on any device -- PGO builds its Jacobians with pypose,
    possibly on the CPU (optim_utils.py:222-255).  The solve runs on the GPU
    (the current device when res is a CPU tensor) and delta comes back on
    res.device."""
    out_dev = res.device
    dev = res.device if res.is_cuda else torch.device("cuda", torch.cuda.current_device())
    Ji = J_Ginv_i.to(dev, torch.float32).contiguous()
    Jj = J_Ginv_j.to(dev, torch.float32).contiguous()
    rr = res.to(dev, torch.float32).contiguous().view(-1, 7)
    ii, jj = H.idx64(ii.to(dev)), H.idx64(jj.to(dev))
    r = rr.shape[0]
    if Ji.shape != (r, 7, 7) or Jj.shape != (r, 7, 7) or ii.numel() != r or jj.numel() != r:
        raise RuntimeError("solve_system: J_Ginv_i/J_Ginv_j must be [r, 7, 7], ii/jj [r], res [r, 7]")
    n = int(torch.maximum(ii.max(), jj.max()).item()) + 1 if r else 0
    m = 7 * n if int(freen) < 0 else min(7 * int(freen), 7 * n)
    A = H.empty(m, m, dtype=torch.float64, device=dev)
    b = H.empty(m, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    H.check(H.lib().dpvo_solve_system_assemble(H.ptr(Ji), H.ptr(Jj), H.ptr(ii), H.ptr(jj), H.ptr(rr), r, m,
                                               float(ep), float(lm), H.ptr(A), H.ptr(b), H.ptr(status),
                                               H.stream_of(rr)))
    if int(status.item()):
        raise RuntimeError("solve_system: an edge with ii == jj (the reference exits the process, ba.cpp:205)")
    delta = torch.zeros(7 * n, dtype=torch.float32, device=dev)
    if m:
        L = torch.linalg.cholesky(A)
        delta[:m] = torch.cholesky_solve(b[:, None], L)[:, 0].float()
    return [delta.view(n, 7).to(out_dev)]
