"""ctypes front-end of the CPU oracle (``oracle/dpvo_oracle.c``).

TEST INFRASTRUCTURE ONLY -- the parity checker.  Imported by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg; never by
the product package.  Every function takes/returns numpy arrays and restates
one reference routine (citations in ``dpvo_oracle.c``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

F16, F32, F64, F16_ACC64 = 0, 1, 2, 3
OPS = {"exp": 0, "log": 1, "inv": 2, "mul": 3, "adj": 4, "adjT": 5, "act": 6, "act4": 7,
       "matrix": 8, "projector": 9, "Jinv": 10}
SO3, RXSO3, SE3, SIM3 = 1, 2, 3, 4


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "dpvo_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        # one thread unless a caller asks for more (bench.cpu_baseline): test
        # processes share the box with the GPU run and need no thread team
        _lib.oracle_set_threads(ctypes.c_int(int(os.environ.get("DPVO_ORACLE_THREADS", "1"))))
    return _lib


def set_threads(n):
    """OpenMP threads of the oracle's parallel loops (the altcorr edge loop);
    1 = the scalar port."""
    lib().oracle_set_threads(ctypes.c_int(int(n)))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _i64(seq):
    return np.ascontiguousarray(np.asarray(seq, dtype=np.int64))


def _elem_strides(a):
    return _i64([s // a.itemsize for s in a.strides])


# ----------------------------------------------------------------------------
# altcorr
# ----------------------------------------------------------------------------
def corr_forward(fmap1, fmap2, coords, ii, jj, radius, mode=None):
    """Reference ``cuda_corr.forward`` (correlation_kernel.cu:193-233).

    fmap1 [B,N1,C,P,P], fmap2 [B,N2,C,H2,W2] (float16/float32/float64 numpy,
    any strides), coords [B,E,2,P,P] float32.  Returns the reference's
    *pre-permute* memory, shape [B,E,2r+1,2r+1,P,P] (dims = y-offset,
    x-offset, i0, j0); the reference's returned view is
    ``out.transpose(0,1,3,2,4,5)``.
    mode defaults to the bit-exact emulation of the input dtype.
    """
    assert fmap1.dtype == fmap2.dtype
    if mode is None:
        mode = {np.dtype(np.float16): F16, np.dtype(np.float32): F32, np.dtype(np.float64): F64}[fmap1.dtype]
    coords = np.asarray(coords, dtype=np.float32)
    B, E, _, H, W = coords.shape
    Do = 2 * radius + 1
    odt = {F16: np.float16, F32: np.float32, F64: np.float64, F16_ACC64: np.float64}[mode]
    out = np.zeros((B, E, Do, Do, H, W), dtype=odt)
    f1 = fmap1.view(np.uint16) if fmap1.dtype == np.float16 else fmap1
    f2 = fmap2.view(np.uint16) if fmap2.dtype == np.float16 else fmap2
    rc = lib().oracle_corr_forward(
        ctypes.c_int(mode), _p(f1), _p(_i64(fmap1.shape)), _p(_elem_strides(fmap1)),
        _p(f2), _p(_i64(fmap2.shape)), _p(_elem_strides(fmap2)),
        _p(coords), _p(_i64(coords.shape)), _p(_elem_strides(coords)),
        _p(_i64(ii)), _p(_i64(jj)), ctypes.c_int(radius), _p(out))
    assert rc == 0
    return out


def corr_pyramid(gmap, fmaps, coords, ii, jj, radius=3, levels=(1, 4), mode=None):
    """dpvo.py:326-333 ``DPVO.corr``: both levels, stacked -> [B, E, 2*49*P*P].

    Returns the stacked tensor in the reference's logical order
    [B][E][x-offset][y-offset][i0][j0][level] flattened."""
    outs = []
    for f, lvl in zip(fmaps, levels):
        c = (np.asarray(coords, np.float32) / np.float32(lvl)).astype(np.float32)
        o = corr_forward(gmap, f, c, ii, jj, radius, mode)
        outs.append(o.transpose(0, 1, 3, 2, 4, 5))
    st = np.stack(outs, axis=-1)
    return st.reshape(st.shape[0], st.shape[1], -1)


def patchify_forward(net, coords, radius):
    """``cuda_corr.patchify_forward`` (correlation_kernel.cu:17-47, :288-308)."""
    B, C, H, W = net.shape
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    M = coords.shape[1]
    D = 2 * radius + 2
    out = np.zeros((B, M, C, D, D), dtype=net.dtype)
    rc = lib().oracle_patchify_forward(ctypes.c_int(net.itemsize), _p(net), _p(_i64(net.shape)),
                                       _p(_elem_strides(net)), _p(coords), ctypes.c_int64(M),
                                       ctypes.c_int(radius), _p(out))
    assert rc == 0
    return out


# ----------------------------------------------------------------------------
# fastba
# ----------------------------------------------------------------------------
def ba_forward(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, iterations=2):
    """``fastba.BA`` (ba_cuda.cu:422-540).  Returns (poses, patches, status)
    as new float32 arrays; status > 0 is the failing Cholesky minor."""
    poses = np.array(poses, dtype=np.float32, copy=True).reshape(-1, 7)
    P = patches.shape[-1]
    patches = np.array(patches, dtype=np.float32, copy=True).reshape(-1, 3, P, P)
    intr = np.ascontiguousarray(intrinsics, dtype=np.float32).reshape(-1, 4)
    target = np.ascontiguousarray(target, dtype=np.float32).reshape(-1, 2)
    weight = np.ascontiguousarray(weight, dtype=np.float32).reshape(-1, 2)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    st = lib().oracle_ba_forward(_p(poses), _p(patches), _p(intr), _p(target), _p(weight),
                                 ctypes.c_float(float(np.asarray(lmbda).reshape(-1)[0])),
                                 _p(ii), _p(jj), _p(kk), ctypes.c_int64(len(ii)), ctypes.c_int(P),
                                 ctypes.c_int(t0), ctypes.c_int(t1), ctypes.c_int(iterations))
    return poses, patches, st


def reproject(poses, patches, intrinsics, ii, jj, kk):
    """``fastba.reproject`` (ba_cuda.cu:368-418, :543-575): [1,E,2,P,P]."""
    poses = np.ascontiguousarray(poses, dtype=np.float32).reshape(-1, 7)
    P = patches.shape[-1]
    patches = np.ascontiguousarray(patches, dtype=np.float32).reshape(-1, 3, P, P)
    intr = np.ascontiguousarray(intrinsics, dtype=np.float32).reshape(-1, 4)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    out = np.zeros((len(ii), 2, P, P), dtype=np.float32)
    lib().oracle_reproject(_p(poses), _p(patches), _p(intr), _p(ii), _p(jj), _p(kk),
                           ctypes.c_int64(len(ii)), ctypes.c_int(P), _p(out))
    return out.reshape(1, len(ii), 2, P, P)


def neighbors(ii, jj):
    """``fastba.neighbors`` (ba.cpp:113-158)."""
    ii, jj = _i64(ii), _i64(jj)
    ix = np.empty_like(ii)
    jx = np.empty_like(ii)
    lib().oracle_neighbors(_p(ii), _p(jj), ctypes.c_int64(len(ii)), _p(ix), _p(jx))
    return ix, jx


# ----------------------------------------------------------------------------
# lietorch (SO3 / RxSO3 / SE3 / Sim3) and projective ops, in double
# ----------------------------------------------------------------------------
DIMS = {SO3: (3, 4), RXSO3: (4, 5), SE3: (6, 7), SIM3: (7, 8)}  # group -> (K, N)
_OUT_DIM = {
    (SO3, "exp"): 4, (SO3, "log"): 3, (SO3, "inv"): 4, (SO3, "mul"): 4, (SO3, "adj"): 3, (SO3, "adjT"): 3,
    (SO3, "act"): 3, (SO3, "act4"): 4, (SO3, "matrix"): 16, (SO3, "projector"): 16, (SO3, "Jinv"): 3,
    (SE3, "exp"): 7, (SE3, "log"): 6, (SE3, "inv"): 7, (SE3, "mul"): 7, (SE3, "adj"): 6, (SE3, "adjT"): 6,
    (SE3, "act"): 3, (SE3, "act4"): 4, (SE3, "matrix"): 16, (SE3, "projector"): 49, (SE3, "Jinv"): 6,
}
for _g in (RXSO3, SIM3):
    _K, _N = DIMS[_g]
    _OUT_DIM.update({(_g, "exp"): _N, (_g, "log"): _K, (_g, "inv"): _N, (_g, "mul"): _N, (_g, "adj"): _K,
                     (_g, "adjT"): _K, (_g, "act"): 3, (_g, "act4"): 4, (_g, "matrix"): 16, (_g, "projector"): _N * _N,
                     (_g, "Jinv"): _K})


def lie_forward(op, group, X, Y=None):
    """Forward lietorch operator on flat [n, dim] inputs (lietorch.cpp:18-283)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n = X.shape[0]
    Yc = np.ascontiguousarray(Y, dtype=np.float64) if Y is not None else X
    out = np.zeros((n, _OUT_DIM[(group, op)]), dtype=np.float64)
    rc = lib().oracle_lie_forward(ctypes.c_int(OPS[op]), ctypes.c_int(group), _p(X), _p(Yc), _p(out),
                                  ctypes.c_int64(n))
    if rc != 0:
        raise NotImplementedError(f"oracle: group {group} op {op}")
    if op == "matrix":
        out = out.reshape(n, 4, 4)
    elif op == "projector":
        d = DIMS[group][1]
        out = out.reshape(n, d, d)
    return out


def transform(poses, patches, intrinsics, ii, jj, kk, depth=False, valid=False, tonly=False):
    """``projective_ops.transform`` (projective_ops.py:53-68): [1,E,P,P,2|3]."""
    poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 7)
    P = patches.shape[-1]
    patches = np.ascontiguousarray(patches, dtype=np.float64).reshape(-1, 3, P, P)
    intr = np.ascontiguousarray(intrinsics, dtype=np.float64).reshape(-1, 4)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    E = len(ii)
    out = np.zeros((E, P, P, 3 if depth else 2))
    v = np.zeros((E, P, P)) if valid else None
    lib().oracle_transform(_p(poses), _p(patches), _p(intr), _p(ii), _p(jj), _p(kk), ctypes.c_int64(E),
                           ctypes.c_int(P), ctypes.c_int(int(depth)), ctypes.c_int(int(tonly)), _p(out),
                           _p(v) if v is not None else ctypes.c_void_p(0))
    out = out.reshape(1, E, P, P, -1)
    return (out, v.reshape(1, E, P, P)) if valid else out


def point_cloud_centre(poses, patches, intrinsics, ix):
    """dpvo.py:747-749: centre pixel of ``pops.point_cloud`` divided by w."""
    poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 7)
    P = patches.shape[-1]
    patches = np.ascontiguousarray(patches, dtype=np.float64).reshape(-1, 3, P, P)
    intr = np.ascontiguousarray(intrinsics, dtype=np.float64).reshape(-1, 4)
    ix = _i64(ix)
    out = np.zeros((len(ix), 3))
    lib().oracle_point_cloud_centre(_p(poses), _p(patches), _p(intr), _p(ix), ctypes.c_int64(len(ix)),
                                    ctypes.c_int(P), _p(out))
    return out


def softagg(f, s, group, groups, eps=1e-12):
    """SoftAgg's grouped softmax-weighted sum (reference dpvo/blocks.py:40-48,
    torch_scatter 2.1.2 ``scatter_softmax`` + ``scatter_sum`` over dim 1),
    in float64: w = exp(s - max_g s) / (sum_g exp(s - max_g s) + eps);
    y[g] = sum_{e in g} f[e] * w[e].  f, s: [E, D]; group: [E] in [0, groups).
    torch_scatter is not under /root/reference: restated from its published
    scatter_softmax (max-recentred, eps added to the group sum) -- parity
    unpinned by reference fixtures."""
    f = np.asarray(f, np.float64)
    s = np.asarray(s, np.float64)
    group = np.asarray(group, np.int64)
    D = f.shape[1]
    gmax = np.full((groups, D), -np.inf)
    np.maximum.at(gmax, group, s)
    ex = np.exp(s - gmax[group])
    den = np.zeros((groups, D))
    np.add.at(den, group, ex)
    w = ex / (den + eps)[group]
    y = np.zeros((groups, D))
    np.add.at(y, group, f * w)
    return y


def gather_rows(x, idx):
    """mask_ix * net[:, ix] of Update.forward (reference dpvo/net.py:82-85):
    rows of x at idx, zero where idx < 0."""
    x = np.asarray(x)
    idx = np.asarray(idx, np.int64)
    out = np.zeros((len(idx), x.shape[1]), x.dtype)
    ok = idx >= 0
    out[ok] = x[idx[ok]]
    return out


def solve_system(Ji, Jj, ii, jj, res, ep, lm, freen):
    """cuda_ba.solve_system (reference dpvo/fastba/ba.cpp:174-234) in float64
    numpy: J (7r x 7n) from the per-edge 7x7 blocks, A = J^T J, b = -J^T res,
    diag(A) += lm diag(A) + ep; solves all of A (freen < 0) or its top-left
    7*freen block (rest of delta zero).  Eigen's SimplicialCholesky there; a
    dense solve here (same solution up to rounding)."""
    Ji = np.asarray(Ji, np.float64)
    Jj = np.asarray(Jj, np.float64)
    res = np.asarray(res, np.float64).reshape(-1, 7)
    ii = np.asarray(ii, np.int64)
    jj = np.asarray(jj, np.int64)
    r = len(ii)
    n = int(max(ii.max(), jj.max())) + 1
    J = np.zeros((7 * r, 7 * n))
    for x in range(r):
        J[7 * x:7 * x + 7, 7 * ii[x]:7 * ii[x] + 7] += Ji[x]
        J[7 * x:7 * x + 7, 7 * jj[x]:7 * jj[x] + 7] += Jj[x]
    A = J.T @ J
    b = -(J.T @ res.reshape(-1))
    A[np.diag_indices_from(A)] += A.diagonal() * lm + ep
    m = 7 * n if freen < 0 else 7 * freen
    delta = np.zeros(7 * n)
    delta[:m] = np.linalg.solve(A[:m, :m], b[:m])
    return delta.reshape(n, 7).astype(np.float32)
