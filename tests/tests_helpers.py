"""Synthetic DPVO patch-graph states for tests (seeded, numpy only)."""
import numpy as np

from oracle import oracle


def dpvo_edges(n, M, lifetime=13, removal=None):
    """Edge construction of dpvo.py:756-769 replayed frame by frame, with the
    removal rule of dpvo.py:657 (patch frame < n - REMOVAL_WINDOW) applied
    after every frame when `removal` is given."""
    ii = np.zeros(0, np.int64)
    jj = np.zeros(0, np.int64)
    kk = np.zeros(0, np.int64)
    for t in range(1, n + 1):
        k_f = np.arange(M * max(t - lifetime, 0), M * max(t - 1, 0))
        j_f = np.full(len(k_f), t - 1)
        kb = np.arange(M * (t - 1), M * t)
        jb = np.arange(max(t - lifetime, 0), t)
        k_b = np.repeat(kb, len(jb))
        j_b = np.tile(jb, len(kb))
        kk = np.concatenate([kk, k_f, k_b])
        jj = np.concatenate([jj, j_f, j_b])
        ii = np.concatenate([ii, k_f // M, k_b // M])
        if removal is not None:
            keep = ii >= t - removal
            ii, jj, kk = ii[keep], jj[keep], kk[keep]
    return ii.astype(np.int64), jj.astype(np.int64), kk.astype(np.int64)


def global_edges(n):
    """Frame pairs of the global BA's fixed pattern (dpvo.py:448-458):
    i -> i+1, and every 5th frame i -> i+10 .. i+19."""
    ie = list(range(n - 1))
    je = list(range(1, n))
    for i in range(0, n, 5):
        for j in range(i + 10, min(i + 20, n)):
            ie.append(i)
            je.append(j)
    return np.asarray(ie, np.int64), np.asarray(je, np.int64)


def dpvo_frames(seed, n, M, wd=128, ht=96, intr=(80.0, 80.0, 80.0, 60.0)):
    """Random-walk poses and random patches (centres on the 1/4-res grid,
    inverse depth U[0.2, 1], constant over 3x3)."""
    g = np.random.default_rng(seed)
    poses = np.zeros((n, 7))
    poses[:, 6] = 1.0
    for i in range(1, n):
        xi = np.concatenate([g.normal(0, 0.05, 3), g.normal(0, 0.01, 3)])
        dq = oracle.lie_forward("exp", oracle.SE3, xi[None])
        poses[i] = oracle.lie_forward("mul", oracle.SE3, dq, poses[i - 1:i])[0]
    xs = g.integers(1, wd - 1, size=(n, M)).astype(np.float64)
    ys = g.integers(1, ht - 1, size=(n, M)).astype(np.float64)
    d = g.uniform(0.2, 1.0, size=(n, M))
    patches = np.zeros((n, M, 3, 3, 3))
    off = np.arange(3) - 1
    patches[:, :, 0] = xs[:, :, None, None] + off[None, None, None, :]
    patches[:, :, 1] = ys[:, :, None, None] + off[None, None, :, None]
    patches[:, :, 2] = d[:, :, None, None]
    patches = patches.reshape(n * M, 3, 3, 3)
    intrinsics = np.tile(np.asarray(intr), (n, 1))
    return g, poses, patches, intrinsics


def with_edges(g, n, M, poses, patches, intrinsics, ii, jj, kk):
    """targets = reprojected centres + N(0, 1) px, weights U[0, 1]."""
    coords = oracle.transform(poses, patches, intrinsics, ii, jj, kk)[0]
    target = coords[:, 1, 1, :] + g.normal(0, 1.0, size=(len(ii), 2))
    weight = g.uniform(0.0, 1.0, size=(len(ii), 2))
    return dict(n=n, M=M, poses=poses.astype(np.float32), patches=patches.astype(np.float32),
                intrinsics=intrinsics.astype(np.float32), ii=ii, jj=jj, kk=kk,
                target=target.astype(np.float32)[None], weight=weight.astype(np.float32)[None])


def dpvo_state(seed, n=40, M=16, lifetime=13, removal=22, wd=128, ht=96, intr=(80.0, 80.0, 80.0, 60.0)):
    g, poses, patches, intrinsics = dpvo_frames(seed, n, M, wd, ht, intr)
    ii, jj, kk = dpvo_edges(n, M, lifetime, removal)
    return with_edges(g, n, M, poses, patches, intrinsics, ii, jj, kk)


def global_state(seed, n=160, M=6):
    """The global BA's patch edges (dpvo.py:461-474): every patch of frame i
    on every frame pair (i, j) of the fixed pattern."""
    g, poses, patches, intrinsics = dpvo_frames(seed, n, M)
    ie, je = global_edges(n)
    ii = np.repeat(ie, M)
    jj = np.repeat(je, M)
    kk = (ie[:, None] * M + np.arange(M)[None]).reshape(-1).astype(np.int64)
    return with_edges(g, n, M, poses, patches, intrinsics, ii, jj, kk)


def first_diff(a, b):
    """None when a and b hold the same bits (NaNs compared by pattern), else a
    message naming the first differing element: flat index, its coordinates
    and both values."""
    import torch
    if a.shape != b.shape or a.dtype != b.dtype:
        return f"shape / dtype {tuple(a.shape)} {a.dtype} vs {tuple(b.shape)} {b.dtype}"
    x, y = a.detach().contiguous().reshape(-1), b.detach().contiguous().reshape(-1)
    if x.dtype.is_floating_point:
        ib = {2: torch.int16, 4: torch.int32, 8: torch.int64}[x.element_size()]
        x, y = x.view(ib), y.view(ib)
    ne = (x != y).nonzero()
    if ne.numel() == 0:
        return None
    i = int(ne[0, 0])
    coord = np.unravel_index(i, tuple(a.shape)) if a.dim() else ()
    av, bv = a.reshape(-1)[i].item(), b.reshape(-1)[i].item()
    return (f"{ne.shape[0]} of {x.numel()} elements differ; first at flat {i}, index "
            f"{tuple(int(c) for c in coord)}: {av!r} vs {bv!r}")


def assert_same_bits(a, b, what="tensor"):
    msg = first_diff(a, b)
    assert msg is None, f"{what}: {msg}"


def same(a, b, what="tensor"):
    """torch.equal for the bit-identity tests: True, or an AssertionError that
    names the first differing element (first_diff).  Tensors of different
    dtypes fall back to torch.equal's value comparison."""
    import torch
    if a.dtype != b.dtype:
        if not torch.equal(a, b):
            raise AssertionError(f"{what}: values differ ({a.dtype} vs {b.dtype})")
        return True
    msg = first_diff(a, b)
    if msg is not None:
        raise AssertionError(f"{what}: {msg}")
    return True
