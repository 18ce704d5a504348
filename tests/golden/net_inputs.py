"""Deterministic inputs and weights for the learned-module fixtures
(update_ref.npz, encoder_ref.npz).

Shared by tests/golden/make_golden.py (which runs the REFERENCE's own modules,
dpvo/net.py:28-93 Update and dpvo/extractor.py:200-264 BasicEncoder4, on them
in this container) and by the tests (which load the same weights into this
repo's mirror modules and run the native HIP path).  Weights and inputs are
regenerated from seeds with numpy's PCG64 instead of being stored: the
fixtures then hold only the parameter spec (names + shapes, i.e. the
reference's state_dict layout), checksums of what was generated, and the
reference outputs.  Test infrastructure only.
"""
import json

import numpy as np

UPDATE_SEED = 31
ENCODER_SEED = 41


def spec_json(state_dict):
    """the (name, shape) list of a torch state_dict, in its own order"""
    return json.dumps([[k, list(v.shape)] for k, v in state_dict.items()])


def make_params(spec, seed):
    """name -> float32 array for every entry of `spec` (a spec_json string).

    Linear / conv weights: U(-a, a) with a = 2 / sqrt(fan_in) (twice torch's
    default bound, so LayerNorms, gates and ReLUs see O(1) activations);
    1-D weights (LayerNorm gamma): U(0.5, 1.5); biases: U(-0.1, 0.1)
    (LayerNorm beta included) -- non-trivial values everywhere, so a swapped
    gamma / beta or a missing bias shows up in the outputs."""
    g = np.random.default_rng(seed)
    out = {}
    for name, shape in json.loads(str(spec)):
        shape = tuple(shape)
        if name.endswith("weight") and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            a = 2.0 / np.sqrt(fan_in)
            out[name] = g.uniform(-a, a, size=shape).astype(np.float32)
        elif name.endswith("weight"):
            out[name] = g.uniform(0.5, 1.5, size=shape).astype(np.float32)
        else:
            out[name] = g.uniform(-0.1, 0.1, size=shape).astype(np.float32)
    return out


def update_edges(n=12, M=72, seed=UPDATE_SEED):
    """Edge lists of the tracker's rules (dpvo.py:756-769) over n frames of M
    patches, with ~8 % of the edges dropped at random (ragged groups, -1
    neighbours inside a patch's run, frame-pair groups both >= 64 and < 64
    edges long)."""
    ii, jj, kk = [], [], []
    for t in range(1, n + 1):
        for k in range(M * max(t - 13, 0), M * max(t - 1, 0)):
            kk.append(k); jj.append(t - 1); ii.append(k // M)
        for k in range(M * (t - 1), M * t):
            for j in range(max(t - 13, 0), t):
                kk.append(k); jj.append(j); ii.append(k // M)
    ii, jj, kk = (np.asarray(a, np.int64) for a in (ii, jj, kk))
    g = np.random.default_rng(seed + 1)
    keep = g.uniform(size=len(ii)) > 0.08
    return ii[keep], jj[keep], kk[keep]


def update_inputs(E, seed=UPDATE_SEED):
    """net (fp32, the tracker's edge state dtype), inp (fp16, the context
    rows) and corr (fp16, altcorr's 882-wide rows) for E edges."""
    g = np.random.default_rng(seed + 2)
    net = g.standard_normal((E, 384)).astype(np.float32)
    inp = (0.5 * g.standard_normal((E, 384))).astype(np.float16)
    corr = g.standard_normal((E, 882)).astype(np.float16)
    return net, inp, corr


def update_rows(E):
    """the rows whose 384-wide outputs are stored (all rows' delta / weight are)"""
    return np.unique(np.concatenate([np.arange(0, E, max(E // 1536, 1)), [E - 1]])).astype(np.int64)


def texture_image(H, W, seed):
    """uint8 [3, H, W]: smooth value noise (bilinear upsampled 1/16 grid) plus
    pixel noise, the synthetic frame of SURVEY.md 8(d)"""
    g = np.random.default_rng(seed)
    gh, gw = H // 16 + 2, W // 16 + 2
    coarse = g.uniform(0, 255, size=(3, gh, gw))
    ys = np.linspace(0, gh - 1.001, H)
    xs = np.linspace(0, gw - 1.001, W)
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[None, :, None], (xs - x0)[None, None, :]
    c = coarse
    img = ((1 - fy) * (1 - fx) * c[:, y0][:, :, x0] + (1 - fy) * fx * c[:, y0][:, :, x0 + 1] +
           fy * (1 - fx) * c[:, y0 + 1][:, :, x0] + fy * fx * c[:, y0 + 1][:, :, x0 + 1])
    img = img + g.normal(0, 12.0, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


ENCODER_FRAMES = ((384, 512, "texture"), (100, 134, "noise"))


def encoder_image(H, W, kind, seed=ENCODER_SEED):
    if kind == "noise":
        return np.random.default_rng(seed + H).integers(0, 256, size=(3, H, W)).astype(np.uint8)
    return texture_image(H, W, seed + H)


def encoder_centres(h, w, M=96, seed=ENCODER_SEED):
    """patch centres as drawn by the Patchifier (net.py:151-152): x in [1, w-1), y in [1, h-1)"""
    g = np.random.default_rng(seed + 7)
    return g.integers(1, w - 1, size=M).astype(np.int64), g.integers(1, h - 1, size=M).astype(np.int64)


def encoder_rows(h):
    """fmap rows stored for the full-size frame (all rows for small frames)"""
    if h <= 32:
        return np.arange(h, dtype=np.int64)
    return np.unique(np.concatenate([[0, 1, 2], np.arange(3, h - 3, 7), [h - 3, h - 2, h - 1]])).astype(np.int64)


def checksum(a):
    a = np.asarray(a, np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * np.arange(a.size).reshape(a.shape) % 7).sum()])


# ----------------------------------------------------------------------------
# one whole DPVO.update() (dpvo.py:711-749) from an injected steady-state
# patch graph: update_step_ref.npz
# ----------------------------------------------------------------------------
STEP_SEED = 51
# the Update's delta head (d.1, net.py:66) scaled by this factor for the
# update_step fixture: seeded random weights put ~1 px of incoherent noise on
# every target, and two Gauss-Newton steps then drive a few poorly observed
# patches' inverse depths into fastba's / ba.py's different clamps (SURVEY 8c
# (i)), where the reference's two BA implementations disagree by design
STEP_DSCALE = 0.25
# default.yaml (REMOVAL_WINDOW 22, OPTIMIZATION_WINDOW 10, PATCH_LIFETIME 13)
# with M = 12 patches per frame, a 48-frame buffer, n = 40 keyframes (the
# 36-slot feature rings wrap), 128 x 96 frames (32 x 24 feature maps)
STEP = dict(n=40, M=12, N=48, pmem=36, ht=96, wd=128, lifetime=13, removal=22, opt_window=10,
            intrinsics=(20.0, 20.0, 16.0, 12.0), iters=2, file="update_step_ref.npz")
# C2's per-update workload (BASELINE.json configs[1]: default.yaml with M = 96,
# 8 BA iterations): E = 497 M = 47,712 edges in steady state at n = 40, on
# 512 x 384 frames (128 x 96 feature maps, the tartan intrinsics / 4)
STEP_C2 = dict(n=40, M=96, N=48, pmem=36, ht=384, wd=512, lifetime=13, removal=22, opt_window=10,
               intrinsics=(80.0, 80.0, 64.0, 48.0), iters=8, file="update_step_c2_ref.npz", dscale=1.0)
# C3's per-update workload (BASELINE.json configs[2], the metric's config:
# dpvo_2k.yaml, M = 192, 2 BA iterations -- dpvo.py:734): E = 497 M = 95,424
# edges in steady state at n = 40, on 512 x 384 frames.  (dpvo_2k.yaml has
# default.yaml's windows; only KEYFRAME_THRESH differs, which update() does
# not read.)
STEP_C3 = dict(n=40, M=192, N=48, pmem=36, ht=384, wd=512, lifetime=13, removal=22, opt_window=10,
               intrinsics=(80.0, 80.0, 64.0, 48.0), iters=2, file="update_step_c3_ref.npz", dscale=1.0,
               preset="dpvo_2k")
STEPS = {"small": STEP, "c2": STEP_C2, "c3": STEP_C3}


def _qmul(a, b):
    """Hamilton product of [x, y, z, w] quaternions"""
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def step_edges(n, M, lifetime, removal):
    """the edge set update() sees at n keyframes in steady state: the append
    rules of dpvo.py:756-769 for the recent frames, then the removal rule of
    dpvo.py:657 as of the previous keyframe (dpvo/synthetic.py restated)"""
    ii, jj, kk = [], [], []
    for t in range(max(1, n - removal - 2), n + 1):
        for k in range(M * max(t - lifetime, 0), M * max(t - 1, 0)):
            ii.append(k // M); jj.append(t - 1); kk.append(k)
        for k in range(M * (t - 1), M * t):
            for j in range(max(t - lifetime, 0), t):
                ii.append(k // M); jj.append(j); kk.append(k)
    ii, jj, kk = (np.asarray(a, np.int64) for a in (ii, jj, kk))
    keep = ii >= n - 1 - removal
    return ii[keep], jj[keep], kk[keep]


def update_step_state(seed=STEP_SEED, S=None):
    """Every input of one update(): poses [N][7] (rows >= n zero), patches
    [N*M][3][3][3], intrinsics [N][4] (all fp32), the fp16 rings fmap1
    [pmem][128][h][w], fmap2 [pmem][128][h/4][w/4] (4x4 average of fmap1),
    gmap [pmem][M][128][3][3] (3x3 windows of fmap1 at the patch centres, the
    Patchifier's patchify), imap [pmem][M][384], the edges ii / jj / kk and the
    fp32 edge state net [E][384].  S: STEP (default) or STEP_C2."""
    S = STEP if S is None else S
    n, M, N, pmem = S["n"], S["M"], S["N"], S["pmem"]
    h, w = S["ht"] // 4, S["wd"] // 4
    g = np.random.default_rng(seed)
    poses = np.zeros((N, 7), np.float64)
    poses[0, 6] = 1.0
    for i in range(1, n):
        dq = np.concatenate([0.5 * g.normal(0, 0.01, 3), [1.0]])
        q = _qmul(dq / np.linalg.norm(dq), poses[i - 1, 3:])
        poses[i, 3:] = q / np.linalg.norm(q)
        poses[i, :3] = poses[i - 1, :3] + g.normal(0, 0.05, 3)
    xs = g.integers(1, w - 1, size=(n, M)).astype(np.float64)
    ys = g.integers(1, h - 1, size=(n, M)).astype(np.float64)
    d = g.uniform(0.2, 1.0, size=(n, M))
    patches = np.zeros((N, M, 3, 3, 3))
    off = np.arange(3) - 1.0
    patches[:n, :, 0] = xs[:, :, None, None] + off[None, None, None, :]
    patches[:n, :, 1] = ys[:, :, None, None] + off[None, None, :, None]
    patches[:n, :, 2] = d[:, :, None, None]
    intrinsics = np.zeros((N, 4))
    intrinsics[:n] = S["intrinsics"]
    fmap1 = (0.25 * g.standard_normal((pmem, 128, h, w))).astype(np.float16)
    fmap2 = fmap1.astype(np.float32).reshape(pmem, 128, h // 4, 4, w // 4, 4).mean((3, 5)).astype(np.float16)
    gmap = np.zeros((pmem, M, 128, 3, 3), np.float16)
    imap = np.zeros((pmem, M, 384), np.float16)
    for f in range(n - pmem, n):
        s = f % pmem
        for p in range(M):
            x, y = int(xs[f, p]), int(ys[f, p])
            gmap[s, p] = fmap1[s, :, y - 1:y + 2, x - 1:x + 2]
        imap[s] = g.standard_normal((M, 384)).astype(np.float16)
    ii, jj, kk = step_edges(n, M, S["lifetime"], S["removal"])
    net = (0.1 * g.standard_normal((len(ii), 384))).astype(np.float32)
    return dict(poses=poses.astype(np.float32), patches=patches.reshape(N * M, 3, 3, 3).astype(np.float32),
                intrinsics=intrinsics.astype(np.float32), fmap1=fmap1, fmap2=fmap2, gmap=gmap, imap=imap,
                ii=ii, jj=jj, kk=kk, net=net)
