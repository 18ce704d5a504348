"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference.  The fixtures are data (seeded inputs + expected
outputs); nothing from the reference travels with them.

What pins what
--------------
* ``lietorch_*.npz`` / ``pops_*.npz`` / ``ba_python_*.npz``: the reference's
  OWN Python (``dpvo/lietorch/groups.py``, ``broadcasting.py``,
  ``dpvo/projective_ops.py``, ``dpvo/ba.py``) executed as imported code.  The
  reference's native modules cannot be built here (no nvcc, no Eigen; see
  SURVEY.md 8c), so ``lietorch_backends`` is served by the CPU oracle's
  restatement of ``lietorch/include/{so3,rxso3,se3,sim3}.h``, which is first checked by
  the reference's own property tests (``dpvo/lietorch/run_tests.py``
  test_exp_log / test_inv / test_adj / test_act, executed below).
  ``torch_scatter.scatter_sum`` (torch-scatter 2.1.2, absent) is restated as
  ``index_add``; ``cv2`` is stubbed (import only).
* ``altcorr_*.npz``: the reference has no CPU/Python altcorr.  The expected
  outputs come from an independent torch-CPU-float16 restatement of
  ``correlation_kernel.cu:83-135`` whose epilogue executes the reference's
  own ATen expression (``:221-232``) on float16 tensors; the C oracle must
  agree with it bit for bit (tests/test_oracle.py).
* ``neighbors_*.npz``: a Python restatement of ``ba.cpp:113-158``.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import copy
import importlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import oracle  # noqa: E402
import net_inputs as NI  # noqa: E402


# ----------------------------------------------------------------------------
# stand-ins for the reference's un-buildable native / absent third-party deps
# ----------------------------------------------------------------------------
def _lie_backend_module():
    m = types.ModuleType("lietorch_backends")

    def make(op):
        def f(group_id, X, Y=None):
            Xn = X.detach().cpu().double().numpy().reshape(X.shape[0], -1)
            Yn = None if Y is None else Y.detach().cpu().double().numpy().reshape(Y.shape[0], -1)
            out = oracle.lie_forward(op, group_id, Xn, Yn)
            return torch.from_numpy(out).to(X.dtype)
        return f

    for name, op in [("expm", "exp"), ("logm", "log"), ("inv", "inv"), ("mul", "mul"), ("adj", "adj"),
                     ("adjT", "adjT"), ("act", "act"), ("act4", "act4"), ("as_matrix", "matrix"),
                     ("projector", "projector"), ("Jinv", "Jinv")]:
        setattr(m, name, make(op))

    def no_backward(*a, **k):
        raise NotImplementedError("backward not restated in the oracle")

    for name in ["expm_backward", "logm_backward", "inv_backward", "mul_backward", "adj_backward",
                 "adjT_backward", "act_backward", "act4_backward"]:
        setattr(m, name, no_backward)
    return m


def _torch_scatter_module():
    m = types.ModuleType("torch_scatter")

    def scatter_sum(src, index, dim=-1, dim_size=None):
        dim = dim % src.dim()
        if dim_size is None:
            dim_size = int(index.max()) + 1 if index.numel() else 0
        shape = list(src.shape)
        shape[dim] = dim_size
        out = torch.zeros(shape, dtype=src.dtype)
        return out.index_add_(dim, index, src)

    def _bcast(index, src, dim):
        # torch_scatter.utils.broadcast: a 1-D index along `dim`, expanded to src
        view = [1] * src.dim()
        view[dim] = -1
        return index.view(view).expand_as(src)

    def scatter_softmax(src, index, dim=-1, eps=1e-12, dim_size=None):
        # torch-scatter 2.1.2 composite/softmax.py: recentre on the group max,
        # exp, divide by (group sum + eps)
        dim = dim % src.dim()
        if dim_size is None:
            dim_size = int(index.max()) + 1 if index.numel() else 0
        idx = _bcast(index, src, dim)
        shape = list(src.shape)
        shape[dim] = dim_size
        gmax = torch.zeros(shape, dtype=src.dtype).scatter_reduce(dim, idx, src, "amax", include_self=False)
        ex = (src - gmax.gather(dim, idx)).exp()
        den = scatter_sum(ex, index, dim, dim_size) + eps
        return ex / den.gather(dim, idx)

    m.scatter_sum = scatter_sum
    m.scatter_softmax = scatter_softmax
    return m


def _neighbors_stub(ii, jj):
    """cuda_ba.neighbors (ba.cpp:106-151) := the Python restatement below"""
    ix, jx = neighbors_py(ii.cpu().numpy(), jj.cpu().numpy())
    return [torch.from_numpy(ix), torch.from_numpy(jx)]


def import_reference():
    for name in list(sys.modules):
        if name == "dpvo" or name.startswith("dpvo."):
            del sys.modules[name]
    sys.modules["lietorch_backends"] = _lie_backend_module()
    sys.modules["torch_scatter"] = _torch_scatter_module()
    for stub in ["cuda_ba", "cuda_corr", "cv2"]:
        mod = types.ModuleType(stub)
        for attr in ["neighbors", "reproject", "forward", "backward", "patchify_forward", "patchify_backward"]:
            setattr(mod, attr, None)
        sys.modules[stub] = mod
    sys.modules["cuda_ba"].neighbors = _neighbors_stub
    sys.path.insert(0, REF)
    pops = importlib.import_module("dpvo.projective_ops")
    ba = importlib.import_module("dpvo.ba")
    lie = importlib.import_module("dpvo.lietorch")
    return pops, ba, lie


# ----------------------------------------------------------------------------
# lietorch: run the reference's own forward property tests against the oracle
# ----------------------------------------------------------------------------
def lietorch_fixtures(lie):
    sys.path.insert(0, os.path.join(REF, "dpvo", "lietorch"))
    sys.modules["lietorch"] = lie
    sys.modules.setdefault("gradcheck", types.ModuleType("gradcheck"))
    sys.modules["gradcheck"].gradcheck = None
    sys.modules["gradcheck"].get_analytical_jacobian = None
    rt = importlib.import_module("run_tests")
    torch.manual_seed(0)
    for G in [lie.SO3, lie.RxSO3, lie.SE3, lie.Sim3]:
        rt.test_exp_log(G, device="cpu")
        rt.test_inv(G, device="cpu")
        rt.test_adj(G, device="cpu")
        rt.test_act(G, device="cpu")

    # vectors through the reference Python surface (broadcasting + views)
    g = torch.Generator().manual_seed(1)
    out = {}
    for name, G in [("SE3", lie.SE3), ("SO3", lie.SO3), ("RxSO3", lie.RxSO3), ("Sim3", lie.Sim3)]:
        D = G.manifold_dim
        a = 0.7 * torch.randn(5, 4, D, generator=g, dtype=torch.float64)
        b = 0.7 * torch.randn(5, 4, D, generator=g, dtype=torch.float64)
        X, Y = G.exp(a), G.exp(b)
        p3 = torch.randn(5, 4, 3, generator=g, dtype=torch.float64)
        p4 = torch.cat([p3, torch.rand(5, 4, 1, generator=g, dtype=torch.float64) + 0.1], -1)
        t = torch.randn(5, 4, D, generator=g, dtype=torch.float64)
        Xb = G.exp(0.7 * torch.randn(5, 1, D, generator=g, dtype=torch.float64))  # broadcast case
        out.update({
            f"{name}_a": a.numpy(), f"{name}_b": b.numpy(), f"{name}_p3": p3.numpy(), f"{name}_p4": p4.numpy(),
            f"{name}_t": t.numpy(), f"{name}_Xb": Xb.data.numpy(),
            f"{name}_exp": X.data.numpy(), f"{name}_log": X.log().numpy(), f"{name}_inv": X.inv().data.numpy(),
            f"{name}_mul": (X * Y).data.numpy(), f"{name}_act": X.act(p3).numpy(), f"{name}_act4": X.act(p4).numpy(),
            f"{name}_adj": X.adj(t).numpy(), f"{name}_adjT": X.adjT(t).numpy(), f"{name}_matrix": X.matrix().numpy(),
            f"{name}_Jinv": X.Jinv(t).numpy(), f"{name}_bmul": (Xb * X).data.numpy(),
            f"{name}_bact4": Xb.act(p4).numpy(),
        })
    np.savez_compressed(os.path.join(HERE, "lietorch_ref.npz"), **out)
    print("lietorch: reference run_tests forward checks passed; vectors saved")


# ----------------------------------------------------------------------------
# synthetic patch-graph state (scaled down)
# ----------------------------------------------------------------------------
def synth_state(seed, n=12, M=8, P=3, wd=32, ht=24, intr=(20.0, 20.0, 16.0, 12.0), rot=0.01, trans=0.05):
    g = np.random.default_rng(seed)
    poses = np.zeros((n, 7), np.float64)
    poses[:, 6] = 1.0
    for i in range(1, n):
        xi = np.concatenate([g.normal(0, trans, 3), g.normal(0, rot, 3)])
        dq = oracle.lie_forward("exp", oracle.SE3, xi[None])
        poses[i] = oracle.lie_forward("mul", oracle.SE3, dq, poses[i - 1:i])[0]
    xs = g.integers(1, wd - 1, size=(n, M)).astype(np.float64)
    ys = g.integers(1, ht - 1, size=(n, M)).astype(np.float64)
    d = g.uniform(0.2, 1.0, size=(n, M))
    patches = np.zeros((n, M, 3, P, P))
    off = np.arange(P) - P // 2
    patches[:, :, 0] = xs[:, :, None, None] + off[None, None, None, :]
    patches[:, :, 1] = ys[:, :, None, None] + off[None, None, :, None]
    patches[:, :, 2] = d[:, :, None, None]
    intrinsics = np.tile(np.asarray(intr, np.float64), (n, 1))
    return poses.astype(np.float32), patches.reshape(n * M, 3, P, P).astype(np.float32), intrinsics.astype(np.float32)


def dpvo_edges(n, M, lifetime=13):
    """Edge rules of dpvo.py:756-769 applied frame by frame, removal :657."""
    ii, jj, kk = [], [], []
    for t in range(1, n + 1):
        t0, t1 = M * max(t - lifetime, 0), M * max(t - 1, 0)
        for k in range(t0, t1):
            kk.append(k); jj.append(t - 1); ii.append(k // M)
        for k in range(M * (t - 1), M * t):
            for j in range(max(t - lifetime, 0), t):
                kk.append(k); jj.append(j); ii.append(k // M)
    return np.array(ii, np.int64), np.array(jj, np.int64), np.array(kk, np.int64)


def pops_fixtures(pops, lie):
    poses, patches, intr = synth_state(2)
    n, M = 12, 8
    ii, jj, kk = dpvo_edges(n, M)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    Gs = lie.SE3(T(poses)[None])
    pt, it = T(patches)[None], T(intr)[None]
    c = pops.transform(Gs, pt, it, T(ii), T(jj), T(kk))
    cd, v = pops.transform(Gs, pt, it, T(ii), T(jj), T(kk), depth=True, valid=True)
    ct = pops.transform(Gs, pt, it, T(ii), T(jj), T(kk), tonly=True)
    x1, vj, (Ji, Jj, Jz) = pops.transform(Gs, pt, it, T(ii), T(jj), T(kk), jacobian=True)
    ix = torch.arange(n).repeat_interleave(M)
    pc = pops.point_cloud(Gs, pt, it, ix)
    fm = pops.flow_mag(Gs, pt, it, T(ii[:40]), T(jj[:40]), T(kk[:40]), beta=0.5)
    np.savez_compressed(os.path.join(HERE, "pops_ref.npz"), poses=poses, patches=patches, intrinsics=intr,
                        ii=ii, jj=jj, kk=kk, coords=c.numpy(), coords_depth=cd.numpy(), valid=v.numpy(),
                        coords_tonly=ct.numpy(), Ji=Ji.numpy(), Jj=Jj.numpy(), Jz=Jz.numpy(),
                        point_cloud=pc.numpy(), ix=ix.numpy(), flow_mag=fm.numpy())
    print("pops: transform / point_cloud / flow_mag vectors saved, E =", len(ii))


def ba_fixtures(ba, lie):
    """The reference Python BA (dpvo/ba.py:207-309) with the arguments that
    make it the same Gauss-Newton step as the live CUDA fastba:
    ep=1.0, lmbda=1e-4, bounds=[-64,-64,2cx+64,2cy+64], fixedp=t0,
    patches_est=0.  One call per iteration."""
    out = {}
    for case, (seed, n, M, t0, iters, structure_only) in {
        "window": (3, 12, 8, 2, 2, False),
        "full": (4, 10, 6, 1, 3, False),
        "structure": (5, 8, 6, 8, 2, True),
    }.items():
        poses, patches, intr = synth_state(seed, n=n, M=M)
        ii, jj, kk = dpvo_edges(n, M)
        g = np.random.default_rng(seed + 100)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
        coords = oracle.transform(poses, patches, intr, ii, jj, kk)[0]  # [E,P,P,2]
        target = coords[:, 1, 1, :] + g.normal(0, 0.5, size=(len(ii), 2))
        weight = g.uniform(0.2, 1.0, size=(len(ii), 2))
        target = target.astype(np.float32)[None]
        weight = weight.astype(np.float32)[None]
        cx, cy = float(intr[0, 2]), float(intr[0, 3])
        bounds = [-64, -64, 2 * cx + 64, 2 * cy + 64]
        Gs = lie.SE3(T(poses.copy())[None])
        pt = T(patches.copy())[None]
        est = torch.zeros_like(pt)
        for _ in range(iters):
            Gs, pt = ba.BA(Gs, pt, T(intr)[None], T(target), T(weight), 1e-4, T(ii), T(jj), T(kk), bounds,
                           ep=1.0, fixedp=t0, structure_only=structure_only, patches_est=est)
        t1 = t0 if structure_only else int(max(ii.max(), jj.max())) + 1
        out.update({f"{case}_poses": poses, f"{case}_patches": patches, f"{case}_intrinsics": intr,
                    f"{case}_target": target, f"{case}_weight": weight, f"{case}_ii": ii, f"{case}_jj": jj,
                    f"{case}_kk": kk, f"{case}_t0": np.int64(t0), f"{case}_t1": np.int64(t1),
                    f"{case}_iters": np.int64(iters),
                    f"{case}_poses_out": Gs.data[0].numpy(), f"{case}_patches_out": pt[0].numpy()})
    np.savez_compressed(os.path.join(HERE, "ba_python_ref.npz"), **out)
    print("ba: reference Python BA vectors saved")


# ----------------------------------------------------------------------------
# altcorr: torch-CPU float16 restatement of correlation_kernel.cu
# ----------------------------------------------------------------------------
def torch_corr_f16(fmap1, fmap2, coords, ii, jj, radius, dtype=torch.float16):
    """correlation_kernel.cu:83-135 with c10::Half arithmetic (each product
    and each sum rounded to binary16), then the reference's ATen epilogue
    (:221-232) verbatim on float16 tensors.  Returns the returned view
    (permuted) as a contiguous tensor [B,E,2r+1(x),2r+1(y),H,W].
    dtype=torch.float64: the same sums and epilogue in float64 (the exact
    answer for fp16 inputs)."""
    fmap1, fmap2 = fmap1.to(dtype), fmap2.to(dtype)
    R, D = radius, 2 * radius + 2
    B, M, _, H, W = coords.shape
    C, H2, W2 = fmap1.shape[2], fmap2.shape[3], fmap2.shape[4]
    x, y = coords[:, :, 0], coords[:, :, 1]
    fy, fx = torch.floor(y).long(), torch.floor(x).long()
    a = torch.arange(D).view(1, 1, 1, 1, D, 1)
    b = torch.arange(D).view(1, 1, 1, 1, 1, D)
    i1 = fy[..., None, None] + (a - R)
    j1 = fx[..., None, None] + (b - R)
    inb = (i1 >= 0) & (i1 < H2) & (j1 >= 0) & (j1 < W2)
    i1c, j1c = i1.clamp(0, H2 - 1), j1.clamp(0, W2 - 1)
    s = torch.zeros(B, M, H, W, D, D, dtype=dtype)
    bidx = torch.arange(B).view(B, 1, 1, 1, 1, 1)
    jx = jj.view(1, M, 1, 1, 1, 1)
    f1 = fmap1[torch.arange(B).view(B, 1), ii.view(1, M)]  # [B,M,C,H,W]
    for c in range(C):
        f2 = fmap2[bidx, jx, c, i1c, j1c]  # [B,M,H,W,D,D]
        s = s + f1[:, :, c, :, :, None, None] * f2
    s = torch.where(inb, s, torch.zeros((), dtype=dtype))
    corr = s.permute(0, 1, 4, 5, 2, 3).contiguous()  # [B,M,D(a),D(b),H,W]
    # --- the reference's ATen epilogue, correlation_kernel.cu:221-232 ---
    xx = coords[:, :, 0, None, None]
    yy = coords[:, :, 1, None, None]
    dx = xx - xx.floor(); dx = dx.to(dtype)
    dy = yy - yy.floor(); dy = dy.to(dtype)
    out = (1 - dx) * (1 - dy) * corr[:, :, 0:D - 1, 0:D - 1]
    out += (dx) * (1 - dy) * corr[:, :, 0:D - 1, 1:D]
    out += (1 - dx) * (dy) * corr[:, :, 1:D, 0:D - 1]
    out += (dx) * (dy) * corr[:, :, 1:D, 1:D]
    return out.permute(0, 1, 3, 2, 4, 5).contiguous()


def altcorr_fixtures():
    g = torch.Generator().manual_seed(7)
    cases = {}
    # (a) DPVO-shaped: two pyramid levels, 3x3 patches, radius 3
    N1, C, N2, H2, W2, E = 20, 128, 3, 16, 24, 48
    gmap = (0.25 * torch.randn(1, N1, C, 3, 3, generator=g)).half()
    fmap1 = (0.25 * torch.randn(1, N2, C, H2, W2, generator=g)).half()
    fmap2 = torch.nn.functional.avg_pool2d(fmap1[0].float(), 4, 4).half()[None]
    ii = torch.randint(0, N1, (E,), generator=g)
    jj = torch.randint(0, N2, (E,), generator=g)
    base = torch.stack([torch.rand(E, generator=g) * (W2 + 8) - 4, torch.rand(E, generator=g) * (H2 + 8) - 4], -1)
    off = torch.stack(torch.meshgrid(torch.arange(3.) - 1, torch.arange(3.) - 1, indexing="ij")[::-1], 0)
    jitter = 0.3 * torch.randn(E, 2, 3, 3, generator=g)
    coords = (base[:, :, None, None] + off[None] + jitter)[None].float()
    coords[0, :4] = torch.floor(coords[0, :4])  # integer coordinates
    lv1 = torch_corr_f16(gmap, fmap1, coords / 1, ii, jj, 3)
    lv2 = torch_corr_f16(gmap, fmap2, coords / 4, ii, jj, 3)
    stacked = torch.stack([lv1, lv2], -1).view(1, E, -1)
    cases.update(dict(gmap=gmap.view(torch.int16).numpy(), fmap1=fmap1.view(torch.int16).numpy(),
                      fmap2=fmap2.view(torch.int16).numpy(), coords=coords.numpy(), ii=ii.numpy(), jj=jj.numpy(),
                      corr_l1=lv1.view(torch.int16).numpy(), corr_l2=lv2.view(torch.int16).numpy(),
                      corr_stacked=stacked.view(torch.int16).numpy()))
    # (b) odd shapes: radius 1, 5x5 "patches", C=40, batch 2
    B, N1b, Cb, Pb, H2b, W2b, Eb = 2, 6, 40, 5, 9, 11, 10
    gb = (torch.randn(B, N1b, Cb, Pb, Pb, generator=g)).half()
    fb = (torch.randn(B, 3, Cb, H2b, W2b, generator=g)).half()
    iib = torch.randint(0, N1b, (Eb,), generator=g)
    jjb = torch.randint(0, 3, (Eb,), generator=g)
    cb = (torch.rand(B, Eb, 2, Pb, Pb, generator=g) * 14 - 2).float()
    ob = torch_corr_f16(gb, fb, cb, iib, jjb, 1)
    cases.update(dict(b_gmap=gb.view(torch.int16).numpy(), b_fmap=fb.view(torch.int16).numpy(),
                      b_coords=cb.numpy(), b_ii=iib.numpy(), b_jj=jjb.numpy(), b_corr=ob.view(torch.int16).numpy()))
    np.savez_compressed(os.path.join(HERE, "altcorr_ref.npz"), **cases)
    print("altcorr: torch-f16 restatement vectors saved")


# ----------------------------------------------------------------------------
# neighbors (ba.cpp:113-158) restated in Python
# ----------------------------------------------------------------------------
def neighbors_py(ii, jj):
    uniq, perm = np.unique(ii, return_inverse=True)
    index = [[] for _ in range(len(uniq))]
    for i in range(len(ii)):
        index[perm[i]].append(i)
    ix = np.empty(len(ii), np.int64)
    jx = np.empty(len(ii), np.int64)
    for idx in index:
        idx = sorted(idx, key=lambda e: jj[e])  # Python sort is stable
        for i, e in enumerate(idx):
            ix[e] = idx[i - 1] if i > 0 else -1
            jx[e] = idx[i + 1] if i < len(idx) - 1 else -1
    return ix, jx


def neighbors_fixtures():
    ii, jj, kk = dpvo_edges(20, 6)
    g = np.random.default_rng(9)
    keep = g.uniform(size=len(ii)) > 0.2
    kk2, jj2 = kk[keep], jj[keep]
    ix, jx = neighbors_py(kk2, jj2)
    r_kk = g.integers(0, 7, 300)
    r_jj = g.integers(0, 5, 300)
    rix, rjx = neighbors_py(r_kk, r_jj)
    np.savez_compressed(os.path.join(HERE, "neighbors_ref.npz"), kk=kk2, jj=jj2, ix=ix, jx=jx,
                        r_kk=r_kk, r_jj=r_jj, r_ix=rix, r_jx=rjx)
    print("neighbors: vectors saved")


# ----------------------------------------------------------------------------
# the learned modules: reference Update (net.py:28-93) and BasicEncoder4
# (extractor.py:200-264) executed as imported code
# ----------------------------------------------------------------------------
def _load(module, spec, seed):
    params = NI.make_params(spec, seed)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    module.load_state_dict(sd, strict=True)
    return params


def _err_stats(a, ref):
    d = (np.asarray(a, np.float64) - np.asarray(ref, np.float64))
    return np.array([np.sqrt((d ** 2).mean()), np.abs(d).max()])


def update_fixtures():
    """Update.forward (net.py:75-93) of the reference module on seeded
    weights / inputs: in float64 (the exact answer) and under CPU fp16
    autocast (the reference's own fp16 execution; its error against float64
    is the scale the native fp16 path is held to)."""
    net_mod = importlib.import_module("dpvo.net")
    torch.manual_seed(0)
    upd = net_mod.Update(3)
    spec = NI.spec_json(upd.state_dict())
    params = _load(upd, spec, NI.UPDATE_SEED)
    ii, jj, kk = NI.update_edges()
    E = len(ii)
    net, inp, corr = NI.update_inputs(E)
    T = torch.from_numpy
    with torch.no_grad():
        u64 = copy.deepcopy(upd).double()
        n64, (d64, w64, _) = u64(T(net).double()[None], T(inp).double()[None], T(corr).double()[None], None,
                                 T(ii), T(jj), T(kk))
        with torch.autocast("cpu", dtype=torch.float16):
            n16, (d16, w16, _) = upd(T(net)[None], T(inp)[None], T(corr)[None], None, T(ii), T(jj), T(kk))
    rows = NI.update_rows(E)
    n64, d64, w64 = n64[0].numpy(), d64[0].numpy(), w64[0].numpy()
    n16, d16, w16 = n16[0].float().numpy(), d16[0].float().numpy(), w16[0].float().numpy()
    ix, jx = neighbors_py(kk, jj)
    np.savez_compressed(
        os.path.join(HERE, "update_ref.npz"), spec=np.array(spec), seed=np.int64(NI.UPDATE_SEED),
        param_checksum=np.stack([NI.checksum(params[k]) for k in sorted(params)]),
        ii=ii, jj=jj, kk=kk, input_checksum=np.stack([NI.checksum(x) for x in (net, inp, corr)]),
        rows=rows, net_out=n64[rows].astype(np.float32), delta=d64.astype(np.float32), weight=w64.astype(np.float32),
        net_out64_rows_sum=n64[rows].sum(1), n_ix_neg=np.int64((ix < 0).sum()), n_jx_neg=np.int64((jx < 0).sum()),
        amp_err_net=_err_stats(n16[rows], n64[rows]), amp_err_delta=_err_stats(d16, d64),
        amp_err_weight=_err_stats(w16, w64))
    print(f"update: reference Update.forward vectors saved, E = {E}; CPU-amp error rms/max net "
          f"{_err_stats(n16, n64)}, delta {_err_stats(d16, d64)}, weight {_err_stats(w16, w64)}")


def encoder_fixtures():
    """fnet = BasicEncoder4(128, 'instance') and inet = BasicEncoder4(384,
    'none') (net.py:100-101) of the reference on seeded weights, in float64,
    on the Patchifier's input 2 (img / 255) - 0.5 and its /4 scale
    (net.py:119-122): fmap (stored rows) and imap at the patch centres."""
    ext = importlib.import_module("dpvo.extractor")
    torch.manual_seed(0)
    fnet = ext.BasicEncoder4(output_dim=128, norm_fn="instance")
    inet = ext.BasicEncoder4(output_dim=384, norm_fn="none")
    fspec, ispec = NI.spec_json(fnet.state_dict()), NI.spec_json(inet.state_dict())
    fp = _load(fnet, fspec, NI.ENCODER_SEED)
    ip = _load(inet, ispec, NI.ENCODER_SEED + 1)
    out = dict(fspec=np.array(fspec), ispec=np.array(ispec),
               param_checksum=np.stack([NI.checksum(d[k]) for d in (fp, ip) for k in sorted(d)]))
    fnet, inet = fnet.double().eval(), inet.double().eval()
    for f, (H, W, kind) in enumerate(NI.ENCODER_FRAMES):
        img = NI.encoder_image(H, W, kind)
        x = 2 * (torch.from_numpy(img).double()[None, None] / 255.0) - 0.5
        with torch.no_grad():
            fmap = (fnet(x) / 4.0)[0, 0].numpy()
            imap = (inet(x) / 4.0)[0, 0].numpy()
        h, w = fmap.shape[-2:]
        xs, ys = NI.encoder_centres(h, w)
        rows = NI.encoder_rows(h)
        out.update({f"f{f}_image_checksum": NI.checksum(img), f"f{f}_hw": np.array([h, w]), f"f{f}_rows": rows,
                    f"f{f}_fmap": fmap[:, rows].astype(np.float32), f"f{f}_xs": xs, f"f{f}_ys": ys,
                    f"f{f}_imap": imap[:, ys, xs].T.astype(np.float32)})
        print(f"encoders: frame {H}x{W} ({kind}) -> fmap {fmap.shape}, |fmap| max {np.abs(fmap).max():.3g}")
    np.savez_compressed(os.path.join(HERE, "encoder_ref.npz"), **out)
    print("encoders: reference BasicEncoder4 vectors saved")


def update_step_fixtures(pops, ba, lie, dscale=None, save=True, which="small"):
    """One whole DPVO.update() (dpvo.py:711-749) of the reference from the
    injected steady-state graph of net_inputs.update_step_state(), through the
    reference's own modules:
      reproject  = projective_ops.transform (+ the permute of dpvo.py:338),
      corr       = the CUDA-only altcorr restated (torch_corr_f16, both levels,
                   coords / 1 and / 4, ring slots kk % (M pmem), jj % pmem,
                   dpvo.py:326-333),
      ctx        = imap[:, kk % (M pmem)]  (dpvo.py:718),
      network    = net.Update on the update_ref.npz weights,
      target     = coords[..., 1, 1] + delta, weight  (dpvo.py:722-724),
      BA         = ba.py with the fastba argument mapping, twice,
                   t0 = n - OPTIMIZATION_WINDOW (dpvo.py:730-734),
      points     = projective_ops.point_cloud centre / w (dpvo.py:747-749).
    Run twice: "f64" in float64 throughout (the exact answer for these inputs)
    and "r16" with the reference's own precisions (fp16 altcorr chain, Update
    under fp16 autocast, fp32 BA) -- its distance from f64 is the reference's
    own error at this state.  The C oracle's restatement of ba_cuda.cu is run
    on the r16 targets as a cross-check of the ba.py mapping."""
    net_mod = importlib.import_module("dpvo.net")
    C = NI.STEPS[which]
    S = NI.update_step_state(NI.STEP_SEED, C)
    iters = C["iters"]
    n, M, pmem = C["n"], C["M"], C["pmem"]
    m = n * M
    t0 = n - C["opt_window"]
    torch.manual_seed(0)
    upd = net_mod.Update(3)
    spec = NI.spec_json(upd.state_dict())
    _load(upd, spec, NI.UPDATE_SEED)
    dscale = C.get("dscale", NI.STEP_DSCALE) if dscale is None else dscale
    with torch.no_grad():   # the delta head scaled (net_inputs.STEP_DSCALE): see there
        upd.d[1].weight.mul_(dscale)
        upd.d[1].bias.mul_(dscale)
    upd.eval()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    ii, jj, kk = T(S["ii"]), T(S["jj"]), T(S["kk"])
    E = len(ii)
    gmap = T(S["gmap"]).view(1, pmem * M, 128, 3, 3)
    fmap1, fmap2 = T(S["fmap1"])[None], T(S["fmap2"])[None]
    imap = T(S["imap"]).view(1, pmem * M, 384)
    ix = torch.arange(C["N"]).repeat_interleave(M)
    rows = NI.update_rows(E)[::4]
    crow = rows[::3]
    cx, cy = C["intrinsics"][2], C["intrinsics"][3]
    bounds = [-64, -64, 2 * cx + 64, 2 * cy + 64]
    out = dict(seed=np.int64(NI.STEP_SEED), dscale=np.float64(dscale), update_seed=np.int64(NI.UPDATE_SEED), spec=np.array(spec),
               t0=np.int64(t0), n=np.int64(n), rows=rows, corr_rows=crow, which=np.array(which), iters=np.int64(iters),
               state_checksum=np.stack([NI.checksum(S[k]) for k in sorted(S)]))
    touched = np.unique(S["kk"])
    out["touched"] = touched
    res = {}
    for mode, dt, cdt in (("f64", torch.float64, torch.float64), ("r16", torch.float32, torch.float16)):
        poses = T(S["poses"]).to(dt)[None]
        patches = T(S["patches"]).to(dt)[None]
        intr = T(S["intrinsics"]).to(dt)[None]
        with torch.no_grad():
            coords = pops.transform(lie.SE3(poses), patches, intr, ii, jj, kk)
            coords = coords.permute(0, 1, 4, 2, 3).contiguous()          # DPVO.reproject
            ii1, jj1 = kk % (M * pmem), jj % pmem
            corr1 = torch_corr_f16(gmap, fmap1, coords / 1, ii1, jj1, 3, dtype=cdt)
            corr2 = torch_corr_f16(gmap, fmap2, coords / 4, ii1, jj1, 3, dtype=cdt)
            corr = torch.stack([corr1, corr2], -1).view(1, E, -1)
            ctx = imap[:, kk % (M * pmem)]
            net = T(S["net"])[None]
            if mode == "f64":
                u64 = copy.deepcopy(upd).double()
                net_o, (delta, weight, _) = u64(net.double(), ctx.double(), corr, None, ii, jj, kk)
            else:
                with torch.autocast("cpu", dtype=torch.float16):
                    net_o, (delta, weight, _) = upd(net, ctx, corr, None, ii, jj, kk)
            weight = weight.to(dt)
            target = coords[..., 1, 1] + delta.to(dt)
            Gs, pt = lie.SE3(poses.clone()), patches.clone()
            est = torch.zeros_like(pt)
            for _ in range(iters):
                Gs, pt = ba.BA(Gs, pt, intr, target, weight, 1e-4, ii, jj, kk, bounds, ep=1.0, fixedp=t0,
                               structure_only=False, patches_est=est)
                dep = pt[0, touched, 2].numpy()
                print(f"update_step {mode}: touched depths in [{dep.min():.4g}, {dep.max():.4g}]")
                assert dep.min() > 1e-3 and dep.max() < 10.0, (mode, dep.min(), dep.max())
            pc = pops.point_cloud(Gs, pt[:, :m], intr, ix[:m])
            points = (pc[..., 1, 1, :3] / pc[..., 1, 1, 3:]).reshape(-1, 3)
        r = dict(poses=Gs.data[0].numpy().astype(np.float64), depth=pt[0, touched, 2, 1, 1].numpy().astype(np.float64),
                 points=points.numpy().astype(np.float64), net=net_o[0].float().numpy()[rows].astype(np.float64),
                 delta=delta[0].float().numpy().astype(np.float64),
                 weight=weight[0].float().numpy().astype(np.float64),
                 target=target[0].numpy().astype(np.float64), corr=corr[0].numpy()[crow])
        res[mode] = r
        for k in ("poses", "depth", "points", "net", "delta", "weight", "target"):
            small = k in ("poses", "depth", "points") and mode == "f64"
            out[f"{mode}_{k}"] = r[k] if small else r[k].astype(np.float32)
        if mode == "r16":
            # the C restatement of ba_cuda.cu on the same fp32 targets / weights
            rp, rq, st = oracle.ba_forward(S["poses"], S["patches"], S["intrinsics"], target.numpy(),
                                           weight.numpy(), 1e-4, S["ii"], S["jj"], S["kk"], t0, n, iters)
            assert st == 0
            dpose = np.abs(rp[t0:n] - r["poses"][t0:n]).max()
            ddep = np.abs(rq[touched, 2, 1, 1] - r["depth"]).max()
            print(f"update_step: ba.py vs the oracle's ba_cuda restatement: poses {dpose:.3g}, depths {ddep:.3g}")
            assert dpose < 1e-4 and ddep < 1e-4
    out["f64_corr"] = res["f64"]["corr"].astype(np.float32)   # exact corr rows (fp16 inputs, fp64 sums)
    for k in ("poses", "depth", "points", "net", "delta", "weight", "target"):
        a, b = res["r16"][k], res["f64"][k]
        if k == "poses":
            a, b = a[t0:n], b[t0:n]
        rel = np.abs(a - b) / (np.abs(b) + 1e-12)
        nrm = np.linalg.norm(a - b) / np.linalg.norm(b)
        extra = ""
        if k == "points":
            pp = np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)
            extra = f", per point max {pp.max():.3g}"
        print(f"update_step: reference fp16 path vs float64, {k}: max abs {np.abs(a - b).max():.3g}, "
              f"max rel (|x| > 1e-3) {rel[np.abs(b) > 1e-3].max():.3g}, norm-wise {nrm:.3g}{extra}")
        out[f"r16_err_{k}"] = _err_stats(a, b)
    moved = np.abs(res["f64"]["poses"][t0:n] - S["poses"][t0:n]).max()
    print(f"update_step: E = {E}, window poses moved by up to {moved:.3g}; fixture saved")
    if save:
        np.savez_compressed(os.path.join(HERE, C["file"]), **out)


if __name__ == "__main__":
    # python make_golden.py [part ...]: parts lietorch, pops, ba, altcorr, neighbors, update, encoder, step,
    # step_c2, step_c3 (not in the default set: ~10 / ~20 min of CPU)
    torch.set_num_threads(8)
    parts = set(sys.argv[1:]) or {"lietorch", "pops", "ba", "altcorr", "neighbors", "update", "encoder", "step"}
    pops, ba, lie = import_reference()
    if "lietorch" in parts:
        lietorch_fixtures(lie)
    if "pops" in parts:
        pops_fixtures(pops, lie)
    if "ba" in parts:
        ba_fixtures(ba, lie)
    if "altcorr" in parts:
        altcorr_fixtures()
    if "neighbors" in parts:
        neighbors_fixtures()
    if "update" in parts:
        update_fixtures()
    if "encoder" in parts:
        encoder_fixtures()
    if "step" in parts:
        update_step_fixtures(pops, ba, lie)
    if "step_c2" in parts:
        update_step_fixtures(pops, ba, lie, which="c2")
    if "step_c3" in parts:
        update_step_fixtures(pops, ba, lie, which="c3")
