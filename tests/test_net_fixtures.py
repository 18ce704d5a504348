"""The mirror's learned modules against fixtures produced by the REFERENCE's
own modules (tests/golden/make_golden.py: dpvo/net.py:28-93 ``Update`` and
dpvo/extractor.py:200-264 ``BasicEncoder4`` imported and run in float64).

CPU tests: the mirror modules (dpvo/net.py, dpvo/blocks.py, dpvo/extractor.py)
take the reference's state_dict layout unchanged and, in float64 on the CPU,
reproduce the reference outputs to rounding.  This pins the module structure
(layer order, LayerNorm eps, residual order, gating, SoftAgg) that the native
GPU path is built from; tests/test_gpu_net_fixtures.py then holds the native
path itself to the same fixtures.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import net_inputs as NI  # noqa: E402


def _fix(name):
    return np.load(os.path.join(GOLDEN, name))


def _spec(model):
    return [[k, list(v.shape)] for k, v in model.state_dict().items()]


def _load(model, spec, seed):
    params = NI.make_params(spec, seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
    return params


def _neighbors_cpu(kk, jj):
    """fastba.neighbors (ba.cpp:106-151) on the host: previous / next edge of
    the same patch in stable jj order, -1 at the ends (test stand-in for the
    device kernel, which tests/test_gpu_updateop.py checks separately)."""
    kk_n, jj_n = kk.numpy(), jj.numpy()
    order = np.lexsort((np.arange(len(kk_n)), jj_n, kk_n))
    ix = np.full(len(kk_n), -1, np.int64)
    jx = np.full(len(kk_n), -1, np.int64)
    same = kk_n[order[1:]] == kk_n[order[:-1]]
    ix[order[1:][same]] = order[:-1][same]
    jx[order[:-1][same]] = order[1:][same]
    return torch.from_numpy(ix), torch.from_numpy(jx)


def test_update_fixture_spec_and_inputs():
    """the mirror Update has the reference's state_dict layout (so dpvo.pth
    loads), and the seeded weights / inputs regenerate bit for bit"""
    from dpvo.net import Update
    f = _fix("update_ref.npz")
    spec = str(f["spec"])
    assert _spec(Update(3)) == json.loads(spec)
    params = NI.make_params(spec, int(f["seed"]))
    np.testing.assert_array_equal(np.stack([NI.checksum(params[k]) for k in sorted(params)]), f["param_checksum"])
    E = len(f["ii"])
    ii, jj, kk = NI.update_edges()
    assert np.array_equal(ii, f["ii"]) and np.array_equal(jj, f["jj"]) and np.array_equal(kk, f["kk"])
    np.testing.assert_array_equal(np.stack([NI.checksum(x) for x in NI.update_inputs(E)]), f["input_checksum"])
    # the edge set exercises what the operator's kernels special-case
    _, counts = np.unique(ii * 12345 + jj, return_counts=True)
    assert counts.max() >= 64 and counts.min() < 64          # long and short frame-pair groups
    assert int(f["n_ix_neg"]) > 0 and int(f["n_jx_neg"]) > 0  # -1 neighbours


def test_update_mirror_float64_matches_reference(monkeypatch):
    """Update.forward of the mirror (torch path, float64, CPU) == the
    reference module's float64 outputs"""
    from dpvo import fastba
    from dpvo.net import Update
    f = _fix("update_ref.npz")
    upd = Update(3)
    _load(upd, str(f["spec"]), int(f["seed"]))
    upd = upd.double()
    monkeypatch.setattr(fastba, "neighbors", _neighbors_cpu)
    ii, jj, kk = (torch.from_numpy(f[k]) for k in ("ii", "jj", "kk"))
    net, inp, corr = (torch.from_numpy(x).double()[None] for x in NI.update_inputs(len(ii)))
    # the torch path with autograd on (the inference path's SoftAgg is the HIP kernel)
    net.requires_grad_(True)
    out, (d, w, _) = upd(net, inp, corr, None, ii, jj, kk)
    rows = torch.from_numpy(f["rows"])
    np.testing.assert_allclose(out[0, rows].detach().numpy(), f["net_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(d[0].detach().numpy(), f["delta"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(w[0].detach().numpy(), f["weight"], rtol=1e-5, atol=1e-6)


def test_encoder_fixture_spec():
    from dpvo.extractor import BasicEncoder4
    f = _fix("encoder_ref.npz")
    assert _spec(BasicEncoder4(128, "instance")) == json.loads(str(f["fspec"]))
    assert _spec(BasicEncoder4(384, "none")) == json.loads(str(f["ispec"]))
    fp = NI.make_params(str(f["fspec"]), NI.ENCODER_SEED)
    ip = NI.make_params(str(f["ispec"]), NI.ENCODER_SEED + 1)
    np.testing.assert_array_equal(np.stack([NI.checksum(d[k]) for d in (fp, ip) for k in sorted(d)]),
                                  f["param_checksum"])


@pytest.mark.parametrize("frame", range(len(NI.ENCODER_FRAMES)))
def test_encoder_mirror_float64_matches_reference(frame):
    """fnet / inet of the mirror in float64 == the reference's (net.py:119-122
    input scaling and /4 output scale included)"""
    from dpvo.extractor import BasicEncoder4
    f = _fix("encoder_ref.npz")
    fnet, inet = BasicEncoder4(128, "instance"), BasicEncoder4(384, "none")
    _load(fnet, str(f["fspec"]), NI.ENCODER_SEED)
    _load(inet, str(f["ispec"]), NI.ENCODER_SEED + 1)
    H, W, kind = NI.ENCODER_FRAMES[frame]
    img = NI.encoder_image(H, W, kind)
    np.testing.assert_array_equal(NI.checksum(img), f[f"f{frame}_image_checksum"])
    x = 2 * (torch.from_numpy(img).double()[None, None] / 255.0) - 0.5
    with torch.no_grad():
        fmap = (fnet.double()(x) / 4.0)[0, 0].numpy()
        imap = (inet.double()(x) / 4.0)[0, 0].numpy()
    assert tuple(fmap.shape[-2:]) == tuple(f[f"f{frame}_hw"])
    np.testing.assert_allclose(fmap[:, f[f"f{frame}_rows"]], f[f"f{frame}_fmap"], rtol=1e-5, atol=1e-6)
    xs, ys = f[f"f{frame}_xs"], f[f"f{frame}_ys"]
    np.testing.assert_allclose(imap[:, ys, xs].T, f[f"f{frame}_imap"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("which", ["small", "c2", "c3"])
def test_update_step_inputs_regenerate(which):
    """update_step_ref.npz's (M = 12), update_step_c2_ref.npz's (C2's
    per-update size, M = 96, 8 BA iterations) and update_step_c3_ref.npz's
    (C3's, M = 192, 2 BA iterations) inputs come back bit for bit
    from their seed (the GPU test regenerates them instead of loading the
    state), and each fixture's edge set is the steady state the tracker sees
    (497 M edges)"""
    C = NI.STEPS[which]
    f = np.load(os.path.join(GOLDEN, C["file"]))
    S = NI.update_step_state(int(f["seed"]), C)
    got = np.stack([NI.checksum(S[k]) for k in sorted(S)])
    np.testing.assert_allclose(got, f["state_checksum"], rtol=1e-12, atol=0)
    assert len(S["ii"]) == 497 * C["M"]
    assert np.array_equal(f["touched"], np.unique(S["kk"]))
    assert int(f["iters"] if "iters" in f else 2) == C["iters"]


@pytest.mark.parametrize("which", ["small", "c2", "c3"])
def test_update_step_oracle_chain_matches_reference(monkeypatch, which):
    """the CPU restatement of the whole update() -- oracle.transform, the
    oracle's exact altcorr (F16_ACC64), the mirror Update in float64, the
    oracle's ba_cuda.cu restatement, the oracle's point cloud -- reproduces the
    reference modules' float64 update_step fixture: the oracle chain the GPU
    kernels are tested against is itself pinned end to end."""
    from oracle import oracle
    from dpvo import fastba
    from dpvo.net import Update
    C = NI.STEPS[which]
    f = np.load(os.path.join(GOLDEN, C["file"]))
    S = NI.update_step_state(int(f["seed"]), C)
    n, M, pmem, t0 = C["n"], C["M"], C["pmem"], int(f["t0"])
    m = n * M
    ii, jj, kk = S["ii"], S["jj"], S["kk"]
    E = len(ii)
    coords = oracle.transform(S["poses"], S["patches"], S["intrinsics"], ii, jj, kk)[0].transpose(0, 3, 1, 2)
    corr = oracle.corr_pyramid(S["gmap"].reshape(1, pmem * M, 128, 3, 3), [S["fmap1"][None], S["fmap2"][None]],
                               coords[None], kk % (M * pmem), jj % pmem, mode=oracle.F16_ACC64)[0]
    # (oracle.transform computes the coordinates in fp32, the reference run in
    # fp64: ~1e-5 px at the C2 fixture's 128-px maps, which the bilinear step
    # turns into up to ~2e-5 of the row values)
    sc = 1.0 if which == "small" else 4.0   # (the absolute floors below scale with it)
    np.testing.assert_allclose(corr[f["corr_rows"]], f["f64_corr"], rtol=1e-5, atol=1e-5 * sc)
    upd = Update(3)
    _load(upd, str(f["spec"]), int(f["update_seed"]))
    with torch.no_grad():
        upd.d[1].weight.mul_(float(f["dscale"]))
        upd.d[1].bias.mul_(float(f["dscale"]))
    upd = upd.double()
    monkeypatch.setattr(fastba, "neighbors", _neighbors_cpu)
    ctx = S["imap"].reshape(pmem * M, 384)[kk % (M * pmem)]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    # the torch path with autograd on (the inference path's SoftAgg is the HIP kernel)
    net0 = T(S["net"]).double()[None].requires_grad_(True)
    net, (d, w, _) = upd(net0, T(ctx).double()[None], T(corr).double()[None], None, T(ii), T(jj), T(kk))
    net, d, w = net.detach(), d.detach(), w.detach()
    np.testing.assert_allclose(net[0].numpy()[f["rows"]], f["f64_net"], rtol=1e-5, atol=1e-5 * sc)
    target = coords[:, :, 1, 1] + d[0].numpy()
    np.testing.assert_allclose(target, f["f64_target"], rtol=1e-5, atol=1e-5 * sc)
    np.testing.assert_allclose(w[0].numpy(), f["f64_weight"], rtol=1e-5, atol=1e-6 * sc)
    poses, patches, st = oracle.ba_forward(S["poses"], S["patches"], S["intrinsics"], target, w[0].numpy(), 1e-4,
                                           ii, jj, kk, t0, n, C["iters"])
    assert st == 0
    np.testing.assert_allclose(poses[t0:n], f["f64_poses"][t0:n], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(patches[f["touched"], 2, 1, 1], f["f64_depth"], rtol=1e-4)
    pts = oracle.point_cloud_centre(poses, patches[:m], S["intrinsics"], np.arange(m) // M)
    np.testing.assert_allclose(pts, f["f64_points"], rtol=1e-4, atol=1e-5)
