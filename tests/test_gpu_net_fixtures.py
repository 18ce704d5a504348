"""The native update operator and the native encoders against fixtures made
by the REFERENCE's own modules (tests/golden/make_golden.py runs
dpvo/net.py:28-93 ``Update`` and dpvo/extractor.py:200-264 ``BasicEncoder4``
in float64 on seeded weights and inputs; tests/test_net_fixtures.py shows
the mirror modules reproduce them on the CPU).

Bars:
* update operator, fused fp16 path (csrc/rowgemm.hip + updateop.hip, what
  DPVO.update runs): per output, RMS error against float64 <= 1.5x and max
  error <= 3x the error of the reference module's own fp16-autocast run
  (recorded in the fixture), plus absolute caps;
* update operator, torch path in fp32 on the GPU: rtol 2e-4;
* encoders (csrc/encoder.hip): RMS <= 1.25x and max <= 2x the error of the
  same modules' torch/MIOpen fp16-autocast evaluation, both against the
  reference's float64 outputs.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import net_inputs as NI  # noqa: E402

pytestmark = pytest.mark.gpu


def _fix(name):
    return np.load(os.path.join(GOLDEN, name))


def _load(model, spec, seed):
    params = NI.make_params(spec, seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)


def _update_case():
    from dpvo.net import Update
    f = _fix("update_ref.npz")
    upd = Update(3)
    _load(upd, str(f["spec"]), int(f["seed"]))
    upd = upd.cuda().eval()
    ii, jj, kk = (torch.from_numpy(f[k]).cuda() for k in ("ii", "jj", "kk"))
    net, inp, corr = NI.update_inputs(len(f["ii"]))
    return f, upd, ii, jj, kk, torch.from_numpy(net).cuda()[None], torch.from_numpy(inp).cuda()[None], \
        torch.from_numpy(corr).cuda()[None]


def _err(a, ref):
    d = np.asarray(a, np.float64) - np.asarray(ref, np.float64)
    return np.sqrt((d ** 2).mean()), np.abs(d).max()


def _check_update(f, out, d, w, label):
    rows = f["rows"]
    got = {"net": out[0].float().cpu().numpy()[rows], "delta": d[0].float().cpu().numpy(),
           "weight": w[0].float().cpu().numpy()}
    ref = {"net": f["net_out"], "delta": f["delta"], "weight": f["weight"]}
    caps = {"net": 2e-2, "delta": 1e-2, "weight": 3e-3}     # absolute max-error caps
    for k in got:
        rms, mx = _err(got[k], ref[k])
        arms, amx = f[f"amp_err_{k}"]
        print(f"{label} {k}: rms {rms:.3g} max {mx:.3g} (reference fp16 autocast: rms {arms:.3g} max {amx:.3g})")
        assert rms <= 1.5 * arms, (label, k, rms, arms)
        assert mx <= 3.0 * amx and mx <= caps[k], (label, k, mx, amx)


def test_update_fused_matches_reference_module():
    """Update.forward under fp16 autocast -> the fused native path"""
    f, upd, ii, jj, kk, net, inp, corr = _update_case()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        assert upd._fusable(net, inp, corr)
        out, (d, w, _) = upd(net, inp, corr, None, ii, jj, kk)
    torch.cuda.synchronize()
    assert out.dtype == torch.float32 and d.dtype == torch.float16
    _check_update(f, out, d, w, "fused")


def test_update_fused_tracker_call_matches_reference_module():
    """the tracker's call form (dpvo.py:718-720 as DPVO.update makes it): the
    context passed as a ring + row index, key bounds and the kk group-by given"""
    import update_ops
    f, upd, ii, jj, kk, net, inp, corr = _update_case()
    E = ii.numel()
    g = torch.Generator().manual_seed(3)
    perm = torch.randperm(E, generator=g).cuda()
    ring = torch.empty_like(inp[0])
    ring[perm] = inp[0]                      # ring[perm[e]] = inp[e]
    N = int(max(ii.max(), jj.max())) + 1
    M = int(kk.max()) + 1
    kk_groups = update_ops.group_by(kk, key_bits=update_ops.key_bits_for(M))
    c = torch.zeros(E, 896, dtype=torch.float16, device="cuda")
    c[:, :882] = corr[0]
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        out, (d, w, _) = upd(net, ring[None], c[:, :882][None], None, ii, jj, kk, inp_idx=perm,
                             index_bounds=(M, N), kk_groups=kk_groups)
    torch.cuda.synchronize()
    _check_update(f, out, d, w, "tracker-call")


def test_update_torch_fp32_matches_reference_module():
    """the mirror's torch composition in fp32 on the GPU (native neighbours and
    SoftAgg kernels inside) against the reference float64 outputs"""
    f, upd, ii, jj, kk, net, inp, corr = _update_case()
    with torch.no_grad():
        out, (d, w, _) = upd(net, inp.float(), corr.float(), None, ii, jj, kk)
    rows = torch.from_numpy(f["rows"]).cuda()
    np.testing.assert_allclose(out[0, rows].cpu().numpy(), f["net_out"], rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(d[0].cpu().numpy(), f["delta"], rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(w[0].cpu().numpy(), f["weight"], rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("frame", range(len(NI.ENCODER_FRAMES)))
def test_native_encoders_match_reference_modules(frame):
    import encoder_ops
    from dpvo.extractor import BasicEncoder4
    f = _fix("encoder_ref.npz")
    fnet, inet = BasicEncoder4(128, "instance"), BasicEncoder4(384, "none")
    _load(fnet, str(f["fspec"]), NI.ENCODER_SEED)
    _load(inet, str(f["ispec"]), NI.ENCODER_SEED + 1)
    fnet, inet = fnet.cuda().eval(), inet.cuda().eval()
    H, W, kind = NI.ENCODER_FRAMES[frame]
    img = torch.from_numpy(NI.encoder_image(H, W, kind)).cuda()
    rows = torch.from_numpy(f[f"f{frame}_rows"])
    xs, ys = torch.from_numpy(f[f"f{frame}_xs"]), torch.from_numpy(f[f"f{frame}_ys"])
    with torch.no_grad():
        fmap, imap = encoder_ops.NativeEncoders(fnet, inet).run(img, xs.cuda(), ys.cuda())
        with torch.autocast("cuda", dtype=torch.float16):
            x = 2 * (img[None, None] / 255.0) - 0.5
            fm16, im16 = fnet(x) / 4.0, inet(x) / 4.0
    torch.cuda.synchronize()
    h, w = (int(v) for v in f[f"f{frame}_hw"])
    assert fmap.shape == (1, 1, 128, h, w) and imap.shape == (len(xs), 384)
    nat_f = fmap[0, 0].double().cpu()[:, rows].numpy()
    ref_f = fm16[0, 0].double().cpu()[:, rows].numpy()
    nat_i = imap.double().cpu().numpy()
    ref_i = im16[0, 0].double().cpu()[:, ys, xs].T.numpy()
    for name, nat, r16, gold in (("fmap", nat_f, ref_f, f[f"f{frame}_fmap"]),
                                 ("imap", nat_i, ref_i, f[f"f{frame}_imap"])):
        en, er = _err(nat, gold), _err(r16, gold)
        print(f"{H}x{W} {name}: native rms/max {en[0]:.3g}/{en[1]:.3g}, torch fp16 {er[0]:.3g}/{er[1]:.3g}")
        assert np.isfinite(nat).all()
        assert en[0] <= 1.25 * er[0] + 1e-5, (name, en, er)
        assert en[1] <= 2.0 * er[1] + 1e-4, (name, en, er)
