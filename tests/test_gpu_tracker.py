"""The DPVO tracker (dpvo/dpvo.py mirror) on the GPU: the hot-path pieces of
one update against the oracle, and the full frame-by-frame API."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def slam():
    from dpvo.synthetic import steady_state_tracker
    return steady_state_tracker("dpvo_2k", buffer=72, seed=0)


def test_steady_state_shapes(slam):
    n, M = slam.n, slam.M
    assert n == 64 and M == 192
    assert slam.pg.ii.numel() == 497 * M
    assert torch.unique(slam.pg.kk).numel() == 23 * M


def test_update_pieces_match_oracle(slam):
    """reproject -> corr (bit-exact on an edge sample) -> BA -> point cloud."""
    from dpvo import fastba
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    with torch.no_grad():
        coords = slam.reproject()
        poses = slam.pg.poses_.cpu().numpy()
        patches = slam.pg.patches_.view(-1, 3, 3, 3).cpu().numpy()
        intr = slam.pg.intrinsics_.cpu().numpy()
        ii, jj, kk = (t.cpu().numpy() for t in (slam.pg.ii, slam.pg.jj, slam.pg.kk))
        ref = oracle.transform(poses, patches, intr, ii, jj, kk)[0].transpose(0, 3, 1, 2)
        np.testing.assert_allclose(coords[0].cpu().numpy(), ref, rtol=1e-5, atol=5e-3)

        slam.cfg.EXACT_CORR = True   # the bit-exact fp16-chain kernel (the MFMA default: test_gpu_corr_mfma.py)
        corr = slam.corr(coords)
        slam.cfg.EXACT_CORR = False
        sel = np.linspace(0, len(ii) - 1, 300).astype(np.int64)
        c_np = coords[0].cpu().numpy()[sel][None]
        want = oracle.corr_pyramid(slam.gmap.cpu().numpy(), [slam.fmap1_.contiguous().cpu().numpy(),
                                                              slam.fmap2_.contiguous().cpu().numpy()],
                                   c_np, kk[sel] % (slam.M * slam.pmem), jj[sel] % slam.pmem)
        assert np.array_equal(corr[0].cpu().numpy()[sel].view(np.uint16), want[0].view(np.uint16))

        g = torch.Generator(device=slam.device).manual_seed(5)
        target = coords[..., 1, 1] + torch.randn(1, len(ii), 2, generator=g, device=slam.device)
        weight = torch.rand(1, len(ii), 2, generator=g, device=slam.device)
        t0, t1 = slam.n - 10, slam.n
        rp, rq, st = oracle.ba_forward(poses, patches, intr, target.cpu().numpy(), weight.cpu().numpy(), 1e-4,
                                       ii, jj, kk, t0, t1, 2)
        assert st == 0
        fastba.BA(slam.poses, slam.patches, slam.intrinsics, target, weight, slam._lmbda, slam.pg.ii, slam.pg.jj,
                  slam.pg.kk, t0, t1, 2)
        gp = slam.pg.poses_.cpu().numpy()
        gq = slam.pg.patches_.view(-1, 3, 3, 3).cpu().numpy()
        # per element on what BA moved (the window poses, the touched depths)
        err = np.abs(gp[t0:t1] - rp[t0:t1])
        assert np.all(err <= 1e-3 * np.abs(rp[t0:t1]) + 1e-5), err.max()
        touched = np.unique(kk)
        err = np.abs(gq[touched, 2] - rq[touched, 2])
        assert np.all(err <= 1e-3 * np.abs(rq[touched, 2]) + 1e-5), err.max()
        assert np.array_equal(gp[:t0], poses[:t0])

        m = slam.pg.m
        pc = pops.point_cloud_centre(SE3(slam.poses), slam.patches[:, :m], slam.intrinsics, slam.ix[:m])
        want = oracle.point_cloud_centre(gp, gq[:m], intr, slam.ix[:m].cpu().numpy())
        np.testing.assert_allclose(pc.cpu().numpy(), want, rtol=1e-4, atol=1e-4)


def test_update_runs_and_moves_the_window(slam):
    with torch.no_grad():
        p0 = slam.pg.poses_.clone()
        d0 = slam.pg.patches_[..., 2, 1, 1].clone()
        for _ in range(3):
            slam.update()
        torch.cuda.synchronize()
    moved = (slam.pg.poses_ - p0).abs().amax(dim=1)
    assert moved[: slam.n - 10].max() == 0          # outside the optimisation window: fixed
    assert moved[slam.n - 10: slam.n].max() > 0     # inside: optimised
    assert torch.isfinite(slam.pg.points_[: slam.pg.m]).all()
    assert (slam.pg.patches_[..., 2, 1, 1] != d0).any()


def test_frame_by_frame_api():
    """__call__ -> init (12 updates) -> update + keyframe per frame -> terminate."""
    from dpvo.config import make_cfg
    from dpvo.dpvo import DPVO
    from dpvo.net import VONet
    from dpvo.synthetic import image_stream
    torch.manual_seed(0)
    net = VONet()
    with torch.no_grad():
        net.update.d[1].weight.mul_(40.0)  # random weights: make the motion probe pass
    cfg = make_cfg("fast", BUFFER_SIZE=64)
    intr = torch.tensor([320.0, 320.0, 320.0, 240.0], device="cuda")
    with torch.no_grad():
        slam = DPVO(cfg, net, ht=384, wd=512)
        for t, img in image_stream(24):
            slam(t, img, None, None, intr)
        assert slam.is_initialized
        poses, tstamps = slam.terminate()
    assert poses.shape == (24, 7) and np.isfinite(poses).all()
    assert len(tstamps) == 24


def _reference_keyframe(slam):
    """The reference's keyframe() (dpvo.py:605-658) written out loop by loop:
    boolean-mask edge removal and the per-frame buffer shift."""
    from dpvo.lietorch import SE3
    k = slam.n - slam.cfg.KEYFRAME_INDEX
    i, j = k - 1, k + 1
    m = slam.motionmag(i, j) + slam.motionmag(j, i)
    if m / 2 < slam.cfg.KEYFRAME_THRESH:
        t0, t1 = int(slam.pg.tstamps_[k - 1]), int(slam.pg.tstamps_[k])
        slam.pg.delta[t1] = (t0, SE3(slam.pg.poses_[k]) * SE3(slam.pg.poses_[k - 1]).inv())
        keep = ~((slam.pg.ii == k) | (slam.pg.jj == k))
        slam.pg.weight, slam.pg.target = slam.pg.weight[:, keep], slam.pg.target[:, keep]
        slam.pg.ii, slam.pg.jj, slam.pg.kk = slam.pg.ii[keep], slam.pg.jj[keep], slam.pg.kk[keep]
        slam.pg.net = slam.pg.net[:, keep]
        slam.pg.kk[slam.pg.ii > k] -= slam.M
        slam.pg.ii[slam.pg.ii > k] -= 1
        slam.pg.jj[slam.pg.jj > k] -= 1
        for f in range(k, slam.n - 1):
            g = f + 1
            slam.pg.tstamps_[f] = slam.pg.tstamps_[g]
            for buf in (slam.pg.colors_, slam.pg.poses_, slam.pg.patches_, slam.pg.patches_est_, slam.pg.intrinsics_):
                buf[f] = buf[g]
            slam.imap_[f % slam.pmem] = slam.imap_[g % slam.pmem]
            slam.gmap_[f % slam.pmem] = slam.gmap_[g % slam.pmem]
            slam.fmap1_[0, f % slam.pmem] = slam.fmap1_[0, g % slam.pmem]
            slam.fmap2_[0, f % slam.pmem] = slam.fmap2_[0, g % slam.pmem]
            slam.image_buffer_[f % slam.mem] = slam.image_buffer_[g % slam.mem]
        slam.n -= 1
        slam.pg.m -= slam.M
    old = slam.ix[slam.pg.kk] < slam.n - slam.cfg.REMOVAL_WINDOW
    keep = ~old
    slam.pg.ii_inac = torch.cat((slam.pg.ii_inac, slam.pg.ii[old]))
    slam.pg.jj_inac = torch.cat((slam.pg.jj_inac, slam.pg.jj[old]))
    slam.pg.kk_inac = torch.cat((slam.pg.kk_inac, slam.pg.kk[old]))
    slam.pg.weight_inac = torch.cat((slam.pg.weight_inac, slam.pg.weight[:, old]), dim=1)
    slam.pg.target_inac = torch.cat((slam.pg.target_inac, slam.pg.target[:, old]), dim=1)
    slam.pg.weight, slam.pg.target = slam.pg.weight[:, keep], slam.pg.target[:, keep]
    slam.pg.ii, slam.pg.jj, slam.pg.kk = slam.pg.ii[keep], slam.pg.jj[keep], slam.pg.kk[keep]
    slam.pg.net = slam.pg.net[:, keep]


@pytest.mark.parametrize("drop", [True, False])
def test_keyframe_matches_reference_loop(drop):
    """keyframe() with index-based compaction and gathered buffer shifts ==
    the reference's mask-and-loop version, buffer for buffer."""
    from dpvo.synthetic import steady_state_tracker
    with torch.no_grad():
        a = steady_state_tracker("fast", buffer=96, n=70, seed=4)
        b = steady_state_tracker("fast", buffer=96, n=70, seed=4)
        w, t = torch.rand_like(a.pg.weight), torch.rand_like(a.pg.target)
        for s in (a, b):
            s.cfg.KEYFRAME_THRESH = 1e9 if drop else -1.0
            s.pg.weight, s.pg.target = w.clone(), t.clone()
        a.keyframe()
        _reference_keyframe(b)
    assert a.n == b.n and a.pg.m == b.pg.m
    for name in ("ii", "jj", "kk", "net", "weight", "target", "ii_inac", "jj_inac", "kk_inac", "weight_inac",
                 "target_inac"):
        assert torch.equal(getattr(a.pg, name), getattr(b.pg, name)), name
    for name in ("poses_", "patches_", "intrinsics_", "colors_", "patches_est_"):
        assert torch.equal(getattr(a.pg, name), getattr(b.pg, name)), name
    assert np.array_equal(a.pg.tstamps_, b.pg.tstamps_)
    for name in ("imap_", "gmap_", "fmap1_", "fmap2_", "image_buffer_"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert a.pg.delta.keys() == b.pg.delta.keys()
    # the next update() reads the shifted rings (the packed gmap table is
    # rebuilt after the native shift, as after the reference's index writes)
    with torch.no_grad():
        a.update()
        b.update()
    for name in ("poses_", "patches_"):
        assert torch.equal(getattr(a.pg, name), getattr(b.pg, name)), name
    assert torch.equal(a.pg.net, b.pg.net)


def test_keyframe_raises_on_nan_pose_when_kept():
    """The keep path raises on a NaN pose at the keyframe index (dpvo.py:647),
    read with the motion magnitudes; the drop path removes that frame instead."""
    from dpvo.synthetic import steady_state_tracker
    with torch.no_grad():
        for drop in (False, True):
            s = steady_state_tracker("fast", buffer=96, n=70, seed=4)
            s.cfg.KEYFRAME_THRESH = 1e9 if drop else -1.0
            k = s.n - s.cfg.KEYFRAME_INDEX
            s.pg.poses_[k, 2] = float("nan")
            if drop:
                n0 = s.n
                s.keyframe()
                assert s.n == n0 - 1
            else:
                with pytest.raises(Exception, match="nan"):
                    s.keyframe()


@pytest.mark.parametrize("native", [True, False])
def test_graphed_ingest_matches_eager(native):
    """Patchifier.forward replayed from its captured HIP graph gives the eager
    launches' results bit for bit (same seed -> same patch centres), and each
    call returns fresh tensors (the next replay does not overwrite them);
    native = the HIP encoders, else the torch modules."""
    from dpvo.net import Patchifier
    from dpvo.synthetic import image_stream
    torch.manual_seed(0)
    pf = Patchifier(3).cuda().eval()
    pf.NATIVE_ENCODERS = native
    imgs = [img for _, img in image_stream(3)]
    with torch.no_grad(), torch.autocast("cuda", enabled=True):
        eager = []
        pf.graphed = False
        torch.manual_seed(7)
        for img in imgs:
            eager.append(pf(img, patches_per_image=96, return_color=True))
        pf.graphed = True
        torch.manual_seed(7)
        graphed = [pf(img, patches_per_image=96, return_color=True) for img in imgs]
    assert pf._graph is not None
    for e, g in zip(eager, graphed):
        for a, b in zip(e, g):
            assert a.shape == b.shape and a.dtype == b.dtype
            assert torch.equal(a, b)
    assert not torch.equal(graphed[0][3], graphed[1][3])  # fresh centres, not aliased outputs


@pytest.mark.parametrize("native", [True, False])
def test_graphed_ingest_recaptures_after_reassign(native):
    """The captured ingest graph holds raw parameter addresses: re-placing the
    parameters (load_state_dict(assign=True) with fresh storage, then
    scaling them) must re-capture, not replay reads of freed memory."""
    from dpvo.net import Patchifier
    from dpvo.synthetic import image_stream
    torch.manual_seed(0)
    pf = Patchifier(3).cuda().eval()
    pf.NATIVE_ENCODERS = native
    img = next(iter(image_stream(1)))[1]
    with torch.no_grad(), torch.autocast("cuda", enabled=True):
        pf.graphed = True
        pf(img, patches_per_image=64)
        g0 = pf._graph
        fresh = {k: (v.clone() * 1.5 if v.is_floating_point() else v.clone()) for k, v in pf.state_dict().items()}
        pf.load_state_dict(fresh, assign=True)
        torch.manual_seed(3)
        got = pf(img, patches_per_image=64)
        assert pf._graph is not g0
        pf.graphed = False
        torch.manual_seed(3)
        want = pf(img, patches_per_image=64)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_motion_mag_matches_oracle(slam):
    """DPVO.motionmag (dpvo.py:507-514) as one native launch for both
    directions == the oracle's transform-based flow_mag (projective_ops.py:
    111-121) averaged over the matching edges; NaN without edges."""
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    poses = slam.pg.poses_.cpu().numpy()
    patches = slam.pg.patches_.view(-1, 3, 3, 3).cpu().numpy()
    intr = slam.pg.intrinsics_.cpu().numpy()
    ii, jj, kk = (t.cpu().numpy() for t in (slam.pg.ii, slam.pg.jj, slam.pg.kk))

    def ref(i, j, beta=0.5):
        s = (ii == i) & (jj == j)
        if not s.any():
            return float("nan")
        c0 = oracle.transform(poses, patches, intr, ii[s], ii[s], kk[s])
        c1 = oracle.transform(poses, patches, intr, ii[s], jj[s], kk[s])
        c2 = oracle.transform(poses, patches, intr, ii[s], jj[s], kk[s], tonly=True)
        f = beta * np.linalg.norm(c1 - c0, axis=-1) + (1 - beta) * np.linalg.norm(c2 - c0, axis=-1)
        return float(f.mean())

    n = slam.n
    with torch.no_grad():
        for i, j in ((n - 5, n - 3), (n - 2, n - 1), (n - 12, n - 1), (0, n - 1)):
            got = pops.motion_mag_pair(SE3(slam.poses), slam.patches, slam.intrinsics, slam.pg.ii, slam.pg.jj,
                                       slam.pg.kk, i, j).tolist()
            for g, w in zip(got, (ref(i, j), ref(j, i))):
                if np.isnan(w):
                    assert np.isnan(g)
                else:
                    assert abs(g - w) <= 1e-4 * max(1.0, abs(w)), (i, j, g, w)
        # the tracker's single-direction accessor agrees with the pair
        assert abs(slam.motionmag(n - 5, n - 3) - ref(n - 5, n - 3)) <= 1e-4 * max(1.0, ref(n - 5, n - 3))


class _RefEdges:
    """The reference's edge bookkeeping written out with Python lists:
    __edges_forw / __edges_back appended per frame (dpvo.py:756-769, 860-861),
    keyframe()'s removal and renumbering (:605-640) and the removal window
    (:657).  Independent of the tracker's tensor code."""

    def __init__(self, cfg):
        self.M, self.r = cfg.PATCHES_PER_FRAME, cfg.PATCH_LIFETIME
        self.win, self.kfi = cfg.REMOVAL_WINDOW, cfg.KEYFRAME_INDEX
        self.n = 0
        self.ii, self.jj, self.kk = [], [], []

    def add_frame(self):
        self.n += 1
        n, M, r = self.n, self.M, self.r
        for k in range(M * max(n - r, 0), M * max(n - 1, 0)):       # forward: old patches -> new frame
            self.kk.append(k); self.jj.append(n - 1); self.ii.append(k // M)
        for k in range(M * max(n - 1, 0), M * n):                    # backward: new patches -> recent frames
            for j in range(max(n - r, 0), n):
                self.kk.append(k); self.jj.append(j); self.ii.append(k // M)

    def keyframe(self, drop):
        k = self.n - self.kfi
        e = list(zip(self.ii, self.jj, self.kk))
        if drop:
            e = [(i, j, kk) for i, j, kk in e if i != k and j != k]
            e = [(i - 1 if i > k else i, j - 1 if j > k else j, kk - self.M if i > k else kk) for i, j, kk in e]
            self.n -= 1
        e = [(i, j, kk) for i, j, kk in e if kk // self.M >= self.n - self.win]
        self.ii, self.jj, self.kk = (list(t) for t in zip(*e)) if e else ([], [], [])


def test_edge_construction_follows_reference_rules():
    """Row a9: the tracker's (ii, jj, kk) after every frame equals the
    reference's rules applied to the same frame / keyframe decisions; the
    keyframe threshold alternates so both the drop and the keep path run."""
    from dpvo.config import make_cfg
    from dpvo.dpvo import DPVO
    from dpvo.net import VONet
    from dpvo.synthetic import image_stream
    torch.manual_seed(0)
    net = VONet()
    with torch.no_grad():
        net.update.d[1].weight.mul_(40.0)  # random weights: make the motion probe pass
    cfg = make_cfg("fast", BUFFER_SIZE=64)
    intr = torch.tensor([320.0, 320.0, 320.0, 240.0], device="cuda")
    ref = _RefEdges(cfg)
    decisions = []
    with torch.no_grad():
        slam = DPVO(cfg, net, ht=384, wd=512)
        orig_kf = slam.keyframe

        def keyframe():
            drop = len(decisions) % 2 == 0
            slam.cfg.KEYFRAME_THRESH = float("inf") if drop else -1.0
            decisions.append(drop)
            orig_kf()
        slam.keyframe = keyframe
        for t, img in image_stream(26):
            n0, init0, nd = slam.n, slam.is_initialized, len(decisions)
            slam(t, img, None, None, intr)
            if not init0 and slam.n == n0:
                continue                       # skipped by the motion probe: no frame, no edges
            ref.add_frame()
            if len(decisions) > nd:
                ref.keyframe(decisions[-1])
            assert slam.n == ref.n
            assert slam.pg.ii.tolist() == ref.ii, t
            assert slam.pg.jj.tolist() == ref.jj, t
            assert slam.pg.kk.tolist() == ref.kk, t
    assert True in decisions and False in decisions


def test_deferred_keyframe_equals_immediate():
    """cfg.DEFER_KEYFRAME: the decision applied by the next __call__ (after its
    encoders are enqueued) leaves the same state as the immediate keyframe():
    edges, poses, patches and the trajectory from terminate() bit-identical,
    on a stream that both keeps and drops frames."""
    from dpvo.config import make_cfg
    from dpvo.dpvo import DPVO
    from dpvo.net import VONet
    from dpvo.synthetic import image_stream
    intr = torch.tensor([320.0, 320.0, 320.0, 240.0], device="cuda")
    frames = list(image_stream(24))
    out = []
    for defer in (False, True):
        torch.manual_seed(0)
        net = VONet()
        with torch.no_grad():
            net.update.d[1].weight.mul_(40.0)  # random weights: make the motion probe pass
        cfg = make_cfg("fast", BUFFER_SIZE=64, DEFER_KEYFRAME=defer)
        calls = [0]
        with torch.no_grad():
            slam = DPVO(cfg, net, ht=384, wd=512)
            orig_kf = slam.keyframe

            def keyframe():
                slam.cfg.KEYFRAME_THRESH = float("inf") if calls[0] % 3 == 0 else -1.0
                calls[0] += 1
                orig_kf()
            slam.keyframe = keyframe
            torch.manual_seed(1)
            for t, img in frames:
                slam(t, img, None, None, intr)
            if defer:
                assert slam._kf_pending is not None
            slam.flush_keyframe()
            state = [x.clone() for x in (slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.pg.poses_, slam.pg.patches_,
                                         slam.pg.net)]
            poses, tstamps = slam.terminate()
        out.append((state, poses, tstamps, getattr(slam, "keyframes_dropped", 0), calls[0]))
    (s0, p0, t0, d0, c0), (s1, p1, t1, d1, c1) = out
    assert c0 == c1 and d0 == d1 and 0 < d0 < c0
    for a, b in zip(s0, s1):
        assert a.shape == b.shape and torch.equal(a, b)
    assert np.array_equal(p0, p1) and np.array_equal(t0, t1)


@pytest.mark.parametrize("preset,buffer,n", [("fast", 96, 70), ("dpvo_2k", 2048, 2040)])
def test_window_ij_groups_equal_the_operator_key(preset, buffer, n):
    """DPVO._ij_groups (12-bit window key, counting sort) == the update
    operator's own group_by(ii * 12345 + jj) (net.py:88), and _kk_groups
    (window-relative kk) == group_by(kk): same gid, CSR and group count, so
    SoftAgg, the neighbours and BA's per-patch reduction are bit-identical."""
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    with torch.no_grad():
        s = steady_state_tracker(preset, buffer=buffer, n=n, seed=3)
        got = s._ij_groups()
        key = s.pg.ii * 12345 + s.pg.jj
        want = update_ops.group_by(key, key_bits=update_ops.key_bits_for(s.N * 12345 + 12345))
        got_kk = s._kk_groups()
        want_kk = update_ops.group_by(s.pg.kk, key_bits=update_ops.key_bits_for(s.N * s.M))
        # the one-launch keys update() uses == the torch compositions
        b, ring = s.n - 64, s.M * s.pmem
        kk_key, ij_key, ctx, jslot = update_ops.window_keys(s.pg.ii, s.pg.jj, s.pg.kk, s.M, b, ring, s.pmem)
        assert torch.equal(kk_key, s.pg.kk - s.M * b)
        assert torch.equal(ij_key, (s.pg.ii - b) * 64 + (s.pg.jj - b))
        assert torch.equal(ctx, s.pg.kk % ring)
        assert torch.equal(jslot, s.pg.jj % s.pmem)
    assert got is not None
    for g, w in ((got, want), (got_kk, want_kk)):
        G = int(w[3].item())
        assert torch.equal(g[3], w[3]) and torch.equal(g[0], w[0]) and torch.equal(g[2], w[2])
        assert torch.equal(g[1][:G + 1], w[1][:G + 1])   # offs past the group count is scratch


def test_window_keys_flag_out_of_window_edges():
    """An edge outside the 64-frame key window sets the deferred failure word
    (-2, first failure kept), which check_ba() turns into an error; in-window
    edges leave it alone."""
    import cuda_ba
    import update_ops
    n, M = 100, 8
    ii = torch.tensor([n - 1, n - 5, n - 40], device="cuda")
    jj = torch.tensor([n - 2, n - 1, n - 50], device="cuda")
    kk = ii * M + 3
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    update_ops.window_keys(ii, jj, kk, M, n - 64, M * 36, 36, flag=flag)
    assert int(flag.item()) == 0
    jj[2] = n - 70   # outside [n - 64, n)
    update_ops.window_keys(ii, jj, kk, M, n - 64, M * 36, 36, flag=flag)
    assert int(flag.item()) == -2
    flag.fill_(7)    # an earlier failure is kept
    update_ops.window_keys(ii, jj, kk, M, n - 64, M * 36, 36, flag=flag)
    assert int(flag.item()) == 7
    with pytest.raises(RuntimeError, match="key window"):
        cuda_ba.raise_for_status(-2)


def test_keyframe_masks_and_frame_shift_edges():
    """dpvo_keyframe_masks against the torch expressions it replaces (masks,
    shifted indices, counts, NaN flag), and dpvo_frame_shift against the
    sequential per-frame move on rings that wrap, odd slot sizes included."""
    from dpvo import projective_ops as pops
    g = torch.Generator().manual_seed(3)
    E, M, n, RW, k = 5000, 8, 40, 6, 36
    ix = torch.arange(n + 4, device="cuda").repeat_interleave(M)
    ii = torch.randint(n - 20, n, (E,), generator=g).cuda()
    kk = ii * M + torch.randint(0, M, (E,), generator=g).cuda()
    jj = torch.randint(n - 20, n, (E,), generator=g).cuda()
    mm = torch.tensor([0.25, float("nan")], device="cuda")
    fail = torch.tensor([-3], dtype=torch.int32, device="cuda")
    pose = torch.tensor([0, 0, float("nan"), 0, 0, 0, 1], device="cuda")
    masks, idx, vals = pops.keyframe_masks(ii, jj, kk, ix, k, M, n, RW, mm, fail, pose)
    old_keep = ix[kk] < n - RW
    drop = (ii == k) | (jj == k)
    later = ii > k
    kk_d = torch.where(later, kk - M, kk)
    old_d = (ix[kk_d] < n - 1 - RW) & ~drop
    rm_d = old_d | drop
    assert torch.equal(masks, torch.stack([old_keep, old_d, rm_d]))
    assert torch.equal(idx, torch.stack([torch.where(later, ii - 1, ii), torch.where(jj > k, jj - 1, jj), kk_d]))
    v = vals.cpu().tolist()
    assert v[0] == 0.25 and np.isnan(v[1]) and v[2] == -3.0 and v[3] == 1.0
    assert v[4:] == [float(old_keep.sum()), float(old_d.sum()), float(rm_d.sum())]
    # frame shift: a wrapping ring, a plain buffer with 28-byte slots, a byte buffer
    ring = torch.randn(6, 5, 4, device="cuda")
    plain = torch.randn(20, 7, device="cuda")
    raw = torch.randint(0, 255, (20, 3), dtype=torch.uint8, device="cuda")
    refs = [t.clone() for t in (ring, plain, raw)]
    k, n = 9, 14
    for f in range(k, n - 1):
        refs[0][f % 6] = refs[0][(f + 1) % 6]
        refs[1][f] = refs[1][f + 1]
        refs[2][f] = refs[2][f + 1]
    v0 = ring._version
    pops.frame_shift([(ring, 0, 6), (plain, 0, 0), (raw, 0, 0)], k, n)
    assert ring._version > v0
    for a, b in zip((ring, plain, raw), refs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["all", "none", "subset"])
def test_native_compaction_equals_torch_path(mode):
    """remove_factors with known sizes (dpvo_compact_edges, one stable
    compaction of the index fields, weights, targets, edge state and the
    inactive-list appends) == the torch index path, twice in a row (the second
    call appends to the lists the first one grew)."""
    from dpvo.synthetic import steady_state_tracker
    g = torch.Generator(device="cuda").manual_seed(9)
    with torch.no_grad():
        a = steady_state_tracker("fast", buffer=96, n=70, seed=4)
        b = steady_state_tracker("fast", buffer=96, n=70, seed=4)
        a.NATIVE_COMPACTION = True
        w, t = torch.rand_like(a.pg.weight), torch.rand_like(a.pg.target)
        for s in (a, b):
            s.pg.weight, s.pg.target = w.clone(), t.clone()
        for _ in range(2):
            E = a.pg.ii.numel()
            m = torch.rand(E, generator=g, device="cuda") < 0.3
            store = {"all": True, "none": False, "subset": m & (torch.rand(E, generator=g, device="cuda") < 0.5)}[mode]
            n_store = int(m.sum()) if mode == "all" else 0 if mode == "none" else int(store.sum())
            a.remove_factors(m, store, counts=(E - int(m.sum()), n_store))
            b.remove_factors(m, store)
            for name in ("ii", "jj", "kk", "net", "weight", "target", "ii_inac", "jj_inac", "kk_inac", "weight_inac",
                         "target_inac"):
                x, y = getattr(a.pg, name), getattr(b.pg, name)
                assert x.shape == y.shape and torch.equal(x, y), name
