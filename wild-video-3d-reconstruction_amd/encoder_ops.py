"""Native frame-ingest encoders (csrc/encoder.hip): the Patchifier's fnet
(BasicEncoder4, instance norm) and inet (BasicEncoder4, no norm) -- reference
dpvo/extractor.py:200-264, called from dpvo/net.py:121-122 -- in 11 launches
per frame for both networks.

Inference under fp16 autocast only (what DPVO runs, dpvo.py:785); the modules'
own torch forward stays the training / fp32 path.  Like the other shims there
is no CPU path: the library must load and the tensors must be on the GPU.
"""
import ctypes as _ct
import os

import torch

import _dpvo_hot as H

XPLAIN, XNORM_RELU, XBLOCK = 0, 1, 2
_DBG_NOSTATS = os.environ.get("DPVO_ENC_DBG") == "nostats"   # timing experiments only: skips the IN statistics
if _DBG_NOSTATS:
    import warnings
    warnings.warn("DPVO_ENC_DBG=nostats is set -- a timing experiment; encoder outputs are NOT valid")


class ConvArgs(_ct.Structure):
    _fields_ = [("a", _ct.c_void_p), ("a_ps", _ct.c_int64), ("a_co", _ct.c_int),
                ("a_st", _ct.c_void_p), ("a_st_tiles", _ct.c_int), ("a_st_ld", _ct.c_int),
                ("r", _ct.c_void_p), ("r_ps", _ct.c_int64), ("r_co", _ct.c_int),
                ("r_st", _ct.c_void_p), ("r_st_tiles", _ct.c_int), ("r_st_ld", _ct.c_int),
                ("xout", _ct.c_void_p), ("x_ps", _ct.c_int64),
                ("w", _ct.c_void_p), ("bias", _ct.c_void_p),
                ("out", _ct.c_void_p), ("o_ps", _ct.c_int64), ("o_co", _ct.c_int), ("out_scale", _ct.c_float),
                ("part", _ct.c_void_p), ("eps", _ct.c_float)]


def conv_out(n, ks, s):
    return (n + 2 * (ks // 2) - ks) // s + 1


def swizzle_rows(w):
    """[..., 32] fp16 rows of 32 K values: row r's four 8-value chunks stored
    at chunk c ^ ((r >> 2) & 3) (csrc/encoder.hip wrow(): the kernels copy the
    weights into LDS as they are, and this layout makes the MFMA operand reads
    conflict-free)."""
    rows = w.reshape(-1, 4, 8)
    r = torch.arange(rows.shape[0], device=w.device)
    src = torch.arange(4, device=w.device)[None, :] ^ ((r[:, None] >> 2) & 3)   # physical c holds logical c ^ s
    return torch.gather(rows, 1, src[:, :, None].expand(-1, -1, 8)).reshape(w.shape).contiguous()


def pack_conv(weight):
    """[cout][cin][k][k] -> fp16 [k*k][cin/32][cout][32] (the kernel's operand order), row-swizzled."""
    co, ci, k, _ = weight.shape
    w = weight.detach().to(torch.float16).permute(2, 3, 1, 0).reshape(k * k, ci // 32, 32, co)
    return swizzle_rows(w.permute(0, 1, 3, 2).contiguous())


def pack_stem(weight):
    """conv1 [32][3][7][7] -> fp16 [5][32][32]: K = c*49 + ky*7 + kx zero-padded
    to 160, split into five 32-wide chunks, row-swizzled."""
    w = torch.zeros(weight.shape[0], 160, dtype=torch.float16, device=weight.device)
    w[:, :147] = weight.detach().reshape(weight.shape[0], 147)
    return swizzle_rows(w.view(-1, 5, 32).permute(1, 0, 2).contiguous())


def _half(t):
    return t.detach().to(torch.float16).contiguous()


def _is_instance(enc):
    return enc.norm_fn == "instance"


class _Packed:
    """One encoder's parameters in kernel order (what autocast casts them to)."""

    def __init__(self, enc):
        if enc.norm_fn not in ("instance", "none"):
            raise NotImplementedError(f"native encoder: norm_fn {enc.norm_fn!r} (the Patchifier uses instance / none)")
        l1, l2 = enc.layer1, enc.layer2
        self.instance = _is_instance(enc)
        self.stem = (pack_stem(enc.conv1.weight), _half(enc.conv1.bias))
        self.l1 = [(pack_conv(c.weight), _half(c.bias)) for b in l1 for c in (b.conv1, b.conv2)]
        b0 = l2[0]
        ds = b0.downsample[0]
        comb = torch.zeros(3, 3, 128, 32, dtype=torch.float16, device=ds.weight.device)
        comb[:, :, :64] = b0.conv1.weight.detach().to(torch.float16).permute(2, 3, 0, 1)
        comb[1, 1, 64:] = ds.weight.detach().to(torch.float16)[:, :, 0, 0]
        self.l2_down = (swizzle_rows(comb.reshape(9, 1, 128, 32)), _half(torch.cat([b0.conv1.bias, ds.bias])))
        self.l2 = [(pack_conv(c.weight), _half(c.bias)) for c in (b0.conv2, l2[1].conv1, l2[1].conv2)]
        cw = enc.conv2.weight
        self.out_dim = cw.shape[0]
        self.head = (pack_conv(cw), _half(enc.conv2.bias))                 # full map (fnet)
        self.head_rows = (_half(cw[:, :, 0, 0]), _half(enc.conv2.bias))      # at points (inet)
        self.eps = 1e-5
        for m in enc.modules():
            if isinstance(m, torch.nn.InstanceNorm2d):
                if m.affine or m.track_running_stats:
                    raise NotImplementedError("native encoder: affine / running-stat instance norm")
                self.eps = m.eps


class _Work:
    """Activations and instance-norm partials of one encoder at one frame size
    (reused per frame).  part[l]: the per-tile (sum, sumsq) rows layer l writes
    (l = 0 stem .. 8), or None without norm."""

    def __init__(self, H1, W1, H2, W2, t1, t2, stats, dev):
        z = lambda n, c: H.empty(n, c, dtype=torch.float16, device=dev)
        n1, n2 = H1 * W1, H2 * W2
        self.y = [z(n1, 32) for _ in range(5)]          # y0 .. y4
        self.x0, self.x1 = z(n1, 32), z(n1, 32)
        self.y5d = z(n2, 128)
        self.y6, self.y7, self.y8, self.x3 = z(n2, 64), z(n2, 64), z(n2, 64), z(n2, 64)
        f = lambda t, c: torch.zeros(t, 2 * c, dtype=torch.float32, device=dev)
        self.part = ([f(t1, 32) for _ in range(5)] + [f(t2, 128), f(t2, 64), f(t2, 64), f(t2, 64)]
                     if stats else [None] * 9)


def _ptr(t):
    return t.data_ptr() if t is not None else None


class NativeEncoders:
    """fnet + inet of a Patchifier on the HIP library.

    run(image uint8 [3, H, W], x, y int64 [M]) ->
        fmap fp16 [1, 1, 128, h, w] (channel-last storage: strides of an NHWC
        tensor), imap fp16 [M, 384] = inet(image)[:, :, y, x] / 4."""

    def __init__(self, fnet, inet):
        self.fnet, self.inet = fnet, inet
        self._pk = self._pk_key = None
        self._work = {}

    def _packed(self):
        key = tuple((q.data_ptr(), q._version) for m in (self.fnet, self.inet) for q in m.parameters())
        if self._pk_key != key:
            self._pk = (_Packed(self.fnet), _Packed(self.inet))
            self._pk_key = key
        return self._pk

    def _ws(self, H_, W_, dev, pk):
        k = (H_, W_, dev)
        if k not in self._work:
            H1, W1 = conv_out(H_, 7, 2), conv_out(W_, 7, 2)
            H2, W2 = conv_out(H1, 3, 2), conv_out(W1, 3, 2)
            t1, t2 = H.lib().dpvo_encoder_tiles(H_, W_, 7, 2), H.lib().dpvo_encoder_tiles(H1, W1, 3, 2)
            ws = [_Work(H1, W1, H2, W2, t1, t2, p.instance, dev) for p in pk]
            self._work[k] = (ws, (H1, W1, H2, W2))
        return self._work[k]

    def run(self, image, x, y, fmap_out=None):
        H.on_gpu(image, x, y)
        if image.dtype != torch.uint8 or image.dim() != 3 or image.shape[0] != 3:
            raise RuntimeError("native encoder: image must be uint8 [3, H, W]")
        image = image.contiguous()
        x, y = H.idx64(x.reshape(-1)), H.idx64(y.reshape(-1))
        if x.numel() != y.numel():
            raise RuntimeError("native encoder: x and y must have the same length")
        pk = self._packed()
        dev = image.device
        Hh, Ww = image.shape[1:]
        ws, (H1, W1, H2, W2) = self._ws(Hh, Ww, dev, pk)
        fmap = fmap_out if fmap_out is not None else H.empty(H2 * W2, 128, dtype=torch.float16, device=dev)
        M = x.numel()
        imap = H.empty(M, pk[1].out_dim, dtype=torch.float16, device=dev)

        def st(t):   # a producer's partials as (pointer, tiles, row length)
            if t is None or _DBG_NOSTATS:
                return None, 0, 0
            return t.data_ptr(), t.shape[0], t.shape[1]

        def args(i, a=None, a_ps=0, a_co=0, a_st=None, r=None, r_ps=0, r_co=0, r_st=None, xout=None, x_ps=0,
                 w=None, out=None, o_ps=0, o_co=0, part=None, scale=1.0):
            return ConvArgs(_ptr(a), a_ps, a_co, *st(a_st), _ptr(r), r_ps, r_co, *st(r_st), _ptr(xout), x_ps,
                            _ptr(w[0]), _ptr(w[1]), _ptr(out), o_ps, o_co, scale,
                            None if _DBG_NOSTATS else _ptr(part), pk[i].eps)

        def launch(fn, *lead, build):
            arr = (ConvArgs * 2)(build(0), build(1))
            H.check(fn(*lead, arr, 2, st_))

        st_ = H.stream_of(image)
        lib = H.lib()
        P = [w.part for w in ws]
        # conv1 + norm1 + relu1 (extractor.py:255-257): y0
        launch(lib.dpvo_encoder_stem, image.data_ptr(), Hh, Ww,
               build=lambda i: args(i, w=pk[i].stem, out=ws[i].y[0], o_ps=32, part=P[i][0]))
        # layer1 (two stride-1 blocks, 32 channels)
        conv = lambda xm, build, ks=3, s=1, ci=32, co=32, hi=H1, wi=W1: launch(
            lib.dpvo_encoder_conv, ks, s, ci, co, xm, hi, wi, build=build)
        conv(XNORM_RELU, lambda i: args(i, a=ws[i].y[0], a_ps=32, a_st=P[i][0], xout=ws[i].x0, x_ps=32,
                                        w=pk[i].l1[0], out=ws[i].y[1], o_ps=32, part=P[i][1]))
        conv(XNORM_RELU, lambda i: args(i, a=ws[i].y[1], a_ps=32, a_st=P[i][1],
                                        w=pk[i].l1[1], out=ws[i].y[2], o_ps=32, part=P[i][2]))
        conv(XBLOCK, lambda i: args(i, a=ws[i].y[2], a_ps=32, a_st=P[i][2], r=ws[i].x0, r_ps=32,
                                    xout=ws[i].x1, x_ps=32, w=pk[i].l1[2], out=ws[i].y[3], o_ps=32, part=P[i][3]))
        conv(XNORM_RELU, lambda i: args(i, a=ws[i].y[3], a_ps=32, a_st=P[i][3],
                                        w=pk[i].l1[3], out=ws[i].y[4], o_ps=32, part=P[i][4]))
        # layer2: stride-2 block (conv1 | downsample in one launch), stride-1 block
        conv(XBLOCK, lambda i: args(i, a=ws[i].y[4], a_ps=32, a_st=P[i][4], r=ws[i].x1, r_ps=32,
                                    w=pk[i].l2_down, out=ws[i].y5d, o_ps=128, part=P[i][5]), s=2, co=128)
        c64 = dict(ci=64, co=64, hi=H2, wi=W2)
        conv(XNORM_RELU, lambda i: args(i, a=ws[i].y5d, a_ps=128, a_st=P[i][5],
                                        w=pk[i].l2[0], out=ws[i].y6, o_ps=64, part=P[i][6]), **c64)
        conv(XBLOCK, lambda i: args(i, a=ws[i].y6, a_ps=64, a_st=P[i][6], r=ws[i].y5d, r_ps=128, r_co=64,
                                    r_st=P[i][5], xout=ws[i].x3, x_ps=64,
                                    w=pk[i].l2[1], out=ws[i].y7, o_ps=64, part=P[i][7]), **c64)
        conv(XNORM_RELU, lambda i: args(i, a=ws[i].y7, a_ps=64, a_st=P[i][7],
                                        w=pk[i].l2[2], out=ws[i].y8, o_ps=64, part=P[i][8]), **c64)
        # conv2 (extractor.py:262), / 4 (net.py:121-122): fnet over the whole map
        f = args(0, a=ws[0].y8, a_ps=64, a_st=P[0][8], r=ws[0].x3, r_ps=64, w=pk[0].head, out=fmap, o_ps=128,
                 scale=0.25)
        H.check(lib.dpvo_encoder_conv(1, 1, 64, 128, XBLOCK, H2, W2, (ConvArgs * 1)(f), 1, st_))
        # inet only at the patch centres
        g = args(1, a=ws[1].y8, a_ps=64, a_st=P[1][8], r=ws[1].x3, r_ps=64, w=pk[1].head_rows, out=imap,
                 o_ps=pk[1].out_dim, scale=0.25)
        H.check(lib.dpvo_encoder_head_at(_ct.byref(g), pk[1].out_dim, H2, W2, _ptr(x), _ptr(y), M, st_))
        fmap = fmap.view(1, 1, H2, W2, 128).permute(0, 1, 4, 2, 3)
        return fmap, imap

    def gather(self, image, fmap, imap, x, y, return_color=True):
        """The Patchifier's gathers at the patch centres (net.py:301-315) in one
        launch: fmap / imap as run() returns them, image the uint8 frame ->
        gmap fp32 [1, M, 128, 3, 3], imap fp32 [1, M, DIM, 1, 1], patches fp32
        [1, M, 3, 3, 3], clr fp32 [1, M, 3] (None unless return_color) --
        bit-identical to DPVONet._gather's torch composition."""
        H.on_gpu(image, fmap, imap, x, y)
        if fmap.dtype != torch.float16 or fmap.dim() != 5 or fmap.shape[2] != 128:
            raise RuntimeError("patch gather: fmap must be fp16 [1, 1, 128, h, w]")
        if imap.dtype != torch.float16 or imap.dim() != 2:
            raise RuntimeError("patch gather: imap must be fp16 [M, DIM]")
        x, y = H.idx64(x.reshape(-1)), H.idx64(y.reshape(-1))
        M, dim = x.numel(), imap.shape[1]
        if y.numel() != M or imap.shape[0] != M:
            raise RuntimeError("patch gather: x, y and imap must have M rows")
        imap = imap.contiguous()
        dev = fmap.device
        h, w = fmap.shape[-2:]
        f = fmap[0, 0]
        strides = torch.tensor([f.stride(0), f.stride(1), f.stride(2)], dtype=torch.int64)
        gm = H.empty(1, M, 128, 3, 3, dtype=torch.float32, device=dev)
        im = H.empty(1, M, dim, 1, 1, dtype=torch.float32, device=dev)
        pt = H.empty(1, M, 3, 3, 3, dtype=torch.float32, device=dev)
        clr = lut = img = None
        Hh = Ww = 0
        if return_color:
            if image.dtype != torch.uint8 or image.dim() != 3 or image.shape[0] != 3:
                raise RuntimeError("patch gather: image must be uint8 [3, H, W]")
            img = image.contiguous()
            Hh, Ww = img.shape[1:]
            lut = self._lut(dev)
            clr = H.empty(1, M, 3, dtype=torch.float32, device=dev)
        H.check(H.lib().dpvo_patch_gather(f.data_ptr(), strides.data_ptr(), h, w, imap.data_ptr(), dim, _ptr(img),
                                          Hh, Ww, _ptr(lut), x.data_ptr(), y.data_ptr(), M, gm.data_ptr(),
                                          im.data_ptr(), pt.data_ptr(), _ptr(clr), H.stream_of(fmap)))
        return gm, im, pt, clr

    def _lut(self, dev):
        """lut[v] = 2 (v / 255) - 0.5 evaluated by the same torch ops as the
        frame normalisation of forward() (net.py:116), so each entry is the
        value that expression gives the pixel"""
        lut = getattr(self, "_lut_t", None)
        if lut is None or lut.device != dev:
            v = torch.arange(256, dtype=torch.int32, device=dev).to(torch.uint8)
            lut = self._lut_t = (2 * (v[None, None] / 255.0) - 0.5).reshape(256).contiguous()
        return lut
