"""ctypes binding of libdpvo_hot.so (the C ABI declared in include/dpvo_hot.h).

This is the only place that loads the native library.  There is no CPU or
Python fallback: if the library is missing or a tensor is not on the GPU the
call raises, so a silently-degraded run cannot pass for the HIP path.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPVO_HOT_LIB", os.path.join(HERE, "libdpvo_hot.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "dpvo_hot.h")

F16, F32, F64 = 0, 1, 2
_DTYPES = {torch.float16: F16, torch.float32: F32, torch.float64: F64}

_i64 = ctypes.c_int64
_vp = ctypes.c_void_p
_ip = ctypes.c_int
_fp = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes)
_SIGNATURES = {
    "dpvo_hot_abi_version": (_ip, []),
    "dpvo_hot_last_error": (ctypes.c_char_p, []),
    "dpvo_hot_build_info": (ctypes.c_char_p, []),
    "dpvo_corr_forward": (_ip, [_ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _ip, _vp, _vp]),
    "dpvo_corr_forward_pyramid": (_ip, [_ip, _vp, _vp, _vp, _ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _ip,
                                        _vp, _vp]),
    "dpvo_corr_forward_pyramid_ld": (_ip, [_ip, _vp, _vp, _vp, _ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                           _ip, _vp, _i64, _vp, _vp]),
    "dpvo_corr_table_bytes": (_sz, [_vp]),
    "dpvo_corr_pack": (_ip, [_vp, _vp, _vp, _vp, _vp]),
    "dpvo_corr_pack_mfma_bytes": (_sz, [_vp]),
    "dpvo_corr_pack_mfma": (_ip, [_vp, _vp, _vp, _vp, _vp]),
    "dpvo_corr_pyramid_mfma": (_ip, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "dpvo_edge_order_workspace_bytes": (_sz, [_ip]),
    "dpvo_edge_order": (_ip, [_vp, _i64, _ip, _vp, _vp, _sz, _vp]),
    "dpvo_corr_backward": (_ip, [_ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _ip, _vp, _vp, _vp]),
    "dpvo_patchify_forward": (_ip, [_ip, _vp, _vp, _vp, _vp, _i64, _ip, _vp, _vp]),
    "dpvo_patchify_backward": (_ip, [_ip, _vp, _vp, _i64, _ip, _vp, _vp, _vp]),
    "dpvo_ba_workspace_bytes": (_sz, [_i64, _i64, _ip]),
    "dpvo_ba_forward": (_ip, [_vp, _vp, _i64, _ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _ip, _ip, _ip, _vp, _sz,
                              _vp, _vp]),
    "dpvo_ba_workspace_bytes_ex": (_sz, [_i64, _i64, _ip, _ip]),
    "dpvo_ba_forward_ex": (_ip, [_vp, _vp, _i64, _ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _ip, _ip, _ip, _ip,
                                 _vp, _sz, _vp, _vp]),
    "dpvo_ba_forward_csr": (_ip, [_vp, _vp, _i64, _ip, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _ip, _ip, _ip, _ip,
                                  _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "dpvo_reproject": (_ip, [_vp, _vp, _ip, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "dpvo_solve_system_assemble": (_ip, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _fp, _fp, _vp, _vp, _vp, _vp]),
    "dpvo_neighbors_workspace_bytes": (_sz, [_i64]),
    "dpvo_neighbors": (_ip, [_vp, _vp, _i64, _vp, _vp, _vp, _sz, _vp]),
    "dpvo_lie_forward": (_ip, [_ip, _ip, _ip, _vp, _vp, _vp, _i64, _vp]),
    "dpvo_lie_backward": (_ip, [_ip, _ip, _ip, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "dpvo_pose_extrapolate": (_ip, [_vp, _i64, _fp, _vp]),
    "dpvo_pose_relative": (_ip, [_vp, _vp, _vp, _vp]),
    "dpvo_transform": (_ip, [_vp, _vp, _ip, _vp, _vp, _vp, _vp, _i64, _ip, _vp, _vp, _vp]),
    "dpvo_point_cloud": (_ip, [_vp, _vp, _ip, _vp, _vp, _i64, _ip, _vp, _vp]),
    "dpvo_motion_mag": (_ip, [_vp, _vp, _ip, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _fp, _vp, _vp]),
    "dpvo_motion_mag_workspace_bytes": (ctypes.c_size_t, [_i64]),
    "dpvo_motion_mag_ws": (_ip, [_vp, _vp, _ip, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _fp, _vp, _vp, ctypes.c_size_t,
                                 _vp]),
    "dpvo_keyframe_flow_lds_bytes": (ctypes.c_size_t, [_ip, _i64]),
    "dpvo_keyframe_flow": (_ip, [_vp, _vp, _ip, _vp, _i64, _i64, _fp, _vp, _vp]),
    "dpvo_softagg_workspace_bytes": (_sz, [_i64, _i64]),
    "dpvo_softagg_forward": (_ip, [_ip, _vp, _i64, _vp, _i64, _vp, _i64, _ip, _i64, _fp, _vp, _vp, _sz, _vp]),
    "dpvo_gather_rows": (_ip, [_ip, _vp, _i64, _i64, _vp, _i64, _ip, _ip, _vp, _vp]),
    "dpvo_group_by_workspace_bytes": (_sz, [_i64]),
    "dpvo_group_by_workspace_bytes_for": (_sz, [_i64, _ip]),
    "dpvo_group_by": (_ip, [_vp, _i64, _ip, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dpvo_softagg_csr": (_ip, [_ip, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _ip, _fp, _vp, _vp]),
    "dpvo_softagg_csr_long": (_ip, [_ip, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _ip, _fp, _vp, _vp]),
    "dpvo_neighbors_csr": (_ip, [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp]),
    "dpvo_scatter_csr": (_ip, [_ip, _ip, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _fp, _vp, _i64, _vp, _vp]),
    "dpvo_rowgemm": (_ip, [_vp, _vp]),
    "dpvo_rowgemm_pair": (_ip, [_vp, _vp, _vp]),
    "dpvo_rowgemm_pair_pre": (_ip, [_vp, _vp, _vp, _vp]),
    "dpvo_rowchain": (_ip, [_vp, _vp, _vp]),
    "dpvo_rowchain3": (_ip, [_vp, _vp, _vp, _vp]),
    "dpvo_rowchain_gated": (_ip, [_vp, _vp, _vp, _vp]),
    "dpvo_rowchain_gated_pre": (_ip, [_vp, _vp, _vp, _vp, _vp]),
    "dpvo_rowadd_ln": (_ip, [_vp, _vp]),
    "dpvo_append_edges_count": (_i64, [_i64, _i64, _i64]),
    "dpvo_append_edges": (_ip, [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "dpvo_edge_targets": (_ip, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "dpvo_window_keys": (_ip, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dpvo_window_group_by_workspace_bytes": (_sz, [_i64, _ip]),
    "dpvo_window_group_by": (_ip, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _ip] + [_vp] * 13 + [_sz, _vp]),
    "dpvo_encoder_tiles": (_i64, [_ip, _ip, _ip, _ip]),
    "dpvo_encoder_stem": (_ip, [_vp, _ip, _ip, _vp, _ip, _vp]),
    "dpvo_encoder_conv": (_ip, [_ip] * 7 + [_vp, _ip, _vp]),
    "dpvo_encoder_head_at": (_ip, [_vp, _ip, _ip, _ip, _vp, _vp, _i64, _vp]),
    "dpvo_keyframe_masks_workspace_bytes": (_sz, [_i64]),
    "dpvo_keyframe_masks": (_ip, [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _sz, _vp]),
    "dpvo_frame_shift": (_ip, [_vp, _vp, _vp, _ip, _i64, _i64, _vp]),
    "dpvo_compact_edges_workspace_bytes": (_sz, [_i64]),
    "dpvo_compact_edges": (_ip, [_i64, _vp, _vp, _ip, _vp, _vp, _vp, _vp, _vp, _ip, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                 _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dpvo_patch_gather": (_ip, [_vp, _vp, _ip, _ip, _vp, _ip, _vp, _ip, _ip, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                _vp, _vp]),
}
EXPORTED = tuple(_SIGNATURES)

_lib = None
build_info = None   # the loaded library's dpvo_hot_build_info(), parsed


def source_sha(csrc=None, header=HEADER):
    """sha256 prefix of the HIP sources shipped beside the library, in the
    Makefile's order (csrc/*.hip and csrc/*.hpp sorted by name, then the C-ABI
    header); None when the sources are not present."""
    csrc = csrc or os.path.join(HERE, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")),
                   key=lambda f: "csrc/" + os.path.basename(f))
    if not files or not os.path.exists(header):
        return None
    h = hashlib.sha256()
    for f in files + [header]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def parse_build_info(info):
    out = {}
    for kv in info.split():
        k, _, v = kv.partition("=")
        out[k] = v
    return out


def verify_build(info, src_sha, diag=False):
    """Refuse a library built from other sources than the ones beside it, or
    a diagnostic / experiment build (in-kernel stamps, scripts/build_exp.sh)
    unless diag (DPVO_DIAG=1).  With diag a non-product build may come from
    other sources (an experiment's A/B variant); the product never.  Returns
    the parsed info."""
    b = parse_build_info(info)
    if "sha" not in b or "flavour" not in b:
        raise ImportError(f"libdpvo_hot.so reports no build provenance ({info!r}): rebuild it (make -B)")
    if src_sha is not None and b["sha"] != src_sha and not (diag and b["flavour"] != "product"):
        raise ImportError(f"libdpvo_hot.so is stale: built from sources sha={b['sha']}, the tree holds "
                          f"sha={src_sha}; rebuild it (__graft_entry__.build())")
    if b["flavour"] != "product" and not diag:
        raise ImportError(f"libdpvo_hot.so is the '{b['flavour']}' diagnostic build; set DPVO_DIAG=1 to load it")
    return b


def lib():
    """Load libdpvo_hot.so once; raise if it was not built, is stale against
    the shipped sources, or is the diagnostic build."""
    global _lib, build_info
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libdpvo_hot.so not found at {LIB_PATH}; build it with `python -c \"import __graft_entry__ as g; "
                f"g.build()\"` (hipcc, --offload-arch=gfx950)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        build_info = verify_build(handle.dpvo_hot_build_info().decode(), source_sha(),
                                  diag=os.environ.get("DPVO_DIAG") == "1")
        _lib = handle
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().dpvo_hot_last_error().decode(errors="replace")
        raise RuntimeError(msg or f"dpvo_hot error {rc}")


def on_gpu(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("MI355X build: operands must be GPU (HIP) tensors; this library has no CPU backend")


def dtype_code(t):
    try:
        return _DTYPES[t.dtype]
    except KeyError:
        raise RuntimeError(f"unsupported dtype {t.dtype}") from None


def stream_of(t):
    return _vp(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return _vp(t.data_ptr()) if t is not None else _vp(0)


def i64arr(vals):
    vals = [int(v) for v in vals]
    return (ctypes.c_int64 * max(len(vals), 1))(*vals)


def sizes(t):
    return i64arr(t.shape)


def strides(t):
    return i64arr(t.stride())


# Debug switch: fill every device buffer the shims allocate uninitialised
# (kernel outputs and workspaces) with one byte pattern before the kernel
# sees it -- 0xff is NaN in fp16 / fp32 / fp64 and -1 in the integer types.
# A kernel that reads memory it never wrote then gives different bits under
# two patterns (tests/test_gpu_update_async.py).  DPVO_POISON=0xff at import,
# or set_poison(byte) / set_poison(None).
_POISON = None


def set_poison(byte):
    """byte pattern (0..255) for every buffer empty() hands out, None = off"""
    global _POISON
    _POISON = None if byte is None else int(byte) & 0xFF


def poison():
    return _POISON


if os.environ.get("DPVO_POISON"):
    set_poison(int(os.environ["DPVO_POISON"], 0))


def empty(*size, dtype=torch.float32, device=None):
    """torch.empty, poisoned under set_poison() (device tensors only)"""
    t = torch.empty(*size, dtype=dtype, device=device)
    if _POISON is not None and t.is_cuda and t.numel():
        t.view(torch.uint8).fill_(_POISON)
    return t


def new_empty(like, *size):
    """like.new_empty(*size) through empty()"""
    return empty(*size, dtype=like.dtype, device=like.device)


def idx64(t):
    """int64, contiguous, on the GPU (the reference passes torch.long)."""
    if t.dtype != torch.int64:
        t = t.long()
    return t.contiguous()
