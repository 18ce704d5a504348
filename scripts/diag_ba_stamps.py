"""Where the BA patch kernel's time goes (csrc/fastba.hip bd_patch_kernel,
DPVO_STAMPS build in diag/libdpvo_hot.so): per-wave cycles by phase, on the
bench's steady-state tracker (C2 by default), from the last <APPLY, HESS>
launch of one update()."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPVO_HOT_LIB"] = os.path.join(REPO, "diag", "libdpvo_hot.so")
os.environ["DPVO_DIAG"] = "1"   # the loader refuses the stamps build otherwise
sys.path.insert(0, os.path.join(REPO, "wild-video-3d-reconstruction_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _dpvo_hot as H  # noqa: E402
from dpvo.synthetic import steady_state_tracker  # noqa: E402

SEGS = ["init (LDS zero, tri_rc)", "group rec + depth apply + px/py", "bd_edge (erec + poses)", "C/u sums + mixed",
        "i-terms (33 all-sums + atomics)", "j-terms (LDS atomics)", "E row + slot", "flush", "iteration total",
        "partial write", "kernel total"]


def main(config="C2"):
    cfg = {"C2": ("default", 512, 8, {"PATCHES_PER_FRAME": 96}), "C3": ("dpvo_2k", 2048, 2, {})}[config]
    slam = steady_state_tracker(cfg[0], buffer=cfg[1], seed=0, iterations=cfg[2], device="cuda", **cfg[3])
    with torch.no_grad():
        for _ in range(3):
            slam.update()
    torch.cuda.synchronize()
    W = 4   # BD_WAVES
    buf = np.zeros(512 * W * 16, np.uint64)
    lib = H.lib()
    lib.dpvo_diag_bd_stamps.restype = ctypes.c_int
    lib.dpvo_diag_bd_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.dpvo_diag_bd_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(512, W, 16).astype(np.float64)
    print(f"== {config}: bd_patch_kernel<true, true>, cycles per wave (mean / max over waves)")
    for k, name in enumerate(SEGS):
        print(f"  {name:34s} {st[:, :, k].mean():9.0f} {st[:, :, k].max():9.0f}")


if __name__ == "__main__":
    main(*(sys.argv[1:]))
