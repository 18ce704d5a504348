"""Where rowgemm5's k-loop time goes (csrc/rowgemm.hip, DPVO_STAMPS build in
diag/libdpvo_hot.so): per k-step cycles waiting at the barrier, waiting for
the step's W / A registers (vmcnt), and issuing the step, plus the row
epilogue per tile -- E = 95,424 rows.  Since round 6 the SoftAgg pair (K =
384) runs rowpair6 (A tile resident in LDS, no stamps); rowgemm5's DUAL pass
serves K outside 128..384, so this script drives it at K = 448 (round 5's
records, profiles/r5/, were taken at K = 384)."""
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
import update_ops as U  # noqa: E402


def main(E=95424, K=448):
    g = torch.Generator(device="cuda").manual_seed(0)
    A = (0.5 * torch.randn(E, K, generator=g, device="cuda")).half()
    W = [U.kblock((torch.randn(384, K, generator=g, device="cuda") / 20).half()) for _ in range(2)]
    b = torch.zeros(384, device="cuda").half()
    for _ in range(3):
        U.rowgemm_pair(A, W[0], b, W[1], b)
    torch.cuda.synchronize()
    nb = min((E + 127) // 128, 256)
    buf = np.zeros(1024 * 8 * 16, np.uint64)
    lib = H.lib()
    lib.dpvo_diag_stamps.restype = ctypes.c_int
    lib.dpvo_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.dpvo_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(1024, 8, 16)[:nb].astype(np.float64)
    tiles = (E + 127) // 128 / nb
    steps = tiles * 2 * (K // 32)
    print(f"pair: {nb} blocks, {tiles:.2f} tiles / block, {steps:.0f} k-steps / block")
    for k, name in ((0, "barrier wait / step"), (1, "W+A vmcnt wait / step"), (2, "issue / step")):
        print(f"  {name:26s} {st[:, :, k].mean() / steps:8.0f} cycles (waves: {np.round(st[:, :, k].mean(0) / steps)})")
    print(f"  {'epilogue / pass':26s} {st[:, :, 3].mean() / (tiles * 2):8.0f}")
    print(f"  {'total / block':26s} {st[:, :, 10].mean():8.0f}")


if __name__ == "__main__":
    main()
