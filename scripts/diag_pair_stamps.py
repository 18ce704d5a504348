"""Where the resident-A pair's time goes (rowpair6 in csrc/rowgemm.hip,
DPVO_STAMPS build in diag/libdpvo_hot.so): per tile, the cycles of pass 0's
barrier waits and the rest of its k-steps, the pass-0 row epilogue, pass 1
(from LDS), and the pass-1 epilogue -- for the SoftAgg pair on fp16 rows and
the pair_pre variant (fp32 rows + a gathered fp16 addend) at E = 95,424."""
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

SEGS = ((0, "pass 0 barrier waits"), (1, "pass 0 k-steps (rest)"), (2, "pass 0 epilogue"), (3, "pass 1"),
        (4, "pass 1 epilogue"))


def report(name, nb):
    buf = np.zeros(1024 * 8 * 16, np.uint64)
    lib = H.lib()
    lib.dpvo_diag_stamps.restype = ctypes.c_int
    lib.dpvo_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.dpvo_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(1024, 8, 16)[:nb].astype(np.float64)
    tiles = st[:, 0, 11].mean()
    print(f"{name}: {nb} blocks, {tiles:.2f} tiles / block; cycles per tile (mean over waves; min / max wave)")
    for k, label in SEGS:
        per = st[:, :, k] / np.maximum(st[:, :, 11], 1)
        print(f"  {label:24s} {per.mean():8.0f}   ({per.mean(0).min():.0f} / {per.mean(0).max():.0f})")
    print(f"  {'total / block':24s} {st[:, :, 10].mean():8.0f}")


def main(E=95424, G=4416):
    g = torch.Generator(device="cuda").manual_seed(0)
    A = (0.5 * torch.randn(E, 384, generator=g, device="cuda")).half()
    W = [U.kblock((torch.randn(384, 384, generator=g, device="cuda") / 20).half()) for _ in range(2)]
    b = torch.zeros(384, device="cuda").half()
    a32 = torch.randn(E, 384, generator=g, device="cuda")
    b16 = torch.randn(G, 384, generator=g, device="cuda").half()
    b_idx = torch.randint(-1, G, (E,), generator=g, device="cuda")
    nb = min((E + 127) // 128, torch.cuda.get_device_properties(0).multi_processor_count)
    for _ in range(3):
        U.rowgemm_pair(A, W[0], b, W[1], b)
    torch.cuda.synchronize()
    report("pair", nb)
    for _ in range(3):
        U.rowgemm_pair_pre(a32, b16, b_idx, W[0], b, W[1], b)
    torch.cuda.synchronize()
    report("pair_pre", nb)


if __name__ == "__main__":
    main()
