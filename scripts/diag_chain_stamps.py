"""Where a chain kernel's time goes: the k-loop segments of rowchain_kernel
(csrc/rowgemm.hip, DPVO_STAMPS) from the diagnostic library diag/libdpvo_hot.so
(`make -C wild-video-3d-reconstruction_amd diag`), on c1-shaped inputs
(E = 95,424 rows, K = 384, the A rows gathered through an index, fp32
residual).  Read the SHARES, not the lengths: the stamps' waits forbid
overlaps the product kernel has.  Prints per-tile cycles by segment, loader
waves (0-3) and the other waves (4-7) apart."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPVO_HOT_LIB"] = os.path.join(REPO, "diag", "libdpvo_hot.so")
sys.path.insert(0, os.path.join(REPO, "wild-video-3d-reconstruction_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _dpvo_hot as H  # noqa: E402
import update_ops as U  # noqa: E402

SEGS = ["g1 wait (vmcnt)", "g1 barrier 1", "g1 frags+mfma", "g1 barrier 2", "g1 epilogue batches",
        "g2 wait (vmcnt)", "g2 barrier 1", "g2 frags+mfma", "g2 barrier 2", "row epilogue", "total",
        "acc_to_y + W2 stage 0 + sync", "after g2 (acc_to_y, gate/tri, next tile issue)", "final sync_lds",
        "tile (g1 .. sync)", "-"]


def run(label, flags, ln=False, E=95424, reps=3):
    res = bool(flags & U.RES)
    g = torch.Generator(device="cuda").manual_seed(0)
    A = (0.5 * torch.randn(E, 384, generator=g, device="cuda")).half()
    idx = torch.randperm(E, generator=g, device="cuda")
    idx[::17] = -1
    W1 = (torch.randn(384, 384, generator=g, device="cuda") / 20).half()
    W2 = (torch.randn(384, 384, generator=g, device="cuda") / 20).half()
    b1 = torch.zeros(384, device="cuda").half()
    b2 = torch.zeros(384, device="cuda").half()
    res32 = torch.randn(E, 384, generator=g, device="cuda")
    lnp = (torch.ones(384, device="cuda"), torch.zeros(384, device="cuda"), 1e-3) if ln else None
    for _ in range(reps):
        U.rowchain(A, W1, b1, W2, b2, flags=flags, a_idx=idx, res32=res32 if res else None, ln=lnp, want32=True,
                   want16=True)
    torch.cuda.synchronize()
    nb = min((E + 127) // 128, 256)
    buf = np.zeros(1024 * 8 * 16, np.uint64)
    lib = H.lib()
    lib.dpvo_diag_stamps.restype = ctypes.c_int
    lib.dpvo_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.dpvo_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(1024, 8, 16)[:nb].astype(np.float64)
    tiles = (E + 127) // 128 / nb
    print(f"== {label}: {nb} blocks, {tiles:.2f} tiles per block; cycles per tile (mean over blocks)")
    for k, name in enumerate(SEGS[:15]):
        ld = st[:, :4, k].mean() / tiles
        ot = st[:, 4:, k].mean() / tiles
        print(f"  {name:24s} loaders {ld:10.0f}   waves 4-7 {ot:10.0f}")


if __name__ == "__main__":
    run("c1 chain (RES, deferred epilogue)", U.RES)
    run("LN|LN_RELU chain (epilogue after the GEMMs)", U.LN | U.LN_RELU, ln=True)
