"""Where the LDS-staged altcorr kernel's time goes (csrc/corrstage.hip,
DPVO_STAMPS build in diag/libdpvo_hot.so): per-wave cycles in the task
barriers + region writes, the edge inputs + prefetch issue, level 2, level 1
and the output stores, at C3 (E = 95,424)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPVO_HOT_LIB"] = os.path.join(REPO, "diag", "libdpvo_hot.so")
os.environ["DPVO_DIAG"] = "1"   # the loader refuses the stamps build otherwise
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _dpvo_hot as H  # noqa: E402


def main():
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker("dpvo_2k", buffer=2048, seed=0)
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, _, _ = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status)
        for _ in range(3):
            slam.corr(coords, slots=(ctx, jslot))
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8 * 16, np.uint64)
    lib = H.lib()
    lib.dpvo_diag_cs_stamps.restype = ctypes.c_int
    lib.dpvo_diag_cs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.dpvo_diag_cs_stamps(buf.ctypes.data, buf.nbytes) == 0
    nb = torch.cuda.get_device_properties(0).multi_processor_count
    st = buf.reshape(4096, 8, 16)[:nb].astype(np.float64)
    names = ["barriers + region write", "edge inputs + prefetch issue", "level 2", "level 1", "stores", "total"]
    tasks, edges = st[:, :, 6], st[:, :, 7]
    print(f"{nb} blocks; tasks / block mean {tasks[:, 0].mean():.1f} max {tasks[:, 0].max():.0f}; "
          f"edges / wave mean {edges.mean():.1f} max {edges.max():.0f}")
    for k, n in enumerate(names):
        print(f"  {n:30s} mean {st[:, :, k].mean():12.0f}  max {st[:, :, k].max():12.0f} cycles per wave")
    e = max(edges.mean(), 1)
    tl = st[:, :, 11].mean()
    print(f"  per edge (both levels): setup {st[:, :, 8].mean() / e:.0f}, tile loop {st[:, :, 9].mean() / e:.0f} "
          f"({tl / e:.1f} tiles, {st[:, :, 9].mean() / max(tl, 1):.0f} per tile), epilogue {st[:, :, 10].mean() / e:.0f}")
    print(f"  per edge: level 2 {st[:, :, 2].mean() / e:.0f}, level 1 {st[:, :, 3].mean() / e:.0f}, "
          f"stores {st[:, :, 4].mean() / e:.0f}; per task: barriers {st[:, :, 0].mean() / max(tasks.mean(), 1):.0f}, "
          f"inputs {st[:, :, 1].mean() / max(tasks.mean(), 1):.0f}")


if __name__ == "__main__":
    main()
