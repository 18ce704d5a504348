"""Timing experiment for rowgemm4_kernel (plain K = 384 GEMM over E = 95,424
rows): each DPVO_RG4_DBG variant drops one part of the kernel (1 epilogue,
2 MFMA, 4 A loads, 8 W loads) so the time left shows what bounds it.  Each
variant runs in its own process (the variant is read once per process)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd"), os.path.join(REPO, "scripts")]
    import torch
    import update_ops as U
    from bench_rowgemm import timeit
    E, D, K = 95424, 384, int(os.environ.get("RG_K", "384"))
    torch.manual_seed(0)
    A = torch.randn(E, K, device="cuda").half()
    W16, b16 = U.pack_linear(torch.randn(D, K, device="cuda") / K ** 0.5, torch.randn(D, device="cuda") * 0.1)
    t = timeit(lambda: U.rowgemm(A, W16, b16))
    print(json.dumps({"dbg": os.environ.get("DPVO_RG4_DBG", "0"), "K": K, "us": round(t * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        for d in ["0", "1", "2", "4", "8", "3", "5", "6", "9", "12", "13", "14", "15"]:
            env = dict(os.environ, DPVO_RG4_DBG=d)
            if d == "0":
                env.pop("DPVO_RG4_DBG")
            subprocess.run([sys.executable, __file__, "child"], env=env, check=True, timeout=300)
