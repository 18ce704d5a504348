"""SoftAgg's f / g GEMM pairs at C3's shape (dpvo_rowgemm_pair on fp16 rows,
dpvo_rowgemm_pair_pre on fp32 rows + a gathered fp16 addend), HIP events over
back-to-back launches -- for A/B runs of experiment builds
(DPVO_HOT_LIB=exp/<name>/libdpvo_hot.so DPVO_DIAG=1).  Prints the times and
a digest of the outputs (equal digests = same bits).

  python scripts/exp_pair_time.py [--rows 95424] [--reps 40] [--tag name]
"""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]

import torch  # noqa: E402


def _time(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(round(a.elapsed_time(b) / reps, 4))
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=95424)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tag", default=os.environ.get("DPVO_HOT_LIB", "product"))
    args = ap.parse_args()
    import update_ops as U
    g = torch.Generator(device="cuda").manual_seed(11)
    M, G, dev = args.rows, 4416, "cuda"
    lin = lambda: U.pack_linear(torch.randn(384, 384, device=dev, generator=g) / 20.0,  # noqa: E731
                                torch.randn(384, device=dev, generator=g) * 0.1)
    (Wa, ba), (Wb, bb) = lin(), lin()
    Wa, Wb = U.kblock(Wa), U.kblock(Wb)
    A = (torch.randn(M, 384, device=dev, generator=g) * 0.5).half()
    a32 = torch.randn(M, 384, device=dev, generator=g)
    b16 = torch.randn(G, 384, device=dev, generator=g).half()
    b_idx = torch.randint(-1, G, (M,), device=dev, generator=g)
    with torch.no_grad():
        t_pair = _time(lambda: U.rowgemm_pair(A, Wa, ba, Wb, bb), args.reps)
        t_pre = _time(lambda: U.rowgemm_pair_pre(a32, b16, b_idx, Wa, ba, Wb, bb), args.reps)
        outs = U.rowgemm_pair(A, Wa, ba, Wb, bb) + U.rowgemm_pair_pre(a32, b16, b_idx, Wa, ba, Wb, bb)
        torch.cuda.synchronize()
    h = hashlib.sha256()
    for o in outs:
        h.update(o.contiguous().view(torch.int16).cpu().numpy().tobytes())
    print(json.dumps({"tag": args.tag, "rows": M, "pair_ms": t_pair, "pair_pre_ms": t_pre,
                      "out_sha": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
