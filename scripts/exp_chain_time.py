"""c1 / c2's chain (dpvo_rowchain: gathered A, ReLU, RES epilogue, out32 +
out16) at C3's shape, HIP events over back-to-back launches -- for A/B runs of
experiment builds (DPVO_HOT_LIB=exp/<name>/libdpvo_hot.so DPVO_DIAG=1).
Prints the time and a digest of both outputs (equal digests = same bits).

  python scripts/exp_chain_time.py [--rows 95424] [--reps 40] [--tag name]
"""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=95424)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tag", default=os.environ.get("DPVO_HOT_LIB", "product"))
    args = ap.parse_args()
    import update_ops as U
    g = torch.Generator(device="cuda").manual_seed(7)
    M, dev = args.rows, "cuda"
    A = (torch.randn(M, 384, device=dev, generator=g) * 0.5).half()
    W1, b1 = U.pack_linear(torch.randn(384, 384, device=dev, generator=g) / 20.0,
                           torch.randn(384, device=dev, generator=g) * 0.1)
    W2, b2 = U.pack_linear(torch.randn(384, 384, device=dev, generator=g) / 20.0,
                           torch.randn(384, device=dev, generator=g) * 0.1)
    W1, W2 = U.kblock(W1), U.kblock(W2)
    res32 = torch.randn(M, 384, device=dev, generator=g)
    # neighbour-like gather: mostly nearby rows, some absent (-1)
    idx = torch.arange(M, device=dev) + torch.randint(-200, 200, (M,), device=dev, generator=g)
    idx = torch.where((idx < 0) | (idx >= M), torch.full_like(idx, -1), idx)
    fn = lambda: U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.RES, res32=res32,  # noqa: E731
                            want32=True)
    with torch.no_grad():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / args.reps)
        o32, o16, _ = fn()
        torch.cuda.synchronize()
    h = hashlib.sha256(o32.contiguous().view(torch.int32).cpu().numpy().tobytes())
    h.update(o16.contiguous().view(torch.int16).cpu().numpy().tobytes())
    print(json.dumps({"tag": args.tag, "rows": M, "chain_ms": [round(t, 4) for t in ts],
                      "out_sha": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
