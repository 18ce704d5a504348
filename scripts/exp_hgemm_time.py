"""SoftAgg's h Linear on the groups (dpvo_rowgemm with a device row count:
G rows of an upper bound E) at C3's shape, HIP events over back-to-back
launches -- for A/B runs of experiment builds (DPVO_HOT_LIB=... DPVO_DIAG=1).

  python scripts/exp_hgemm_time.py [--rows 95424] [--groups 4416,600] [--tag name]
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
    ap.add_argument("--groups", default="4416,600")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tag", default=os.environ.get("DPVO_HOT_LIB", "product"))
    args = ap.parse_args()
    import update_ops as U
    g = torch.Generator(device="cuda").manual_seed(13)
    E, dev = args.rows, "cuda"
    W, b = U.pack_linear(torch.randn(384, 384, device=dev, generator=g) / 20.0,
                         torch.randn(384, device=dev, generator=g) * 0.1)
    W = U.kblock(W)
    y = (torch.randn(E, 384, device=dev, generator=g) * 0.5).half()
    res, h = {}, hashlib.sha256()
    with torch.no_grad():
        for G in (int(x) for x in args.groups.split(",")):
            Gd = torch.tensor([G], dtype=torch.int64, device=dev)
            out = torch.zeros(E, 384, dtype=torch.float16, device=dev)
            fn = lambda: U.rowgemm(y, W, b, M_dev=Gd, out16=out)  # noqa: E731
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    fn()
                z.record()
                torch.cuda.synchronize()
                ts.append(round(a.elapsed_time(z) / args.reps * 1000, 2))
            res[f"G{G}_us"] = ts
            h.update(out[:G].contiguous().view(torch.int16).cpu().numpy().tobytes())
    print(json.dumps({"tag": args.tag, **res, "out_sha": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
