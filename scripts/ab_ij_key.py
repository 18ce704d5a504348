"""A/B of DPVO._ij_groups (12-bit window key, counting sort) against the
update operator's own ii * 12345 + jj radix group-by, interleaved on one C3
steady-state tracker (update() ms, median of 5 rounds of 20)."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def main():
    from dpvo.synthetic import steady_state_tracker
    s = steady_state_tracker("dpvo_2k", buffer=2048, seed=0)
    res = {True: [], False: []}
    with torch.no_grad():
        for _ in range(3):
            s.update()
        for _ in range(5):
            for on in (True, False):
                s.cfg.WINDOW_IJ_KEY = on   # both window keys (kk and ii, jj)
                s.update()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    s.update()
                b.record()
                torch.cuda.synchronize()
                res[on].append(a.elapsed_time(b) / 20)
    print({"window_key_ms": round(statistics.median(res[True]), 4),
           "operator_key_ms": round(statistics.median(res[False]), 4)}, flush=True)


if __name__ == "__main__":
    main()
