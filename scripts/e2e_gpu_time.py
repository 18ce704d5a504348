"""End-to-end frames vs their GPU time: run bench.py's
end_to_end loop (C3, keep / drop alternating) with a 0.5 s idle gap before the
timed frames, under rocprofv3 --kernel-trace; then

    python scripts/e2e_gpu_time.py run                     # (inside rocprofv3)
    python scripts/e2e_gpu_time.py report <kernel_trace.csv> <frames> <wall json>

reports the GPU busy time per timed frame (sum of kernel durations after the
gap: one stream, so they do not overlap) beside the wall-clock ms per frame."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]


def run(defer=True, frames=32):
    import torch
    import bench
    with torch.no_grad():
        r = bench.end_to_end(bench.CONFIGS["C3"], 2048, 2, frames, device="cuda", defer=defer, mark_gap=0.5)
    print(json.dumps(r), flush=True)


def report(trace, frames, wall):
    import csv
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
    i = max(k for k, g in enumerate(gaps) if g > 300e6) + 1
    seg = rows[i:]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / frames / 1e6
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / frames / 1e6
    w = json.load(open(wall))
    print(json.dumps({"frames": frames, "gpu_busy_ms_per_frame": round(busy, 3),
                      "trace_span_ms_per_frame": round(span, 3), "kernels_per_frame": round(len(seg) / frames, 1),
                      "wall_ms_per_frame": w["ms_per_frame"], "deferred_keyframe": w["deferred_keyframe"],
                      "wall_over_gpu": round(w["ms_per_frame"] / busy, 3)}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(defer=os.environ.get("DEFER", "1") == "1")
    else:
        report(sys.argv[2], int(sys.argv[3]), sys.argv[4])
