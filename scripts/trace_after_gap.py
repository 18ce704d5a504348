"""Per-replay GPU busy time from a rocprofv3 kernel trace: the kernels after
the last idle gap over 0.3 s (prof_encoder.py sleeps before its replays), divided by
the replay count.  usage: trace_after_gap.py run_kernel_trace.csv 20"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
big = [k for k, g in enumerate(gaps) if g > 300e6]   # the last idle gap over 0.3 s (the script's sleep)
i = (big[-1] if big else max(range(len(gaps)), key=gaps.__getitem__)) + 1
seg = rows[i:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
span = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
print(f"kernels per replay {len(seg) / n:.1f}, GPU busy {busy / n / 1e3:.1f} us, span {span / n / 1e3:.1f} us per replay")
