"""Average each PMC counter per dispatch over the passes under a gpu_pmc.sh output dir."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{sys.argv[1]}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:96]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
