"""Print the top kernels of a rocprofv3 --stats run: name, calls, average us, share."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in list(csv.DictReader(open(f)))[:n]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):6.2f}%")
