#!/bin/bash
# rocprofv3 kernel stats of a short script (default: native encoders x 20);
# prints the per-kernel averages of kernels matching $KPAT.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
S=${SCRIPT:-scripts/prof_encoder.py}
T=${TAG:-enc}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_$T -o run -- python $R/$S > $R/gpurun_out/prof_$T.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R; f=$(find gpurun_out/prof_$T -name "*kernel_stats.csv" | head -1)
python - "$f" "${KPAT:-enc_}" <<'PY'
import csv, sys
tot = 0
for r in csv.DictReader(open(sys.argv[1])):
    tot += float(r["TotalDurationNs"])
    if sys.argv[2] in r["Name"]:
        print(r["Name"][:100], r["Calls"], r["AverageNs"])
print(f"all kernels: {tot / 1e3:.1f} us in total")
PY
