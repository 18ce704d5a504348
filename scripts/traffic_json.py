"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the fused altcorr
kernel to profiles/altcorr_traffic.json (HBM-side bytes per launch).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) counts
wide streaming reads at half their bytes -> x2; WRITE_SIZE (KB) is exact.
Both are L2 memory-side counters: Infinity-Cache hits are included.

  python scripts/traffic_json.py <fetch_dir> <write_dir> <edges> [out.json]
"""
import csv
import glob
import json
import os
import re
import sys

KERNEL = re.compile(os.environ.get("KREGEX", r"corr_mfma_kernel|corr_s?fast_kernel<2"))


NAMES = set()


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and KERNEL.search(r["Kernel_Name"]):
                NAMES.add(r["Kernel_Name"].split("(")[0])
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for the altcorr kernel under {d}")
    return sorted(vals.values())


def main():
    fetch_dir, write_dir, edges = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                               "altcorr_traffic.json")
    fk = per_dispatch(fetch_dir, "FETCH_SIZE")
    wk = per_dispatch(write_dir, "WRITE_SIZE")
    med = lambda v: v[len(v) // 2]
    fetch = med(fk) * 1024 * 2      # KB -> B, gfx950 x2 for 16-B/lane streaming reads
    write = med(wk) * 1024
    res = {"kernel": " / ".join(sorted(NAMES)), "edges": edges, "fetch_bytes": round(fetch),
           "write_bytes": round(write), "hbm_bytes_per_launch": round(fetch + write),
           "bytes_per_edge": round((fetch + write) / edges, 1), "dispatches": [len(fk), len(wk)],
           "note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; FETCH x2 (gfx950); "
                   "L2 memory-side counters, Infinity-Cache hits included"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
