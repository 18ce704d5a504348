"""Reduce rocprofv3 --pmc passes over `bench.py` (C3) to profiles/counters_c3.json,
the counter record bench.py's roofline objects read.

  python scripts/counters_json.py <pmc_dir> <edges> [out.json]

<pmc_dir> holds one sub-directory per pass (scripts/gpu_pmc.sh layout: p1, p2,
...), each with rocprofv3's *counter_collection.csv.  Passes must include
FETCH_SIZE and WRITE_SIZE (separate passes: TCC slots) and may include
TA_BUSY_avr + GRBM_GUI_ACTIVE.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) counts
16-B/lane streaming reads at half their bytes -> x 2; WRITE_SIZE (KB) is exact.
Both are the L2's memory-side counters (Infinity-Cache hits included).

Records, per kernel: dispatches, bytes per dispatch; and the two groups the
bench line uses:
  corr      = edge_hist + edge_scatter + corr_mfma (one altcorr phase per update)
  update_op = rowgemm (incl. the narrow GEMM) / rowpair / rowchain / rowadd_ln /
              sa_reduce / nb_csr kernels,
              bytes per update() (total / corr_mfma dispatches: every update,
              and every phase_breakdown repetition, runs altcorr once)
plus the sha of the HIP sources (bench.py uses the record only when they match).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

CORR = re.compile(r"corr_mfma_kernel|edge_hist_kernel|edge_scatter_kernel")
UPD = re.compile(r"rowgemm\w*_kernel|rowpair\d?_kernel|rowchain\d?_kernel|rowadd_ln_kernel|sa_reduce_csr|nb_csr_kernel")


def short(name):
    return re.sub(r"\(.*$", "", name.replace("void ", "").replace("dpvo::", "").replace("(anonymous namespace)::", ""))


def read(pmc_dir):
    """kernel -> counter -> {dispatch id: value}"""
    out = defaultdict(lambda: defaultdict(dict))
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = out[k][r["Counter_Name"]]
            key = (f, r["Dispatch_Id"])
            d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
    return out


def main():
    pmc_dir, edges = sys.argv[1], int(sys.argv[2])
    out_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "profiles", "counters_c3.json")
    data = read(pmc_dir)
    kern = {}
    for k, cs in data.items():
        rec = {}
        if "FETCH_SIZE" in cs:
            v = list(cs["FETCH_SIZE"].values())
            rec["dispatches"] = len(v)
            rec["fetch_bytes"] = sum(v) / len(v) * 1024 * 2
            rec["fetch_total"] = sum(v) * 1024 * 2
        if "WRITE_SIZE" in cs:
            v = list(cs["WRITE_SIZE"].values())
            rec["write_bytes"] = sum(v) / len(v) * 1024
            rec["write_total"] = sum(v) * 1024
        if "TA_BUSY_avr" in cs and "GRBM_GUI_ACTIVE" in cs:
            ta = sum(cs["TA_BUSY_avr"].values()) / len(cs["TA_BUSY_avr"])
            gr = sum(cs["GRBM_GUI_ACTIVE"].values()) / len(cs["GRBM_GUI_ACTIVE"])
            rec["ta_busy_avr"] = ta
            rec["grbm_gui_active"] = gr
            rec["ta_busy_frac"] = ta / (gr / 8.0)   # GRBM counts per XCD, summed over the 8 XCDs
        if rec:
            kern[k] = rec
    corr_k = {k: v for k, v in kern.items() if CORR.search(k)}
    upd_k = {k: v for k, v in kern.items() if UPD.search(k)}
    mf = [v for k, v in corr_k.items() if "corr_mfma_kernel" in k]
    if not mf or "fetch_bytes" not in mf[0] or "write_bytes" not in mf[0]:
        raise SystemExit("no FETCH_SIZE / WRITE_SIZE rows for corr_mfma_kernel")
    updates = mf[0]["dispatches"]
    corr_bytes = sum(v.get("fetch_total", 0) + v.get("write_total", 0) for v in corr_k.values()) / updates
    upd_bytes = sum(v.get("fetch_total", 0) + v.get("write_total", 0) for v in upd_k.values()) / updates
    import bench
    res = {
        "edges": edges,
        "sha": {"corr": bench.source_sha(*bench.CORR_SOURCES), "update_op": bench.source_sha(*bench.UPD_SOURCES)},
        "updates_profiled": updates,
        "corr": {"hbm_bytes_per_launch": round(corr_bytes),
                 "kernel_bytes": round(mf[0]["fetch_bytes"] + mf[0]["write_bytes"]),
                 "ta_busy_frac": round(mf[0]["ta_busy_frac"], 4) if "ta_busy_frac" in mf[0] else None,
                 "kernels": sorted(corr_k)},
        "update_op": {"hbm_bytes_per_update": round(upd_bytes), "kernels": sorted(upd_k)},
        "per_kernel": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                       for k, v in sorted(kern.items())},
        "note": "rocprofv3 --pmc, one pass per counter group; FETCH_SIZE x 2 (gfx950), WRITE_SIZE exact; "
                "L2 memory-side counters (Infinity-Cache hits included); corr = per altcorr phase, "
                "update_op = per update()",
    }
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("edges", "sha", "corr", "update_op")}, indent=1))


if __name__ == "__main__":
    main()
