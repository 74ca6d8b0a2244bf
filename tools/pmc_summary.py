"""Per-kernel PMC summary from the rocprofv3 --pmc passes of tools/gpu_round.sh.

    python tools/pmc_summary.py gpurun_out/<tag>  > pmc_summary.json

For every kernel: dispatch count, mean duration, and the mean per-dispatch value of every counter
collected (one counter set per pass; passes are separate runs of the same command).  HBM bytes
per launch = FETCH_SIZE + WRITE_SIZE (both reported in KiB).  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE under-reports 16-B/lane streaming reads by exactly 2x on gfx950 (the encoder's input
loads), WRITE_SIZE is exact for 16-B stores; other access widths are uncalibrated, so both the raw
sum and the 16-B-corrected figure are given.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("ldpc5g_impl::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                key = (k, r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                durs[k][(p, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        e = {"dispatches": max(len(v) for v in cs.values()),
             "mean_duration_ns": round(sum(durs[k].values()) / max(len(durs[k]), 1), 1)}
        for c, v in sorted(cs.items()):
            e[c] = sum(v) / len(v)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_raw"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            e["hbm_bytes_fetch16_corrected"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        out[k] = e
    # the format bench.py reads (profiles/pmc_latest.json): {"source": ..., "kernels": {name: ...}}
    json.dump({"source": f"{d} (tools/gpu_round.sh pmc passes -> tools/pmc_summary.py)", "kernels": out},
              sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
