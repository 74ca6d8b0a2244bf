"""Per-kernel summary (calls, total/avg/min/max duration in ns) from a rocprofv3 output:
either the rocpd SQLite database (ROCm 7.2 default) or a --output-format csv kernel trace.

    python tools/rocpd_summary.py gpurun_out/<tag>/prof [--skip N] > profiles/rNN/<name>_kernel_stats.csv

--skip N drops the first N dispatches of every kernel (in start-time order): the bench's warmup
launches, so a kernel's average is over the timed launches only.
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    n = name.replace("ldpc5g_impl::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0] if n.startswith("void ") or "<" in n else n


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select k.display_name, d.\"end\" - d.start, d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol k on d.kernel_id = k.id").fetchall()
    return rows


def from_csv(path):
    with open(path) as f:
        return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                 int(r["Start_Timestamp"])) for r in csv.DictReader(f)]


def main(d, skip=0):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        rows += from_db(p)
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += from_csv(p)
    agg = defaultdict(list)
    for n, t, _ in sorted(rows, key=lambda r: r[2]):
        agg[short(n)].append(t)
    agg = {n: v[skip:] for n, v in agg.items() if len(v) > skip}
    tot = sum(sum(v) for v in agg.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([n, len(v), sum(v), round(sum(v) / len(v), 1), round(100 * sum(v) / tot, 3),
                    min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0)
