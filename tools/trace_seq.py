"""Print the kernel sequence (duration, gap) around the last occurrences of a kernel in a rocprofv3
kernel trace (dev tool):  python tools/trace_seq.py gpurun_out/<tag>/prof/run_kernel_trace.csv demod 12"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
prev = None
for r in rows[max(0, i0 - 2):i0 + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'][:70]:70s} dur={(e - s) / 1e3:9.1f}us gap={gap:8.1f}us grid={r['Grid_Size_X']}")
    prev = e
