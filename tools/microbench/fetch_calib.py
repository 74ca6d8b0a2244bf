"""FETCH_SIZE / WRITE_SIZE per byte moved, by access width, from the rocprofv3 --pmc passes over
tools/microbench/fetch_calib (tools/gpu_round.sh calib).  Each kernel moves exactly 1 GiB.

    python tools/microbench/fetch_calib.py gpurun_out/<tag>   > fetch_calib.json
"""
import csv
import glob
import json
import os
import sys

BYTES = 1 << 30


def per_kernel(d, counter):
    out = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                name = r["Kernel_Name"]
                key = (name, r["Dispatch_Id"])
                out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    return out


def width(name):
    if "B16" in name:
        return 16
    if "B8" in name:
        return 8
    return 4


def main(d):
    res = {"bytes_per_kernel": BYTES, "fetch_size_bytes_per_byte": {}, "write_size_bytes_per_byte": {},
           "source": f"{d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over tools/microbench/fetch_calib "
                     "(1 GiB streamed per kernel with W-byte lane accesses, W = 4 / 8 / 16)"}
    for counter, kind, key in (("FETCH_SIZE", "rd_kernel", "fetch_size_bytes_per_byte"),
                               ("WRITE_SIZE", "wr_kernel", "write_size_bytes_per_byte")):
        for (name, _), v in per_kernel(os.path.join(d, "calib_fetch" if counter == "FETCH_SIZE" else "calib_write"),
                                       counter).items():
            if kind in name:
                res[key][str(width(name))] = round(v * 1024 / BYTES, 4)   # counters are in KiB
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
