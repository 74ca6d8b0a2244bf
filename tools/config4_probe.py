"""BASELINE config 4 alone (bench.bench_config4, one GPU), printing its JSON block (dev tool; run
under rocprofv3 --kernel-trace to see the per-kernel timeline of the timed step)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from python_5gtoolbox_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _lib.lib()
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    r = bench.bench_config4(torch, None, 1, dev, 0, steps)
    print(json.dumps(r, indent=1), flush=True)


if __name__ == "__main__":
    main()
