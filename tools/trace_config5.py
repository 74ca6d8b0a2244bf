"""Config 5 alone (dev tool, GPU): the PDSCH 256QAM TB stream of bench.py (TX and RX chains,
32 TBs x 129 codeblocks), for a per-kernel rocprofv3 breakdown of the receive chain:

    rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -o run -- python tools/trace_config5.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from python_5gtoolbox_amd import _lib  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _lib.lib()
    print(json.dumps(bench.bench_config5(torch, dist, 1, dev, 0, 5)))
