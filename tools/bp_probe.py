"""BP / BF decode timing probe (development tool, not the bench contract): 1024 BG1 Zc=384
codeblocks at -3 dB, L=8, HIP events, plus the VALU counter pass target for rocprofv3.

    python tools/bp_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402


def main():
    B, Zc = 1024, 384
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ck = torch.randint(0, 2, (B, 22 * Zc), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (3 / 20)
    llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, device="cuda", dtype=torch.float64,
                                                              generator=g)) / sigma ** 2).contiguous()
    for algo in ("BP", "BF"):
        fn = lambda: D.nr_decode_ldpc_batch(llr, Zc, 1, 8, algo)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f"{algo}: {ms:.3f} ms per {B} codeblocks = {B / ms * 1e3 / 1e3:.1f} k CB/s", flush=True)


if __name__ == "__main__":
    main()
