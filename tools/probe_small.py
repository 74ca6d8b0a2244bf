"""Small-codeblock decode latency probe (development tool): one BG2 Zc=8 codeblock (BASELINE
config 1) and a few other small lifting sizes, float64 flooding NMS alpha=0.75 L=8, event-timed
per call on the device (no host copies): the product path (nr_decode_ldpc_batch) beside the
sparse CSR/CSC kernel on the same expanded graph; decisions compared.

    python tools/probe_small.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402
from python_5gtoolbox_amd.ldpc_info import code_dims  # noqa: E402


def timeit(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for bg, Zc, B, snr in [(2, 8, 1, 1.0), (2, 8, 1, -3.0), (1, 8, 1, -3.0), (2, 16, 1, -3.0),
                           (2, 64, 1, -3.0), (2, 8, 8, -3.0), (1, 64, 1, -3.0), (1, 128, 1, -3.0),
                           (1, 384, 1, -3.0), (1, 384, 1, 1.0), (2, 384, 1, -3.0), (1, 384, 4, -3.0)]:
        K, N, Nf = code_dims(bg, Zc)
        ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
        dn = E.encode_ldpc_batch(ck, bg)
        sigma = 10 ** (-snr / 20)
        llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                                  generator=g)) / sigma ** 2).contiguous()
        out = (torch.empty((B, Nf), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
               torch.empty((B,), dtype=torch.int32, device="cuda"))
        us = timeit(lambda: D.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, "flooding", out=out))
        full = torch.zeros((B, Nf), dtype=torch.float64, device="cuda")
        full[:, 2 * Zc:] = llr
        sg = D.SparseGraph.from_base_graph(bg, Zc, "cuda")
        out2 = (torch.empty((B, Nf), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
                torch.empty((B,), dtype=torch.int32, device="cuda"))
        us2 = timeit(lambda: D.decode_ldpc_batch(full, sg, 8, "min-sum", 0.75, 0.0, out=out2))
        same = torch.equal(out[0], out2[0]) and torch.equal(out[1], out2[1])
        print(f"BG{bg} Zc={Zc} B={B} snr {snr}: product {us:.1f} us/call, sparse {us2:.1f} us/call, "
              f"iters {out[2].float().mean().item():.2f}, same={same}", flush=True)


if __name__ == "__main__":
    main()
