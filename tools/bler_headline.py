"""BLER / iteration characterisation of the headline configuration (dev tool, GPU): BG1 Zc=384,
NMS alpha=0.75, L=8, codeblocks from the batched for_test_5g_ldpc_encoder (sim_ldpc.gen_codeblocks:
CRC24A-terminated info bits, BPSK + AWGN at the reference's SNR definition).  The same LLRs go
through the layered float32 kernel (the headline), the flooding float32 kernel and the float64
flooding kernel (the reference's arithmetic); a fixed number of codeblocks per point (no stopping
rule), so the three columns share their trials.

    python tools/bler_headline.py [n_per_point]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd.nr_ldpc_decode import nr_decode_ldpc_batch  # noqa: E402
from python_5gtoolbox_amd.sim_ldpc import gen_codeblocks  # noqa: E402

ZC, BG, ALPHA, L = 384, 1, 0.75, 8
K = 22 * ZC


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2026)
    print(f"BG{BG} Zc={ZC} NMS alpha={ALPHA} L={L}, {n} codeblocks per SNR point")
    print(f"{'snr_db':>7} | {'BLER layered f32':>16} {'iters':>5} | {'BLER flood f32':>14} {'iters':>5} | "
          f"{'BLER flood f64':>14} {'iters':>5}")
    for snr in [-1.5, -1.25, -1.0, -0.75, -0.5, -0.25, 0.0, 0.25, 0.5, 1.0]:
        res = {k: [0, 0.0] for k in ("lay", "f32", "f64")}
        done = 0
        while done < n:
            b = min(10000, n - done)
            blk, llr = gen_codeblocks(ZC, BG, snr, "24A", b, gen, dev)
            for key, x, sch in (("lay", llr.float(), "layered"), ("f32", llr.float(), "flooding"),
                                ("f64", llr, "flooding")):
                ck, st, it = nr_decode_ldpc_batch(x, ZC, BG, L, "min-sum", ALPHA, 0.0, sch)
                res[key][0] += int((ck[:, :K] != blk).any(dim=1).sum().item())
                res[key][1] += float(it.float().sum().item())
            done += b
        row = " | ".join(f"{res[k][0] / n:16.5f} {res[k][1] / n:5.2f}" if k == "lay" else
                         f"{res[k][0] / n:14.5f} {res[k][1] / n:5.2f}" for k in ("lay", "f32", "f64"))
        print(f"{snr:7.2f} | {row}", flush=True)


if __name__ == "__main__":
    main()
