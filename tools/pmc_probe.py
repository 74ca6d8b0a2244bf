"""PMC driver (development tool, not the bench contract): each kernel the bench's roofline lines
read counters of, launched a few times on the bench's shapes, so one rocprofv3 --pmc pass per
counter set covers them all quickly (tools/gpu_round.sh pmc):
    f64 frame kernel (4096 x BG1 Zc=384, -3 dB, L=8; config 3's headline), layered f32 (perf mode),
    encoder (4096; config 2), BF and BP (1024 codeblocks, float64, L=8).
    python tools/pmc_probe.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B, ZC = 4096, 384
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    ck = torch.randint(0, 2, (B, 22 * ZC), dtype=torch.int8, device="cuda", generator=g)
    dn = torch.empty((B, 66 * ZC), dtype=torch.int8, device="cuda")
    sigma = 10 ** (3 / 20)
    E.encode_ldpc_batch(ck, 1, out=dn)
    llr = (2 * ((1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda", generator=g)) / sigma ** 2)
    llr64 = llr.double()
    out = (torch.empty((B, 68 * ZC), dtype=torch.int8, device="cuda"),
           torch.empty((B,), dtype=torch.uint8, device="cuda"), torch.empty((B,), dtype=torch.int32, device="cuda"))
    for _ in range(reps):
        E.encode_ldpc_batch(ck, 1, out=dn)
        D.nr_decode_ldpc_batch(llr64, ZC, 1, 8, "min-sum", 0.75, 0.0, "flooding", out=out)
        D.nr_decode_ldpc_batch(llr, ZC, 1, 8, "min-sum", 0.75, 0.0, "layered", out=out)
        for algo in ("BF", "BP"):
            D.nr_decode_ldpc_batch(llr64[:1024], ZC, 1, 8, algo, 1.0, 0.0)
    torch.cuda.synchronize()
    print("pmc_probe done", flush=True)


if __name__ == "__main__":
    main()
