"""Latency probe of the multi-workgroup float64 flooding kernel (ldpc5g_dec_split.hip; development
tool): one (or a few) BG1 Zc=384 codeblocks, NMS alpha=0.75 L=8, event-timed per call.  With a
library built with -DLDPC5G_SPLIT_TS (LDPC5G_LIB=...), also prints workgroup 0's phase timestamps
(us since kernel start).

    python tools/split_probe.py [B] [snr_dB] [bg] [Zc]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402
from python_5gtoolbox_amd.ldpc_info import code_dims  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    snr = float(sys.argv[2]) if len(sys.argv) > 2 else -3.0
    bg = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    Zc = int(sys.argv[4]) if len(sys.argv) > 4 else 384
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    K, N, Nf = code_dims(bg, Zc)
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, bg)
    sigma = 10 ** (-snr / 20)
    llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                              generator=g)) / sigma ** 2).contiguous()
    out = (torch.empty((B, Nf), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
           torch.empty((B,), dtype=torch.int32, device="cuda"))
    fn = lambda: D.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, "flooding", out=out)  # noqa: E731
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"BG{bg} Zc={Zc} B={B} snr {snr}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us/call, "
          f"iters {out[2].float().mean().item():.2f}", flush=True)
    ts = out[0][0, :128].cpu().numpy().view(np.uint64).astype(np.int64)
    if ts[1] > ts[0] > 0:
        names = ["start", "prologue+bar", "A0", "barA0", "B0", "barB0", "A1", "barA1", "B1", "barB1",
                 "loop end", "final pass", "final bar", "end"]
        prev = ts[0]
        for i, n in enumerate(names):
            if ts[i] == 0:
                continue
            print(f"  {n:>13}: {(ts[i] - ts[0]) / 100:8.2f} us  (+{(ts[i] - prev) / 100:.2f})")
            prev = ts[i]


if __name__ == "__main__":
    main()
