"""Time algo='BP' (float64 sum-product) on the bench's BP shape: 1024 BG1 Zc=384 codeblocks,
L=8, -3 dB (dev tool).  LDPC5G_LIB selects the library.

    python tools/bp_probe.py [B] [snr]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    snr = float(sys.argv[2]) if len(sys.argv) > 2 else -3.0
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ck = torch.randint(0, 2, (B, 22 * 384), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (-snr / 20)
    y = (1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda", generator=g)
    llr = (2 * y / sigma ** 2).double().contiguous()
    for _ in range(2):
        out = D.nr_decode_ldpc_batch(llr, 384, 1, 8, "BP")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        out = D.nr_decode_ldpc_batch(llr, 384, 1, 8, "BP")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"BP B={B} snr={snr}: {ms:.3f} ms per call = {B / ms:.1f} k CB/s, "
          f"mean iters {out[2].float().mean().item():.2f}, converged {int(out[1].sum().item())}", flush=True)


if __name__ == "__main__":
    main()
