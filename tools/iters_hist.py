"""Iteration statistics of the layered decoder at one SNR (dev tool): mean iterations, mean of
the per-workgroup maximum (2 codeblocks per workgroup at Zc=384), histogram.
    python tools/iters_hist.py SNR_DB [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402

snr = float(sys.argv[1])
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
g = torch.Generator(device="cuda")
g.manual_seed(99)
ck = torch.randint(0, 2, (B, 22 * 384), dtype=torch.int8, device="cuda", generator=g)
dn = E.encode_ldpc_batch(ck, 1)
sigma = 10 ** (-snr / 20)
llr = (2 * ((1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda", generator=g)) / sigma ** 2)
_, st, it = D.nr_decode_ldpc_batch(llr.contiguous(), 384, 1, 8, "min-sum", 0.75, 0.0, "layered")
it = it.long().cpu()
pm = it.view(-1, 2).max(dim=1).values.float().mean().item()
print(f"snr {snr} dB: mean iters {it.float().mean().item():.3f}, mean per-workgroup max {pm:.3f}, "
      f"converged {st.float().mean().item():.4f}, hist {torch.bincount(it, minlength=9).tolist()}")
