"""Per-workgroup phase timing of the layered decoder (dev tool): run with
LDPC5G_LIB=build/alt/lay_ts.so (or flood_ts.so; tools/ab/make_variants.py), which writes 7
real-time clock stamps (100 MHz) per workgroup into the first 56 bytes of its first ck row.

    LDPC5G_LIB=build/alt/lay_ts.so python tools/ts_probe.py layered 4096 [L]
    LDPC5G_LIB=build/alt/flood_ts.so python tools/ts_probe.py flooding64 4096 [L]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402


def main():
    what = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    sched, G = ("layered", 2) if what == "layered" else ("flooding", 1)
    Zc, K, N, NF = 384, 22 * 384, 66 * 384, 68 * 384
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (3 / 20)
    llr = 2 * ((1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda", generator=g)) / sigma ** 2
    if what == "flooding64":
        llr = llr.double()
    out = (torch.empty((B, NF), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
           torch.empty((B,), dtype=torch.int32, device="cuda"))
    for _ in range(3):
        D.nr_decode_ldpc_batch(llr, Zc, 1, L, "min-sum", 0.75, 0.0, sched, out=out)
    torch.cuda.synchronize()
    ts = out[0][::G, :56].contiguous().cpu().numpy().view(np.uint64).astype(np.int64)   # [nwg, 7]
    ts = ts[:, [0, 6, 1, 2, 3, 4, 5]]
    d = np.diff(ts, axis=1) * 10e-3   # us
    names = ["prologue loads", "prologue rest", "iteration 1", f"iterations 2..{L}", "final syndrome", "ck store"]
    tot = (ts[:, 6] - ts[:, 0]) * 10e-3
    span = (ts[:, 6].max() - ts[:, 0].min()) * 10e-3
    print(f"{what} B={B} L={L}: {len(ts)} workgroups, launch span {span:.1f} us, per-WG total mean {tot.mean():.2f} us")
    for k, n in enumerate(names):
        print(f"  {n:18s} mean {d[:, k].mean():8.2f} us  min {d[:, k].min():8.2f}  max {d[:, k].max():8.2f}")
    # gaps between consecutive workgroups on a CU are not visible here; idle = span * CUs - sum
    cus = 256
    print(f"  sum of WG times / (span x {cus} CUs) = {tot.sum() / (span * cus):.3f}")


if __name__ == "__main__":
    main()
