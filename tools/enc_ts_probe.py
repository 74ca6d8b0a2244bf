"""Encoder phase timing (development tool): with a library built with -DLDPC5G_ENC_TS (LDPC5G_LIB=...),
every codeblock's workgroup writes its phase timestamps over the first 64 output bytes; prints the
mean phase durations, the per-codeblock lifetime and the launch's concurrency profile.

    python tools/enc_ts_probe.py [B]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_encode as E  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K, N = 22 * 384, 66 * 384
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda")
    dn = torch.empty((B, N), dtype=torch.int8, device="cuda")
    for _ in range(5):
        E.encode_ldpc_batch(ck, 1, out=dn)
    torch.cuda.synchronize()
    raw = dn[:, :72].cpu().numpy().copy().view(np.int64).reshape(B, 9)
    ts = raw[:, :8].astype(np.float64) / 100.0  # us
    cu = raw[:, 8]
    t0 = ts[:, 0].min()
    ts -= t0
    names = ["loads+pack", "sync1", "X ext", "recursion", "core parity", "ext rows", "drain"]
    d = np.diff(ts, axis=1)
    print(f"B={B}: launch span {ts[:, 7].max():.1f} us; per-codeblock lifetime mean {np.mean(ts[:, 7] - ts[:, 0]):.2f} us "
          f"(p10 {np.percentile(ts[:, 7] - ts[:, 0], 10):.2f}, p90 {np.percentile(ts[:, 7] - ts[:, 0], 90):.2f})")
    for i, n in enumerate(names):
        print(f"  {n:>12}: mean {d[:, i].mean():6.2f} us  p90 {np.percentile(d[:, i], 90):6.2f}")
    # most workgroups resident together on one CU (by __smid), over the launch
    t0s, t1s = ts[:, 0] - ts[:, 0].min(), ts[:, 7] - ts[:, 0].min()
    peak = []
    for c in np.unique(cu):
        m = cu == c
        ev = sorted([(a, 1) for a in t0s[m]] + [(b, -1) for b in t1s[m]], key=lambda x: (x[0], x[1]))
        cur = best = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
        peak.append(best)
    print(f"  CUs seen {len(peak)}, resident workgroups per CU: max {max(peak)}, median {int(np.median(peak))}, min {min(peak)}")
    for q in (0.1, 0.25, 0.5, 0.75, 0.9, 1.0):
        t = ts[:, 7].max() * q
        live = np.sum((ts[:, 0] <= t) & (ts[:, 7] >= t))
        print(f"  at {q:4.2f} of the span: {live} codeblocks in flight ({live / 256:.1f} per CU)")


if __name__ == "__main__":
    main()
