"""Config-4 decode split by (BG, Zc) group (development tool): bench.bench_config4's 12 groups,
each decoded alone through MixedBatch (layered OMS beta=0.5, L=8, rate-matched), event-timed, with
its lane-op fraction on the algorithmic count, beside the whole mixed batch.

    python tools/c4_groups_probe.py [f64]

f64: the reference-precision plan instead (float64 rows, float64 flooding OMS beta=0.5).
Per group also the workgroups of its plan and their CU time (workgroups x time when they all fit
on the GPU at once: a lower bound on what the group costs inside the mixed plan).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from python_5gtoolbox_amd.ldpc_info import code_dims  # noqa: E402
from python_5gtoolbox_amd.nr_ldpc_decode_mixed import MixedBatch  # noqa: E402
from python_5gtoolbox_amd.sch import SchRaterecoverPlan, cfg_from_codeblocks, sch_ratematch_batch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(404)
    g = torch.Generator(device=dev)
    g.manual_seed(404)
    n_per, snr = 341, 1.0
    cfgs, llrs, meta = [], [], []
    for Zc in (12, 40, 72, 176, 208, 384):
        for bg in (1, 2):
            K, N, _ = code_dims(bg, Zc)
            Qm = int(rng.choice([2, 4, 6, 8]))
            rv = int(rng.integers(0, 4))
            E = Qm * int(rng.integers(-(-K // Qm), int(1.6 * N) // Qm + 1))
            cfg = cfg_from_codeblocks(n_per, K, K, Zc, bg, Qm, n_per * E, 1, rv)
            ck = torch.randint(0, 2, (n_per, K), dtype=torch.int8, device=dev, generator=g)
            gs = sch_ratematch_batch(ck, cfg, 1)
            sigma = 10 ** (-snr / 20)
            y = (1 - 2 * gs.float()) + sigma * torch.randn(gs.shape, device=dev, generator=g)
            llrs.append((2 * y / sigma ** 2).reshape(-1))
            cfgs.append(cfg)
            meta.append((bg, Zc, K, N, E))
    rrp = SchRaterecoverPlan(cfgs, dev)
    lay = rrp.lay
    llr = torch.zeros((len(cfgs), lay["max_E"]), dtype=torch.float32, device=dev)
    for t_, x in enumerate(llrs):
        llr[t_, :x.numel()] = x
    f64 = "f64" in sys.argv[1:]
    dt = torch.float64 if f64 else torch.float32
    sched = "flooding" if f64 else "layered"
    dn = rrp(llr, torch.empty((lay["dn"],), dtype=dt, device=dev))
    groups = [(bg, Zc, dn[r[2]:r[2] + r[1] * N].view(r[1], N)) for (bg, Zc, K, N, E), r in zip(meta, lay["rows"])]
    tot = cu_tot = 0.0
    for (bg, Zc, K, N, E), grp in zip(meta, groups):
        mb = MixedBatch([grp])
        ms = bench.ev_ms(torch, lambda: mb.decode(8, 1.0, 0.5, sched, True), reps=10)
        _, st, it = mb.decode(8, 1.0, 0.5, sched, True)
        nwg = _nwg(mb, sched)
        edges = int(it.sum().item()) * sum(bench._ROW_DEG[bg]) * Zc
        frac = edges * 13 / (ms * 1e-3) / 78.6e12
        tot += ms
        cu_us = nwg * ms * 1e3 if nwg <= 256 else 256 * ms * 1e3
        cu_tot += cu_us
        print(f"BG{bg} Zc={Zc:3d} E/N={E / N:.2f}: {ms * 1e3:7.1f} us  mean it {it.float().mean().item():.2f}  "
              f"max it {int(it.max().item())}  alg frac {frac:.3f}  ({n_per / ms * 1e3 / 1e6:.2f} M CB/s)  "
              f"{nwg} wg  {cu_us:8.0f} CU-us", flush=True)
    mb = MixedBatch(groups, flat=dn)
    ms = bench.ev_ms(torch, lambda: mb.decode(8, 1.0, 0.5, sched, True), reps=10)
    print(f"sum of groups alone {tot * 1e3:.1f} us; CU time {cu_tot:.0f} CU-us = {cu_tot / 256:.1f} us on 256 CUs; "
          f"all groups in one plan {ms * 1e3:.1f} us")


def _nwg(mb, sched):
    """workgroups of the plan (its header: magic, schedule, nw1, nw2, ...)"""
    host = mb._plans[sched][0]
    hdr = host[:24].cpu().numpy().view(np.int32)
    return int(hdr[2] + hdr[3])


if __name__ == "__main__":
    main()
