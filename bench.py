#!/usr/bin/env python
"""bench.py — BASELINE.json metric: LDPC codeblocks/s + info-Gbit/s, BG1 Zc=384 NMS L=8.

Workload (BASELINE.json configs[2]): per GPU, a batch of 4096 BG1 Zc=384 rate-1/3 codeblocks
(K = 8448 info bits incl. CRC, N = 25344 float32 AWGN LLRs each), layered normalised min-sum
alpha=0.75, L=8.  One step = one decode launch over the whole batch, LLRs resident in HBM.
The headline runs at snr -3 dB, where no codeblock converges, so every step does all 8
iterations plus the final syndrome pass (worst case); `early_exit` repeats it at 1 dB.
Synthetic data: random info bits -> GPU encoder -> BPSK + AWGN (torch RNG) — no datasets.

Multi-GPU: one process per GPU (torch.distributed.run), each decodes its own 4096-codeblock
shard (weak scaling, no collective on the data path); timing = barrier + synchronize around
the K steps, max over ranks.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BG, ZC = 1, 384
K_INFO, N_TX, N_FULL = 22 * ZC, 66 * ZC, 68 * ZC
EDGES = 316 * ZC
DEC_BYTES_PER_CB = 4 * N_TX + N_FULL + 1 + 4       # f32 LLR in, int8 ck out, status, iters
ENC_BYTES_PER_CB = K_INFO + N_TX                     # int8 bits in, int8 dn out
HBM_PEAK_GBS = 8000.0                                # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12        # 256 CU x 4 SIMD32 x 2.4 GHz = 78.6 T/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="codeblocks per GPU")
    ap.add_argument("--schedule", default="layered", choices=["layered", "flooding"])
    ap.add_argument("--snr", type=float, default=-3.0)
    ap.add_argument("--alpha", type=float, default=0.75)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the bounded CPU-baseline sample (0 disables)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary measurements (early exit, flooding, encoder)")
    return ap.parse_args()


def make_llr(torch, enc, B, snr_db, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    ck = torch.randint(0, 2, (B, K_INFO), dtype=torch.int8, device=dev, generator=g)
    dn = enc.encode_ldpc_batch(ck, BG)
    sigma = 10 ** (-snr_db / 20)
    y = (1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device=dev, generator=g)
    llr = (2 * y / sigma ** 2).contiguous()
    del y
    return ck, dn, llr


def timed(torch, dist, world, fn, steps, warmup):
    """warmup, then exactly `steps` calls bracketed by barrier + synchronize; returns
    (max-over-ranks wall seconds, this rank's event-timed seconds)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev = e0.elapsed_time(e1) / 1e3
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, ev


def cpu_baseline(seconds, schedule, alpha, L):
    """Oracle (numpy restatement, one core) on a bounded sample of the same workload."""
    import numpy as np
    from oracle import ldpc_oracle as O
    rng = np.random.default_rng(11)
    n = 8
    ck = rng.integers(0, 2, (n, K_INFO)).astype(np.int8)
    llr = O.bpsk_awgn_llr(O.encode(ck, BG), -3.0, rng).astype(np.float32)
    fn = (lambda: O.decode_layered(llr, ZC, BG, L, alpha, 0.0)) if schedule == "layered" else \
        (lambda: O.decode_flooding(llr, ZC, BG, L, alpha, 0.0, np.float32))
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(done / el, 3), "unit": "codeblocks/s", "cores": 1, "kind": "port",
            "sample": f"{done} BG1 Zc=384 codeblocks ({n} per call), {schedule} NMS alpha={alpha} "
                      f"L={L}, snr -3 dB (all iterations), oracle/ldpc_oracle.py numpy, "
                      f"{el:.1f} s on 1 host core",
            "reference_measured_in_build_container": {
                "value": 0.073, "unit": "codeblocks/s", "cores": 1,
                "note": "py5gphy nr_decode_ldpc itself, 13.2-14.1 s per BG1 Zc=384 CB at L=8 "
                        "(BASELINE.md §2); the reference cannot travel to the GPU box"}}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from python_5gtoolbox_amd import _lib, nr_ldpc_decode as D, nr_ldpc_encode as E
    _lib.lib()

    B = args.batch
    ck, dn, llr = make_llr(torch, E, B, args.snr, 1234 + rank, dev)
    out = (torch.empty((B, N_FULL), dtype=torch.int8, device=dev),
           torch.empty((B,), dtype=torch.uint8, device=dev),
           torch.empty((B,), dtype=torch.int32, device=dev))

    def step():
        D.nr_decode_ldpc_batch(llr, ZC, BG, args.L, "min-sum", args.alpha, 0.0, args.schedule,
                               out=out)

    wall, ev = timed(torch, dist, world, step, args.steps, args.warmup)
    iters = out[2].float().mean().item()
    conv = int(out[1].sum().item())
    total_cb = B * world * args.steps
    value = total_cb / wall
    launch_s = ev / args.steps
    achieved = B * DEC_BYTES_PER_CB / launch_s / 1e9
    edge_rate = B * EDGES * iters / launch_s
    res = {
        "metric": "LDPC codeblocks/s + info-Gbit/s, BG1 Zc=384 NMS L=8, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "codeblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (random info bits -> GPU LDPC encode -> BPSK + AWGN, torch RNG)",
        "config": {"workload": f"BASELINE config 3: decode {B} codeblocks/GPU BG1 Zc=384 "
                               f"rate-1/3, {args.schedule} NMS alpha={args.alpha} L={args.L}",
                   "codeblocks_per_gpu": B, "bgn": BG, "Zc": ZC, "L": args.L,
                   "alpha": args.alpha, "beta": 0.0, "schedule": args.schedule,
                   "snr_db": args.snr, "mean_iterations": round(iters, 3),
                   "converged": conv, "parallelism": f"cb-shard x{world}"},
        "info_gbit_s": round(value * K_INFO / 1e9, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": f"ldpc_dec_kernel<1,float,{args.schedule == 'layered'}>",
                     "algorithmic_bytes_per_cb": DEC_BYTES_PER_CB,
                     "launch_ms": round(launch_s * 1e3, 4),
                     "note": "decode is VALU/LDS-bound (~99 lane-op/B); see valu"},
        "valu": {"edge_updates_per_s": round(edge_rate / 1e12, 4), "unit": "T edge-updates/s",
                 "peak_lane_ops": round(VALU_PEAK_TLANE, 1),
                 "lane_ops_per_edge_update_at_peak": round(VALU_PEAK_TLANE * 1e12 / edge_rate, 2)},
    }

    if not args.no_extras:
        ex = {}
        _, _, llr1 = make_llr(torch, E, B, 1.0, 99 + rank, dev)

        def step1():
            D.nr_decode_ldpc_batch(llr1, ZC, BG, args.L, "min-sum", args.alpha, 0.0,
                                   args.schedule, out=out)
        w1, e1 = timed(torch, dist, world, step1, max(3, args.steps // 2), 1)
        it1 = out[2].float().mean().item()
        ex["early_exit_snr1dB"] = {"codeblocks_per_s": round(B * world * max(3, args.steps // 2) / w1, 1),
                                   "mean_iterations": round(it1, 3),
                                   "converged_frac": round(out[1].float().mean().item(), 4)}
        del llr1
        other = "flooding" if args.schedule == "layered" else "layered"

        def step2():
            D.nr_decode_ldpc_batch(llr, ZC, BG, args.L, "min-sum", args.alpha, 0.0, other, out=out)
        w2, e2 = timed(torch, dist, world, step2, max(3, args.steps // 2), 1)
        ex[f"{other}_f32_snr{args.snr:g}dB"] = {
            "codeblocks_per_s": round(B * world * max(3, args.steps // 2) / w2, 1),
            "mean_iterations": round(out[2].float().mean().item(), 3)}
        # BASELINE config 2: encode-only
        dnb = torch.empty((B, N_TX), dtype=torch.int8, device=dev)

        def step3():
            E.encode_ldpc_batch(ck, BG, out=dnb)
        es = 50
        w3, e3 = timed(torch, dist, world, step3, es, 5)
        enc_launch = e3 / es
        ach = B * ENC_BYTES_PER_CB / enc_launch / 1e9
        ex["encode_config2"] = {"codeblocks_per_s": round(B * world * es / w3, 1),
                                "info_gbit_s": round(B * world * es / w3 * K_INFO / 1e9, 2),
                                "launch_ms": round(enc_launch * 1e3, 4),
                                "roofline": {"bound": "hbm", "achieved": round(ach, 1),
                                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                             "frac": round(ach / HBM_PEAK_GBS, 4),
                                             "algorithmic_bytes_per_cb": ENC_BYTES_PER_CB}}
        res["extras"] = ex

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        res["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.schedule, args.alpha, args.L)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
