#!/usr/bin/env python
"""bench.py — BASELINE.json metric: LDPC codeblocks/s + info-Gbit/s, BG1 Zc=384 NMS L=8.

Workload (BASELINE.json configs[2]): per GPU, a batch of 4096 BG1 Zc=384 rate-1/3 codeblocks
(K = 8448 info bits incl. CRC, N = 25344 AWGN LLRs each), normalised min-sum alpha=0.75, L=8.
One step = one decode launch over the whole batch, LLRs resident in HBM.  The headline (top-level
`value`) decodes in the reference's own schedule and arithmetic: float64 flooding, bit-identical to
py5gphy nr_decode_ldpc (float32 LLRs widened to float64).  `perf_mode` is the same workload through
the float32 layered kernel (the schedule BASELINE's wording names, not the reference's).
Both run at snr -3 dB, where no codeblock converges, so every step does all 8 iterations plus the
final syndrome pass (worst case); `early_exit_*` repeat it at 1 dB.
Synthetic data: random info bits -> GPU encoder -> BPSK + AWGN (torch RNG) — no datasets.

Multi-GPU: one process per GPU (torch.distributed.run, or `--gpus N` alone, which starts the N
rank processes itself), each decodes its own 4096-codeblock shard (weak scaling, no collective on
the data path); timing = barrier + synchronize around the K steps, max over ranks.  Rank 0 prints
ONE JSON line.
"""
import argparse
import json
import math
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
DEC64_BYTES_PER_CB = 8 * N_TX + N_FULL + 1 + 4       # f64 LLR in, int8 ck out, status, iters
HBM_PEAK_GBS = 8000.0                                # MI355X_MICROARCH.md chip table (spec)
# rocprofv3 PMC summary of this code version (tools/gpu_round.sh pmc step -> tools/pmc_summary.py),
# committed: FETCH_SIZE / WRITE_SIZE per launch cannot be collected inside the timed run.
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")
# exact kernel names as rocprofv3 reports them for the 4096-codeblock BG1 Zc=384 launches (the
# flooding kernel's 4th/5th template arguments are its plan: 2 parts x 384 slots; the last one of
# both kernels is DEAD, the LDPC5G_RATE_MATCHED variant, false for the headline; then the
# compile-time lifting size, 384 for the Zc = 384 kernels, 0 for the runtime-Zc ones)
DEC_KERNEL = {"layered": "void ldpc_dec_kernel_l<1, float, true, false, false, 384>",
              "flooding": "void ldpc_flood_kernel<1, float, false, 2, 384, false, 384>"}
# the float64 Zc = 384 batches run the frame kernel (ldpc5g_dec_frame.h: <BG, OFS, DEAD>)
DEC64_KERNEL = "void ldpc_frame_kernel<1, false, false>"
BP_KERNEL = "void ldpc_bp_kernel<1>"
BF_KERNEL = "void ldpc_bf_kernel<1, double>"
ENC_KERNEL = "void ldpc_enc_fast_kernel<1, true>"


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary, or None: 2 x FETCH_SIZE +
    WRITE_SIZE.  The factor is calibrated on this GPU (profiles/r06/fetch_calib.json,
    tools/microbench/fetch_calib.hip): streaming 1 GiB with 4-, 8- and 16-B lane loads reports
    FETCH_SIZE = 0.50 of the bytes for all three widths, and W-byte stores WRITE_SIZE = 1.00 of them
    (MI355X_MICROARCH.md §HBM had calibrated only the 16-B read)."""
    e = pmc_entry(kernel)
    if e is None:
        return None
    try:
        return int(e["hbm_bytes_fetch16_corrected"])
    except (KeyError, ValueError, TypeError):
        return None


def pmc_entry(kernel):
    """The committed PMC summary of exactly this kernel (no fuzzy match: a renamed or re-templated
    kernel reports None until its counters are collected again)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        return d.get("kernels", d)[kernel]   # (a bare per-kernel dict is accepted too)
    except (OSError, KeyError, ValueError, AttributeError):
        return None


VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12        # 256 CU x 4 SIMD32 x 2.4 GHz = 78.6 T/s
ALG_OPS_PER_EDGE = 13                                # lane-ops per edge-update


def pmc_valu_insts(kernel):
    """VALU wave-instructions per launch of `kernel` (4096-codeblock batch) from the committed PMC
    summary (SQ_INSTS_VALU), or None."""
    e = pmc_entry(kernel)
    try:
        return float(e["SQ_INSTS_VALU"]) if e else None
    except (KeyError, ValueError, TypeError):
        return None


def valu_block(edge_rate, launch_s, kernel, B):
    """The decoder's binding resource: VALU issue.  Measured lane-ops/s = SQ_INSTS_VALU per launch
    (committed PMC summary of the same kernel) x 64 lanes / this run's launch time, against the
    full-rate peak (every lane of every SIMD32 issuing each cycle; min/max/med3, compares and
    SGPR-operand ops issue at half that rate, tools/microbench/valu_rates.hip)."""
    v = {"edge_updates_per_s": round(edge_rate / 1e12, 4), "unit": "T edge-updates/s",
         "peak_lane_ops": round(VALU_PEAK_TLANE, 1),
         "lane_ops_per_edge_update_at_peak": round(VALU_PEAK_TLANE * 1e12 / edge_rate, 2)}
    insts = pmc_valu_insts(kernel) if B == 4096 else None
    if insts:
        lane_ops = insts * 64 / launch_s / 1e12
        v.update({"measured_lane_ops": round(lane_ops, 2), "measured_unit": "T lane-op/s",
                  "frac_of_full_rate_peak": round(lane_ops / VALU_PEAK_TLANE, 4),
                  "valu_insts_per_edge_update": round(insts * 64 / (edge_rate * launch_s), 2),
                  "source": "SQ_INSTS_VALU per launch, profiles/pmc_latest.json"})
    return v


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="codeblocks per GPU")
    ap.add_argument("--headline", default="reference", choices=["reference", "layered"],
                    help="top-level line: the float64 flooding decode (bit-identical to the "
                         "reference, default) or the float32 layered perf kernel")
    ap.add_argument("--snr", type=float, default=-3.0)
    ap.add_argument("--alpha", type=float, default=0.75)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the bounded CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU-baseline processes (default: min(16, os.cpu_count()), the box's "
                         "CPU share per GPU)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse the "
                         "multi-rank control flow with several ranks on one GPU)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary measurements (early exit, flooding, encoder)")
    ap.add_argument("--no-perf", action="store_true",
                    help="time only the --headline line (skip the other schedule's config-3 line)")
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
        t = torch.tensor([wall], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, ev


def _cpu_worker(job):
    """One host process of the CPU baseline: the oracle (numpy) decoding 8-codeblock batches of
    the headline workload until `seconds` have passed.  schedule "flooding64" is the reference's
    own algorithm and arithmetic (float64 flooding, nr_ldpc_decode.py:51-143)."""
    seconds, schedule, alpha, L, seed = job
    import numpy as np
    from oracle import ldpc_oracle as O
    rng = np.random.default_rng(seed)
    n = 8
    ck = rng.integers(0, 2, (n, K_INFO)).astype(np.int8)
    llr = O.bpsk_awgn_llr(O.encode(ck, BG), -3.0, rng).astype(np.float32)
    if schedule == "layered":
        fn = lambda: O.decode_layered(llr, ZC, BG, L, alpha, 0.0)   # noqa: E731
    elif schedule == "flooding64":
        llr64 = llr.astype(np.float64)
        fn = lambda: O.decode_flooding(llr64, ZC, BG, L, alpha, 0.0, np.float64)   # noqa: E731
    else:
        fn = lambda: O.decode_flooding(llr, ZC, BG, L, alpha, 0.0, np.float32)   # noqa: E731
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += n
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def host_info():
    """The host the CPU baseline runs on: CPU model, physical cores (sockets x cores per socket
    from /proc/cpuinfo), logical CPUs, and the CPUs this process may run on."""
    import platform
    model, phys = platform.processor() or platform.machine(), set()
    try:
        pid = core = None
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name":
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    core = v
                elif not k and pid is not None:
                    phys.add((pid, core))
                    pid = core = None
            if pid is not None:
                phys.add((pid, core))
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count()
    return {"model": model, "physical_cores": len(phys) or None, "logical_cpus": os.cpu_count(),
            "affinity_cpus": aff}


def _host_cpu():
    h = host_info()
    return (f"host {h['model']}, {h['physical_cores']} physical cores / {h['logical_cpus']} logical "
            f"CPUs ({h['affinity_cpus']} in this process's affinity)")


def cpu_baseline(seconds, schedule, alpha, L, procs):
    """Oracle (numpy restatement, kind "port") on a bounded sample of the same workload, one
    process per host core up to `procs`.  Runs before this process touches
    the GPU, so the spawned workers never inherit a GPU context.  `procs` defaults to the GPU
    box's CPU share per GPU (16): the pool allots that many host CPUs to a one-GPU job although
    os.cpu_count() shows the whole machine, so the whole-host figure is reported as a per-core
    extrapolation (the workers share nothing, so the rate scales with cores), not measured."""
    import multiprocessing as mp
    jobs = [(seconds, schedule, alpha, L, 11 + i) for i in range(procs)]
    if procs == 1:
        res = [_cpu_worker(jobs[0])]
    else:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, jobs)
    done = sum(d for d, _ in res)
    el = max(e for _, e in res)
    h = host_info()
    what = {"layered": "layered float32", "flooding": "flooding float32",
            "flooding64": "flooding float64 (the reference's algorithm and arithmetic)"}[schedule]
    per_core = done / el / procs
    return {"value": round(done / el, 3), "unit": "codeblocks/s", "cores": procs, "kind": "port",
            "sample": f"{done} BG1 Zc=384 codeblocks (8 per call) over {procs} processes, "
                      f"{what} NMS alpha={alpha} L={L}, snr -3 dB (all iterations), "
                      f"oracle/ldpc_oracle.py numpy, {el:.1f} s; {_host_cpu()}",
            "host": h, "per_core": round(per_core, 3),
            "all_physical_cores_extrapolated": (round(per_core * h["physical_cores"], 1)
                                                if h["physical_cores"] else None),
            "reference_measured_in_build_container": {
                "value": 0.073, "unit": "codeblocks/s", "cores": 1,
                "note": "py5gphy nr_decode_ldpc itself, 13.2-14.1 s per BG1 Zc=384 CB at L=8 "
                        "(BASELINE.md §2); the reference cannot travel to the GPU box"}}


def bench_config1(rank, n=300):
    """BASELINE config 1 shape on the GPU: ONE BG2 Zc=8 codeblock per call through the
    reference-style drop-ins (numpy in / numpy out, as scripts/internal/sim_ldpc_internal.py:51-58
    calls them): us per encode_ldpc and per nr_decode_ldpc (float64 flooding, NMS alpha=.75,
    L=8), host round trip included.  The reference itself: 1.2-2.2 ms per encode, 30-57 ms per
    decode on one core."""
    import numpy as np
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    rng = np.random.default_rng(7 + rank)
    ck = rng.integers(0, 2, 80).astype(np.int8)
    llr = 2 * ((1 - 2 * E.encode_ldpc(ck.copy(), 2)) + 0.8 * rng.normal(size=400)) / 0.64
    for _ in range(20):
        E.encode_ldpc(ck.copy(), 2)
        D.nr_decode_ldpc(llr, 8, 2, 8, "min-sum", 0.75, 0)
    t0 = time.perf_counter()
    for _ in range(n):
        E.encode_ldpc(ck.copy(), 2)
    t1 = time.perf_counter()
    for _ in range(n):
        D.nr_decode_ldpc(llr, 8, 2, 8, "min-sum", 0.75, 0)
    t2 = time.perf_counter()
    return {"workload": "BASELINE config 1: single BG2 Zc=8 codeblock per call, drop-in API",
            "encode_us_per_call": round((t1 - t0) / n * 1e6, 1),
            "decode_us_per_call": round((t2 - t1) / n * 1e6, 1), "calls": n,
            "reference_cpu_ms_per_call": {"encode": "1.2-2.2", "decode": "30-57"}}


def bench_dlsch_caller(rank, reps=5):
    """Per-codeblock drop-in latency in the reference's own caller shape: DLSCHDecode's loop over
    the C codeblocks of one TB (/root/reference/py5gphy/nr_pdsch/nr_dlsch_decode.py:62-103: rate
    recovery, nr_decode_ldpc, CB CRC per codeblock, then the TB CRC) restated here over this
    package's drop-ins — what a user gets who swaps only the py5gphy.ldpc / crc modules ("codec-only
    swap") — beside the module swap, where DLSCHDecode itself is the drop-in that runs the whole TB
    through the GPU chain in one call.  TB: A = 193,728 bits, C = 23 BG1 Zc=384 codeblocks, 256QAM,
    2 layers, R = 700/1024, G = 278,016, float64 flooding NMS alpha=0.75 L=8, 30 dB BPSK LLRs."""
    import numpy as np
    from python_5gtoolbox_amd import crc, ldpc_info, nr_dlsch, nr_dlsch_decode, nr_ldpc_decode, \
        nr_ldpc_ratematch, nr_ldpc_raterecover
    A, Qm, R, NL, rv, LBRM, G = 193728, 8, 700, 2, 0, 1081512, 278016
    dec = {"L": 8, "algo": "min-sum", "alpha": 0.75, "beta": 0.0}
    rng = np.random.default_rng(11 + rank)
    tb = rng.integers(0, 2, A).astype(np.int8)
    g = nr_dlsch.DLSCHEncode(tb, A, Qm, R, NL, rv, LBRM, G)
    llr = (1 - 2 * g.astype(np.float64)) * 20.0 + rng.normal(0, 0.5, G)

    def codec_only():   # nr_dlsch_decode.py:16-106 with the codec modules swapped
        B, poly = A + 24, "24A"
        bgn = 1
        C, cbz, Lc, F, K, Zc = ldpc_info.get_cbs_info(B, bgn)
        K_apo = cbz + Lc
        N = 66 * Zc
        Ncb = min(N, math.floor(LBRM / (C * 2 / 3)))
        k0 = nr_ldpc_ratematch.get_k0(Ncb, bgn, rv, Zc)
        Er = nr_ldpc_ratematch.get_Er_ldpc(G, C, Qm, NL)
        tbb = np.zeros(B)
        to = go = 0
        for c in range(C):
            E = Er[c]
            dn = nr_ldpc_raterecover.raterecover_ldpc(llr[go:go + E], Ncb, N, k0, Qm, Zc, K_apo, K)
            go += E
            blkandcrc, ck, status = nr_ldpc_decode.nr_decode_ldpc(dn, Zc, bgn, dec["L"], dec["algo"],
                                                                  dec["alpha"], dec["beta"])
            cbblk, err = crc.nr_crc_decode(blkandcrc[0:K_apo], "24B")
            tbb[to:to + cbz] = cbblk
            to += cbz
        blk, e = crc.nr_crc_decode(tbb.astype(np.int8), poly)
        return e == 0, blk

    def module_swap():
        ok, blk, _ = nr_dlsch_decode.DLSCHDecode(llr, A, Qm, R, NL, rv, LBRM, dec)
        return ok, blk

    res = {}
    for name, fn in (("codec_only_swap", codec_only), ("module_swap", module_swap)):
        ok, blk = fn()
        res[name + "_tb_bits_match"] = bool(ok and np.array_equal(np.asarray(blk, np.int8), tb))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        res[name + "_ms_per_tb"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
    return {"workload": "one 23-codeblock DL-SCH TB (BG1 Zc=384) through DLSCHDecode's per-codeblock "
                        "loop (nr_dlsch_decode.py:62-103) with only the codec swapped, vs DLSCHDecode "
                        "swapped (whole TB on the GPU in one call); float64 flooding, host arrays in/out",
            **res, "codeblocks_per_tb": 23,
            "codec_only_ms_per_codeblock": round(res["codec_only_swap_ms_per_tb"] / 23, 3)}


def bench_single_cb(torch, rank):
    """One large codeblock per call (the per-codeblock drop-ins' shape at Zc=384, DLSCHDecode's
    loop): float64 flooding NMS alpha=0.75 L=8 at -3 dB (all 8 iterations run), the multi-workgroup
    kernel (ldpc5g_dec_split.hip: one codeblock over 18 CUs for BG1).  Device-resident call
    (nr_decode_ldpc_batch, event-timed on the stream, scratch allocation included) and the numpy
    drop-in nr_decode_ldpc (host wall, host<->device copies included)."""
    import numpy as np
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    from python_5gtoolbox_amd.ldpc_info import code_dims
    res = {"workload": "one BG1/BG2 Zc=384 codeblock per call, float64 flooding NMS alpha=0.75 L=8, -3 dB"}
    g = torch.Generator(device="cuda")
    g.manual_seed(5 + rank)
    for bg in (1, 2):
        Zc = 384
        K, N, Nf = code_dims(bg, Zc)
        ck = torch.randint(0, 2, (1, K), dtype=torch.int8, device="cuda", generator=g)
        dn = E.encode_ldpc_batch(ck, bg)
        sigma = 10 ** (3 / 20)
        llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                                  generator=g)) / sigma ** 2).contiguous()
        out = (torch.empty((1, Nf), dtype=torch.int8, device="cuda"), torch.empty((1,), dtype=torch.uint8, device="cuda"),
               torch.empty((1,), dtype=torch.int32, device="cuda"))
        fn = lambda: D.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, "flooding", out=out)  # noqa: E731
        for _ in range(10):
            fn()
        us = ev_ms(torch, fn, reps=200) * 1e3
        x = llr[0].cpu().numpy()
        for _ in range(5):
            D.nr_decode_ldpc(x, Zc, bg, 8, "min-sum", 0.75, 0.0)
        t0 = time.perf_counter()
        for _ in range(50):
            D.nr_decode_ldpc(x, Zc, bg, 8, "min-sum", 0.75, 0.0)
        host_us = (time.perf_counter() - t0) / 50 * 1e6
        res[f"bg{bg}"] = {"device_us_per_call": round(us, 1), "dropin_host_us_per_call": round(host_us, 1),
                          "iterations": int(out[2].item())}
    # a whole BG1 transport block of 23 Zc=384 codeblocks in one call (DLSCHDecode swapped whole, or
    # sch_decode_batch): the multi-workgroup kernel with two chunks per wave, 207 workgroups; beside
    # it the one-workgroup-per-codeblock batch kernel's time for the same call is ~220 us
    B, Zc = 23, 384
    K, N, Nf = code_dims(1, Zc)
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (3 / 20)
    llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                              generator=g)) / sigma ** 2).contiguous()
    out = (torch.empty((B, Nf), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
           torch.empty((B,), dtype=torch.int32, device="cuda"))
    fn = lambda: D.nr_decode_ldpc_batch(llr, Zc, 1, 8, "min-sum", 0.75, 0.0, "flooding", out=out)  # noqa: E731
    for _ in range(10):
        fn()
    us = ev_ms(torch, fn, reps=200) * 1e3
    res["bg1_tb23"] = {"device_us_per_call": round(us, 1), "codeblocks": B,
                       "max_iterations": int(out[2].max().item())}
    return res


def ev_ms(torch, fn, reps=5):
    """Event-timed milliseconds per call of fn (one untimed call first), on torch's current
    stream — the stream the library launches on."""
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def hbm_line(alg_bytes, ms):
    """Algorithmic-byte roofline of one kernel call: bytes it must move / its event time."""
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    return {"ms": round(ms, 4), "algorithmic_bytes": int(alg_bytes), "achieved_GBps": round(gbs, 1),
            "peak_GBps": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4), "bound": "hbm"}


def valu_line(edges, ms):
    """Lane-op roofline of a decode call: 13 lane-ops per edge-update."""
    t = edges * ALG_OPS_PER_EDGE / (ms * 1e-3) / 1e12
    return {"ms": round(ms, 4), "edge_updates": int(edges), "achieved": round(t, 3),
            "peak": round(VALU_PEAK_TLANE, 1), "unit": "T lane-op/s",
            "frac": round(t / VALU_PEAK_TLANE, 4), "bound": "valu"}


def _config4_groups(rng):
    """BASELINE config 4's 12 (Zc, BG) groups with their random (Qm, rv, E in [K, 1.6N])."""
    from python_5gtoolbox_amd.ldpc_info import code_dims
    out = []
    for Zc in (12, 40, 72, 176, 208, 384):
        for bg in (1, 2):
            K, N, _ = code_dims(bg, Zc)
            Qm = int(rng.choice([2, 4, 6, 8]))
            rv = int(rng.integers(0, 4))
            E = Qm * int(rng.integers(-(-K // Qm), int(1.6 * N) // Qm + 1))
            out.append((bg, Zc, K, N, Qm, rv, E))
    return out


C4_N_PER, C4_SNR, C4_SEED = 341, 1.0, 404


def _c4_executed(its, dnh, meta, rows, Gw_of):
    """(algorithmic, executed) edge-updates of a config-4 decode and the per-codeblock iterations
    its workgroups run: the plan's workgroups (per (bgn, Zc) group a partial workgroup of n % G
    codeblocks first, then full ones of G = Gw_of(Zc) — ldpc5g_capi.hip build_plan)."""
    import numpy as np
    alg_edges = exe_edges = wg_iters = 0
    cb0 = 0
    for (bg, Zc, K, N), r in zip(meta, rows):
        n = r[1]
        Gw = Gw_of(Zc)
        rows_cb = dnh[r[2]:r[2] + n * N].reshape(n, N)
        # extension column c of the transmitted row layout: columns 2..(N/Zc+1) of the full graph;
        # ext row i (>= 4) <-> full column KB + i <-> transmitted column KB + i - 2
        kb = 22 if bg == 1 else 10
        mb_rows = 46 if bg == 1 else 42
        live_col = np.abs(rows_cb.reshape(n, N // Zc, Zc)).max(axis=2) != 0   # (n, N/Zc)
        row_deg = _ROW_DEG[bg]
        starts = [0] + list(range(n % Gw, n, Gw)) if n % Gw else list(range(0, n, Gw))
        bounds = starts + [n]
        for w0, w1 in zip(bounds[:-1], bounds[1:]):
            if w1 <= w0:
                continue
            live = np.ones(mb_rows, bool)
            lc = live_col[w0:w1].any(axis=0)
            for i in range(4, mb_rows):
                live[i] = lc[kb + i - 2]
            e_live = int(sum(row_deg[i] for i in range(mb_rows) if live[i]))
            exe_edges += int(its[cb0 + w0:cb0 + w1].max()) * (w1 - w0) * e_live * Zc
            wg_iters += int(its[cb0 + w0:cb0 + w1].max()) * (w1 - w0)
        alg_edges += int(its[cb0:cb0 + n].sum()) * sum(row_deg) * Zc
        cb0 += n
    return alg_edges, exe_edges, wg_iters


def _cpu_worker_c4(job):
    """One host process of config 4's reference-precision CPU baseline: the oracle's float64 rate
    recovery (raterecover, nr_ldpc_raterecover.py:6-65) + float64 flooding OMS beta=0.5 L=8
    (decode_ldpc, nr_ldpc_decode.py:51-143) over `n` codeblocks of each of the 12 groups, repeated
    until `seconds` have passed."""
    seconds, seed, n = job
    import numpy as np
    from oracle import ldpc_oracle as O
    rng = np.random.default_rng(C4_SEED)   # the GPU line's groups (rank 0)
    groups = _config4_groups(rng)
    rng = np.random.default_rng(seed)
    work = []
    for bg, Zc, K, N, Qm, rv, E in groups:
        k0 = O.get_k0(N, bg, rv, Zc)
        ck = rng.integers(0, 2, (n, K)).astype(np.int8)
        dn = O.encode(ck, bg)
        sigma = 10 ** (-C4_SNR / 20)
        fe = [2 * ((1 - 2 * O.ratematch(d, N, E, k0, Qm).astype(np.float64)) + sigma * rng.normal(size=E)) / sigma ** 2
              for d in dn]
        work.append((bg, Zc, K, N, Qm, k0, fe))
    done, t0 = 0, time.perf_counter()
    while True:
        for bg, Zc, K, N, Qm, k0, fe in work:
            rows = np.stack([O.raterecover(x, N, N, k0, Qm, Zc, K, K) for x in fe])
            O.decode_flooding(rows, Zc, bg, 8, 1.0, 0.5, np.float64)
            done += len(fe)
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def cpu_baseline_c4(seconds, procs, n=2):
    """config 4 at the reference's precision on the host (kind "port"), procs processes."""
    import multiprocessing as mp
    jobs = [(seconds, 41 + i, n) for i in range(procs)]
    if procs == 1:
        res = [_cpu_worker_c4(jobs[0])]
    else:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker_c4, jobs)
    done = sum(d for d, _ in res)
    el = max(e for _, e in res)
    return {"value": round(done / el, 3), "unit": "codeblocks/s", "cores": procs, "kind": "port",
            "sample": f"{done} codeblocks ({n} of each of the 12 (Zc, BG) groups per round) over "
                      f"{procs} processes: oracle float64 raterecover + float64 flooding OMS "
                      f"beta=0.5 L=8 (the reference's algorithm and arithmetic), {el:.1f} s; "
                      f"{_host_cpu()}"}


def bench_config4(torch, dist, world, dev, rank, steps, cpu_c4=None):
    """BASELINE config 4: mixed-Zc batch {12,40,72,176,208,384} x BG1/BG2, 341 codeblocks per
    (Zc, BG) = 4092, each group rate-matched with its own random (Qm, rv, E in [K, 1.6N]) on the
    GPU chain (encode -> rate match -> BPSK+AWGN), OMS beta=0.5, L=8.  The timed step is the
    receive side: the 12 groups' rate recovery in ONE launch (ldpc5g_sch_raterecover_multi_plan,
    per-group geometry uploaded once) + the mixed-Zc decode (ldpc5g_decode_ms_mixed_plan, plan
    built once).  Two lines: the float32 layered perf kernel (top level), and
    `reference_precision`: the reference's own arithmetic — float64 LLRs rate-recovered into
    float64 rows (nr_ldpc_raterecover.py:62) and decoded by float64 flooding (nr_dlsch_decode.py:91
    -> nr_ldpc_decode.py:51-143), bit-identical to it, with a same-algorithm CPU baseline.  Each
    decode's lane-op roofline is reported twice: on the algorithmic count (all rows x each
    codeblock's iterations) and on the work the kernel executes (live rows only — a row whose
    extension column was never transmitted is skipped — x the iterations of the slowest codeblock
    of each workgroup, which every codeblock packed into that workgroup runs)."""
    import numpy as np
    from python_5gtoolbox_amd.nr_ldpc_decode_mixed import MixedBatch
    from python_5gtoolbox_amd.sch import SchRaterecoverPlan, cfg_from_codeblocks, sch_ratematch_batch
    rng = np.random.default_rng(C4_SEED + rank)
    g = torch.Generator(device=dev)
    g.manual_seed(C4_SEED + rank)
    n_per, snr = C4_N_PER, C4_SNR
    cfgs, llrs, info_bits, meta = [], [], 0, []
    ebytes = nbytes = 0
    for bg, Zc, K, N, Qm, rv, E in _config4_groups(rng):
        cfg = cfg_from_codeblocks(n_per, K, K, Zc, bg, Qm, n_per * E, 1, rv)
        ck = torch.randint(0, 2, (n_per, K), dtype=torch.int8, device=dev, generator=g)
        gs = sch_ratematch_batch(ck, cfg, 1)
        sigma = 10 ** (-snr / 20)
        y = (1 - 2 * gs.float()) + sigma * torch.randn(gs.shape, device=dev, generator=g)
        llrs.append((2 * y / sigma ** 2).reshape(-1))
        cfgs.append(cfg)
        ebytes += n_per * E
        nbytes += n_per * N
        meta.append((bg, Zc, K, N))
        info_bits += n_per * K
    rrp = SchRaterecoverPlan(cfgs, dev)   # geometry validated and uploaded once
    lay = rrp.lay
    llr = torch.zeros((len(cfgs), lay["max_E"]), dtype=torch.float32, device=dev)
    for t_, x in enumerate(llrs):
        llr[t_, :x.numel()] = x
    del llrs

    def line(dt, schedule, Gw_of):
        x = llr if dt == torch.float32 else llr.to(dt)
        dn = rrp(x, torch.empty((lay["dn"],), dtype=dt, device=dev))
        groups = [(bg, Zc, dn[r[2]:r[2] + r[1] * N].view(r[1], N))
                  for (bg, Zc, K, N), r in zip(meta, lay["rows"])]
        mb = MixedBatch(groups, flat=dn)
        B = mb.B

        def step():   # rate recovery (one launch) + decode (<= 3 launches), all on the GPU
            rrp(x, dn)
            mb.decode(8, 1.0, 0.5, schedule, True)
        wall, ev = timed(torch, dist, world, step, steps, 2)
        _, st, it = mb.decode(8, 1.0, 0.5, schedule, True)
        rr_ms = ev_ms(torch, lambda: rrp(x, dn))
        dec_ms = ev_ms(torch, lambda: mb.decode(8, 1.0, 0.5, schedule, True))
        its = it.cpu().numpy().astype(np.int64)
        alg_edges, exe_edges, wg_iters = _c4_executed(its, dn.cpu().numpy(), meta, lay["rows"], Gw_of)
        dec_alg = valu_line(alg_edges, dec_ms)
        dec_exe = valu_line(exe_edges, dec_ms)
        es = x.element_size()
        return {"codeblocks_per_gpu": B, "codeblocks_per_s": round(B * world * steps / wall, 1),
                "info_gbit_s": round(info_bits * world * steps / wall / 1e9, 3),
                "ms_per_step": round(wall / steps * 1e3, 4),
                "mean_iterations": round(float(its.mean()), 3),
                "converged_frac": round(st.float().mean().item(), 4),
                "kernels": {
                    "decode": {**dec_alg, "frac_executed": dec_exe["frac"],
                               "achieved_executed": dec_exe["achieved"], "edge_updates_executed": exe_edges,
                               "iterations_run_per_codeblock": round(wg_iters / max(B, 1), 3),
                               "note": "frac: 13 lane-ops x (every row's edges x each codeblock's "
                                       "iterations); frac_executed: the same over the work the kernel "
                                       "runs — live rows only x the slowest codeblock's iterations of "
                                       "each workgroup, for every codeblock packed in it"},
                    "raterecover": {**hbm_line(es * (ebytes + nbytes), rr_ms),
                                    "note": f"all 12 groups in ONE launch ({x.dtype} in, {x.dtype} rows "
                                            f"out: {es}E + {es}N bytes per codeblock), inside the timed step"}}}
    perf = line(torch.float32, "layered", lambda Zc: 768 // Zc)
    ref = line(torch.float64, "flooding", lambda Zc: max(1, 384 // Zc))
    ref.update({"dtype": "f64", "schedule": "flooding",
                "what": "float64 LLRs -> float64 rate recovery (one launch) -> float64 flooding OMS "
                        "beta=0.5 L=8 (LDPC5G_RATE_MATCHED): the reference's own arithmetic "
                        "(DLSCHDecode: nr_dlsch_decode.py:62-91), bit-identical to it",
                "cpu_baseline": cpu_c4})
    if cpu_c4:
        ref["vs_cpu_baseline"] = round(ref["codeblocks_per_s"] / cpu_c4["value"], 1)
    return {"workload": "BASELINE config 4: 12 (Zc, BG) groups x 341 CBs, random (Qm, rv, E), "
                        "GPU rate match, snr 1 dB, timed step = rate recovery (one launch) + "
                        "layered OMS beta=0.5 L=8 decode (LDPC5G_RATE_MATCHED); float32 perf mode",
            "dtype": "f32", "schedule": "layered", **perf, "reference_precision": ref}


# base-graph row degrees (TS 38.212 Tables 5.3.2-2/-3: edges per base row)
_ROW_DEG = {1: [19, 19, 19, 19, 3, 8, 9, 7, 10, 9, 7, 8, 7, 6, 7, 7, 6, 6, 6, 6, 6, 6, 5, 5, 6, 5, 5, 4, 5,
                5, 5, 5, 5, 5, 5, 5, 5, 4, 5, 5, 4, 5, 4, 5, 5, 4],
            2: [8, 10, 8, 10, 4, 6, 6, 6, 4, 5, 5, 5, 4, 5, 5, 4, 5, 5, 4, 4, 4, 4, 3, 4, 4, 3, 5, 3, 4,
                3, 5, 3, 4, 4, 4, 4, 4, 3, 4, 4, 4, 4]}


C5 = dict(A=1081512, Qm=8, R=948, NL=4, rv=0, G=8 * 4 * 36036)


def _cpu_worker_c5(job):
    """One host process of config 5's reference-precision CPU baseline: the oracle DL-SCH receive
    chain at 30 dB — 256QAM soft demodulation of complex128 symbols (float32 LLRs, as
    nr_Demodulation.py returns them) + descrambling, float64 rate recovery of the 129 codeblocks,
    float64 flooding NMS alpha=0.75 L=8, TB reassembly + CRCs — on one transport block, repeated
    until `seconds` have passed."""
    seconds, seed = job
    import numpy as np
    from oracle import ldpc_oracle as O
    rng = np.random.default_rng(seed)
    c = C5
    p = O.sch_params(c["A"], c["Qm"], c["R"], c["NL"], c["rv"], c["A"], c["G"])
    tb = rng.integers(0, 2, c["A"]).astype(np.int8)
    cinit = 7 + seed
    g = O.sch_encode(tb, c["A"], c["Qm"], c["R"], c["NL"], c["rv"], c["A"], c["G"])
    sym = O.modulate(g ^ O.prbs(cinit, g.size), c["Qm"]).astype(np.complex128)
    nvar = 10 ** (-30.0 / 10)
    y = sym + (rng.normal(size=sym.size) + 1j * rng.normal(size=sym.size)) * (nvar / 2) ** 0.5
    nv = np.full(sym.size, nvar, np.float32)
    done, ok, t0 = 0, 0, time.perf_counter()
    while True:
        llr = O.descramble(O.demodulate(y, nv, c["Qm"]), cinit)
        rows = O.sch_raterecover(llr, p)
        ck, _, _ = O.decode_flooding(rows, p["Zc"], p["bgn"], 8, 0.75, 0.0, np.float64)
        tb_ok, blk, _ = O.sch_tb_check(ck, p)
        done += 1
        ok += bool(tb_ok) and np.array_equal(blk[:c["A"]], tb)
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el, ok


def cpu_baseline_c5(seconds, procs):
    """config 5 at the reference's precision on the host (kind "port"), procs processes."""
    import multiprocessing as mp
    jobs = [(seconds, 51 + i) for i in range(procs)]
    if procs == 1:
        res = [_cpu_worker_c5(jobs[0])]
    else:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker_c5, jobs)
    done = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    return {"value": round(done / el, 4), "unit": "TB/s", "cores": procs, "kind": "port",
            "codeblocks_per_s": round(done * 129 / el, 2),
            "tb_crc_ok": f"{sum(r[2] for r in res)}/{done}",
            "sample": f"{done} transport blocks (TBS {C5['A']}, 129 BG1 Zc=384 codeblocks, 256QAM, "
                      f"30 dB) over {procs} processes: oracle demodulation (complex128 -> float32 "
                      f"LLRs) + descrambling + float64 rate recovery + float64 flooding NMS "
                      f"alpha=0.75 L=8 + TB CRC (the reference's algorithm and arithmetic), "
                      f"{el:.1f} s; {_host_cpu()}"}


def bench_config5(torch, dist, world, dev, rank, steps, T=32, cpu_c5=None):
    """BASELINE config 5: PDSCH 273 PRB 256QAM MCS27 4 layers TB stream (TBS 1,081,512 ->
    129 BG1 Zc=384 codeblocks per TB, G = 8*4*36036), T TBs per GPU, every step on the GPU:
    TX = ldpc5g_sch_encode + scrambling/256QAM mapping; RX = soft demodulation/descrambling +
    ldpc5g_sch_decode (rate recovery, decode, CB/TB CRCs).  Two RX lines: the perf mode (complex64
    symbols, float32 rate recovery, layered NMS L=8: the top level) and `reference_precision`
    (DLSCHDecode's own arithmetic: complex128 symbols demodulated to float32 LLRs as
    nr_Demodulation.py does, float64 rate recovery, float64 flooding NMS L=8 — bit-identical to
    it), each with a per-kernel split.  Channel: complex AWGN on the symbols (outside the timed
    regions), at 30 dB (easy: ~3 iterations) and at each line's threshold point (the highest SNR of
    a list at which that line's decoder needs >= 6 mean iterations, the same SNR on every rank),
    each with its TB CRC pass rate; per-kernel split + rooflines at the threshold."""
    from python_5gtoolbox_amd import phy
    from python_5gtoolbox_amd.nr_ldpc_decode import nr_decode_ldpc_batch
    from python_5gtoolbox_amd.sch import SchWorkspace, sch_config, sch_decode_batch, \
        sch_encode_batch, sch_raterecover_batch, sch_tb_check_batch
    from python_5gtoolbox_amd.shard import decode_tbs_sharded
    A, Qm, R, NL, rv, G = (C5[k] for k in ("A", "Qm", "R", "NL", "rv", "G"))
    cfg = sch_config(A, Qm, R, NL, rv, A, G)
    g = torch.Generator(device=dev)
    g.manual_seed(505 + rank)
    tb = torch.randint(0, 2, (T, A), dtype=torch.int8, device=dev, generator=g)
    cinit = (torch.arange(T, device=dev, dtype=torch.int64) + 1000 * rank) * 2 ** 15 + 7
    ws = SchWorkspace(cfg, T, dev)
    sym = torch.empty((T, G // Qm), dtype=torch.complex64, device=dev)

    def tx():
        bits = sch_encode_batch(tb, cfg, ws)
        phy.scramble_modulate(bits, Qm, cinit, out=sym)
    wt, _ = timed(torch, dist, world, tx, steps, 2)
    tx()
    llr = torch.empty((T, G), dtype=torch.float32, device=dev)
    cur = {}

    def channel(snr):
        nvar = 10 ** (-snr / 10)
        noise = torch.complex(torch.randn(sym.shape, device=dev, generator=g),
                              torch.randn(sym.shape, device=dev, generator=g)) * (nvar / 2) ** 0.5
        cur["y"] = (sym + noise).contiguous()
        cur["y128"] = cur["y"].to(torch.complex128)
        del noise
        cur["nv"] = torch.full(sym.shape, nvar, dtype=torch.float32, device=dev)

    last = {}
    MODES = {"perf": ("y", "layered", torch.float32), "ref": ("y128", "flooding", torch.float64)}

    def rx_local(y_local, mode):
        _, sched, dnt = MODES[mode]
        phy.demod_descramble(y_local, cur["nv"], Qm, cinit, out=llr)
        r = sch_decode_batch(llr, cfg, 8, "min-sum", 0.75, 0.0, sched, dn_dtype=dnt, ws=ws)
        last["r"] = r
        return r.tb_ok, r.tbblk
    tm = {}
    gather = world == 1 or dist.get_backend() == "nccl"   # gloo cannot gather device tensors

    def rx(mode):
        # this rank's TBs (round robin over T*world) -> records -> ONE RCCL gather to rank 0
        y = cur[MODES[mode][0]]
        if gather:
            return decode_tbs_sharded(y, cfg, 8, T_total=T * world,
                                      decode_fn=lambda yl: rx_local(yl, mode), timing=tm)
        return rx_local(y, mode)

    def rx_line(snr, mode="perf"):
        channel(snr)
        wr, _ = timed(torch, dist, world, lambda: rx(mode), steps, 2)
        res = rx(mode)
        r = last["r"]
        ok = r.tb_ok.bool()
        # TBs that pass their CRC carry the transmitted bits
        good = bool(torch.equal(r.tbblk[:, :A][ok], tb[ok]))
        if gather and rank == 0:   # rank 0's own TBs, back through pack -> gather -> unpack
            good = good and bool(torch.equal(res[1][0::world][:, :A][ok], tb[ok])) and \
                bool(torch.equal(res[0][0::world], r.tb_ok.to(torch.uint8)))
        return {"snr_db": snr, "rx_tb_per_s": round(T * world * steps / wr, 2),
                "rx_codeblocks_per_s": round(T * cfg.C * world * steps / wr, 1),
                "rx_info_gbit_s": round(T * A * world * steps / wr / 1e9, 3),
                "rx_ms_per_batch": round(wr / steps * 1e3, 4),
                "tb_crc_ok_frac": round(ok.float().mean().item(), 4),
                "tb_bits_match_where_crc_ok": good,
                "mean_iterations": round(r.iters.float().mean().item(), 3)}

    def split(mode):
        """per-kernel split of the RX step at the current channel (event-timed, the same calls
        rx makes), with rooflines"""
        ykey, sched, dnt = MODES[mode]
        y = cur[ykey]
        t_demod = ev_ms(torch, lambda: phy.demod_descramble(y, cur["nv"], Qm, cinit, out=llr))
        dn = sch_raterecover_batch(llr, cfg, None, dnt, ws)
        t_rr = ev_ms(torch, lambda: sch_raterecover_batch(llr, cfg, None, dnt, ws))
        dec_out = (ws.dec_ck, ws.status, ws.iters)
        t_dec = ev_ms(torch, lambda: nr_decode_ldpc_batch(dn, cfg.Zc, cfg.bgn, 8, "min-sum", 0.75, 0.0,
                                                          sched, out=dec_out, rate_matched=True))
        t_chk = ev_ms(torch, lambda: sch_tb_check_batch(ws.dec_ck, cfg, T, ws))
        n_sym, ncb = T * (G // Qm), T * cfg.C
        it_mean = ws.iters.float().mean().item()
        ys, es = y.element_size(), dn.element_size()
        out = {
            "demod_descramble": {**hbm_line(n_sym * (ys + 4) + T * G * 4 + 2 * T * G // 8, t_demod),
                                 "note": f"{y.dtype} symbol + float32 noise variance in, Qm float32 "
                                         "LLRs out, packed scrambling words written + read (PRBS "
                                         "kernel included)"},
            "raterecover": {**hbm_line(T * cfg.E_total * 4 + ncb * cfg.N * es, t_rr),
                            "note": f"E float32 LLRs in, N {dn.dtype} rate-recovered LLRs out per CB"},
            "decode": {**valu_line(ncb * 316 * cfg.Zc * it_mean, t_dec),
                       "mean_iterations": round(it_mean, 3), "schedule": sched, "dtype": str(dn.dtype),
                       "note": f"{sched}, LDPC5G_RATE_MATCHED (dead extension rows skipped: fewer "
                               "edge-updates done than counted)"},
            "tb_check": hbm_line(ncb * (cfg.K_apo + cfg.cbz), t_chk),
        }
        out["sum_ms"] = round(t_demod + t_rr + t_dec + t_chk, 4)
        return out

    easy = rx_line(30.0)
    # threshold search (untimed): mean decoder iterations per candidate SNR, averaged over ranks
    cands = [29.0, 28.5, 28.0, 27.5, 27.0, 26.5, 26.25, 26.0, 25.5, 25.0, 24.0]

    def search(mode):
        its = []
        for snr in cands:
            channel(snr)
            rx_local(cur[MODES[mode][0]], mode)
            its.append(last["r"].iters.float().mean().item())
        if world > 1:
            v = torch.tensor(its, dtype=torch.float64,
                             device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(v)
            its = (v / world).tolist()
        return next((c for c, m in zip(cands, its) if m >= 6.0), cands[-1]), its
    pick, its = search("perf")
    thr = rx_line(pick)
    thr_split = split("perf")
    # the reference's precision: 30 dB and its own threshold point (float64 flooding needs a
    # higher SNR than layered for the same iterations: at the layered threshold it fails every TB)
    ref_easy = rx_line(30.0, "ref")
    ref_pick, ref_its = search("ref")
    ref_thr = rx_line(ref_pick, "ref")
    ref_split = split("ref")
    ref = {**{k: ref_easy[k] for k in ("rx_tb_per_s", "rx_codeblocks_per_s", "rx_info_gbit_s",
                                       "rx_ms_per_batch", "tb_crc_ok_frac", "mean_iterations")},
           "snr_db": 30.0, "tb_bits_match": ref_easy["tb_bits_match_where_crc_ok"],
           "dtype": "f64", "schedule": "flooding",
           "what": "complex128 symbols -> float32 LLRs (nr_Demodulation.py) -> float64 rate recovery "
                   "-> float64 flooding NMS alpha=0.75 L=8 -> CB/TB CRCs: DLSCHDecode's arithmetic "
                   "(nr_dlsch_decode.py:62-106), bit-identical to it",
           "threshold": {**ref_thr, "search": {"snr_db": cands,
                                               "mean_iterations": [round(m, 3) for m in ref_its]},
                         "kernels": ref_split},
           "cpu_baseline": cpu_c5}
    if cpu_c5:
        ref["vs_cpu_baseline"] = round(ref["rx_tb_per_s"] / cpu_c5["value"], 1)
    return {"workload": f"BASELINE config 5: {T} TBs/GPU x 129 CBs (TBS {A}, 256QAM, BG1 Zc=384, "
                        f"Ncb {cfg.Ncb}, E {cfg.E_lo}/{cfg.E_hi}), complex AWGN; RX float32 layered "
                        "(perf mode)",
            "tb_per_gpu": T, "codeblocks_per_tb": cfg.C, "dtype": "f32", "schedule": "layered",
            **{k: easy[k] for k in ("rx_tb_per_s", "rx_codeblocks_per_s", "rx_info_gbit_s",
                                    "rx_ms_per_batch", "tb_crc_ok_frac", "mean_iterations")},
            "snr_db": easy["snr_db"], "tb_bits_match": easy["tb_bits_match_where_crc_ok"],
            "tx_tb_per_s": round(T * world * steps / wt, 2),
            "tx_info_gbit_s": round(T * A * world * steps / wt / 1e9, 3),
            "tx_ms_per_batch": round(wt / steps * 1e3, 4),
            "threshold": {**thr, "search": {"snr_db": cands,
                                           "mean_iterations": [round(m, 3) for m in its]},
                          "kernels": thr_split},
            "reference_precision": ref,
            "gather": ({"what": "TB round robin over ranks; (tb_ok, tbblk) packed into "
                                f"{tm.get('gather_bytes', 0) // max(world, 1) // max(T, 1)}-B records, "
                                "ONE dist.gather (RCCL) to rank 0, unpacked there — inside rx",
                        "gather_ms": round(tm["gather_s"] * 1e3, 3),
                        "gather_bytes": tm["gather_bytes"], "ranks": world}
                       if tm else None)}


def bench_perf_mode(torch, dist, world, llr, out, args, cpu_res):
    """BASELINE config 3 with the float32 layered NMS kernel (the perf schedule BASELINE's wording
    names; not the reference's arithmetic): same LLRs, same timing contract (warmup, barrier +
    synchronize, max over ranks), launch time from HIP events on the launch stream."""
    B = llr.shape[0]
    D = sys.modules["python_5gtoolbox_amd.nr_ldpc_decode"]

    def step():
        D.nr_decode_ldpc_batch(llr, ZC, BG, args.L, "min-sum", args.alpha, 0.0, "layered", out=out)
    wall, ev = timed(torch, dist, world, step, args.steps, args.warmup)
    iters = out[2].float().mean().item()
    conv = int(out[1].sum().item())
    value = B * world * args.steps / wall
    launch_s = ev / args.steps
    achieved = B * DEC_BYTES_PER_CB / launch_s / 1e9
    edge_rate = B * EDGES * iters / launch_s
    alg_lane_ops = edge_rate * ALG_OPS_PER_EDGE
    return {
        "what": "BASELINE config 3 with the float32 layered NMS kernel (perf mode: a different "
                "schedule than the reference's flooding; bit-exact vs oracle.decode_layered, BLER "
                "pinned one-sided to the reference's published values)",
        "value": round(value, 1), "unit": "codeblocks/s", "dtype": "f32", "schedule": "layered",
        "ms_per_step": round(wall / args.steps * 1e3, 4), "launch_ms": round(launch_s * 1e3, 4),
        "steps": args.steps, "warmup": args.warmup,
        "info_gbit_s": round(value * K_INFO / 1e9, 3), "mean_iterations": round(iters, 3),
        "converged": conv,
        "roofline": {"bound": "valu", "achieved": round(alg_lane_ops / 1e12, 3),
                     "peak": round(VALU_PEAK_TLANE, 1), "unit": "T lane-op/s",
                     "frac": round(alg_lane_ops / 1e12 / VALU_PEAK_TLANE, 4),
                     "traffic": pmc_traffic(DEC_KERNEL["layered"]) if B == 4096 else None,
                     "kernel": DEC_KERNEL["layered"], "launch_ms": round(launch_s * 1e3, 4),
                     "algorithmic": f"{ALG_OPS_PER_EDGE} lane-ops per edge-update (SURVEY.md "
                                    f"§8(d)) x 121,344 edges x mean iterations per codeblock",
                     "hbm_achieved_GBps": round(achieved, 2), "hbm_peak_GBps": HBM_PEAK_GBS,
                     "hbm_frac": round(achieved / HBM_PEAK_GBS, 5),
                     "algorithmic_bytes_per_cb": DEC_BYTES_PER_CB,
                     "traffic_source": "profiles/pmc_latest.json: 2 x FETCH_SIZE + WRITE_SIZE bytes "
                                       "per 4096-CB launch (factor calibrated, profiles/r06/"
                                       "fetch_calib.json; FETCH includes Infinity-Cache hits of the "
                                       "per-iteration ext-column LLR re-reads)"},
        "valu": valu_block(edge_rate, launch_s, DEC_KERNEL["layered"], B),
        "cpu_baseline": cpu_res,
    }


def bench_reference_precision(torch, dist, world, llr, out, args, cpu64):
    """BASELINE config 3 at the reference's precision: float64 flooding NMS, bit-identical to
    nr_decode_ldpc (/root/reference/py5gphy/ldpc/nr_ldpc_decode.py:51-143) — what the drop-in
    nr_decode_ldpc / DLSCHDecode / ULSCH_decoding run.  Same LLRs (widened to float64), same
    timing contract as the headline (warmup, barrier + synchronize, max over ranks), launch time
    from HIP events on the launch stream."""
    B = llr.shape[0]
    llr64 = llr.double()

    def step():
        D = sys.modules["python_5gtoolbox_amd.nr_ldpc_decode"]
        D.nr_decode_ldpc_batch(llr64, ZC, BG, args.L, "min-sum", args.alpha, 0.0, "flooding", out=out)
    wall, ev = timed(torch, dist, world, step, args.steps, args.warmup)
    iters = out[2].float().mean().item()
    launch_s = ev / args.steps
    edge_rate = B * EDGES * iters / launch_s
    lane = edge_rate * ALG_OPS_PER_EDGE / 1e12
    value = B * world * args.steps / wall
    traffic = pmc_traffic(DEC64_KERNEL) if B == 4096 else None
    alg_bytes = B * DEC64_BYTES_PER_CB
    del llr64
    return {
        "what": "BASELINE config 3 at the reference's precision and schedule: float64 flooding NMS "
                "alpha=%g L=%d, bit-identical to py5gphy nr_decode_ldpc (ck and status, 193 reference "
                "goldens)" % (args.alpha, args.L),
        "value": round(value, 1), "unit": "codeblocks/s", "dtype": "f64", "schedule": "flooding",
        "ms_per_step": round(wall / args.steps * 1e3, 4), "launch_ms": round(launch_s * 1e3, 4),
        "steps": args.steps, "warmup": args.warmup,
        "info_gbit_s": round(value * K_INFO / 1e9, 3), "mean_iterations": round(iters, 3),
        "converged": int(out[1].sum().item()),
        "roofline": {"bound": "valu", "achieved": round(lane, 3),
                     "peak": round(VALU_PEAK_TLANE, 1), "unit": "T lane-op/s",
                     "frac": round(lane / VALU_PEAK_TLANE, 4),
                     "f64_issue_ceiling": round(VALU_PEAK_TLANE / 2, 1),
                     "frac_of_f64_ceiling": round(lane / (VALU_PEAK_TLANE / 2), 4),
                     "traffic": traffic, "algorithmic_bytes": alg_bytes,
                     "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic else None,
                     "kernel": DEC64_KERNEL,
                     "hbm_achieved_GBps": round(alg_bytes / launch_s / 1e9, 2),
                     "hbm_frac": round(alg_bytes / launch_s / 1e9 / HBM_PEAK_GBS, 5),
                     "algorithmic": f"{ALG_OPS_PER_EDGE} lane-ops per edge-update x 121,344 edges x "
                                    f"mean iterations per codeblock; bytes {DEC64_BYTES_PER_CB} per "
                                    f"codeblock (f64 LLR in, ck, status, iters)",
                     "note": "two ceilings: the full-rate lane peak (78.6 T) and the float64 issue "
                             "ceiling (39.3 T: v_add/min/max/cmp_f64 issue at half rate on gfx950, "
                             "profiles/r02/r02o_valu_rates_f64.txt); traffic = 2 x FETCH_SIZE + "
                             "WRITE_SIZE bytes per launch (calibrated: profiles/r06/fetch_calib.json), "
                             "profiles/pmc_latest.json"},
        "valu": valu_block(edge_rate, launch_s, DEC64_KERNEL, B),
        "cpu_baseline": cpu64,
    }


def spawn_ranks(args):
    """`bench.py --gpus N` without an external launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, as
    torch.distributed.run would) before this process touches the GPU; exit with the first failing
    rank's code (the other ranks are then stopped by PID)."""
    import socket
    import subprocess
    if args.backend == "nccl":
        import torch   # device_count() does not initialise the GPU
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {ndev} visible "
                             f"(--backend gloo rehearses several ranks on one GPU)\n")
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env))
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in procs:
                    q.kill()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
        sys.exit(2)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cpu_res = cpu64 = cpu_c4 = cpu_c5 = None
    if rank == 0 and args.cpu_seconds > 0:   # before any GPU initialisation
        procs = args.cpu_procs or min(16, os.cpu_count() or 1)
        seconds = args.cpu_seconds
        if world > 1:
            # the other ranks share this host: a short single-process sample only
            procs, seconds = 1, min(args.cpu_seconds, 6.0)
        if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ):
            procs = 1   # a profiler may have initialised the GPU already: no spawned workers
        cpu64 = cpu_baseline(seconds, "flooding64", args.alpha, args.L, procs)
        if not args.no_perf or args.headline == "layered":
            cpu_res = cpu_baseline(seconds, "layered", args.alpha, args.L, procs)
        if not args.no_extras:   # configs 4 / 5 at the reference's precision, shorter samples
            cpu_c4 = cpu_baseline_c4(min(seconds, 8.0), procs)
            cpu_c5 = cpu_baseline_c5(min(seconds, 10.0), procs)
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        sys.stderr.write(f"bench.py: {world} ranks but {ndev} GPUs visible\n")
        sys.exit(2)
    dev = torch.device("cuda", local % max(ndev, 1))   # one rank per GPU (several only to rehearse)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from python_5gtoolbox_amd import _lib, nr_ldpc_decode as D, nr_ldpc_encode as E
    _lib.lib()

    B = args.batch
    ck, dn, llr = make_llr(torch, E, B, args.snr, 1234 + rank, dev)
    out = (torch.empty((B, N_FULL), dtype=torch.int8, device=dev),
           torch.empty((B,), dtype=torch.uint8, device=dev),
           torch.empty((B,), dtype=torch.int32, device=dev))
    lines = {}
    if args.headline == "reference" or not args.no_perf:
        lines["reference"] = bench_reference_precision(torch, dist, world, llr, out, args, cpu64)
    if args.headline == "layered" or not args.no_perf:
        lines["layered"] = bench_perf_mode(torch, dist, world, llr, out, args, cpu_res)
    head = lines[args.headline]
    res = {
        "metric": "LDPC codeblocks/s + info-Gbit/s, BG1 Zc=384 NMS L=8, 1/2/4/8 MI355X",
        "value": head["value"],
        "unit": "codeblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": head["dtype"],
        "data": "synthetic (random info bits -> GPU LDPC encode -> BPSK + AWGN, torch RNG)",
        "config": {"workload": f"BASELINE config 3: decode {B} codeblocks/GPU BG1 Zc=384 rate-1/3, NMS "
                               f"alpha={args.alpha} L={args.L}, " +
                               ("float64 flooding, bit-identical to py5gphy nr_decode_ldpc (the "
                                "reference's own schedule and arithmetic)" if args.headline == "reference"
                                else "float32 layered (perf mode)"),
                   "codeblocks_per_gpu": B, "bgn": BG, "Zc": ZC, "L": args.L,
                   "alpha": args.alpha, "beta": 0.0, "schedule": head["schedule"],
                   "snr_db": args.snr, "mean_iterations": head["mean_iterations"],
                   "converged": head["converged"], "parallelism": f"cb-shard x{world}",
                   "note": "BASELINE config 3 names a layered NMS decode; the reference itself "
                           "decodes with a float64 flooding schedule (nr_ldpc_decode.py:51-143), "
                           "so the headline is the like-for-like float64 flooding line and the "
                           "float32 layered kernel is reported as `perf_mode`"},
        "info_gbit_s": head["info_gbit_s"],
        "roofline": head["roofline"],
        "valu": head["valu"],
    }
    for k, v in lines.items():
        if k != args.headline:
            res["perf_mode" if k == "layered" else "reference_precision"] = v

    if not args.no_extras:
        ex = {}
        _, _, llr1 = make_llr(torch, E, B, 1.0, 99 + rank, dev)
        ns = max(3, args.steps // 2)
        llr1_64 = llr1.double()
        for name, x, sched in (("early_exit_snr1dB", llr1_64, "flooding"),
                               ("early_exit_snr1dB_layered_f32", llr1, "layered")):
            w1, e1 = timed(torch, dist, world, lambda: D.nr_decode_ldpc_batch(
                x, ZC, BG, args.L, "min-sum", args.alpha, 0.0, sched, out=out), ns, 1)
            ex[name] = {"codeblocks_per_s": round(B * world * ns / w1, 1),
                        "dtype": "f64" if x.dtype == torch.float64 else "f32", "schedule": sched,
                        "mean_iterations": round(out[2].float().mean().item(), 3),
                        "converged_frac": round(out[1].float().mean().item(), 4)}
        del llr1, llr1_64
        w2, e2 = timed(torch, dist, world, lambda: D.nr_decode_ldpc_batch(
            llr, ZC, BG, args.L, "min-sum", args.alpha, 0.0, "flooding", out=out), ns, 1)
        ex[f"flooding_f32_snr{args.snr:g}dB"] = {
            "codeblocks_per_s": round(B * world * ns / w2, 1),
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
                                             "traffic": pmc_traffic(ENC_KERNEL)
                                             if B == 4096 else None,
                                             "kernel": ENC_KERNEL,
                                             "algorithmic_bytes_per_cb": ENC_BYTES_PER_CB,
                                             "note": "one 4096-codeblock launch moves 138 MB, "
                                                     "which fits the 256 MB Infinity Cache: "
                                                     "back-to-back launches are partly "
                                                     "cache-assisted; hbm_resident is the rate "
                                                     "with 4x the batch (553 MB per launch)"}}
        del dnb
        Bh = 4 * B                       # buffers well past the MALL: the HBM-resident rate
        ckh = torch.randint(0, 2, (Bh, K_INFO), dtype=torch.int8, device=dev)
        dnh = torch.empty((Bh, N_TX), dtype=torch.int8, device=dev)
        w3h, e3h = timed(torch, dist, world, lambda: E.encode_ldpc_batch(ckh, BG, out=dnh), 20, 3)
        ach_h = Bh * ENC_BYTES_PER_CB / (e3h / 20) / 1e9
        ex["encode_config2"]["hbm_resident"] = {
            "codeblocks_per_launch": Bh, "bytes_per_launch": Bh * ENC_BYTES_PER_CB,
            "launch_ms": round(e3h / 20 * 1e3, 4), "codeblocks_per_s": round(Bh * world * 20 / e3h, 1),
            "codeblocks_per_s_wall": round(Bh * world * 20 / w3h, 1),
            "achieved_GBps": round(ach_h, 1), "frac": round(ach_h / HBM_PEAK_GBS, 4),
            "note": "codeblocks_per_s from the launches' HIP events (the kernel rate); _wall: host "
                    "clock around the 20 calls, which includes the Python call overhead"}
        del ckh, dnh
        ex["config1_per_codeblock"] = bench_config1(rank)
        ex["dlsch_caller_shape"] = bench_dlsch_caller(rank)
        ex["single_codeblock_latency"] = bench_single_cb(torch, rank)
        from python_5gtoolbox_amd.shard import decode_codeblocks_sharded
        if world == 1 or dist.get_backend() == "nccl":   # gloo cannot gather device tensors
            llr64 = llr.double()
            g_lines = {}
            for name, x, sched in (("reference_precision", llr64, "flooding"), ("perf_mode", llr, "layered")):
                tm = {}
                for _ in range(2):   # second run timed (first allocates)
                    decode_codeblocks_sharded(x, ZC, BG, args.L, args.alpha, 0.0, sched,
                                              n_total=B * world, timing=tm)
                g_lines[name] = {"schedule": sched, "dtype": "f64" if x is llr64 else "f32",
                                 "gather_ms": round(tm["gather_s"] * 1e3, 3),
                                 "decode_ms": round(tm["decode_s"] * 1e3, 3),
                                 "gather_bytes": tm["gather_bytes"]}
            del llr64
            ex["multi_gpu_gather"] = {
                "what": "decode this rank's shard, pack info bits + status + iterations into "
                        "1061-B records on the GPU, ONE dist.gather (RCCL) to rank 0, unpack there; "
                        "decode_codeblocks_sharded's default is the reference's float64 flooding",
                **g_lines["reference_precision"], "perf_mode": g_lines["perf_mode"], "ranks": world}
        # algo='BF' / 'BP' (nr_decode_ldpc's other two algorithms) on 1024 codeblocks of the
        # headline shape, float64 LLRs, L iterations (all run at -3 dB)
        Bb = min(B, 1024)
        x64 = llr[:Bb].double()
        for algo in ("BF", "BP"):
            nb = max(3, args.steps // 4)
            wb, eb = timed(torch, dist, world,
                           lambda: D.nr_decode_ldpc_batch(x64, ZC, BG, args.L, algo, 1.0, 0.0), nb, 1)
            _, stb, itb = D.nr_decode_ldpc_batch(x64, ZC, BG, args.L, algo, 1.0, 0.0)
            line = {}
            launch_s = eb / nb
            kern = BP_KERNEL if algo == "BP" else BF_KERNEL
            insts = pmc_valu_insts(kern) if Bb == 1024 else None
            if insts:
                # the executed-instruction roofline: VALU lane-ops issued / the full-rate peak and
                # (BP: mostly float64 arithmetic) the f64 issue ceiling
                lane_ops = insts * 64 / launch_s / 1e12
                line["valu"] = {"bound": "valu", "achieved": round(lane_ops, 3), "unit": "T lane-op/s",
                                "peak": round(VALU_PEAK_TLANE, 1), "frac": round(lane_ops / VALU_PEAK_TLANE, 4),
                                "f64_issue_ceiling": round(VALU_PEAK_TLANE / 2, 1),
                                "frac_of_f64_ceiling": round(lane_ops / (VALU_PEAK_TLANE / 2), 4),
                                "valu_insts_per_edge_update": round(
                                    insts * 64 / (float(itb.sum().item()) * EDGES), 2),
                                "kernel": kern,
                                "source": "SQ_INSTS_VALU per 1024-codeblock launch, profiles/pmc_latest.json"}
            if algo == "BF":
                # hard decisions live in LDS: the HBM side is the float64 LLRs in and the decisions
                # out once per codeblock
                line["roofline"] = hbm_line(Bb * (N_TX * 8 + N_FULL + 5), launch_s * 1e3)
            if algo == "BP":
                # the per-edge messages live in a device scratch: each iteration reads and writes
                # every edge's float64 message once (16 B per edge-update), plus the LLRs in and
                # the decisions out once per codeblock
                it_sum = int(itb.sum().item())
                alg = it_sum * EDGES * 16 + Bb * (N_TX * 8 + N_FULL)
                line.update({"roofline": hbm_line(alg, eb / nb * 1e3),
                             "edge_updates_per_s": round(it_sum * EDGES / (eb / nb), 1)})
            ex[f"{algo.lower()}_decode"] = {
                "codeblocks_per_call": Bb, "codeblocks_per_s": round(Bb * world * nb / wb, 1), **line,
                "launch_ms": round(eb / nb * 1e3, 4), "mean_iterations": round(itb.float().mean().item(), 3),
                "note": ("hard-decision bit flipping (ldpc_decoder_bit_flipping.py:5-73)" if algo == "BF" else
                         "float64 sum-product flooding (_BP_process, nr_ldpc_decode.py:145-176), per-edge "
                         "messages in a device scratch")}
        del x64
        ex["config4_mixed_zc"] = bench_config4(torch, dist, world, dev, rank, max(3, args.steps // 2), cpu_c4)
        ex["config5_tb_stream"] = bench_config5(torch, dist, world, dev, rank, max(3, args.steps // 2),
                                                cpu_c5=cpu_c5)
        res["extras"] = ex

    if rank == 0:
        res["cpu_baseline"] = cpu64 if args.headline == "reference" else cpu_res
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
