"""GPU-batched LDPC BLER harness — the counterpart of the reference's
scripts/internal/sim_ldpc_internal.py:9-91 (run_ldpc_simulation) built on
nr_ldpc_decode.for_test_5g_ldpc_encoder (py5gphy/ldpc/nr_ldpc_decode.py:229-260).

The reference draws ONE codeblock at a time (random K - crc bits -> CRC -> encode -> BPSK + AWGN,
sigma = 10^(-snr/20), LLR = 2y/sigma^2), decodes it and counts a block error when the decoded
blkandcrc differs; it stops at 1000 / 2000 / 4000 codeblocks once 50 / 25 / 10 errors are seen,
else at 10000 (:66-77).  Here the codeblocks are drawn 1000 at a time on the GPU (CRC by
ldpc5g_crc, encoder, torch's RNG for bits and noise) and decoded in one batched launch; the
stopping rule is evaluated at exactly the reference's counts, so each BLER point rests on the
same number of trials as the reference's.

Results are returned (and optionally written as JSON, not pickle) in the reference's shape:
(sim_config, test_config_list, test_results_list).  run_ldpc_simulation_fixed is the fixed-count
variant of scripts/sim_ldpc_decoder_bf.py (200 codeblocks per SNR below 4 dB, 2000 from 4 dB).
"""
import json

from . import _lib
from .ldpc_info import code_dims

TEST_LIMITS = (1000, 2000, 4000, 10000)   # sim_ldpc_internal.py:67 (np.array([200,400,800,2000])*5)
FAIL_LIMITS = (50, 25, 10)                # :68 (np.array([10,5,2])*5)
CRC_LEN = {"24A": 24, "24B": 24, "16": 16}


def test_configs(algo_list, alpha_list, beta_list, mixed_list, L_list):
    """(flag, algo, alpha, beta, L) per test, in the reference's order and naming (:15-41)."""
    out = []
    for algo in algo_list:
        if algo in ["BP", "BF", "min-sum"]:
            n = 1
        elif algo == "NMS":
            n = len(alpha_list)
        elif algo == "OMS":
            n = len(beta_list)
        else:
            n = len(mixed_list)
        for L in L_list:
            for i in range(n):
                if algo in ["BF", "BP", "min-sum"]:
                    out.append((f"{algo} L={L}", algo, 1.0, 0.0, L))
                elif algo == "NMS":
                    out.append((f"NMS-alpha={alpha_list[i]}-L={L}", "min-sum", alpha_list[i], 0.0, L))
                elif algo == "OMS":
                    out.append((f"OMS-beta={beta_list[i]}-L={L}", "min-sum", 1.0, beta_list[i], L))
                else:
                    a, b = mixed_list[i]
                    out.append((f"mixed-MS-[alpha,beta]=[{a},{b}]-L={L}", "min-sum", a, b, L))
    return out


def gen_codeblocks(Zc, bgn, snr_db, crcpoly, n, gen, device):
    """Batched for_test_5g_ldpc_encoder: (blkandcrc (n, K) int8, LLR (n, N) float64) on the GPU."""
    t = _lib.require_gpu()
    from .nr_ldpc_encode import encode_ldpc_batch
    from .sch import crc_rows
    K, N, _ = code_dims(bgn, Zc)
    L = CRC_LEN[crcpoly]
    blk = t.empty((n, K), dtype=t.int8, device=device)
    blk[:, :K - L] = t.randint(0, 2, (n, K - L), dtype=t.int8, device=device, generator=gen)
    rem = crc_rows(blk, crcpoly, nbits=K - L)
    shifts = t.arange(L - 1, -1, -1, device=device, dtype=t.int64)
    blk[:, K - L:] = ((rem[:, None] >> shifts) & 1).to(t.int8)
    dn = encode_ldpc_batch(blk, bgn)
    sigma = 10 ** (-snr_db / 20)
    y = (1 - 2 * dn.double()) + sigma * t.randn(dn.shape, dtype=t.float64, device=device,
                                                  generator=gen)
    return blk, 2 * y / (10 ** (-snr_db / 10))


def bler_point(Zc, bgn, snr_db, crcpoly, algo, alpha, beta, L, gen, device, schedule="flooding",
               batch=1000):
    """(test_count, failed_count) at one SNR with the reference's stopping rule."""
    t = _lib.require_gpu()
    from .nr_ldpc_decode import nr_decode_ldpc_batch
    K, _, _ = code_dims(bgn, Zc)
    assert all(x % batch == 0 for x in TEST_LIMITS)
    count = failed = 0
    while True:
        blk, llr = gen_codeblocks(Zc, bgn, snr_db, crcpoly, batch, gen, device)
        x = llr if schedule == "flooding" else llr.float()
        ck, _, _ = nr_decode_ldpc_batch(x, Zc, bgn, L, algo, alpha, beta, schedule)
        failed += int((ck[:, :K] != blk).any(dim=1).sum().item())
        count += batch
        if count in TEST_LIMITS:
            i = TEST_LIMITS.index(count)
            if i < len(FAIL_LIMITS) and failed >= FAIL_LIMITS[i]:
                break
            if count == TEST_LIMITS[-1]:
                break
    return count, failed


def bler_fixed(Zc, bgn, snr_db, crcpoly, algo, alpha, beta, L, n, gen, device, schedule="flooding",
               batch=1000):
    """(n, failed_count) over exactly n codeblocks: the fixed-count loop of
    scripts/sim_ldpc_decoder_bf.py:77-98 (no stopping rule)."""
    t = _lib.require_gpu()
    from .nr_ldpc_decode import nr_decode_ldpc_batch
    K, _, _ = code_dims(bgn, Zc)
    count = failed = 0
    while count < n:
        b = min(batch, n - count)
        blk, llr = gen_codeblocks(Zc, bgn, snr_db, crcpoly, b, gen, device)
        x = llr if schedule == "flooding" else llr.float()
        ck, _, _ = nr_decode_ldpc_batch(x, Zc, bgn, L, algo, alpha, beta, schedule)
        failed += int((ck[:, :K] != blk).any(dim=1).sum().item())
        count += b
    return count, failed


def run_ldpc_simulation_fixed(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list,
                              L_list, snr_db_list, test_count_seed=200, filename=None, seed=0,
                              schedule="flooding", verbose=False):
    """The fixed-count BLER script scripts/sim_ldpc_decoder_bf.py:43-107 on the GPU: per SNR
    total_count = test_count_seed if snr_db < 4 else 10 * test_count_seed (:77-80), same test
    naming and result shape as run_ldpc_simulation."""
    t = _lib.require_gpu()
    dev = t.device("cuda", t.cuda.current_device())
    gen = t.Generator(device=dev)
    gen.manual_seed(seed)
    flags, results, counts = [], [], []
    for flag, algo, alpha, beta, L in test_configs(algo_list, alpha_list, beta_list, mixed_list,
                                                   L_list):
        flags.append(flag)
        bler, cnt = [], []
        for snr in snr_db_list:
            total = test_count_seed if snr < 4 else test_count_seed * 10
            n, f = bler_fixed(Zc, bgn, snr, crcpoly, algo, alpha, beta, L, total, gen, dev, schedule)
            bler.append(f / n)
            cnt.append([n, f])
            if verbose:
                print(f"finish test {flag}, snr_db={snr}, bler={f / n:2.5f}")
        results.append(bler)
        counts.append(cnt)
    sim_config = {"Zc": Zc, "bgn": bgn}
    if filename:
        with open(filename, "w") as fh:
            json.dump({"sim_config": sim_config, "test_config_list": flags,
                       "test_results_list": results, "trials": counts,
                       "snr_db_list": list(snr_db_list), "schedule": schedule}, fh, indent=1)
    return sim_config, flags, results


def run_ldpc_simulation(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list, L_list,
                        snr_db_list, filename=None, seed=0, schedule="flooding", verbose=False):
    """sim_ldpc_internal.run_ldpc_simulation on the GPU.  Returns (sim_config,
    test_config_list, test_results_list); with `filename`, also writes them as JSON together with
    the trial counts behind every BLER value."""
    t = _lib.require_gpu()
    dev = t.device("cuda", t.cuda.current_device())
    gen = t.Generator(device=dev)
    gen.manual_seed(seed)
    flags, results, counts = [], [], []
    for flag, algo, alpha, beta, L in test_configs(algo_list, alpha_list, beta_list, mixed_list,
                                                   L_list):
        flags.append(flag)
        bler, cnt = [], []
        for snr in snr_db_list:
            n, f = bler_point(Zc, bgn, snr, crcpoly, algo, alpha, beta, L, gen, dev, schedule)
            bler.append(f / n)
            cnt.append([n, f])
            if verbose:
                print(f"finish test {flag}, Zc {Zc}, bgn{bgn},snr_db={snr}, test_count={n},"
                      f"failed_count={f},bler={f / n:2.5f}")
        results.append(bler)
        counts.append(cnt)
    sim_config = {"Zc": Zc, "bgn": bgn}
    if filename:
        with open(filename, "w") as fh:
            json.dump({"sim_config": sim_config, "test_config_list": flags,
                       "test_results_list": results, "trials": counts,
                       "snr_db_list": list(snr_db_list), "schedule": schedule}, fh, indent=1)
    return sim_config, flags, results
