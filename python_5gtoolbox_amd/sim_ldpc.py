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

run_ldpc_simulation writes the reference's result file — pickle.dump([sim_config,
test_config_list, test_results_list]) — and returns None, so the reference's scripts
(scripts/sim_ldpc_decoder.py:45-51 and the three alpha/beta searches) run unchanged once
scripts.internal.sim_ldpc_internal points here (module sim_ldpc_internal); draw_ldpc_decoder_result
plots it like :93-117.  run_ldpc_simulation_fixed is the fixed-count sweep of
scripts/sim_ldpc_decoder_bf.py (200 codeblocks per SNR below 4 dB, 2000 from 4 dB).  simulate()
returns the results together with the trial counts behind every value.
"""
import json
import pickle

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


def simulate(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list, L_list,
             snr_db_list, seed=0, schedule="flooding", verbose=False, fixed_count=None):
    """Run every test of the sweep; returns (sim_config, test_config_list, test_results_list,
    trials) with trials[i][j] = [test_count, failed_count] behind test_results_list[i][j].
    fixed_count=None: the reference's stopping rule (sim_ldpc_internal.py:44-83); else the
    fixed-count loop of scripts/sim_ldpc_decoder_bf.py:74-98 (fixed_count codeblocks below 4 dB,
    10x from 4 dB)."""
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
            if fixed_count is None:
                n, f = bler_point(Zc, bgn, snr, crcpoly, algo, alpha, beta, L, gen, dev, schedule)
            else:
                total = fixed_count if snr < 4 else fixed_count * 10
                n, f = bler_fixed(Zc, bgn, snr, crcpoly, algo, alpha, beta, L, total, gen, dev,
                                  schedule)
            bler.append(f / n)
            cnt.append([n, f])
            if verbose:
                print(f"finish test {flag}, Zc {Zc}, bgn{bgn},snr_db={snr}, test_count={n},"
                      f"failed_count={f},bler={f / n:2.5f}")
        results.append(bler)
        counts.append(cnt)
    return {"Zc": Zc, "bgn": bgn}, flags, results, counts


def _dump(filename, json_filename, sim_config, flags, results, counts, snr_db_list, schedule):
    # the reference's result file (sim_ldpc_internal.py:89-91): [sim_config, labels, bler lists],
    # plain containers only, read back by the scripts with pickle.load (sim_ldpc_decoder.py:49-50)
    with open(filename, "wb") as handle:
        pickle.dump([sim_config, flags, results], handle, protocol=pickle.HIGHEST_PROTOCOL)
    if json_filename:   # extra: the trial counts behind every BLER value
        with open(json_filename, "w") as fh:
            json.dump({"sim_config": sim_config, "test_config_list": flags,
                       "test_results_list": results, "trials": counts,
                       "snr_db_list": list(snr_db_list), "schedule": schedule}, fh, indent=1)


def run_ldpc_simulation(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list, L_list,
                        snr_db_list, filename, *, seed=0, schedule="flooding", verbose=True,
                        json_filename=None):
    """Drop-in for scripts/internal/sim_ldpc_internal.py:9-91 run_ldpc_simulation: the same
    sweep (labels, order, stopping rule), batched on the GPU; writes
    pickle.dump([sim_config, test_config_list, test_results_list]) to `filename` exactly as the
    reference does and returns None.  The keyword-only extras: the RNG seed, the decoder
    schedule ("flooding" = the reference's float64 arithmetic), per-point prints, and a JSON copy
    with the trial counts."""
    sim_config, flags, results, counts = simulate(Zc, bgn, crcpoly, algo_list, alpha_list,
                                                  beta_list, mixed_list, L_list, snr_db_list,
                                                  seed, schedule, verbose)
    _dump(filename, json_filename, sim_config, flags, results, counts, snr_db_list, schedule)


def run_ldpc_simulation_fixed(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list,
                              L_list, snr_db_list, filename, test_count_seed=200, *, seed=0,
                              schedule="flooding", verbose=True, json_filename=None):
    """The fixed-count sweep of scripts/sim_ldpc_decoder_bf.py:43-107 (its main body, which has no
    function of its own in the reference): total_count = test_count_seed below 4 dB, 10x from
    4 dB (:77-80); writes the same pickle to `filename` (:104-107) and returns None."""
    sim_config, flags, results, counts = simulate(Zc, bgn, crcpoly, algo_list, alpha_list,
                                                  beta_list, mixed_list, L_list, snr_db_list,
                                                  seed, schedule, verbose,
                                                  fixed_count=test_count_seed)
    _dump(filename, json_filename, sim_config, flags, results, counts, snr_db_list, schedule)


def draw_ldpc_decoder_result(snr_db_list, sim_config, test_config_list, test_results_list,
                             figfile):
    """scripts/internal/sim_ldpc_internal.py:93-117: BLER vs Eb/N0, one curve per test, log
    scale, saved to `figfile` (host-only plotting, no GPU)."""
    import matplotlib
    if matplotlib.get_backend().lower() not in ("agg", "pdf", "svg", "ps", "cairo"):
        matplotlib.use("Agg")   # headless: the reference saves to a file too (:115)
    import matplotlib.pyplot as plt
    fig = plt.figure()
    markers = [".", "o", "v", "<", ">", "P", "*", "+", "x", "D", "d"]
    plt.xlabel("Eb/N0")
    plt.ylabel("BLER")
    plt.title("ldpc decoder, Zc={}, bgn={}".format(sim_config["Zc"], sim_config["bgn"]))
    plt.yscale("log")
    plt.xlim(snr_db_list[0], snr_db_list[-1])
    plt.ylim(10 ** (-4), 1)
    plt.grid(True)
    for i, label in enumerate(test_config_list):
        plt.plot(snr_db_list, test_results_list[i], marker=markers[i % len(markers)],
                 label="{}".format(label))
    plt.legend(loc="upper right", fontsize=5)
    plt.savefig(figfile)
    plt.close(fig)
