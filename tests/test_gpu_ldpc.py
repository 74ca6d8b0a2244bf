"""GPU parity tests: the HIP kernels (through libldpc5g.so's C ABI) against the reference's golden
vectors and the oracle.  Run on an MI355X with `pytest -m gpu`.

Bars:
  encode ..................... bit-exact with the reference (all 51 Zc x 2 BG, fillers)
  decode float64 flooding .... bit-exact ck + status with the reference (every fixture)
  decode float32 flooding .... bit-exact ck + status + iters with the fp32 oracle restatement
  decode float32 layered ..... bit-exact ck + status + iters with the layered oracle
  full-size (4096 x BG1 Zc=384): codeword syndrome == 0, encode->BPSK->decode round trip
"""
import math
import os

import numpy as np
import pytest

from conftest import load_algo_cases, load_decode_cases
from oracle import ldpc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a ROCm GPU"
    return t


@pytest.fixture(scope="module")
def enc():
    from python_5gtoolbox_amd import nr_ldpc_encode
    return nr_ldpc_encode


@pytest.fixture(scope="module")
def dec():
    from python_5gtoolbox_amd import nr_ldpc_decode
    return nr_ldpc_decode


# ------------------------------------------------------------------------------------- encode
def test_native_library_loaded(torch):
    from python_5gtoolbox_amd import _lib
    assert _lib.lib().ldpc5g_version().startswith(b"ldpc5g")


def test_encode_golden_dropin(torch, enc, encode_cases):
    for bg, Zc, F, ck, dn in encode_cases:
        x = ck.copy()
        out = enc.encode_ldpc(x, bg)
        assert out.dtype == np.int8 and out.shape == dn.shape
        assert np.array_equal(out, dn), (bg, Zc, F)
        exp = ck.copy()
        exp[2 * Zc:][exp[2 * Zc:] == -1] = 0          # in-place filler zeroing (:34-35)
        assert np.array_equal(x, exp)


@pytest.mark.parametrize("bg,Zc", [(1, 384), (2, 384), (1, 7), (2, 13), (1, 208), (2, 2)])
def test_encode_batch_vs_oracle(torch, enc, bg, Zc):
    rng = np.random.default_rng(Zc * bg)
    K = (22 if bg == 1 else 10) * Zc
    B = 300
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    for b in range(0, B, 3):
        F = int(rng.integers(1, K - 2 * Zc))
        ck[b, K - F:] = -1
    assert np.array_equal(enc.encode_ldpc_batch(ck, bg), O.encode(ck, bg))


def test_encode_strided_unaligned(torch, enc):
    """Row stride not a multiple of 16 and a misaligned base pointer take the slow paths."""
    rng = np.random.default_rng(5)
    bg, Zc = 1, 40
    K, N = 22 * Zc, 66 * Zc
    src = torch.from_numpy(rng.integers(0, 2, (33, K + 7)).astype(np.int8)).cuda()
    view = src[:, 3:3 + K]
    out = torch.full((33, N + 5), 7, dtype=torch.int8, device="cuda")
    enc.encode_ldpc_batch(view, bg, out=out)
    got = out.cpu().numpy()
    assert np.array_equal(got[:, :N], O.encode(view.cpu().numpy(), bg))
    assert (got[:, N:] == 7).all()


def test_encode_full_size_codewords(torch, enc):
    """BASELINE config 2 shape: 4096 x BG1 Zc=384; every codeword satisfies H c = 0."""
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    B, Zc = 4096, 384
    ck = torch.randint(0, 2, (B, 22 * Zc), dtype=torch.int8, device="cuda", generator=g)
    dn = enc.encode_ldpc_batch(ck, 1)
    torch.cuda.synchronize()
    c = ck.cpu().numpy()
    d = dn.cpu().numpy()
    for s in range(0, B, 512):
        bits = np.concatenate([c[s:s + 512, :2 * Zc], d[s:s + 512]], axis=1)
        assert not O.syndrome(bits, 1, Zc).any()
    sub = np.arange(0, B, 97)
    assert np.array_equal(d[sub], O.encode(c[sub], 1))


# ------------------------------------------------------------------------------------- decode
def test_decode_golden_fp64_bitexact(torch, dec, decode_cases):
    """nr_decode_ldpc drop-in (float64 flooding kernel) == reference, ck and status, on every
    golden case including the three BG1 Zc=384 codeblocks."""
    for c in decode_cases:
        blk, ck, st = dec.nr_decode_ldpc(c["llr"].astype(np.float64), c["Zc"], c["bg"], c["L"],
                                         "min-sum", c["alpha"], c["beta"])
        K = (22 if c["bg"] == 1 else 10) * c["Zc"]
        assert ck.dtype == np.int8 and isinstance(st, bool)
        assert np.shares_memory(blk, ck) and blk.size == K
        assert np.array_equal(ck, c["ck"]), (c["kind"], c["bg"], c["Zc"], c["L"])
        assert st == c["status"], (c["kind"], c["bg"], c["Zc"])


def _groups(cases):
    g = {}
    for c in cases:
        g.setdefault((c["bg"], c["Zc"], c["L"], c["alpha"], c["beta"]), []).append(c)
    return g


@pytest.mark.parametrize("dtype,schedule", [(np.float64, "flooding"), (np.float32, "flooding"),
                                            (np.float32, "layered")])
def test_decode_golden_vs_oracle(torch, dec, decode_cases, dtype, schedule):
    """Batched kernels == oracle restatement (ck, status, iters) on the golden inputs."""
    for (bg, Zc, L, a, b), cs in _groups(decode_cases).items():
        llr = np.stack([c["llr"] for c in cs]).astype(dtype)
        ck, st, it = dec.nr_decode_ldpc_batch(llr, Zc, bg, L, "min-sum", a, b, schedule)
        if schedule == "layered":
            ock, ost, oit = O.decode_layered(llr, Zc, bg, L, a, b)
        else:
            ock, ost, oit = O.decode_flooding(llr, Zc, bg, L, a, b, dtype)
        assert np.array_equal(ck, ock), (bg, Zc, L, a, b)
        assert np.array_equal(st, ost) and np.array_equal(it, oit), (bg, Zc, L, a, b)


@pytest.mark.parametrize("bg,Zc", [(1, 2), (2, 5), (1, 13), (2, 36), (1, 96), (2, 176)])
@pytest.mark.parametrize("schedule", ["flooding", "layered"])
def test_decode_packed_workgroups(torch, dec, bg, Zc, schedule):
    """Many codeblocks per workgroup (G = 384 // Zc), each exiting early at its own iteration."""
    rng = np.random.default_rng(Zc + 7 * bg)
    K = (22 if bg == 1 else 10) * Zc
    B = 200
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    dn = O.encode(ck, bg)
    snr = rng.uniform(-3.0, 2.5, (B, 1))
    llr = (2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
           10 ** (-snr / 10)).astype(np.float32)
    got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 12, "min-sum", 0.8, 0.1, schedule)
    ref = (O.decode_layered(llr, Zc, bg, 12, 0.8, 0.1) if schedule == "layered"
           else O.decode_flooding(llr, Zc, bg, 12, 0.8, 0.1, np.float32))
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)
    assert got[1].sum() > 0 and len(np.unique(got[2])) > 2   # early exits at different iterations


@pytest.mark.parametrize("bg,Zc,B", [(1, 16, 4), (2, 12, 5), (1, 64, 1), (2, 2, 32), (2, 8, 1), (1, 20, 3)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_decode_flooding_small_launch(torch, dec, bg, Zc, B, dtype):
    """Launches whose codeblocks fit 64 slots run the 16-part flooding configuration
    (ldpc5g_dec_flood16.hip): bit-exact with the oracle for 1..32 codeblocks, early exits included."""
    assert B * Zc <= 64
    rng = np.random.default_rng(Zc * 31 + B)
    K = (22 if bg == 1 else 10) * Zc
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    snr = rng.uniform(-2.0, 3.0, (B, 1))
    dn = O.encode(ck, bg)
    llr = ((2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
            10 ** (-snr / 10))).astype(dtype)
    got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 10, "min-sum", 0.75, 0.25, "flooding")
    ref = O.decode_flooding(llr, Zc, bg, 10, 0.75, 0.25, dtype)
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)


@pytest.mark.parametrize("bg,Zc,B", [(1, 64, 1), (2, 64, 1), (2, 8, 8), (1, 2, 32), (1, 40, 1), (1, 48, 1),
                                     (1, 56, 1)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_decode_small_kernel_edge_cases(torch, dec, bg, Zc, B, dtype):
    """The small-codeblock kernel (ldpc5g_dec_small.h, B * Zc <= 64) on its edge cases, bit-exact
    with the oracle: NMS (beta 0) and OMS, L = 0 / 1 / 8, integer LLRs (|q| ties, argmin order),
    an all-zero codeblock and a noiseless one (exit at iteration 0).  BG1 Zc = 48 / 56 are the
    three-nodes-per-thread (RPT = 3) instantiation; Zc = 56 is the largest BG1 float64 lifting size
    whose LDS fits, so BG1 Zc = 64 float64 exercises the 16-part fallback (small_fits false)."""
    rng = np.random.default_rng(Zc * 7 + B)
    K = (22 if bg == 1 else 10) * Zc
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    dn = O.encode(ck, bg)
    llr = (1 - 2 * dn) * 2.0 + rng.integers(-3, 4, dn.shape)   # integer: ties everywhere
    llr[0] = 0.0
    if B > 1:
        llr[1] = (1 - 2 * dn[1]) * 4.0
    llr = llr.astype(dtype)
    for L, alpha, beta in ((0, 0.75, 0.0), (1, 1.0, 0.5), (8, 0.8, 0.0), (8, 1.0, 0.25)):
        got = dec.nr_decode_ldpc_batch(llr, Zc, bg, L, "min-sum", alpha, beta, "flooding")
        ref = O.decode_flooding(llr, Zc, bg, L, alpha, beta, dtype)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r), (L, alpha, beta)


@pytest.mark.parametrize("schedule,dtype", [("flooding", np.float32), ("layered", np.float32),
                                            ("flooding", np.float64)])
def test_decode_z384_batch_vs_oracle(torch, dec, schedule, dtype):
    """BASELINE config 3 shape (BG1 Zc=384, NMS alpha=0.75, L=8) on 48 codeblocks vs oracle
    (float64 flooding: the reference-exact mode, bit-exact with the oracle's float64 restatement)."""
    rng = np.random.default_rng(384)
    Zc, B = 384, 48
    ck = rng.integers(0, 2, (B, 22 * Zc)).astype(np.int8)
    dn = O.encode(ck, 1)
    snr = np.repeat([-3.0, 0.0, 0.5, 1.0], B // 4)[:, None]
    llr = (2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
           10 ** (-snr / 10)).astype(dtype)
    got = dec.nr_decode_ldpc_batch(llr, Zc, 1, 8, "min-sum", 0.75, 0.0, schedule)
    ref = (O.decode_layered(llr, Zc, 1, 8, 0.75, 0.0) if schedule == "layered"
           else O.decode_flooding(llr, Zc, 1, 8, 0.75, 0.0, dtype))
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)


@pytest.mark.parametrize("schedule,dtype,rm,bg", [("layered", np.float32, False, 1), ("layered", np.float32, True, 1),
                                                  ("flooding", np.float64, False, 1), ("flooding", np.float64, True, 1),
                                                  ("flooding", np.float64, False, 2), ("flooding", np.float64, True, 2)])
def test_decode_z384_kernels_vs_oracle(torch, dec, schedule, dtype, rm, bg):
    """The Zc = 384 kernels (lifting size and shifts compile-time, wrap-table offsets as immediates):
    offset min-sum (beta > 0), an odd batch (a half-empty last workgroup of the layered kernel),
    mixed SNRs, and rate-matched rows (untransmitted extension columns +0.0: the dead-row
    variants), bit-exact with the oracle."""
    rng = np.random.default_rng(7 + rm + 10 * bg)
    # float64: 30 codeblocks run the batch kernels (up to 24 BG1 / 28 BG2 take the split kernel)
    Zc, B = 384, (30 if dtype == np.float64 else 9)
    ck = rng.integers(0, 2, (B, (22 if bg == 1 else 10) * Zc)).astype(np.int8)
    dn = O.encode(ck, bg)
    snr = rng.choice([-1.0, 1.0, 3.0], size=B)[:, None]
    llr = (2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
           10 ** (-snr / 10)).astype(dtype)
    if rm:   # the last 20 extension columns never transmitted
        llr[:, -20 * Zc:] = 0
    got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 6, "min-sum", 1.0, 0.5, schedule, rate_matched=rm)
    ref = (O.decode_layered(llr, Zc, bg, 6, 1.0, 0.5) if schedule == "layered"
           else O.decode_flooding(llr, Zc, bg, 6, 1.0, 0.5, dtype))
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)


@pytest.mark.parametrize("bg", [1, 2])
@pytest.mark.parametrize("pattern", ["ties", "dead_rows"])
@pytest.mark.parametrize("rm", [False, True])
def test_decode_frame_kernel_edge_cases(torch, dec, bg, pattern, rm):
    """The float64 Zc = 384 frame kernel (ldpc5g_dec_frame.h: per-row thread frames, column 0 / 1
    sums in registers, hand-offs through the dead LDS image of columns 0 / 1) on inputs that stress
    its exactness arguments, vs the oracle's float64 decode_ldpc: "ties" — integer LLRs in [-3, 3]
    with +0.0 and -0.0 entries (equal magnitudes, zero messages, zero sums, -0.0 in iteration 0);
    "dead_rows" — the extension columns of BG1's hand-off rows 4, 15, 19 (and BG2's rows 4, 10,
    19) plus the last 12 never transmitted, so with rm (LDPC5G_RATE_MATCHED) whole rows and row
    groups are skipped.  NMS (alpha .75) and OMS (beta .5), 32 codeblocks (the batch kernel)."""
    rng = np.random.default_rng(3 + bg + 10 * rm + (pattern == "ties"))
    Zc, B = 384, 32
    kb = 22 if bg == 1 else 10
    ck = rng.integers(0, 2, (B, kb * Zc)).astype(np.int8)
    dn = O.encode(ck, bg)
    if pattern == "ties":
        llr = ((1 - 2 * dn) * rng.integers(0, 4, dn.shape) + rng.integers(-1, 2, dn.shape)).astype(np.float64)
        llr[:, ::17] = -0.0
        llr[:, 5::23] = 0.0
    else:
        llr = 2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 0.9) / 0.81
        for i in ((4, 15, 19) if bg == 1 else (4, 10, 19)):   # ext column of row i: kb + i - 2
            llr[:, (kb + i - 2) * Zc:(kb + i - 1) * Zc] = 0.0
        llr[:, -12 * Zc:] = 0.0
    for alpha, beta in ((0.75, 0.0), (1.0, 0.5)):
        got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", alpha, beta, "flooding", rate_matched=rm)
        ref = O.decode_flooding(llr, Zc, bg, 8, alpha, beta, np.float64)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r), (alpha, beta)


@pytest.mark.parametrize("bg", [1, 2])
def test_decode_frame_kernel_mixed_liveness(torch, dec, bg):
    """One rate-matched (LDPC5G_RATE_MATCHED) float64 Zc = 384 launch whose codeblocks differ in
    which extension rows are dead: the frame kernel finds each codeblock's live rows from its
    prologue loads (wave ballots) and picks the dead-row or the plain iterations per workgroup, so
    one launch runs both.  Codeblocks with 0 / 1 / 7 / 25 / all-but-one dead extension columns,
    one dead column in the middle (a live row after a dead one), +0.0 vs -0.0 (-0.0 is not dead:
    its bit pattern is not +0.0), filler-like huge LLRs, SNRs from -2 to 4 dB (codeblocks stop at
    different iterations); NMS and OMS; vs the oracle's float64 decode_ldpc."""
    rng = np.random.default_rng(77 + bg)
    Zc, B = 384, 24
    kb, mb = (22, 46) if bg == 1 else (10, 42)
    ck = rng.integers(0, 2, (B, kb * Zc)).astype(np.int8)
    dn = O.encode(ck, bg)
    snr = rng.uniform(-2.0, 4.0, (B, 1))
    llr = 2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) / 10 ** (-snr / 10)
    nx = mb - 4
    for b in range(B):
        kind = b % 8
        if kind == 1:
            llr[b, -1 * Zc:] = 0.0
        elif kind == 2:
            llr[b, -7 * Zc:] = 0.0
        elif kind == 3:
            llr[b, -25 * Zc:] = 0.0
        elif kind == 4:
            llr[b, -(nx - 1) * Zc:] = 0.0
        elif kind == 5:   # one dead column between live ones (ext row 4 + 10)
            c0 = (kb + 2 + 10) * Zc - 2 * Zc
            llr[b, c0:c0 + Zc] = 0.0
        elif kind == 6:   # -0.0 everywhere in the tail: live (not +0.0)
            llr[b, -7 * Zc:] = -0.0
        elif kind == 7:   # a dead tail but one live entry in its last column
            llr[b, -7 * Zc:] = 0.0
            llr[b, -1] = 1.5
    llr[::5, 3:kb * Zc:97] = 10 * np.abs(llr).max()   # filler-like entries (nr_ldpc_raterecover.py)
    for alpha, beta in ((0.75, 0.0), (1.0, 0.5)):
        got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", alpha, beta, "flooding", rate_matched=True)
        ref = O.decode_flooding(llr, Zc, bg, 8, alpha, beta, np.float64)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r), (alpha, beta)


@pytest.mark.parametrize("bg,Zc,B", [(1, 384, 1), (2, 384, 1), (1, 384, 7), (1, 64, 1), (1, 96, 2),
                                     (2, 72, 1), (2, 176, 3), (1, 208, 1), (2, 384, 8),
                                     # two chunks per wave (R = 2): more codeblocks than R = 1 fits
                                     (1, 384, 23), (2, 384, 15), (1, 208, 30), (1, 120, 40)])
def test_decode_split_kernel_vs_oracle(torch, dec, bg, Zc, B):
    """The multi-workgroup float64 flooding kernel (ldpc5g_dec_split.hip: each codeblock over
    ceil(MB*Zc/1024) CUs, barriers over a codeblock's workgroups) that serves launches of a few
    large codeblocks (the per-codeblock drop-ins and whole transport blocks of up to 24 BG1 Zc=384
    codeblocks: one or two 64-slot chunks per wave), bit-exact with the oracle: NMS and OMS,
    L = 0 / 1 / 8, integer LLRs (|q| ties), an all-zero codeblock, a noiseless one, mixed SNRs
    (codeblocks of one launch exiting at different iterations) and rate-matched rows."""
    rng = np.random.default_rng(Zc * 3 + B + 100 * bg)
    K = (22 if bg == 1 else 10) * Zc
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    dn = O.encode(ck, bg)
    snr = rng.uniform(-3.0, 3.0, (B, 1))
    noisy = 2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) / 10 ** (-snr / 10)
    ties = ((1 - 2 * dn) * 2.0 + rng.integers(-3, 4, dn.shape)).astype(np.float64)
    ties[0] = 0.0
    if B > 1:
        ties[1] = (1 - 2 * dn[1]) * 4.0
    for llr in (noisy, ties):
        for L, alpha, beta, rm in ((0, 0.75, 0.0, False), (1, 1.0, 0.5, False), (8, 0.75, 0.0, False),
                                   (8, 1.0, 0.25, False), (6, 0.8, 0.0, True)):
            x = llr.copy()
            if rm:
                x[:, -7 * Zc:] = 0
            got = dec.nr_decode_ldpc_batch(x, Zc, bg, L, "min-sum", alpha, beta, "flooding", rate_matched=rm)
            ref = O.decode_flooding(x, Zc, bg, L, alpha, beta, np.float64)
            for g, r in zip(got, ref):
                assert np.array_equal(g, r), (L, alpha, beta, rm)


def test_decode_split_kernel_concurrent_streams(torch, dec):
    """Three streams each launching the multi-workgroup kernel with 7 BG1 Zc=384 codeblocks (126
    workgroups each, 378 together: more than the CUs hold at once) — the library chains split
    launches of a device one after another, so none can wait forever for CUs the others hold;
    results equal a sequential run."""
    rng = np.random.default_rng(77)
    Zc, B = 384, 7
    xs = []
    for s_ in range(3):
        ck = rng.integers(0, 2, (B, 22 * Zc)).astype(np.int8)
        dn = O.encode(ck, 1)
        llr = 2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (3 / 20)) / 10 ** (3 / 10)
        xs.append(torch.from_numpy(llr).cuda())
    ref = [[t.cpu() for t in dec.nr_decode_ldpc_batch(x, Zc, 1, 8, "min-sum", 0.75, 0.0, "flooding")] for x in xs]
    streams = [torch.cuda.Stream() for _ in xs]
    outs = []
    torch.cuda.synchronize()
    for st, x in zip(streams, xs):
        with torch.cuda.stream(st):
            outs.append(dec.nr_decode_ldpc_batch(x, Zc, 1, 8, "min-sum", 0.75, 0.0, "flooding"))
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        for a, b in zip(o, r):
            assert torch.equal(a.cpu(), b)


def test_decode_split_kernel_two_processes(torch):
    """Two processes on the GPU launching the multi-workgroup kernel at once, 12 BG1 Zc=384
    codeblocks = 216 workgroups per launch (two launches cannot be resident together): parts are
    taken by arrival ticket, so both finish, every repetition equal to the first
    (tools/split_mp_probe.py; the children are new interpreters, started under a time limit)."""
    import signal
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # a session of its own: on the time limit the whole group (the probe AND its GPU children) dies
    p = subprocess.Popen([sys.executable, os.path.join(root, "tools", "split_mp_probe.py"), "2", "300"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        raise
    assert p.returncode == 0, out[-2000:] + err[-2000:]
    assert out.count("mismatches 0") == 2, out


def test_decode_ldpc_full_length(torch, dec):
    """decode_ldpc(LLRin, H, ...) — full-length LLR incl. the punctured columns — matches the
    oracle fed the same full row."""
    from python_5gtoolbox_amd import ldpc_info
    for c in load_decode_cases()[:40:5]:
        Zc, bg = c["Zc"], c["bg"]
        H = ldpc_info.getH(Zc, bg, ldpc_info.find_iLS(Zc))
        rng = np.random.default_rng(Zc)
        full = np.concatenate([rng.normal(size=2 * Zc), c["llr"].astype(np.float64)])
        ck, st = dec.decode_ldpc(full, H, c["L"], "min-sum", c["alpha"], c["beta"])
        # oracle: punctured columns carry LLRs here, so restate via a zero-padded shift trick
        ock, ost = _oracle_full(full, Zc, bg, c["L"], c["alpha"], c["beta"])
        assert np.array_equal(ck, ock) and st == ost


@pytest.mark.parametrize("bg,Zc", [(1, 384), (2, 96), (1, 120)])
def test_decode_split_kernel_full_length(torch, dec, bg, Zc):
    """decode_ldpc with a full-length LLR row (the punctured columns carry LLRs: pc = 0) through
    the multi-workgroup kernel (one large codeblock per call) == the oracle on the same row."""
    from python_5gtoolbox_amd import ldpc_info
    rng = np.random.default_rng(Zc + bg)
    K = (22 if bg == 1 else 10) * Zc
    ck0 = rng.integers(0, 2, (1, K)).astype(np.int8)
    dn = O.encode(ck0, bg)[0]
    full = np.concatenate([1 - 2 * ck0[0, :2 * Zc].astype(np.float64), 1 - 2 * dn.astype(np.float64)])
    full = 2 * (full + rng.normal(size=full.shape) * 0.9) / 0.81
    H = ldpc_info.getH(Zc, bg, ldpc_info.find_iLS(Zc))
    for L, a, b in ((8, 0.75, 0.0), (5, 1.0, 0.3)):
        ck, st = dec.decode_ldpc(full, H, L, "min-sum", a, b)
        ock, ost = _oracle_full(full, Zc, bg, L, a, b)
        assert np.array_equal(ck, ock) and st == ost, (L, a, b)


def _oracle_full(full, Zc, bg, L, a, b):
    """Flooding restatement with caller-provided LLRs on every column (decode_ldpc semantics)."""
    g = O.graph(bg, Zc)
    T = np.float64
    Lfull = full[None].astype(T)
    LQ = Lfull.copy()
    Lr = [np.zeros((1, g.rs[i + 1] - g.rs[i], Zc), T) for i in range(g.Mb)]
    for it in range(L):
        hd = LQ < 0
        if not O._row_hd_fail(hd, g)[0]:
            return hd[0].astype(np.int8), True
        acc = np.zeros_like(LQ)
        for i in range(g.Mb):
            cols = g.rows_cols(i)
            Lr[i] = O._cn_update(LQ[:, cols] - Lr[i], T(a), T(b), T)
            acc[:, cols] += Lr[i]
        LQ = Lfull + acc
    hd = LQ <= 0
    return hd[0].astype(np.int8), not O._row_hd_fail(hd, g)[0]


def test_decode_full_size_round_trip(torch, enc, dec):
    """4096 x BG1 Zc=384 (BASELINE config 3 shape): GPU encode -> BPSK/AWGN at 2 dB -> GPU
    layered NMS decode recovers every codeword (syndrome-checked status and info bits)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    B, Zc = 4096, 384
    ck = torch.randint(0, 2, (B, 22 * Zc), dtype=torch.int8, device="cuda", generator=g)
    dn = enc.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (-2.0 / 20)
    y = (1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda", generator=g)
    llr = (2 * y / sigma ** 2).contiguous()
    for schedule in ("layered", "flooding"):
        out, st, it = dec.nr_decode_ldpc_batch(llr, Zc, 1, 8, "min-sum", 0.75, 0.0, schedule)
        torch.cuda.synchronize()
        assert int(st.sum()) == B
        assert torch.equal(out[:, :22 * Zc], ck)
        assert torch.equal(out[:, 2 * Zc:], dn)
        assert int(it.max()) <= 8


def test_decode_mixed_batch(torch):
    """BASELINE config 4: Zc in {12,40,72,176,208,384} x BG1/BG2 in one mixed call, OMS beta=0.5."""
    from python_5gtoolbox_amd import nr_ldpc_decode_mixed as MX
    rng = np.random.default_rng(44)
    items = []
    for bg in (1, 2):
        for Zc in (12, 40, 72, 176, 208, 384):
            n = 5
            K = (22 if bg == 1 else 10) * Zc
            ck = rng.integers(0, 2, (n, K)).astype(np.int8)
            dn = O.encode(ck, bg)
            llr = O.bpsk_awgn_llr(dn, float(rng.uniform(0, 2)), rng).astype(np.float32)
            for k in range(n):
                items.append((bg, Zc, llr[k]))
    order = rng.permutation(len(items))
    items = [items[i] for i in order]
    # (5 BG1 Zc=384 codeblocks: a partial and two full layered workgroups, the full ones through
    # the Zc = 384 kernel; float64 flooding: all five through it)
    for schedule, dt in (("flooding", np.float32), ("layered", np.float32), ("flooding", np.float64)):
        outs, st, it = MX.decode_mixed([(b, z, l.astype(dt)) for b, z, l in items], 8, 1.0, 0.5, schedule)
        for k, (bg, Zc, llr) in enumerate(items):
            ref = (O.decode_layered(llr[None], Zc, bg, 8, 1.0, 0.5) if schedule == "layered"
                   else O.decode_flooding(llr[None].astype(dt), Zc, bg, 8, 1.0, 0.5, dt))
            assert np.array_equal(outs[k], ref[0][0]) and st[k] == ref[1][0] and it[k] == ref[2][0]


@pytest.mark.parametrize("schedule,dt,n384", [("layered", np.float32, 1031), ("flooding", np.float64, 515)])
def test_decode_mixed_batch_zc384_launch(torch, dec, schedule, dt, n384):
    """A mixed call with enough BG1 Zc=384 codeblocks (>= 512 workgroups) for their own launch of
    the Zc = 384 kernel (ldpc5g_capi.hip launch_plan): every codeblock identical to the uniform
    batch decode of its (bg, Zc), itself bit-exact with the oracle (test_decode_z384_*)."""
    from python_5gtoolbox_amd import nr_ldpc_decode_mixed as MX
    rng = np.random.default_rng(n384)
    groups = {(1, 384): n384, (2, 52): 9}
    items, llrs = [], {}
    for (bg, Zc), n in groups.items():
        K = (22 if bg == 1 else 10) * Zc
        dn = O.encode(rng.integers(0, 2, (n, K)).astype(np.int8), bg)
        llr = O.bpsk_awgn_llr(dn, float(rng.uniform(0, 1.5)), rng).astype(dt)
        llrs[(bg, Zc)] = llr
        items += [(bg, Zc, k) for k in range(n)]
    order = rng.permutation(len(items))
    items = [items[i] for i in order]
    outs, st, it = MX.decode_mixed([(b, z, llrs[(b, z)][k]) for b, z, k in items], 8, 1.0, 0.5, schedule)
    ref = {key: dec.nr_decode_ldpc_batch(v, key[1], key[0], 8, "min-sum", 1.0, 0.5, schedule)
           for key, v in llrs.items()}
    for j, (bg, Zc, k) in enumerate(items):
        rck, rst, rit = ref[(bg, Zc)]
        assert np.array_equal(outs[j], rck[k]) and st[j] == rst[k] and it[j] == rit[k]


def test_decode_errors_are_assertions(torch, dec):
    with pytest.raises(AssertionError):
        dec.nr_decode_ldpc(np.zeros(66 * 17), 17, 1, 8)
    with pytest.raises(AssertionError):
        dec.nr_decode_ldpc(np.zeros(66 * 8), 8, 3, 8)
    with pytest.raises(AssertionError):
        dec.nr_decode_ldpc(np.zeros(66 * 8 + 1), 8, 1, 8)
    with pytest.raises(AssertionError):
        dec.nr_decode_ldpc(np.zeros(66 * 8), 8, 1, 8, "LDPC")


def test_dlsch_encode_chain_with_gpu_encoder(torch, enc):
    """Reference DLSCHEncode chain (nr_dlsch.py:12-74) with the GPU encoder as its encode_ldpc
    reproduces the reference transport-block output g_seq."""
    import os
    from conftest import GOLD
    from python_5gtoolbox_amd import crc, nr_ldpc_cbsegment, nr_ldpc_ratematch as RM
    d = np.load(os.path.join(GOLD, "dlsch_golden.npz"))
    for i, (TBS, Qm, R, NL, rv, LBRM, G) in enumerate(d["meta"].tolist()):
        tb = np.unpackbits(d["tb"][d["tb_off"][i]:d["tb_off"][i + 1]])[:TBS]
        g_ref = np.unpackbits(d["g"][d["g_off"][i]:d["g_off"][i + 1]])[:G]
        blk = crc.nr_crc_encode(tb, "24A" if TBS > 3824 else "16")
        bgn = 2 if (TBS <= 292 or (TBS <= 3824 and R <= 0.67 * 1024) or R <= 0.25 * 1024) else 1
        cbs, Zc = nr_ldpc_cbsegment.ldpc_cbsegment(blk, bgn)
        C = cbs.shape[0]
        Er = RM.get_Er_ldpc(G, C, Qm, NL)
        out = []
        for c in range(C):
            dn = enc.encode_ldpc(cbs[c, :], bgn)
            Ncb = min(dn.size, math.floor(LBRM / (C * 2 / 3)))
            k0 = RM.get_k0(Ncb, bgn, rv, Zc)
            out.append(RM.ratematch_ldpc(dn, Ncb, Er[c], k0, Qm))
        assert np.array_equal(np.concatenate(out), g_ref)


# ---------------------------------------------------------------------------------- BF / BP
def test_decode_bf_golden_bitexact(torch, dec):
    """algo='BF' (ldpc_decoder_bit_flipping.py:5-73): ck (float64 like the reference) and status
    bit-exact on all 40 golden cases; batched kernel == oracle incl. iteration counts."""
    cases = load_algo_cases("BF")
    for c in cases:
        blk, ck, st = dec.nr_decode_ldpc(c["llr"].astype(np.float64), c["Zc"], c["bg"], c["L"], "BF")
        assert ck.dtype == np.float64 and np.array_equal(ck, c["ck"]) and st == c["status"]
    for (bg, Zc, L), cs in _groups3(cases).items():
        llr = np.stack([c["llr"] for c in cs]).astype(np.float64)
        got = dec.nr_decode_ldpc_batch(llr, Zc, bg, L, "BF")
        ref = O.decode_bf(llr, Zc, bg, L)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)


def _groups3(cases):
    g = {}
    for c in cases:
        g.setdefault((c["bg"], c["Zc"], c["L"]), []).append(c)
    return g


def test_decode_bp_golden(torch, dec):
    """algo='BP' (float64 sum-product, _BP_process :145-176): the GPU's tanh/atanh are not
    numpy's, so messages differ in the last ulps.  Bar: identical status on every golden case,
    identical ck whenever the reference decoded successfully."""
    for c in load_algo_cases("BP"):
        blk, ck, st = dec.nr_decode_ldpc(c["llr"].astype(np.float64), c["Zc"], c["bg"], c["L"], "BP")
        assert ck.dtype == np.int8 and st == c["status"], (c["bg"], c["Zc"], c["L"])
        if c["status"]:
            assert np.array_equal(ck, c["ck"]), (c["bg"], c["Zc"])


def test_decode_bp_batch_vs_oracle(torch, dec):
    rng = np.random.default_rng(9)
    for bg, Zc in [(1, 13), (2, 36)]:
        K = (22 if bg == 1 else 10) * Zc
        ck = rng.integers(0, 2, (64, K)).astype(np.int8)
        llr = O.bpsk_awgn_llr(O.encode(ck, bg), 1.0, rng)
        got = dec.nr_decode_ldpc_batch(llr, Zc, bg, 12, "BP")
        ref = O.decode_bp(llr, Zc, bg, 12)
        assert np.array_equal(got[1], ref[1])
        both = ref[1]
        assert np.array_equal(got[0][both], ref[0][both]) and np.array_equal(got[2][both], ref[2][both])


def test_config1_golden_dropins(torch, dec):
    """BASELINE config 1 exactly (BG2 Zc=8, CRC24A, NMS alpha=.75, L=8), against the reference's
    own outputs (tests/golden/config1_golden.npz): for_test_5g_ldpc_encoder under the same
    np.random seed reproduces (blkandcrc, dn, LLR) bit for bit (host CRC + GPU
    encoder), and nr_decode_ldpc (float64 flooding kernel) reproduces ck and status."""
    from conftest import GOLD
    d = np.load(f"{GOLD}/config1_golden.npz")
    for i, seed in enumerate(d["seed"].tolist()):
        np.random.seed(seed)
        blk, dn, llr = dec.for_test_5g_ldpc_encoder(8, 2, float(d["snr"][i]), "24A")
        assert np.array_equal(blk, d["blk"][i]) and np.array_equal(dn, d["dn"][i])
        assert np.array_equal(llr.view(np.uint64), d["llr"][i].view(np.uint64))
        blkandcrc, ck, status = dec.nr_decode_ldpc(llr, 8, 2, 8, "min-sum", 0.75, 0)
        assert status == bool(d["status"][i]) and np.array_equal(ck, d["ck"][i]), i
        assert np.shares_memory(blkandcrc, ck) and blkandcrc.size == 80


def test_config1_layered_vs_oracle(torch, dec):
    """Config 1 through the batched layered perf kernel: bit-exact vs the layered oracle, and
    every codeblock the reference decoded is decoded to the same codeword."""
    from conftest import GOLD
    d = np.load(f"{GOLD}/config1_golden.npz")
    llr = d["llr"].astype(np.float32)
    ck, st, it = dec.nr_decode_ldpc_batch(llr, 8, 2, 8, "min-sum", 0.75, 0.0, "layered")
    rck, rst, rit = O.decode_layered(llr, 8, 2, 8, 0.75, 0.0)
    assert np.array_equal(ck, rck) and np.array_equal(st, rst) and np.array_equal(it, rit)
    ref_ok = d["status"].astype(bool)
    assert st[ref_ok].all() and np.array_equal(ck[ref_ok], d["ck"][ref_ok])


@pytest.mark.parametrize("schedule,dtype,rm", [("layered", "float32", False), ("flooding", "float32", False),
                                               ("flooding", "float64", False), ("flooding", "float64", True)])
def test_mixed_batch_rate_matched_vs_oracle(torch, schedule, dtype, rm):
    """BASELINE config 4 inputs as the bench builds them: 12 (Zc, BG) groups, each rate-matched
    on the GPU with its own (Qm, rv, E) (fillers, punctured zeros, repetitions), BPSK + AWGN,
    rate-recovered (float32 rows, or float64 rows: the reference's precision, nr_ldpc_raterecover.py
    :62); decoded by MixedBatch (plan built once, asynchronous launches, called twice; rm: the
    LDPC5G_RATE_MATCHED variant that skips dead extension rows, what the bench's config-4
    reference-precision line runs) and compared group by group with the oracle (OMS beta=0.5,
    L=8; float64 flooding = the reference's decode_ldpc)."""
    from python_5gtoolbox_amd.ldpc_info import code_dims
    from python_5gtoolbox_amd.nr_ldpc_decode_mixed import MixedBatch
    from python_5gtoolbox_amd.sch import cfg_from_codeblocks, sch_ratematch_batch, sch_raterecover_batch
    rng = np.random.default_rng(404)
    g = torch.Generator(device="cuda")
    g.manual_seed(404)
    groups = []
    for Zc in (12, 40, 72, 176, 208, 384):
        for bg in (1, 2):
            n = 7
            K, N, _ = code_dims(bg, Zc)
            Kapo = K - int(rng.integers(0, K // 8))            # fillers at the end
            Qm = int(rng.choice([1, 2, 4, 6, 8]))
            rv = int(rng.integers(0, 4))
            E = Qm * int(rng.integers(-(-Kapo // Qm), int(1.6 * N) // Qm + 1))
            cfg = cfg_from_codeblocks(n, K, Kapo, Zc, bg, Qm, n * E, 1, rv)
            ck = torch.randint(0, 2, (n, K), dtype=torch.int8, device="cuda", generator=g)
            ck[:, Kapo:] = -1
            gs = sch_ratematch_batch(ck, cfg, 1)
            y = (1 - 2 * gs.float()) + 0.9 * torch.randn(gs.shape, device="cuda", generator=g)
            llr = (2 * y / 0.81).contiguous()
            if dtype == "float64":
                llr = llr.double()
            dn = sch_raterecover_batch(llr, cfg, dn_dtype=getattr(torch, dtype)).clone()
            groups.append((bg, Zc, dn))
    mb = MixedBatch(groups)
    for _ in range(2):
        ck, st, it = mb.decode(8, 1.0, 0.5, schedule, rm)
    ck, st, it = ck.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
    k = 0
    for bg, Zc, dn in groups:
        x = dn.cpu().numpy()
        ref = (O.decode_layered(x, Zc, bg, 8, 1.0, 0.5) if schedule == "layered"
               else O.decode_flooding(x, Zc, bg, 8, 1.0, 0.5, x.dtype.type))
        for r in range(x.shape[0]):
            co, nf = mb.rows[k]
            assert np.array_equal(ck[co:co + nf], ref[0][r]), (bg, Zc, r)
            assert st[k] == ref[1][r] and it[k] == ref[2][r], (bg, Zc, r)
            k += 1


@pytest.mark.parametrize("bg,Zc", [(2, 13), (1, 15), (1, 9), (2, 6)])
@pytest.mark.parametrize("schedule,dtype", [("layered", np.float32), ("flooding", np.float32),
                                            ("flooding", np.float64)])
def test_decode_ck_store_unaligned_rows(torch, dec, bg, Zc, schedule, dtype):
    """The staged ck store (ck_store_staged): rows whose length Nf*Zc is not a multiple of 16 and
    rows in a padded, odd-offset view of a wider buffer take the byte path; slots of several
    workgroups incl. a batch tail.  ck / status / iters == oracle, padding bytes untouched."""
    rng = np.random.default_rng(Zc * 10 + bg)
    K, N, Nf = ((22, 66, 68) if bg == 1 else (10, 50, 52))
    B = 100
    ck0 = rng.integers(0, 2, (B, K * Zc)).astype(np.int8)
    dn = O.encode(ck0, bg)
    snr = np.repeat([-1.0, 1.0, 3.0, 6.0], B // 4)[:, None]
    llr = (2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
           10 ** (-snr / 10)).astype(dtype)
    ref = (O.decode_layered(llr, Zc, bg, 6, 0.75, 0.0) if schedule == "layered"
           else O.decode_flooding(llr, Zc, bg, 6, 0.75, 0.0, dtype))
    x = torch.from_numpy(llr).cuda()
    for pad, off in ((0, 0), (21, 3)):
        wide = torch.full((B, Nf * Zc + pad + off), 0x55, dtype=torch.int8, device="cuda")
        ckv = wide[:, off:off + Nf * Zc]
        st = torch.empty((B,), dtype=torch.uint8, device="cuda")
        it = torch.empty((B,), dtype=torch.int32, device="cuda")
        dec.nr_decode_ldpc_batch(x, Zc, bg, 6, "min-sum", 0.75, 0.0, schedule, out=(ckv, st, it))
        w = wide.cpu().numpy()
        assert np.array_equal(w[:, off:off + Nf * Zc], ref[0]), (pad, off)
        assert np.array_equal(st.cpu().numpy(), ref[1]) and np.array_equal(it.cpu().numpy(), ref[2])
        assert (w[:, :off] == 0x55).all() and (w[:, off + Nf * Zc:] == 0x55).all(), (pad, off)
