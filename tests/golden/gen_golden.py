"""Generate the golden fixtures in tests/golden/ by running the REFERENCE (py5gphy) in this
container.  The reference never travels: only the input/output vectors below are committed.

    cd /root/reference && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/gen_golden.py

(the reference opens its tables through the relative path "py5gphy/ldpc/tables/",
py5gphy/ldpc/ldpc_info.py:110, so the cwd must be the reference root.)

Fixtures (all bit vectors stored np.packbits-packed, LLRs as float32 — the reference is run on
the float64 widening of those float32 values so the fixtures are exact for both precisions):
  encode_golden.npz    encode_ldpc (nr_ldpc_encode.py:8) on 51 Zc x 2 BG x 2 seeds, with fillers
  decode_golden.npz    nr_decode_ldpc (nr_ldpc_decode.py:11), min-sum family, flooding, incl.
                       rate-recovered LLRs (zeros, repetition averages, filler 10*max), integer
                       LLRs (ties), all-zero LLRs, and 3 BG1 Zc=384 codeblocks
  ratematch_golden.npz ratematch_ldpc / raterecover_ldpc / get_k0 / get_Er cases
  crc_golden.json      CRC KATs (the inline vectors of py5gphy/crc/crc.py:167-210) + generated
  dlsch_golden.npz     DLSCHEncode (nr_dlsch.py:12) transport blocks -> g_seq
  sch_golden.npz/.json DLSCHDecode (+HARQ), ULSCH encode/decode, a config-5 DLSCHEncode TB
  sch_negbeta_golden.* DLSCHDecode / ULSCH_decoding with beta < 0 (per-codeblock nr_decode_ldpc)
  demod_golden.npz     nrModulate / nrDemodulate (QPSK..256QAM) / gen_nrPRBS vectors
  decode_bf_golden.npz / decode_bp_golden.npz   nr_decode_ldpc with algo='BF' / 'BP'
  sparse_golden.npz    decode_ldpc (nr_ldpc_decode.py:51) on random binary H (all algorithms), the
                       bit-flipping toy H KAT shape, nr_decode_ldpc with beta < 0
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)

ZLIST = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36,
         40, 44, 48, 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208,
         224, 240, 256, 288, 320, 352, 384]


def _ref():
    from py5gphy.ldpc import nr_ldpc_encode, nr_ldpc_decode
    return nr_ldpc_encode, nr_ldpc_decode


def bpsk_llr(dn, snr_db, rng):
    en = 1 - 2 * np.asarray(dn, np.float64)
    fn = en + rng.normal(0, 10 ** (-snr_db / 20), en.shape)
    return 2 * fn / 10 ** (-snr_db / 10)


# ------------------------------------------------------------------------------------- encode
def gen_encode():
    enc, _ = _ref()
    rng = np.random.default_rng(20251003)
    meta, ckp, dnp = [], [], []
    for bg in (1, 2):
        kb = 22 if bg == 1 else 10
        for Zc in ZLIST:
            K = kb * Zc
            for seed in range(2):
                ck = rng.integers(0, 2, K).astype(np.int8)
                F = 0 if seed == 0 else int(rng.integers(1, K - 2 * Zc))
                if F:
                    ck[K - F:] = -1
                ck_in = ck.copy()
                dn = enc.encode_ldpc(ck_in, bg)
                # reference semantics pinned here: systematic part copied (fillers stay -1) ...
                assert np.array_equal(dn[:K - 2 * Zc], ck[2 * Zc:])
                # ... and fillers zeroed in the caller's array in place (nr_ldpc_encode.py:34-35)
                exp_in = ck.copy()
                exp_in[2 * Zc:][exp_in[2 * Zc:] == -1] = 0
                assert np.array_equal(ck_in, exp_in)
                par = dn[K - 2 * Zc:]
                assert set(np.unique(par)) <= {0, 1}
                meta.append((bg, Zc, F))
                ckp.append(np.packbits(ck == 1))
                dnp.append(np.packbits(par == 1))
    np.savez_compressed(os.path.join(OUT, "encode_golden.npz"), meta=np.array(meta, np.int32),
                        ck_bits=np.concatenate(ckp), ck_off=_offs(ckp),
                        par_bits=np.concatenate(dnp), par_off=_offs(dnp))
    print("encode cases", len(meta))


def _offs(lst):
    return np.concatenate([[0], np.cumsum([x.size for x in lst])]).astype(np.int64)


# ------------------------------------------------------------------------------------- decode
def _decode_case(args):
    (bg, Zc, L, alpha, beta, llr32) = args
    _, dec = _ref()
    t = time.time()
    _, ck, status = dec.nr_decode_ldpc(llr32.astype(np.float64), Zc, bg, L, "min-sum", alpha, beta)
    return np.packbits(ck == 1), bool(status), time.time() - t


def _mk_awgn(rng, bg, Zc, snr):
    import oracle_shim as O
    K = (22 if bg == 1 else 10) * Zc
    ck = rng.integers(0, 2, K).astype(np.int8)
    dn = O.encode(ck, bg)
    return bpsk_llr(dn, snr, rng).astype(np.float32)


def _mk_ratematched(rng, bg):
    """LLRs as the DL-SCH receiver builds them: ratematch -> BPSK+AWGN -> raterecover
    (nr_ldpc_ratematch.py:64 / nr_ldpc_raterecover.py:6) — exact zeros for punctured bits,
    averaged repetitions, 10*max|LLR| on filler positions."""
    from py5gphy.ldpc import ldpc_info, nr_ldpc_ratematch as RM, nr_ldpc_raterecover as RR
    import oracle_shim as O
    while True:
        B = int(rng.integers(60, 3000))
        try:
            C, cbz, Lc, F, K, Zc = ldpc_info.get_cbs_info(B, bg)
            break
        except AssertionError:
            pass
    if Zc > 96:
        return None
    K_apo = K - F
    ck = rng.integers(0, 2, K).astype(np.int8)
    ck[K_apo:] = -1
    dn = O.encode(ck, bg)
    N = dn.size
    Ncb = N if rng.random() < 0.6 else int(rng.integers(K, N + 1))
    Qm = int(rng.choice([1, 2, 4, 6, 8]))
    rv = int(rng.integers(0, 4))
    E = Qm * int(rng.integers(max(1, (K - F) // Qm), int(1.7 * N) // Qm))
    k0 = RM.get_k0(Ncb, bg, rv, Zc)
    fe = RM.ratematch_ldpc(dn, Ncb, E, k0, Qm)
    snr = float(rng.uniform(-1, 3))
    y = bpsk_llr(fe, snr, rng)
    llr = RR.raterecover_ldpc(y, Ncb, N, k0, Qm, Zc, K_apo, K)
    return Zc, llr.astype(np.float32)


def gen_decode(pool):
    rng = np.random.default_rng(77)
    zs = [2, 3, 4, 5, 6, 7, 9, 11, 13, 15, 16, 24, 28, 36, 44, 52, 60, 72]
    ab = [(1.0, 0.0), (0.75, 0.0), (1.0, 0.5), (0.8, 0.3)]
    cases = []   # (kind, bg, Zc, L, alpha, beta, llr32)
    i = 0
    for bg in (1, 2):
        for zi, Zc in enumerate(zs):
            for k in range(4):
                snr = [-1.0, 0.0, 1.0, 2.0][(zi + k) % 4]
                a, b = ab[(zi + 2 * k) % 4]
                L = [8, 32][(zi + k) % 2]
                cases.append(("awgn", bg, Zc, L, a, b, _mk_awgn(rng, bg, Zc, snr)))
                i += 1
    n = 0
    while n < 32:
        bg = 1 + n % 2
        r = _mk_ratematched(rng, bg)
        if r is None:
            continue
        Zc, llr = r
        a, b = ab[n % 4]
        cases.append(("ratematched", bg, Zc, [8, 16][n % 2], a, b, llr))
        n += 1
    # integer-valued LLRs: many exact ties in the two-min selection (tie rules :195-199)
    for n in range(12):
        bg = 1 + n % 2
        Zc = [4, 6, 10, 12, 20, 26][n % 6]
        K = (22 if bg == 1 else 10) * Zc
        import oracle_shim as O
        dn = O.encode(rng.integers(0, 2, K).astype(np.int8), bg)
        llr = (1 - 2 * dn.astype(np.float32)) * rng.integers(1, 4, dn.size)
        flip = rng.random(dn.size) < 0.12
        llr[flip] = -llr[flip]
        zero = rng.random(dn.size) < 0.05
        llr[zero] = 0
        cases.append(("ties", bg, Zc, 8, *ab[n % 4], llr.astype(np.float32)))
    # all-zero LLRs: decision 0, syndrome 0 -> immediate success (nr_ldpc_decode.py:107-114)
    for bg, Zc in ((1, 8), (2, 15)):
        N = (66 if bg == 1 else 50) * Zc
        cases.append(("zeros", bg, Zc, 8, 1.0, 0.0, np.zeros(N, np.float32)))
    print("decode cases (small)", len(cases))
    t = time.time()
    res = pool.map(_decode_case, [c[1:] for c in cases], chunksize=1)
    print("small decode done", time.time() - t)
    # 3 full-size BG1 Zc=384 codeblocks (the BASELINE config-3 shape), run serially (7.7 GB each)
    big = [(0.5, 0.75, 0.0), (-2.0, 0.75, 0.0), (1.5, 1.0, 0.0)]
    for snr, a, b in big:
        llr = _mk_awgn(rng, 1, 384, snr)
        cases.append(("z384", 1, 384, 8, a, b, llr))
        r = _decode_case((1, 384, 8, a, b, llr))
        print("z384 snr", snr, "status", r[1], "t", round(r[2], 1))
        res.append(r)
    kinds = sorted(set(c[0] for c in cases))
    np.savez_compressed(
        os.path.join(OUT, "decode_golden.npz"),
        kind=np.array([kinds.index(c[0]) for c in cases], np.int8), kinds=np.array(kinds),
        bg=np.array([c[1] for c in cases], np.int32), Zc=np.array([c[2] for c in cases], np.int32),
        L=np.array([c[3] for c in cases], np.int32), alpha=np.array([c[4] for c in cases]),
        beta=np.array([c[5] for c in cases]),
        llr=np.concatenate([c[6] for c in cases]), llr_off=_offs([c[6] for c in cases]),
        ck_bits=np.concatenate([r[0] for r in res]), ck_off=_offs([r[0] for r in res]),
        status=np.array([r[1] for r in res]))
    print("decode cases", len(cases), "status True", sum(r[1] for r in res))


# ------------------------------------------------------------------------------ BF / BP
def _decode_algo_case(args):
    (bg, Zc, L, algo, llr32) = args
    _, dec = _ref()
    t = time.time()
    _, ck, status = dec.nr_decode_ldpc(llr32.astype(np.float64), Zc, bg, L, algo, 1, 0)
    return np.packbits(np.asarray(ck) != 0), bool(status), time.time() - t


def gen_bf_bp(pool):
    """nr_decode_ldpc(..., algo='BF') (ldpc_decoder_bit_flipping.py:5-73) and algo='BP'
    (nr_ldpc_decode.py:145-176) on small lifting sizes."""
    rng = np.random.default_rng(123)
    cases = []
    for algo, snrs in (("BF", [3.0, 4.0, 5.0, 6.0]), ("BP", [-1.0, 0.0, 1.0, 2.0])):
        for n in range(40):
            bg = 1 + n % 2
            Zc = [2, 3, 5, 7, 9, 11, 13, 15, 8, 12, 20, 26, 36, 40][n % 14]
            snr = snrs[n % 4]
            L = [8, 16][(n // 4) % 2]
            cases.append((algo, bg, Zc, L, _mk_awgn(rng, bg, Zc, snr)))
    t = time.time()
    res = pool.map(_decode_algo_case, [(c[1], c[2], c[3], c[0], c[4]) for c in cases], chunksize=1)
    print("bf/bp decode done", time.time() - t)
    for algo in ("BF", "BP"):
        idx = [k for k, c in enumerate(cases) if c[0] == algo]
        np.savez_compressed(
            os.path.join(OUT, f"decode_{algo.lower()}_golden.npz"),
            bg=np.array([cases[k][1] for k in idx], np.int32),
            Zc=np.array([cases[k][2] for k in idx], np.int32),
            L=np.array([cases[k][3] for k in idx], np.int32),
            llr=np.concatenate([cases[k][4] for k in idx]), llr_off=_offs([cases[k][4] for k in idx]),
            ck_bits=np.concatenate([res[k][0] for k in idx]), ck_off=_offs([res[k][0] for k in idx]),
            status=np.array([res[k][1] for k in idx]))
        print(algo, "cases", len(idx), "status True", sum(res[k][1] for k in idx))


# ---------------------------------------------------------------- arbitrary H (decode_ldpc)
TOY_H = np.array([[1, 1, 0, 1, 0, 0],      # ldpc_decoder_bit_flipping.py:115-118
                  [0, 1, 1, 0, 1, 0],
                  [1, 0, 0, 0, 1, 1],
                  [0, 0, 1, 1, 0, 1]])


def gf2_nullspace(H):
    """Basis of {x : H x = 0 mod 2} (rows of the returned array) — codewords for random H."""
    A = (np.asarray(H) & 1).astype(np.uint8).copy()
    M, N = A.shape
    piv, r = [], 0
    for c in range(N):
        p = next((i for i in range(r, M) if A[i, c]), None)
        if p is None:
            continue
        A[[r, p]] = A[[p, r]]
        for i in range(M):
            if i != r and A[i, c]:
                A[i] ^= A[r]
        piv.append(c)
        r += 1
        if r == M:
            break
    free = [c for c in range(N) if c not in piv]
    basis = []
    for f in free:
        x = np.zeros(N, np.uint8)
        x[f] = 1
        for i, c in enumerate(piv):
            x[c] = A[i, f]
        basis.append(x)
    return np.array(basis, np.uint8).reshape(-1, N)


def _random_H(rng, M, N, wmin=2, wmax=7, dead_cols=0):
    H = np.zeros((M, N), np.uint8)
    live = np.arange(dead_cols, N)
    for m in range(M):
        w = int(rng.integers(wmin, min(wmax, live.size) + 1))
        H[m, rng.choice(live, w, replace=False)] = 1
    perm = rng.permutation(N)            # degree-0 columns land anywhere
    return H[:, perm]


def _sparse_case(args):
    (H, L, algo, alpha, beta, llr) = args
    _, dec = _ref()
    ck, status = dec.decode_ldpc(llr.astype(np.float64), H, L, algo, alpha, beta)
    return np.asarray(ck).astype(np.int8), bool(status)


def gen_sparse(pool):
    """decode_ldpc(LLRin, H, L, algo, alpha, beta) (nr_ldpc_decode.py:51-143) on random binary H
    (not TS 38.212 expansions), all algorithms, plus the reference's 4x6 bit-flipping toy H with
    every 1- and 2-bit LLR sign flip of every codeword (ldpc_decoder_bit_flipping.py:115-143), and
    nr_decode_ldpc with a negative offset beta (decode_ldpc's literal zero branches)."""
    rng = np.random.default_rng(4242)
    shapes = [(6, 12), (8, 16), (10, 20), (12, 18), (15, 30), (20, 32), (24, 48), (32, 64),
              (40, 60), (48, 96), (60, 120)]
    abl = [(1.0, 0.0), (0.75, 0.0), (1.0, 0.5), (0.8, 0.3), (1.0, -0.25), (0.7, -0.1)]
    cases = []          # (tag, H, L, algo, alpha, beta, llr)
    for n in range(96):
        M, N = shapes[n % len(shapes)]
        H = _random_H(rng, M, N, dead_cols=int(n % 5 == 0))
        basis = gf2_nullspace(H)
        x = (rng.integers(0, 2, basis.shape[0]) @ basis % 2) if basis.size else np.zeros(N, np.uint8)
        assert not ((H.astype(np.int64) @ x) % 2).any()
        kind = n % 4
        if kind == 3:    # integer LLRs with ties and exact zeros
            llr = (1 - 2 * x.astype(np.float64)) * rng.integers(1, 4, N)
            flip = rng.random(N) < 0.15
            llr[flip] = -llr[flip]
            llr[rng.random(N) < 0.08] = 0.0
        else:
            llr = bpsk_llr(x, float(rng.uniform(-1.0, 4.0)), rng)
        llr = llr.astype(np.float32)
        algo = ["min-sum", "min-sum", "BP", "BF"][n % 4] if n % 7 else "min-sum"
        a, b = abl[n % len(abl)]
        L = [1, 5, 12, 25][(n // 4) % 4]
        cases.append(("rand", H, L, algo, a, b, llr))
    # all-zero LLRs: LQ = 0 -> decision 0 -> syndrome 0 at the first check
    for algo in ("min-sum", "BP", "BF"):
        H = _random_H(rng, 10, 20)
        cases.append(("zeros", H, 8, algo, 1.0, 0.0, np.zeros(20, np.float32)))
    # the reference's toy KAT shape: every codeword, 1-bit and 2-bit sign flips, BF / min-sum / BP
    cw = [x for x in (np.array([(v >> k) & 1 for k in range(6)], np.uint8) for v in range(64))
          if not ((TOY_H @ x) % 2).any()]
    for x in cw:
        base = (2 * (1 - 2 * x.astype(np.float64)) / 10 ** (-255 / 10)).astype(np.float32)
        for m in range(6):
            for two in (False, True):
                llr = base.copy()
                llr[m] = -llr[m]
                if two:
                    llr[(m + 1) % 6] = -llr[(m + 1) % 6]
                for algo in ("BF", "min-sum", "BP"):
                    cases.append(("toy", TOY_H.astype(np.uint8), 8, algo, 1.0, 0.0, llr))
    t = time.time()
    res = pool.map(_sparse_case, [c[1:] for c in cases], chunksize=4)
    print("sparse decode done", time.time() - t)
    # nr_decode_ldpc with beta < 0 on the 38.212 graph (min-sum zero branches as written)
    nr = []
    _, dec = _ref()
    for bg, Zc, snr, a, b in ((2, 4, 1.0, 1.0, -0.3), (1, 3, 0.5, 0.8, -0.2), (2, 6, -0.5, 0.75, -0.5)):
        llr = _mk_awgn(rng, bg, Zc, snr)
        _, ck, st = dec.nr_decode_ldpc(llr.astype(np.float64), Zc, bg, 8, "min-sum", a, b)
        nr.append((bg, Zc, a, b, llr, np.asarray(ck, np.int8), bool(st)))
    kinds = sorted(set(c[0] for c in cases))
    np.savez_compressed(
        os.path.join(OUT, "sparse_golden.npz"),
        kind=np.array([kinds.index(c[0]) for c in cases], np.int8), kinds=np.array(kinds),
        M=np.array([c[1].shape[0] for c in cases], np.int32),
        N=np.array([c[1].shape[1] for c in cases], np.int32),
        H=np.concatenate([np.packbits(c[1].reshape(-1)) for c in cases]),
        H_off=_offs([np.packbits(c[1].reshape(-1)) for c in cases]),
        L=np.array([c[2] for c in cases], np.int32),
        algo=np.array([c[3] for c in cases]),
        alpha=np.array([c[4] for c in cases]), beta=np.array([c[5] for c in cases]),
        llr=np.concatenate([c[6] for c in cases]), llr_off=_offs([c[6] for c in cases]),
        ck_bits=np.concatenate([np.packbits(r[0] == 1) for r in res]),
        ck_off=_offs([np.packbits(r[0] == 1) for r in res]),
        status=np.array([r[1] for r in res]),
        nr_meta=np.array([(r[0], r[1]) for r in nr], np.int32),
        nr_ab=np.array([(r[2], r[3]) for r in nr]),
        nr_llr=np.concatenate([r[4] for r in nr]), nr_llr_off=_offs([r[4] for r in nr]),
        nr_ck=np.concatenate([np.packbits(r[5] == 1) for r in nr]),
        nr_ck_off=_offs([np.packbits(r[5] == 1) for r in nr]),
        nr_status=np.array([r[6] for r in nr]))
    print("sparse cases", len(cases), "status True", sum(r[1] for r in res),
          "nr beta<0 cases", len(nr), [r[6] for r in nr])


# --------------------------------------------------------------------------- rate matching
def gen_ratematch():
    from py5gphy.ldpc import ldpc_info, nr_ldpc_ratematch as RM, nr_ldpc_raterecover as RR
    import oracle_shim as O
    rng = np.random.default_rng(5)
    rows = []
    dns, fes, llrs, rrs = [], [], [], []
    n = 0
    while n < 16:
        bg = 1 + n % 2
        B = int(rng.integers(100, 3000))
        try:
            C, cbz, Lc, F, K, Zc = ldpc_info.get_cbs_info(B, bg)
        except AssertionError:
            continue
        K_apo = K - F
        ck = rng.integers(0, 2, K).astype(np.int8)
        ck[K_apo:] = -1
        dn = O.encode(ck, bg)
        N = dn.size
        Ncb = N if n % 3 else int(rng.integers(K, N + 1))
        Qm = [1, 2, 4, 6, 8][n % 5]
        rv = n % 4
        E = Qm * int(rng.integers(max(1, K // (2 * Qm)), int(1.8 * N) // Qm))
        k0 = RM.get_k0(Ncb, bg, rv, Zc)
        fe = RM.ratematch_ldpc(dn, Ncb, E, k0, Qm)
        y = rng.normal(size=E).astype(np.float32).astype(np.float64)   # stored as float32
        rr = RR.raterecover_ldpc(y, Ncb, N, k0, Qm, Zc, K_apo, K)
        rows.append((bg, Zc, K, K_apo, N, Ncb, E, k0, Qm, rv))
        dns.append(dn)
        fes.append(fe)
        llrs.append(y)
        rrs.append(rr)
        n += 1
    er = []
    for G, C, Qm, NL in [(100000, 5, 2, 1), (36036 * 8 * 4, 129, 8, 4), (12345 * 6, 7, 6, 1),
                         (24000, 3, 4, 2)]:
        er.append((G, C, Qm, NL, RM.get_Er_ldpc(G, C, Qm, NL)))
    np.savez_compressed(os.path.join(OUT, "ratematch_golden.npz"),
                        meta=np.array(rows, np.int64),
                        dn=np.concatenate(dns), dn_off=_offs(dns),
                        fe=np.concatenate(fes), fe_off=_offs(fes),
                        llr=np.concatenate(llrs).astype(np.float32), llr_off=_offs(llrs),
                        rr=np.concatenate(rrs), rr_off=_offs(rrs))
    with open(os.path.join(OUT, "er_golden.json"), "w") as f:
        json.dump([{"G": a, "C": b, "Qm": c, "NL": d, "Er": e} for a, b, c, d, e in er], f)
    print("ratematch cases", len(rows))


# -------------------------------------------------------------------------------------- CRC
def gen_crc():
    from py5gphy.crc import crc
    rng = np.random.default_rng(9)
    out = []
    for poly in ["6", "11", "16", "24A", "24B", "24C"]:
        for mask in (0, 1, 12345, 45678):
            for n in (1, 8, 37, 200):
                blk = rng.integers(0, 2, n)
                out.append({"poly": poly, "mask": mask, "blk": blk.tolist(),
                            "out": crc.nr_crc_encode(blk, poly, mask).tolist()})
    with open(os.path.join(OUT, "crc_golden.json"), "w") as f:
        json.dump(out, f)
    print("crc cases", len(out))


# ------------------------------------------------------------------------------------ DL-SCH
def gen_dlsch():
    from py5gphy.nr_pdsch import nr_dlsch
    rng = np.random.default_rng(11)
    rows, tbs, gs = [], [], []
    # (TBS, Qm, R*1024, NL, rv, TBS_LBRM, G): a BG2 single-CB TB and BG1 multi-CB TBs
    for TBS, Qm, R, NL, rv, LBRM, G in [(1800, 2, 308, 1, 0, 40000, 6000),
                                        (24000, 6, 658, 2, 1, 100000, 40008),
                                        (12000, 4, 517, 1, 2, 30000, 25000)]:
        trblk = rng.integers(0, 2, TBS)
        g = nr_dlsch.DLSCHEncode(trblk, TBS, Qm, R, NL, rv, LBRM, G)
        rows.append((TBS, Qm, R, NL, rv, LBRM, G))
        tbs.append(np.packbits(trblk.astype(np.uint8)))
        gs.append(np.packbits(g == 1))
    np.savez_compressed(os.path.join(OUT, "dlsch_golden.npz"), meta=np.array(rows, np.int64),
                        tb=np.concatenate(tbs), tb_off=_offs(tbs),
                        g=np.concatenate(gs), g_off=_offs(gs))
    print("dlsch cases", len(rows))


# ------------------------------------------------------------------ SCH chain (TX + RX, DL + UL)
def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def gen_sch():
    """DLSCHDecode / ULSCH_decoding (+ HARQ) and UL-SCH encode, and one full-size config-5
    transport block through DLSCHEncode.  LLRs are stored float32 and the reference runs on
    their float64 widening; new_LLr_dns is pinned by a sha256 of its float64 bytes."""
    from py5gphy.nr_pdsch import nr_dlsch, nr_dlsch_decode
    from py5gphy.nr_pusch import nr_ulsch, nr_ulsch_decode
    rng = np.random.default_rng(21)
    cases, blobs = [], {}
    dec_cfg = {"L": 6, "algo": "min-sum", "alpha": 0.8, "beta": 0.0}
    # (kind, TBS, Qm, R*1024, NL, rv, LBRM, G, snr_db)
    specs = [("dl", 12000, 4, 517, 1, 0, 30000, 25000, 3.0),
             ("dl", 12000, 4, 517, 1, 0, 30000, 25000, -1.0),
             ("dl", 1800, 2, 308, 1, 0, 40000, 6000, 1.0),
             ("ul", 8000, 2, 600, 1, 0, 0, 16000, 2.0),
             ("ul", 2000, 4, 200, 1, 3, 0, 9000, 0.0)]
    for n, (kind, TBS, Qm, R, NL, rv, LBRM, G, snr) in enumerate(specs):
        trblk = rng.integers(0, 2, TBS)
        if kind == "dl":
            g = nr_dlsch.DLSCHEncode(trblk, TBS, Qm, R, NL, rv, LBRM, G)
        else:
            cbs, Zc, bgn = nr_ulsch.ULSCH_Crc_CodeBlockSegment(trblk, TBS, R)
            blobs[f"cbs{n}"] = np.packbits((cbs.reshape(-1) == 1).astype(np.uint8))
            blobs[f"cbsfill{n}"] = np.array([cbs.shape[0], cbs.shape[1], int(np.sum(cbs[0] == -1))])
            g = nr_ulsch.ULSCH_encoding_ratematch(cbs, Zc, bgn, Qm, G, NL, rv)
        llr = bpsk_llr(g, snr, rng).astype(np.float32)
        x = llr.astype(np.float64)
        if kind == "dl":
            ok, tbblk, new = nr_dlsch_decode.DLSCHDecode(x, TBS, Qm, R, NL, rv, LBRM, dec_cfg)
            # HARQ retransmission (rv 2) combined with the first decoder input
            g2 = nr_dlsch.DLSCHEncode(trblk, TBS, Qm, R, NL, 2, LBRM, G)
            llr2 = bpsk_llr(g2, snr, rng).astype(np.float32)
            ok2, tb2, new2 = nr_dlsch_decode.DLSCHDecode(llr2.astype(np.float64), TBS, Qm, R, NL, 2,
                                                         LBRM, dec_cfg, True, new)
        else:
            ok, tbblk, new = nr_ulsch_decode.ULSCH_decoding(x, TBS, R, Qm, G, NL, rv, dec_cfg)
            llr2, ok2, tb2, new2 = np.zeros(1, np.float32), ok, tbblk, new
        cases.append({"kind": kind, "TBS": TBS, "Qm": Qm, "R": R, "NL": NL, "rv": rv,
                      "LBRM": LBRM, "G": G, "snr": snr, "ok": bool(ok), "ok2": bool(ok2),
                      "new_sha": _sha(new), "new2_sha": _sha(new2), "new_shape": list(new.shape),
                      "new_sum": float(np.sum(new))})
        blobs[f"trblk{n}"] = np.packbits(trblk.astype(np.uint8))
        blobs[f"g{n}"] = np.packbits((g == 1).astype(np.uint8))
        blobs[f"llr{n}"] = llr
        blobs[f"llr2_{n}"] = llr2
        blobs[f"tbblk{n}"] = np.packbits(np.asarray(tbblk).astype(np.uint8))
        blobs[f"tbblk2_{n}"] = np.packbits(np.asarray(tb2).astype(np.uint8))
        print("sch case", n, kind, "ok", ok, "ok2", ok2, flush=True)
    # config 5: 273 PRB 256QAM 4 layers, TBS 1,081,512 (dl_tbsize.py:308-317), C = 129
    TBS, Qm, R, NL, rv, G = 1081512, 8, 948, 4, 0, 8 * 4 * 36036
    trblk = rng.integers(0, 2, TBS)
    g = nr_dlsch.DLSCHEncode(trblk, TBS, Qm, R, NL, rv, TBS, G)
    cases.append({"kind": "dl-encode", "TBS": TBS, "Qm": Qm, "R": R, "NL": NL, "rv": rv,
                  "LBRM": TBS, "G": G})
    n = len(cases) - 1
    blobs[f"trblk{n}"] = np.packbits(trblk.astype(np.uint8))
    blobs[f"g{n}"] = np.packbits((g == 1).astype(np.uint8))
    np.savez_compressed(os.path.join(OUT, "sch_golden.npz"), **blobs)
    with open(os.path.join(OUT, "sch_golden.json"), "w") as f:
        json.dump(cases, f, indent=0)
    print("sch cases", len(cases))


def gen_sch_negbeta():
    """DLSCHDecode / ULSCH_decoding with a negative offset beta: the reference decodes every
    codeblock through nr_decode_ldpc (nr_dlsch_decode.py:91, nr_ulsch_decode.py:92), whose
    min-sum keeps its literal zero branches for beta < 0 (nr_ldpc_decode.py:186-225)."""
    from py5gphy.nr_pdsch import nr_dlsch, nr_dlsch_decode
    from py5gphy.nr_pusch import nr_ulsch, nr_ulsch_decode
    rng = np.random.default_rng(31)
    cases, blobs = [], {}
    specs = [("dl", 12000, 4, 517, 1, 0, 30000, 25000, 1.0, -0.25),
             ("ul", 2000, 4, 200, 1, 3, 0, 9000, 0.0, -0.5)]
    for n, (kind, TBS, Qm, R, NL, rv, LBRM, G, snr, beta) in enumerate(specs):
        dec_cfg = {"L": 5, "algo": "min-sum", "alpha": 0.8, "beta": beta}
        trblk = rng.integers(0, 2, TBS)
        if kind == "dl":
            g = nr_dlsch.DLSCHEncode(trblk, TBS, Qm, R, NL, rv, LBRM, G)
        else:
            cbs, Zc, bgn = nr_ulsch.ULSCH_Crc_CodeBlockSegment(trblk, TBS, R)
            g = nr_ulsch.ULSCH_encoding_ratematch(cbs, Zc, bgn, Qm, G, NL, rv)
        llr = bpsk_llr(g, snr, rng).astype(np.float32)
        x = llr.astype(np.float64)
        if kind == "dl":
            ok, tbblk, new = nr_dlsch_decode.DLSCHDecode(x, TBS, Qm, R, NL, rv, LBRM, dec_cfg)
        else:
            ok, tbblk, new = nr_ulsch_decode.ULSCH_decoding(x, TBS, R, Qm, G, NL, rv, dec_cfg)
        cases.append({"kind": kind, "TBS": TBS, "Qm": Qm, "R": R, "NL": NL, "rv": rv,
                      "LBRM": LBRM, "G": G, "snr": snr, "dec": dec_cfg, "ok": bool(ok),
                      "new_sha": _sha(new), "new_shape": list(new.shape)})
        blobs[f"llr{n}"] = llr
        blobs[f"tbblk{n}"] = np.packbits(np.asarray(tbblk).astype(np.uint8))
        print("sch beta<0 case", n, kind, "ok", ok, flush=True)
    np.savez_compressed(os.path.join(OUT, "sch_negbeta_golden.npz"), **blobs)
    with open(os.path.join(OUT, "sch_negbeta_golden.json"), "w") as f:
        json.dump(cases, f, indent=0)


# ------------------------------------------------------- modulation / demodulation / PRBS (f4)
def gen_demod():
    """nrModulate (common/nrModulation.py:4-41), nrDemodulate (demodulation/nr_Demodulation.py:
    12-46) for QPSK..256QAM, gen_nrPRBS (common/nrPRBS.py:5-25)."""
    from py5gphy.common import nrModulation, nrPRBS
    from py5gphy.demodulation import nr_Demodulation
    rng = np.random.default_rng(17)
    blobs, meta = {}, []
    for k, (mod, Qm, scale) in enumerate([("qpsk", 2, 2), ("16qam", 4, 10), ("64qam", 6, 42),
                                          ("256qam", 8, 170)]):
        n = 3000
        bits = rng.integers(0, 2, n * Qm)
        sym = nrModulation.nrModulate(bits, mod)
        A = 1 / np.sqrt(scale)
        # noisy symbols + exact decision-threshold values (multiples of A) + zeros
        y = sym.astype(np.complex128) + (rng.normal(0, 0.3, n) + 1j * rng.normal(0, 0.3, n)) * A * 3
        th = rng.integers(-16, 17, 400) * A
        y[:400] = th + 1j * th[::-1]
        y[400:410] = 0.0
        nv = rng.uniform(0.01, 1.0, n)
        _, llr = nr_Demodulation.nrDemodulate(y, mod, nv)
        blobs[f"bits{k}"] = np.packbits(bits.astype(np.uint8))
        blobs[f"sym{k}"] = np.asarray(sym)                      # reference modulation output
        blobs[f"y{k}"] = y
        blobs[f"nv{k}"] = nv.astype(np.float32)
        blobs[f"llr{k}"] = np.asarray(llr, np.float32)
        meta.append((Qm, n))
    prbs = []
    for j, (cinit, N) in enumerate([(0, 64), (1, 1000), (12345 * 2 ** 15 + 7, 100003),
                                    (2 ** 31 - 1, 4096), (65535 * 2 ** 15 + 1023, 1153152)]):
        seq = nrPRBS.gen_nrPRBS(cinit, N)
        blobs[f"prbs{j}"] = np.packbits(seq.astype(np.uint8))
        prbs.append((cinit, N))
    np.savez_compressed(os.path.join(OUT, "demod_golden.npz"), meta=np.array(meta, np.int64),
                        prbs_meta=np.array(prbs, np.int64), **blobs)
    print("demod cases", len(meta), "prbs cases", len(prbs))


def gen_demod2():
    """The remaining modulations of nrModulate / nrDemodulate: BPSK, pi/2-BPSK, 1024QAM
    (common/nrModulation.py:15-21,38-42; demodulation/demod_bpsk.py, demod_pi2_bpsk.py,
    demod_1024qam.py), and all seven with complex64 input symbols (numpy >= 2 evaluates the
    per-symbol formulas in float32 then; complex128 input keeps them in float64)."""
    from py5gphy.common import nrModulation
    from py5gphy.demodulation import nr_Demodulation
    rng = np.random.default_rng(29)
    mods = [("bpsk", 1, 2), ("pi/2-bpsk", 1, 2), ("qpsk", 2, 2), ("16qam", 4, 10),
            ("64qam", 6, 42), ("256qam", 8, 170), ("1024qam", 10, 682)]
    blobs, meta = {}, []
    for k, (mod, Qm, scale) in enumerate(mods):
        n = 3001 if Qm == 1 else 3000      # odd length: pi/2-BPSK's odd/even split
        bits = rng.integers(0, 2, n * Qm)
        sym = nrModulation.nrModulate(bits, mod)
        A = 1 / np.sqrt(scale)
        lev = int(np.sqrt(scale * 2)) if Qm > 1 else 2
        y = sym.astype(np.complex128) + (rng.normal(0, 0.3, n) + 1j * rng.normal(0, 0.3, n)) * A * 3
        th = rng.integers(-2 * lev, 2 * lev + 1, 400) * A     # exact decision thresholds
        y[:400] = th + 1j * th[::-1]
        y[400:410] = 0.0
        nv = rng.uniform(0.01, 1.0, n)
        _, llr = nr_Demodulation.nrDemodulate(y, mod, nv)
        y64 = y.astype(np.complex64)
        _, llr64 = nr_Demodulation.nrDemodulate(y64, mod, nv)
        blobs[f"bits{k}"] = np.packbits(bits.astype(np.uint8))
        blobs[f"sym{k}"] = np.asarray(sym)
        blobs[f"y{k}"] = y
        blobs[f"nv{k}"] = nv.astype(np.float32)
        blobs[f"llr{k}"] = np.asarray(llr)                  # float64 for BPSK (demod_bpsk.py:9)
        blobs[f"llr_c64_{k}"] = np.asarray(llr64)
        meta.append((k, Qm, n))
    np.savez_compressed(os.path.join(OUT, "demod2_golden.npz"), meta=np.array(meta, np.int64),
                        mods=np.array([m[0] for m in mods]), **blobs)
    print("demod2 cases", len(meta))


def gen_config1():
    """BASELINE config 1 exactly: BG2 Zc=8, CRC24A, for_test_5g_ldpc_encoder (nr_ldpc_decode.py:
    229-260, global numpy RNG seeded per case) then nr_decode_ldpc(..., L=8, 'min-sum', 0.75, 0)
    (NMS alpha=.75), 7 SNRs x 6 codeblocks."""
    _, dec = _ref()
    rows = []
    blk_l, dn_l, llr_l, ck_l = [], [], [], []
    for snr in (-3.0, -2.0, -1.0, 0.0, 1.0, 2.0, 3.0):
        for j in range(6):
            seed = 1000 + len(rows)
            np.random.seed(seed)
            blk, dn, llr = dec.for_test_5g_ldpc_encoder(8, 2, snr, "24A")
            _, ck, status = dec.nr_decode_ldpc(llr, 8, 2, 8, "min-sum", 0.75, 0)
            rows.append((seed, snr, int(bool(status))))
            blk_l.append(np.asarray(blk, np.int8))
            dn_l.append(np.asarray(dn, np.int8))
            llr_l.append(np.asarray(llr, np.float64))
            ck_l.append(np.asarray(ck, np.int8))
    np.savez_compressed(os.path.join(OUT, "config1_golden.npz"),
                        seed=np.array([r[0] for r in rows], np.int64),
                        snr=np.array([r[1] for r in rows], np.float64),
                        status=np.array([r[2] for r in rows], np.uint8),
                        blk=np.stack(blk_l), dn=np.stack(dn_l), llr=np.stack(llr_l),
                        ck=np.stack(ck_l))
    print("config1 cases", len(rows), "converged", sum(r[2] for r in rows))


class _NoGlobals(__import__("pickle").Unpickler):
    """Loads plain containers only: any class or function reference in the stream raises, so
    nothing from the file can execute."""
    def find_class(self, module, name):
        raise __import__("pickle").UnpicklingError(f"blocked {module}.{name}")


# BLER pickles written by scripts/internal/sim_ldpc_internal.py:89-91 ([sim_config, labels,
# bler_lists]) and the SNR lists of the scripts that wrote them (the pickles do not store them).
# Two pickles come from FIXED-COUNT harnesses instead of the stopping rule (FIXED_PIN_FILES).
PIN_FILES = (
    [(f"NMS_search_alpha_ZC{z}_bgn{b}.pickle", "scripts/NMS_ldpc_search_best_alpha.py:13-27", [-0.5])
     for z in (8, 12, 28, 40, 72, 176, 208, 384) for b in (1, 2) if (z, b) != (384, 2)] +
    [(f"OMS_search_beta_ZC{z}_bgn{b}.pickle", "scripts/OMS_ldpc_search_best_beta.py:13-27", [-0.5])
     for z in (12, 28, 40, 72, 176, 208) for b in (1, 2)] +
    [("OMS_search_beta_ZC2_bgn1.pickle", "scripts/OMS_ldpc_search_best_beta.py:13 (commented list)", [-0.5])] +
    [(f"mixed_MS_search_pair_ZC{z}_bgn{b}.pickle", "scripts/mixed_MS_ldpc_search_best_pair.py:13-27", [-1.0, -0.5])
     for z, b in ((12, 1), (12, 2), (28, 1))] +
    [("ldpc_decode_result_opt.pickle", "scripts/sim_ldpc_decoder.py:20-40 (L=32 run)", [-1.0, -0.5, 0.0, 0.5, 1.0]),
     ("ldpc_decode_result_opt_2.pickle", "scripts/sim_ldpc_decoder.py:20-40", [-1.0, -0.5, 0.0, 0.5, 1.0]),
     ("ldpc_decode_result_for_L.pickle", "scripts/sim_ldpc_decoder.py:57-81", [-1.0, -0.5, 0.0, 0.5])])


# Fixed trial counts per SNR (no stopping rule):
#  * ldpc_decode_result_BF.pickle — scripts/sim_ldpc_decoder_bf.py:19-33,73-98: Zc=10 BG1 'BF',
#    L in {16,32,64}, snr 2..5.5 step 0.5, total_count = 200 if snr < 4 else 2000;
#  * ldpc_decode_result_all.pickle — Zc=10 BG1 L=32, BP / min-sum / NMS .8,.5 / OMS .3,.1 / mixed
#    (.8,.3) at snr -1..1 step 0.5 (the axis of out/ldpc_decode_result_all.png).  The harness that
#    wrote it is not in the snapshot; its count per SNR is inferred as the least common denominator
#    of that SNR's published values (every value is a whole number of failures at that count):
#    300, 300, 1200, 4500, 4500.
FIXED_PIN_FILES = (
    ("ldpc_decode_result_BF.pickle", "scripts/sim_ldpc_decoder_bf.py:19-33,73-98",
     [2.0, 2.5, 3.0, 3.5, 4.0, 4.5, 5.0, 5.5], lambda snr, col: 200 if snr < 4 else 2000),
    ("ldpc_decode_result_all.pickle", "Zc=10 BG1 L=32 algorithm comparison (fixed counts inferred)",
     [-1.0, -0.5, 0.0, 0.5, 1.0], lambda snr, col: _lcd(col)),
)


def _lcd(values):
    """Least common denominator of the BLER values (limit 10^5): the smallest trial count at
    which every value is a whole number of failures."""
    from fractions import Fraction
    from math import lcm
    d = 1
    for v in values:
        d = lcm(d, Fraction(v).limit_denominator(100000).denominator)
    return d


def _parse_label(s):
    """'NMS-alpha=0.7-L=32' / 'OMS-beta=0.5-L=16' / 'mixed-MS-[alpha,beta]=[0.8,0.3]-L=32' /
    'BP L=32' / 'min-sum L=32' -> (algo, alpha, beta, L), the reverse of the reference's
    label format (sim_ldpc_internal.py:15-41)."""
    import re
    m = re.fullmatch(r"NMS-alpha=([\d.]+)-L=(\d+)", s)
    if m:
        return "min-sum", float(m[1]), 0.0, int(m[2])
    m = re.fullmatch(r"OMS-beta=([\d.]+)-L=(\d+)", s)
    if m:
        return "min-sum", 1.0, float(m[1]), int(m[2])
    m = re.fullmatch(r"mixed-MS-\[alpha,beta\]=\[([\d.]+),([\d.]+)\]-L=(\d+)", s)
    if m:
        return "min-sum", float(m[1]), float(m[2]), int(m[3])
    m = re.fullmatch(r"(BP|min-sum|BF) L=(\d+)", s)
    return m[1], 1.0, 0.0, int(m[2])


def gen_pins():
    """tests/golden/bler_pins.json: every LDPC BLER value the reference published in out/."""
    pins = []
    for fname, src, snrs in PIN_FILES:
        with open(os.path.join(REF, "out", fname), "rb") as fh:
            cfg, labels, results = _NoGlobals(fh).load()
        for lab, bl in zip(labels, results):
            assert len(bl) == len(snrs), (fname, lab)
            algo, alpha, beta, L = _parse_label(lab)
            for snr, p in zip(snrs, bl):
                pins.append({"file": "out/" + fname, "Zc": cfg["Zc"], "bgn": cfg["bgn"],
                             "label": lab, "algo": algo, "alpha": alpha, "beta": beta, "L": L,
                             "snr": snr, "bler": p, "config": src})
    for fname, src, snrs, count in FIXED_PIN_FILES:
        with open(os.path.join(REF, "out", fname), "rb") as fh:
            cfg, labels, results = _NoGlobals(fh).load()
        for k, snr in enumerate(snrs):
            col = [bl[k] for bl in results]
            n_ref = count(snr, col)
            for lab, bl in zip(labels, results):
                assert len(bl) == len(snrs), (fname, lab)
                p = bl[k]
                assert abs(p * n_ref - round(p * n_ref)) < 1e-6, (fname, lab, snr, p, n_ref)
                algo, alpha, beta, L = _parse_label(lab)
                pins.append({"file": "out/" + fname, "Zc": cfg["Zc"], "bgn": cfg["bgn"],
                             "label": lab, "algo": algo, "alpha": alpha, "beta": beta, "L": L,
                             "snr": snr, "bler": p, "config": src, "n_ref": n_ref,
                             "rule": "fixed"})
    doc = {"_source": "BLER values the reference published in /root/reference/out/*.pickle "
                      "(written by scripts/internal/sim_ldpc_internal.py:89-91), read by "
                      "tests/golden/gen_golden.py gen_pins() with a no-globals unpickler; SNR "
                      "lists from the scripts named in 'config'.  Every point is per-BPSK-symbol "
                      "Es/N0 (nr_ldpc_decode.py:253-257), CRC24A, the reference's stopping rule "
                      "(sim_ldpc_internal.py:66-77) except pins with rule 'fixed': n_ref trials "
                      "per point (scripts/sim_ldpc_decoder_bf.py:73-98; the _all pickle's counts "
                      "inferred per SNR, gen_golden.py FIXED_PIN_FILES).",
           "pins": pins}
    with open(os.path.join(OUT, "bler_pins.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print("bler pins", len(pins))


if __name__ == "__main__":
    os.chdir(REF)
    sys.path.insert(0, OUT)    # oracle_shim: the build's oracle, used only to make codewords
    which = sys.argv[1:] or ["encode", "crc", "ratematch", "dlsch", "sch", "demod", "decode", "bfbp",
                             "demod2", "config1", "pins", "sparse"]
    if "demod2" in which:
        gen_demod2()
    if "config1" in which:
        gen_config1()
    if "pins" in which:
        gen_pins()
    if "encode" in which:
        gen_encode()
    if "crc" in which:
        gen_crc()
    if "ratematch" in which:
        gen_ratematch()
    if "dlsch" in which:
        gen_dlsch()
    if "sch" in which:
        gen_sch()
    if "sch_negbeta" in which:
        gen_sch_negbeta()
    if "demod" in which:
        gen_demod()
    if "decode" in which:
        with mp.get_context("fork").Pool(6) as pool:
            gen_decode(pool)
    if "bfbp" in which:
        with mp.get_context("fork").Pool(6) as pool:
            gen_bf_bp(pool)
    if "sparse" in which:
        with mp.get_context("fork").Pool(6) as pool:
            gen_sparse(pool)
