"""CPU ORACLE for the py5gphy/ldpc hot path — TEST INFRASTRUCTURE ONLY.

This module is a numpy restatement of the reference algorithms (xu753x/python_5gtoolbox,
``py5gphy/ldpc``).  It is imported only by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — as the checker / the timed CPU baseline, never as the
product path.  The product (``python_5gtoolbox_amd``) runs the HIP kernels and fails loudly when
they are unavailable.

Parity pinning: every function below is checked against golden vectors produced by the reference
itself in the build container (``tests/golden/gen_golden.py``; fixtures in ``tests/golden/``).

Contents (reference file:line each restates):
  find_iLS, get_cbs_info ........ py5gphy/ldpc/ldpc_info.py:81-97, :5-78
  graph / getH ................... py5gphy/ldpc/ldpc_info.py:99-139 (edge-list form, no dense H)
  encode ......................... py5gphy/ldpc/nr_ldpc_encode.py:8-50, :52-115 (optimised A/B/C path)
  decode_flooding ................ py5gphy/ldpc/nr_ldpc_decode.py:11-49, :51-143, :178-227
  decode_layered ................. (no reference: the build's layered perf schedule)
  decode_bf ...................... py5gphy/ldpc/ldpc_decoder_bit_flipping.py:5-73
  decode_bp ...................... py5gphy/ldpc/nr_ldpc_decode.py:51-143, :145-176
  decode_sparse .................. py5gphy/ldpc/nr_ldpc_decode.py:51-227 (any binary H, dense form),
                                   ldpc_decoder_bit_flipping.py:5-73
  crc_encode / crc_decode ........ py5gphy/crc/crc.py:4-88
  get_Er / get_k0 / ratematch / raterecover  py5gphy/ldpc/nr_ldpc_ratematch.py:5-97,
                                              py5gphy/ldpc/nr_ldpc_raterecover.py:6-65
  cbsegment ...................... py5gphy/ldpc/nr_ldpc_cbsegment.py:7-33
"""
import json
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_NPZ = os.path.join(os.path.dirname(_HERE), "python_5gtoolbox_amd", "data", "nr_ldpc_bg.npz")

ZSETS = [[2, 4, 8, 16, 32, 64, 128, 256], [3, 6, 12, 24, 48, 96, 192, 384],
         [5, 10, 20, 40, 80, 160, 320], [7, 14, 28, 56, 112, 224], [9, 18, 36, 72, 144, 288],
         [11, 22, 44, 88, 176, 352], [13, 26, 52, 104, 208], [15, 30, 60, 120, 240]]
ZLIST = sorted(z for s in ZSETS for z in s)

_TAB = None


def tables():
    global _TAB
    if _TAB is None:
        d = np.load(_NPZ)
        _TAB = {1: d["BG1"], 2: d["BG2"]}
    return _TAB


def find_iLS(Zc):
    """ldpc_info.py:81-97 — lifting-set index, 255 when Zc is not a legal lifting size."""
    for s, zs in enumerate(ZSETS):
        if Zc in zs:
            return s
    return 255


def get_cbs_info(B, bgn):
    """ldpc_info.py:5-78 — (C, cbz, L, F, K, Zc) of TS 38.212 §5.2.2 CB segmentation."""
    Kcb = 8448 if bgn == 1 else 3840
    if B <= Kcb:
        L, C, Bd = 0, 1, B
    else:
        L = 24
        C = int(math.ceil(B / (Kcb - L)))
        Bd = B + C * L
    cbz = B // C
    assert B % C == 0
    Kd = Bd // C
    assert Bd % C == 0
    if bgn == 1:
        Kb = 22
    else:
        Kb = 10 if B > 640 else 9 if B > 560 else 8 if B > 192 else 6
    Zc = next(v for v in ZLIST if v * Kb >= Kd)
    K = 22 * Zc if bgn == 1 else 10 * Zc
    return C, cbz, L, K - Kd, K, Zc


class Graph:
    """Expanded QC parity-check structure for (bgn, Zc) as edge lists (ldpc_info.py:124-137:
    block (i,j) is I_Zc right-shifted by V(i,j) mod Zc, so row i*Zc+m connects column
    j*Zc+(m+V)%Zc)."""

    def __init__(self, bgn, Zc):
        assert bgn in (1, 2)
        iLS = find_iLS(Zc)
        assert iLS < 8
        V = tables()[bgn][iLS].astype(np.int64)
        self.bgn, self.Zc, self.iLS = bgn, Zc, iLS
        self.Mb, self.Nb = V.shape
        self.Kb = 22 if bgn == 1 else 10
        self.K = self.Kb * Zc
        self.N = (66 if bgn == 1 else 50) * Zc        # transmitted length
        self.Nf = self.Nb * Zc                        # full codeword (2Zc punctured + N)
        self.Kcore = self.Kb + 4                      # columns of degree > 1
        ii, jj = np.nonzero(V >= 0)
        self.bi, self.bj = ii, jj
        self.bv = V[ii, jj] % Zc
        self.rs = np.searchsorted(ii, np.arange(self.Mb + 1))
        self.V = V
        m = np.arange(Zc)
        # per base edge b: columns hit by rows m = 0..Zc-1
        self.ecol = jj[:, None] * Zc + (m[None, :] + self.bv[:, None]) % Zc   # (Eb, Zc)

    def shift(self, i, j):
        return int(self.V[i, j]) % self.Zc

    def rows_cols(self, i):
        """(deg, Zc) column indices of base row i's edges."""
        return self.ecol[self.rs[i]:self.rs[i + 1]]


_GRAPHS = {}


def graph(bgn, Zc):
    key = (bgn, Zc)
    if key not in _GRAPHS:
        _GRAPHS[key] = Graph(bgn, Zc)
    return _GRAPHS[key]


def getH(Zc, bgn, iLS=None):
    """ldpc_info.py:99-139 — dense int8 H (small Zc only; used by tests)."""
    g = graph(bgn, Zc)
    H = np.zeros((g.Mb * Zc, g.Nf), np.int8)
    m = np.arange(Zc)
    for b in range(len(g.bi)):
        H[g.bi[b] * Zc + m, g.ecol[b]] = 1
    return H


# ----------------------------------------------------------------------------------- encode
def _rot(x, s):
    """(P_s x)[m] = x[(m+s) % Zc] along the last axis (one shifted-identity block times x)."""
    Zc = x.shape[-1]
    return x[..., (np.arange(Zc) + s) % Zc]


def encode(ck, bgn):
    """nr_ldpc_encode.py:8-50 + _gen_ldpc_parity_bit :52-115 (the optimised A/B/C method), batched.

    ck: (B, K) or (K,) integer array, values 0/1 and -1 for filler bits.  Parity arithmetic is
    the reference's int8 mat-vec mod 2, i.e. the XOR of the LSBs; fillers at k >= 2Zc are zeroed
    first (:32-37), fillers before 2Zc keep LSB 1 as in the reference's -1 entries.
    Returns dn (B, N) int8: dn[0:K-2Zc] = ck[2Zc:K] (fillers stay -1), dn[K-2Zc:] = parity.
    Does NOT mutate ck (the product wrapper reproduces the in-place filler zeroing)."""
    ck = np.asarray(ck)
    one = ck.ndim == 1
    ck2 = np.atleast_2d(ck).astype(np.int64)
    B, K = ck2.shape
    Kb = 22 if bgn == 1 else 10
    Zc = K // Kb
    g = graph(bgn, Zc)
    assert K == g.K
    bits = (ck2 & 1).astype(np.uint8)
    tail = ck2[:, 2 * Zc:] == -1
    bits[:, 2 * Zc:][tail] = 0
    blk = bits.reshape(B, Kb, Zc)
    lam = np.zeros((4, B, Zc), np.uint8)
    for i in range(4):
        for b in range(g.rs[i], g.rs[i + 1]):
            j = g.bj[b]
            if j < Kb:
                lam[i] ^= _rot(blk[:, j], g.bv[b])
    L2 = lam[0] ^ lam[1] ^ lam[2] ^ lam[3]
    if bgn == 1:
        p1 = np.roll(L2, g.shift(1, 22), axis=1)
        p2 = lam[0] ^ _rot(p1, g.shift(0, 22))
        p4 = lam[3] ^ _rot(p1, g.shift(3, 22))
        p3 = lam[2] ^ _rot(p4, g.shift(2, 25))
    else:
        p1 = np.roll(L2, g.shift(2, 10), axis=1)
        p2 = lam[0] ^ _rot(p1, g.shift(0, 10))
        p4 = lam[3] ^ _rot(p1, g.shift(3, 10))
        p3 = lam[1] ^ _rot(p2, g.shift(1, 11))
    x = np.concatenate([blk, np.stack([p1, p2, p3, p4], 1)], axis=1)   # (B, Kb+4, Zc)
    pe = np.zeros((B, g.Mb - 4, Zc), np.uint8)
    for i in range(4, g.Mb):
        for b in range(g.rs[i], g.rs[i + 1]):
            j = g.bj[b]
            if j < Kb + 4:
                pe[:, i - 4] ^= _rot(x[:, j], g.bv[b])
    dn = np.empty((B, g.N), np.int8)
    dn[:, :K - 2 * Zc] = ck2[:, 2 * Zc:].astype(np.int8)
    dn[:, K - 2 * Zc:K + 2 * Zc] = np.stack([p1, p2, p3, p4], 1).reshape(B, 4 * Zc)
    dn[:, K + 2 * Zc:] = pe.reshape(B, -1)
    return dn[0] if one else dn


def syndrome(bits, bgn, Zc):
    """(H @ bits) % 2 for bits (B, Nf) — used to check codewords."""
    g = graph(bgn, Zc)
    bits = np.atleast_2d(bits).astype(np.uint8)
    s = np.zeros((bits.shape[0], g.Mb, Zc), np.uint8)
    for i in range(g.Mb):
        s[:, i] = np.bitwise_xor.reduce(bits[:, g.rows_cols(i)], axis=1)
    return s.reshape(bits.shape[0], -1)


# ----------------------------------------------------------------------------------- decode
def _row_hd_fail(hd, g):
    """True where any parity check of hd (B, Nf) bool fails (nr_ldpc_decode.py:111-112)."""
    fail = np.zeros(hd.shape[0], bool)
    for i in range(g.Mb):
        par = np.bitwise_xor.reduce(hd[:, g.rows_cols(i)], axis=1)
        fail |= par.any(axis=1)
    return fail


def _cn_update(q, alpha, beta, T):
    """Min-sum check-node update of one base row, q: (B, d, Zc) of dtype T.

    Restates _min_sum_process (nr_ldpc_decode.py:178-227): for every edge,
    Lr = alpha * prod_{others} sign(Lq) * max(min_{others} |Lq| - beta, 0).
    Two-min form: mag = min2 on the edge(s) equal to min1, else min1 (ties give min2 == min1);
    sign(0) taken as +1 — the reference's zero branches (:203-225) are exactly this (a zero
    among the others forces magnitude 0, and an edge's own sign cancels in s*sign(e))."""
    a = np.abs(q)
    min1 = a.min(axis=1, keepdims=True)
    eq = a == min1
    cnt = eq.sum(axis=1, keepdims=True)
    min2 = np.where(eq, T(np.inf), a).min(axis=1, keepdims=True)
    min2 = np.where(cnt >= 2, min1, min2)
    neg = q < 0
    s = np.bitwise_xor.reduce(neg, axis=1, keepdims=True)
    mag = np.where(eq, min2, min1)
    m = alpha * np.maximum(mag - beta, T(0))
    return np.where(neg ^ s, -m, m).astype(T)


def decode_flooding(llr, Zc, bgn, L, alpha=1.0, beta=0.0, dtype=np.float64):
    """nr_decode_ldpc + decode_ldpc (nr_ldpc_decode.py:11-49, :51-143), flooding schedule, batched.

    llr: (B, N) with N = 66Zc (BG1) / 50Zc (BG2); LLR = log P0/P1.
    Returns ck (B, Nf) int8, status (B,) bool, iters (B,) int32 — iters = number of check-node
    updates performed (the reference's loop index at its early return, or L).

    Semantics (restated exactly):
      LQ = [0]*2Zc ++ llr; Lq = LQ on edges; Lr = 0            (:43, :94-101)
      for it < L: ck = LQ<0; if syndrome == 0 -> return       (:105-114)
                  Lr = CN(Lq) for every row                    (:117-123)
                  LQ = LLR + sum_rows Lr  (row-ascending sum)  (:126)
                  Lq = LQ - Lr on edges                        (:129-131)
      ck = LQ<=0; status = syndrome == 0                       (:133-143)
    dtype float64 reproduces the reference bit for bit; float32 is the same algorithm with
    every operation rounded to fp32 (alpha, beta cast to fp32)."""
    T = np.dtype(dtype).type
    llr = np.atleast_2d(np.asarray(llr))
    g = graph(bgn, Zc)
    B = llr.shape[0]
    assert llr.shape[1] == g.N
    alpha, beta = T(alpha), T(beta)
    Lfull = np.concatenate([np.zeros((B, 2 * Zc), T), llr.astype(T)], axis=1)
    LQ = Lfull.copy()
    Lr = [np.zeros((B, g.rs[i + 1] - g.rs[i], Zc), T) for i in range(g.Mb)]
    done = np.zeros(B, bool)
    ck = np.zeros((B, g.Nf), np.int8)
    status = np.zeros(B, bool)
    iters = np.full(B, L, np.int32)
    for it in range(L):
        hd = LQ < 0
        ok = ~_row_hd_fail(hd, g) & ~done
        ck[ok] = hd[ok]
        status[ok] = True
        iters[ok] = it
        done |= ok
        if done.all():
            break
        act = ~done
        acc = np.zeros((B, g.Nf), T)
        newLr = []
        for i in range(g.Mb):
            cols = g.rows_cols(i)
            q = LQ[:, cols] - Lr[i]
            r = _cn_update(q, alpha, beta, T)
            newLr.append(r)
            acc[:, cols] += r          # columns within one base row are distinct
        LQn = Lfull + acc
        LQ[act] = LQn[act]
        for i in range(g.Mb):
            Lr[i][act] = newLr[i][act]
    rem = ~done
    if rem.any():
        hd = LQ <= 0
        fail = _row_hd_fail(hd, g)
        ck[rem] = hd[rem]
        status[rem] = ~fail[rem]
    return ck, status, iters


def decode_layered(llr, Zc, bgn, L, alpha=1.0, beta=0.0):
    """Layered (row-block serial) normalized/offset min-sum in fp32 — the build's perf schedule.

    No reference counterpart (the reference only has flooding, nr_ldpc_decode.py:105-131); this is
    the exact arithmetic of the HIP layered kernel, so the kernel is checked bit
    for bit against it, and against the reference by codeword/BLER agreement.
      APP = [0]*2Zc ++ llr on the Kb+4 core columns; degree-1 extension columns keep no APP:
      their variable-to-check message is the channel LLR itself and APP = llr + r.
      per iteration, per base row i (layer):
         q = APP[c] - r_old (ext: q = llr);  r_new = CN(q) (same CN as the flooding path)
         APP[c] = q + r_new (ext: llr + r_new)
      stopping rule, after each iteration: if no hard decision (APP < 0) changed over the
      iteration and the hard decisions satisfy every check -> ck = APP < 0, status True,
      iters = it+1.  After L iterations: ck = APP <= 0, status = syndrome == 0, iters = L."""
    T = np.float32
    llr = np.atleast_2d(np.asarray(llr)).astype(T)
    g = graph(bgn, Zc)
    B = llr.shape[0]
    assert llr.shape[1] == g.N
    alpha, beta = T(alpha), T(beta)
    Lfull = np.concatenate([np.zeros((B, 2 * Zc), T), llr], axis=1)
    APP = Lfull.copy()
    R = [np.zeros((B, g.rs[i + 1] - g.rs[i], Zc), T) for i in range(g.Mb)]
    done = np.zeros(B, bool)
    ck = np.zeros((B, g.Nf), np.int8)
    status = np.zeros(B, bool)
    iters = np.full(B, L, np.int32)

    def cur_app():
        a = APP.copy()
        for i in range(4, g.Mb):      # extension row i owns degree-1 column Kb+i (last edge)
            cols = g.rows_cols(i)[-1]
            a[:, cols] = Lfull[:, cols] + R[i][:, -1]
        return a

    hd_prev = cur_app() < 0
    for it in range(L):
        act = ~done
        for i in range(g.Mb):
            cols = g.rows_cols(i)                       # (d, Zc)
            core = g.bj[g.rs[i]:g.rs[i + 1]] < g.Kcore  # (d,)
            q = APP[:, cols] - R[i]
            q[:, ~core] = Lfull[:, cols[~core]]
            r = _cn_update(q, alpha, beta, T)
            app_new = q + r
            cc = cols[core]
            APP[np.ix_(act, cc.reshape(-1))] = app_new[act][:, core].reshape(act.sum(), -1)
            R[i][act] = r[act]
        hd = cur_app() < 0
        cand = act & (hd == hd_prev).all(axis=1)
        if cand.any():
            conv = cand & ~_row_hd_fail(hd, g)
            ck[conv] = hd[conv]
            status[conv] = True
            iters[conv] = it + 1
            done |= conv
        hd_prev = hd
        if done.all():
            break
    rem = ~done
    if rem.any():
        a = cur_app()
        hd = a <= 0
        f = _row_hd_fail(hd, g)
        ck[rem] = hd[rem]
        status[rem] = ~f[rem]
    return ck, status, iters


def decode_bf(llr, Zc, bgn, L, full=False):
    """nr_decode_ldpc(..., algo='BF') -> ldpc_decoder_BF (ldpc_decoder_bit_flipping.py:5-73),
    batched.  Returns ck (B, Nf) int8 (the reference returns the same 0/1 values as float64),
    status (B,) bool, iters (B,) int32.
      ck = LLR<0 (LLR==0 stays 0)                            (:41-43)
      for it < L: S = H ck mod 2; if S == 0 -> (ck, True)   (:47-56)
                  En = (2S-1) H; flip every bit with En == max(En)   (:61-70)
      (ck, False)                                            (:72-73)"""
    llr = np.atleast_2d(np.asarray(llr))
    g = graph(bgn, Zc)
    B = llr.shape[0]
    Lfull = llr if full else np.concatenate([np.zeros((B, 2 * Zc)), llr], axis=1)
    assert Lfull.shape[1] == g.Nf
    ck = (Lfull < 0).astype(np.uint8)
    done = np.zeros(B, bool)
    status = np.zeros(B, bool)
    iters = np.full(B, L, np.int32)
    for it in range(L):
        S = np.zeros((B, g.Mb, Zc), np.int64)
        for i in range(g.Mb):
            S[:, i] = np.bitwise_xor.reduce(ck[:, g.rows_cols(i)], axis=1)
        ok = ~S.reshape(B, -1).any(axis=1) & ~done
        status[ok] = True
        iters[ok] = it
        done |= ok
        if done.all():
            break
        En = np.zeros((B, g.Nf), np.int64)
        for b in range(len(g.bi)):   # column ecol[b, m] meets row bi*Zc + m
            En[:, g.ecol[b]] += 2 * S[:, g.bi[b]] - 1
        flip = En == En.max(axis=1, keepdims=True)
        act = ~done
        ck[act] ^= flip[act].astype(np.uint8)
    return ck.astype(np.int8), status, iters


def _bp_update(q):
    """_BP_process (nr_ldpc_decode.py:145-176) on q: (B, d, Zc) float64, every row at once."""
    B, d, Zc = q.shape
    t = np.tanh(q / 2)
    zero = q == 0
    nz = zero.sum(axis=1)
    prod = t[:, 0].copy()
    for k in range(1, d):                     # np.prod: left-to-right
        prod = prod * t[:, k]
    with np.errstate(divide="ignore", invalid="ignore"):
        tmp2 = prod[:, None, :] / t
        r = np.where(tmp2 >= 1, 2 * 19.07, np.where(tmp2 <= -1, -2 * 19.07,
                                                     2 * np.arctanh(np.clip(tmp2, -1, 1))))
    r = np.where((nz == 0)[:, None, :], r, 0.0)
    # one zero: that edge gets prod(t[0:zk]) * prod(t[zk+1:]) (no atanh, as the reference)
    one = nz == 1
    if one.any():
        zk = np.argmax(zero, axis=1)
        pa = np.ones((B, Zc))
        pb = np.ones((B, Zc))
        first_a = np.ones((B, Zc), bool)
        first_b = np.ones((B, Zc), bool)
        for k in range(d):
            ina = k < zk
            pa = np.where(ina, np.where(first_a, t[:, k], pa * t[:, k]), pa)
            first_a &= ~ina
            inb = k > zk
            pb = np.where(inb, np.where(first_b, t[:, k], pb * t[:, k]), pb)
            first_b &= ~inb
        val = pa * pb
        for k in range(d):
            r[:, k] = np.where(one & (zk == k), val, r[:, k])
    return r


def decode_bp(llr, Zc, bgn, L, full=False):
    """nr_decode_ldpc(..., algo='BP'): the flooding loop of decode_ldpc (:51-143) with the
    sum-product check-node update _BP_process (:145-176), float64, batched."""
    T = np.float64
    llr = np.atleast_2d(np.asarray(llr, T))
    g = graph(bgn, Zc)
    B = llr.shape[0]
    Lfull = llr.copy() if full else np.concatenate([np.zeros((B, 2 * Zc), T), llr], axis=1)
    LQ = Lfull.copy()
    Lr = [np.zeros((B, g.rs[i + 1] - g.rs[i], Zc), T) for i in range(g.Mb)]
    done = np.zeros(B, bool)
    ck = np.zeros((B, g.Nf), np.int8)
    status = np.zeros(B, bool)
    iters = np.full(B, L, np.int32)
    for it in range(L):
        hd = LQ < 0
        ok = ~_row_hd_fail(hd, g) & ~done
        ck[ok] = hd[ok]
        status[ok] = True
        iters[ok] = it
        done |= ok
        if done.all():
            break
        act = ~done
        acc = np.zeros((B, g.Nf), T)
        newLr = []
        for i in range(g.Mb):
            cols = g.rows_cols(i)
            r = _bp_update(LQ[:, cols] - Lr[i])
            newLr.append(r)
            acc[:, cols] += r
        LQn = Lfull + acc
        LQ[act] = LQn[act]
        for i in range(g.Mb):
            Lr[i][act] = newLr[i][act]
    rem = ~done
    if rem.any():
        hd = LQ <= 0
        fail = _row_hd_fail(hd, g)
        ck[rem] = hd[rem]
        status[rem] = ~fail[rem]
    return ck, status, iters


# ------------------------------------------------------------------- arbitrary parity-check H
def _pymax0(v):
    """Python's max(v, 0) elementwise: 0 when 0 > v, else v (nr_ldpc_decode.py:201, :220)."""
    return np.where(0 > v, 0.0, v)


def decode_sparse(llr, H, L, algo="min-sum", alpha=1.0, beta=0.0):
    """decode_ldpc(LLRin, H, L, algo, alpha, beta) (nr_ldpc_decode.py:51-143) for an ARBITRARY
    0/1 matrix H, batched over rows of llr (B, N), float64, written as the reference writes it:
    dense Lq / Lr, the per-row branches of _min_sum_process (:178-227) / _BP_process (:145-176),
    LQ = LLRin + Lr.sum(axis=0) summed row by row (:126), ldpc_decoder_BF for algo='BF'
    (ldpc_decoder_bit_flipping.py:5-73).  Small H only.
    Returns ck (B, N) int8, status (B,) bool, iters (B,) int32.  A min-sum update on a row with
    fewer than 2 edges raises IndexError, as the reference's np.sort(...)[1] does."""
    H = np.asarray(H)
    M, N = H.shape
    Hi = (H == 1).astype(np.int64)
    llr = np.atleast_2d(np.asarray(llr, np.float64))
    B = llr.shape[0]
    assert llr.shape[1] == N
    A = [np.nonzero(Hi[m])[0] for m in range(M)]
    ck = np.zeros((B, N), np.int8)
    status = np.zeros(B, bool)
    iters = np.full(B, L, np.int32)
    if algo == "BF":
        for b in range(B):
            c = (llr[b] < 0).astype(np.int64)                   # LLR == 0 stays 0 (:41-43)
            for it in range(L):
                S = (Hi @ c) % 2
                if not S.any():
                    status[b], iters[b] = True, it
                    break
                En = (2 * S - 1) @ Hi                            # (:61)
                c = np.where(En == En.max(), 1 - c, c)           # (:70)
            ck[b] = c
        return ck, status, iters
    for b in range(B):
        LLR = llr[b]
        LQ = LLR.copy()
        Lr = np.zeros((M, N))
        Lq = Hi * LLR
        done = False
        for it in range(L):
            c = (LQ < 0).astype(np.int64)
            if not ((Hi @ c) % 2).any():
                ck[b], status[b], iters[b], done = c, True, it, True
                break
            for m in range(M):
                a = A[m]
                q = Lq[m, a]
                Lr[m, a] = 0.0
                if algo == "BP":
                    zero = np.nonzero(q == 0)[0]
                    t = np.tanh(q / 2)
                    if zero.size == 0:
                        pv = np.prod(t)
                        for k in range(a.size):
                            x = pv / t[k]
                            Lr[m, a[k]] = 2 * 19.07 if x >= 1 else (-2 * 19.07 if x <= -1
                                                                     else 2 * np.arctanh(x))
                    elif zero.size == 1:
                        z = zero[0]
                        Lr[m, a[z]] = np.prod(t[0:z]) * np.prod(t[z + 1:])
                    continue
                zero = np.nonzero(q == 0)[0]
                if zero.size == 0:
                    sp = np.prod(np.sign(q))
                    srt = np.sort(np.abs(q))
                    f1, f2 = srt[0], srt[1]                      # IndexError for degree < 2
                    minv = np.where(np.abs(q) == f1, f2, f1)
                    Lr[m, a] = alpha * sp * np.sign(q) * _pymax0(minv - beta)
                elif zero.size == 1:
                    z = zero[0]
                    others = np.delete(q, z)
                    if others.size == 0:
                        raise IndexError("min-sum row with a single edge")
                    Lr[m, a[z]] = alpha * np.prod(np.sign(others)) * _pymax0(np.min(np.abs(others)) - beta)
            acc = Lr[0].copy()
            for m in range(1, M):                                # Lr.sum(axis=0), row by row
                acc = acc + Lr[m]
            LQ = LLR + acc
            Lq = np.where(Hi == 1, LQ[None, :] - Lr, Lq)         # (:129-131)
        if not done:
            c = (LQ <= 0).astype(np.int64)
            ck[b], status[b] = c, not ((Hi @ c) % 2).any()
    return ck, status, iters


def bpsk_awgn_llr(dn, snr_db, rng):
    """for_test_5g_ldpc_encoder (nr_ldpc_decode.py:251-257): BPSK 0->+1, sigma = 10^(-snr/20),
    LLR = 2y/sigma^2 (float64)."""
    en = 1 - 2 * np.asarray(dn, np.float64)
    fn = en + rng.normal(0, 10 ** (-snr_db / 20), en.shape)
    return 2 * fn / 10 ** (-snr_db / 10)


# -------------------------------------------------------------------------------------- CRC
_POLY = {
    "6": [1, 0, 0, 0, 0, 1],
    "11": [1, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1],
    "16": [0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1],
    "24A": [1, 0, 0, 0, 0, 1, 1, 0, 0, 1, 0, 0, 1, 1, 0, 0, 1, 1, 1, 1, 1, 0, 1, 1],
    "24B": [1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 1, 1],
    "24C": [1, 0, 1, 1, 0, 0, 1, 0, 1, 0, 1, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 1, 1, 1],
}


def _crc_rem(bits, poly, L):
    g = 0
    for b in poly:
        g = (g << 1) | b
    mask = (1 << L) - 1
    reg = 0
    for b in bits:
        top = (reg >> (L - 1)) & 1
        reg = ((reg << 1) & mask) | 0
        if top ^ int(b):
            reg ^= g
    return reg


def crc_encode(blk, poly, mask=0):
    """crc.py:4-41 — blk ++ CRC (int8).  The reference's shift register with appended zeros is the
    standard MSB-first polynomial remainder, restated here in register form."""
    p = _POLY[poly.upper()]
    L = len(p)
    blk = np.asarray(blk).astype(np.int64)
    assert ((blk >= 0) & (blk <= 1)).all()
    rem = _crc_rem(blk.tolist(), p, L)
    if mask:
        rem ^= mask & ((1 << L) - 1)
    out = np.zeros(blk.size + L, np.int8)
    out[:blk.size] = blk
    out[blk.size:] = [(rem >> (L - 1 - i)) & 1 for i in range(L)]
    return out


def crc_decode(blkandcrc, poly, mask=0):
    """crc.py:43-88 — (blk, err)."""
    p = _POLY[poly.upper()]
    L = len(p)
    x = np.asarray(blkandcrc).astype(np.int64)
    A = x.size - L
    rem = _crc_rem(x[:A].tolist(), p, L)
    if mask:
        rem ^= mask & ((1 << L) - 1)
    tx = 0
    for b in x[A:].tolist():
        tx = (tx << 1) | int(b)
    return x[:A].astype(np.int8), int(rem != tx)


# ----------------------------------------------------------------- segmentation / rate matching
def cbsegment(inbits, bgn):
    """nr_ldpc_cbsegment.py:7-33 — (cbs (C,K) int8 with -1 fillers, Zc)."""
    inbits = np.asarray(inbits)
    C, cbz, L, F, K, Zc = get_cbs_info(inbits.size, bgn)
    cbs = -np.ones((C, K), np.int8)
    if C == 1:
        cbs[0, :cbz] = inbits
    else:
        for c in range(C):
            cbs[c, :cbz + L] = crc_encode(inbits[c * cbz:(c + 1) * cbz], "24B")
    return cbs, Zc


def get_Er(G, C, Qm, NL):
    """nr_ldpc_ratematch.py:5-27."""
    out = []
    for j in range(C):
        if j <= (C - ((G / (NL * Qm)) % C) - 1):
            out.append(NL * Qm * math.floor(G / (NL * Qm * C)))
        else:
            out.append(NL * Qm * math.ceil(G / (NL * Qm * C)))
    return out


def get_k0(Ncb, bgn, rv, Zc):
    """nr_ldpc_ratematch.py:29-61."""
    num = {1: (0, 17, 33, 56), 2: (0, 13, 25, 43)}[bgn][rv]
    den = 66 if bgn == 1 else 50
    return math.floor(num * Ncb / (den * Zc)) * Zc


def ratematch(dn, Ncb, E, k0, Qm):
    """nr_ldpc_ratematch.py:64-97 — bit selection skipping fillers, then Qm-row interleave."""
    dn = np.asarray(dn)
    pos = (k0 + np.arange(Ncb)) % Ncb
    sel = pos[dn[pos] != -1]
    reps = -(-E // sel.size)
    ek = dn[np.tile(sel, reps)[:E]]
    return ek.reshape(Qm, E // Qm).T.reshape(E).astype(np.int8)


def raterecover(llr_fe, Ncb, N, k0, Qm, Zc, K_apo, K):
    """nr_ldpc_raterecover.py:6-65 — de-interleave, average repetitions, 0 for punctured,
    10*max|LLR| on filler positions.  Same float64 operation order: per-position sum over
    repetition passes (rows of tmp_buf summed top to bottom) divided by the visit count."""
    llr_fe = np.asarray(llr_fe, np.float64)
    E = llr_fe.size
    ek = llr_fe.reshape(E // Qm, Qm).T.reshape(E)
    max_llr = np.max(np.abs(llr_fe)) * 10
    filler = np.arange(K_apo, K) - 2 * Zc
    isfill = np.zeros(Ncb, bool)
    isfill[filler[(filler >= 0) & (filler < Ncb)]] = True
    size = Ncb - filler.size
    rep_num = int(np.ceil(E / size))
    tmp = np.zeros((rep_num, Ncb))
    cnt = np.zeros(Ncb)
    k = 0
    j = 0
    rep = -1
    while k < E:
        p = (k0 + j) % Ncb
        if p == k0:
            rep += 1
        if not isfill[p]:
            tmp[rep, p] = ek[k]
            k += 1
        cnt[p] += 1
        j += 1
    cnt[cnt == 0] = 10000
    out = np.zeros(N)
    out[:Ncb] = np.sum(tmp, axis=0) / cnt
    out[filler] = max_llr
    return out


# -------------------------------------------------------------------- DL-SCH / UL-SCH chains
def sch_params(A, Qm, R, NL, rv, TBS_LBRM, G):
    """Shared geometry of DLSCHEncode / DLSCHDecode (nr_dlsch.py:30-66, nr_dlsch_decode.py:16-60);
    TBS_LBRM = 0 selects the UL-SCH Ncb = N (nr_ulsch.py:55-58, nr_ulsch_decode.py:49-54)."""
    B, poly = (A + 24, "24A") if A > 3824 else (A + 16, "16")
    bgn = 2 if (A <= 292 or (A <= 3824 and R <= 0.67 * 1024) or R <= 0.25 * 1024) else 1
    C, cbz, L, F, K, Zc = get_cbs_info(B, bgn)
    N = (66 if bgn == 1 else 50) * Zc
    Ncb = min(N, math.floor(TBS_LBRM / (C * 2 / 3))) if TBS_LBRM else N
    return dict(A=A, B=B, poly=poly, bgn=bgn, C=C, cbz=cbz, L=L, F=F, K=K, Zc=Zc, N=N, Ncb=Ncb,
                K_apo=cbz + L, k0=get_k0(Ncb, bgn, rv, Zc), Er=get_Er(G, C, Qm, NL), Qm=Qm)


def sch_encode(trblk, A, Qm, R, NL, rv, TBS_LBRM, G):
    """DLSCHEncode (nr_dlsch.py:12-74) / ULSCH encode (nr_ulsch.py:13-70) -> g (int8, G)."""
    p = sch_params(A, Qm, R, NL, rv, TBS_LBRM, G)
    cbs, _ = cbsegment(crc_encode(np.asarray(trblk), p["poly"]), p["bgn"])
    g = np.zeros(G, np.int8)
    off = 0
    for c in range(p["C"]):
        dn = encode(cbs[c], p["bgn"])
        E = p["Er"][c]
        g[off:off + E] = ratematch(dn, p["Ncb"], E, p["k0"], Qm)
        off += E
    return g


def sch_raterecover(llr, p, harq=None):
    """Per-codeblock rate recovery + HARQ combining (nr_dlsch_decode.py:62-88) -> (C, N)."""
    llr = np.asarray(llr, np.float64)
    out = np.zeros((p["C"], p["N"]))
    off = 0
    for c in range(p["C"]):
        E = p["Er"][c]
        d = raterecover(llr[off:off + E], p["Ncb"], p["N"], p["k0"], p["Qm"], p["Zc"],
                        p["K_apo"], p["K"])
        off += E
        if harq is not None:
            h = harq[c]
            d = np.where((d == 0) | (h == 0), d + h, (d + h) / 2)
        out[c] = d
    return out


def sch_tb_check(ck, p):
    """TB reassembly + CRC checks (nr_dlsch_decode.py:93-106) of decoded (C, >=K_apo) bits ->
    (tb_ok, tbblk int8[A], cb_crc_ok bool[C])."""
    cbz, C = p["cbz"], p["C"]
    tb = np.zeros(p["B"], np.int8)
    cb_ok = np.ones(C, bool)
    for c in range(C):
        if C > 1:
            _, err = crc_decode(ck[c, :p["K_apo"]], "24B")
            cb_ok[c] = err == 0
        tb[c * cbz:(c + 1) * cbz] = ck[c, :cbz]
    blk, err = crc_decode(tb, p["poly"])
    return err == 0, blk, cb_ok


# ------------------------------------- scrambling, modulation, soft demodulation
def prbs(c_init, N):
    """gen_nrPRBS (py5gphy/common/nrPRBS.py:5-25): Gold sequence c(n) = x1(n+1600) + x2(n+1600)
    mod 2; x1 = 1,0,..,0, x2 = bits of c_init; x1(n+31) = x1(n+3)+x1(n),
    x2(n+31) = x2(n+3)+x2(n+2)+x2(n+1)+x2(n).  Generated 28 bits per step (the recurrences
    only reach back 31 - 3 = 28 positions)."""
    assert N > 0
    L = 1600 + N + 31
    x1 = np.zeros(L + 28, np.int8)
    x2 = np.zeros(L + 28, np.int8)
    x1[0] = 1
    x2[:31] = [(c_init >> i) & 1 for i in range(31)]
    for m in range(0, L - 31, 28):
        x1[m + 31:m + 59] = x1[m + 3:m + 31] ^ x1[m:m + 28]
        x2[m + 31:m + 59] = x2[m + 3:m + 31] ^ x2[m + 2:m + 30] ^ x2[m + 1:m + 29] ^ x2[m:m + 28]
    return (x1[1600:1600 + N] ^ x2[1600:1600 + N]).astype(np.int8)


# modulation id (ABI convention): the order Qm for QPSK..1024QAM, 1 BPSK, -1 pi/2-BPSK
_QAM_SCALE = {-1: 2, 1: 2, 2: 2, 4: 10, 6: 42, 8: 170, 10: 682}


def modulate(bits, mod):
    """nrModulate (py5gphy/common/nrModulation.py:4-42), all seven: float32 levels, then numpy's
    complex64 division by the real scalar sqrt(scale), which multiplies by the float32 reciprocal
    1 / float32(sqrt(scale)) (Smith's algorithm with a zero imaginary divisor)."""
    Qm = abs(mod)
    b = np.asarray(bits).astype(np.float32).reshape(-1, Qm)
    u = 1 - 2 * b                                   # float32
    if Qm == 1:
        re, im = u[:, 0].copy(), u[:, 0]
        if mod == -1:                               # pi/2-BPSK: odd symbols (2b - 1) + j(1 - 2b)
            re[1::2] = 2 * b[1::2, 0] - 1
    elif Qm == 2:
        re, im = u[:, 0], u[:, 1]
    elif Qm == 4:
        re, im = u[:, 0] * (2 - u[:, 2]), u[:, 1] * (2 - u[:, 3])
    elif Qm == 6:
        re = u[:, 0] * (4 - u[:, 2] * (2 - u[:, 4]))
        im = u[:, 1] * (4 - u[:, 3] * (2 - u[:, 5]))
    elif Qm == 8:
        re = u[:, 0] * (8 - u[:, 2] * (4 - u[:, 4] * (2 - u[:, 6])))
        im = u[:, 1] * (8 - u[:, 3] * (4 - u[:, 5] * (2 - u[:, 7])))
    else:
        re = u[:, 0] * (16 - u[:, 2] * (8 - u[:, 4] * (4 - u[:, 6] * (2 - u[:, 8]))))
        im = u[:, 1] * (16 - u[:, 3] * (8 - u[:, 5] * (4 - u[:, 7] * (2 - u[:, 9]))))
    scl = np.float32(1) / np.float32(math.sqrt(_QAM_SCALE[mod]))
    return (re * scl + 1j * (im * scl)).astype(np.complex64)


# Piecewise-linear soft-demodulation segments of demod_{qpsk,16qam,64qam,256qam,1024qam}.py, per
# PAM bit pair p (bits 2p / 2p+1 from the real / imaginary part): (upper threshold in units of A,
# k, s, c) meaning  r < thr*A  ->  LLR = (k*A) * (s*r + (s*c)*A) / noise_var  (= s (k A)(r + c A)
# / noise_var up to the sign of zero, which follows the reference's written form; c = 0: (k*A)*r).
# 1024QAM: oracle/demod1024_segments.json (tools/gen_demod_tables.py, from demod_1024qam.py).
_INF = float("inf")
DEMOD_SEGMENTS = {
    2: [[(_INF, 4, 1, 0)]],
    4: [[(-2, 8, 1, 1), (2, 4, 1, 0), (_INF, 8, 1, -1)],
        [(0, 4, 1, 2), (_INF, 4, -1, -2)]],
    6: [[(-6, 16, 1, 3), (-4, 12, 1, 2), (-2, 8, 1, 1), (2, 4, 1, 0), (4, 8, 1, -1),
         (6, 12, 1, -2), (_INF, 16, 1, -3)],
        [(-6, 8, 1, 5), (-2, 4, 1, 4), (0, 8, 1, 3), (2, 8, -1, -3), (6, 4, -1, -4),
         (_INF, 8, -1, -5)],
        [(-4, 4, 1, 6), (0, 4, -1, 2), (4, 4, 1, -2), (_INF, 4, -1, -6)]],
    8: [[(-14, 32, 1, 7), (-12, 28, 1, 6), (-10, 24, 1, 5), (-8, 20, 1, 4), (-6, 16, 1, 3),
         (-4, 12, 1, 2), (-2, 8, 1, 1), (2, 4, 1, 0), (4, 8, 1, -1), (6, 12, 1, -2),
         (8, 16, 1, -3), (10, 20, 1, -4), (12, 24, 1, -5), (14, 28, 1, -6), (_INF, 32, 1, -7)],
        [(-14, 16, 1, 11), (-12, 12, 1, 10), (-10, 8, 1, 9), (-6, 4, 1, 8), (-4, 8, 1, 7),
         (-2, 12, 1, 6), (0, 16, 1, 5), (2, 16, -1, -5), (4, 12, -1, -6), (6, 8, -1, -7),
         (10, 4, -1, -8), (12, 8, -1, -9), (14, 12, -1, -10), (_INF, 16, -1, -11)],
        [(-14, 8, 1, 13), (-10, 4, 1, 12), (-8, 8, 1, 11), (-6, 8, -1, 5), (-2, 4, -1, 4),
         (0, 8, -1, 3), (2, 8, 1, -3), (6, 4, 1, -4), (8, 8, 1, -5), (10, 8, -1, -11),
         (14, 4, -1, -12), (_INF, 8, -1, -13)],
        [(-12, 4, 1, 14), (-8, 4, -1, 10), (-4, 4, 1, 6), (0, 4, -1, 2), (4, 4, 1, -2),
         (8, 4, -1, -6), (12, 4, 1, -10), (_INF, 4, -1, -14)]],
}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "demod1024_segments.json")) as _f:
    DEMOD_SEGMENTS[10] = [[(_INF if t is None else t, k, s, c) for t, k, s, c in segs]
                          for segs in json.load(_f)["segments"]]


def demodulate(sym, noise_var, mod):
    """nrDemodulate (demodulation/nr_Demodulation.py:12-46 -> demod_*.py), all seven, in the
    reference's precision: the expressions are evaluated on numpy arrays of the symbols' real
    type with the reference's Python-float constants, so numpy (>= 2, NEP 50) applies the same
    rules as to the reference's scalars: float64 for complex128 input, float32 (constants and
    thresholds rounded to float32) for complex64.  Returns float32 LLRs, except BPSK on
    complex128 input: float64 (demod_bpsk.py:9 stores nothing)."""
    y = np.asarray(sym).reshape(-1)
    if y.dtype != np.complex64:
        y = y.astype(np.complex128)
    nv = np.asarray(noise_var).real.reshape(-1).astype(np.float32)
    Qm = abs(mod)
    A = 1 / math.sqrt(_QAM_SCALE[mod])
    re, im = y.real, y.imag
    if mod == 1:
        return 4 * (re + im) * A / nv
    out = np.zeros(y.size * Qm, np.float32)
    if mod == -1:
        out[0::2] = 4 * (re[0::2] + im[0::2]) * A / nv[0::2]
        out[1::2] = 4 * (-re[1::2] + im[1::2]) * A / nv[1::2]
        return out
    for p, segs in enumerate(DEMOD_SEGMENTS[Qm]):
        for part, r in ((0, re), (1, im)):
            v = np.zeros(r.size, r.dtype)
            done = np.zeros(r.size, bool)
            for t, k, s, c in segs:      # the if / elif chain: first segment with r < t*A
                m = ~done if t == _INF else (~done) & (r < t * A)
                x = r[m] if c == 0 else s * r[m] + (s * c) * A
                v[m] = (k * A) * x / nv[m]
                done |= m
            out[2 * p + part::Qm] = v
    return out


def descramble(llr, c_init):
    """nr_pdsch.py:268-274: LLR * (1 - 2 c(n))."""
    llr = np.asarray(llr)
    return llr * (1 - 2 * prbs(c_init, llr.size)).astype(llr.dtype)
