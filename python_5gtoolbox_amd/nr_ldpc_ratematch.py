"""LDPC rate matching (TS 38.212 §5.4.2) — mirror of py5gphy/ldpc/nr_ldpc_ratematch.py:5-97.

Per-codeblock host drop-in (the reference's call surface) around the GPU encoder.  Batched GPU
rate matching is `ratematch_kernel` (`ldpc5g_sch_ratematch`, sch.py)."""
import math

import numpy as np


def get_Er_ldpc(G, C, Qm, NL):
    """nr_ldpc_ratematch.py:5-27 — rate-matching output length per codeblock."""
    Er_list = [0] * C
    for j in range(C):
        if j <= (C - ((G / (NL * Qm)) % C) - 1):
            Er_list[j] = NL * Qm * math.floor(G / (NL * Qm * C))
        else:
            Er_list[j] = NL * Qm * math.ceil(G / (NL * Qm * C))
    return Er_list


def get_k0(Ncb, bgn, rv, Zc):
    """nr_ldpc_ratematch.py:29-61 — starting position of redundancy version rv."""
    assert rv in [0, 1, 2, 3]
    assert bgn in [1, 2]
    num = (0, 17, 33, 56)[rv] if bgn == 1 else (0, 13, 25, 43)[rv]
    den = 66 if bgn == 1 else 50
    return math.floor(num * Ncb / (den * Zc)) * Zc


def ratematch_ldpc(dn, Ncb, E, k0, Qm):
    """nr_ldpc_ratematch.py:64-97 — circular bit selection from k0 skipping fillers (-1),
    then the Qm-row bit interleaver.  Returns int8 fe of length E."""
    dn = np.asarray(dn)
    N = dn.size
    assert N >= Ncb
    pos = (k0 + np.arange(Ncb)) % Ncb
    sel = pos[dn[pos] != -1]
    ek = dn[np.tile(sel, -(-E // sel.size))[:E]]
    return ek.reshape(Qm, E // Qm).T.reshape(E).astype("i1")
