"""LDPC rate recovery (inverse of §5.4.2) — mirror of py5gphy/ldpc/nr_ldpc_raterecover.py:6-65.

Produces the decoder input LLRs: de-interleave, average repeated transmissions, 0 for
punctured bits, 10*max|LLR| on filler positions.  Per-codeblock host drop-in (the reference's
call surface); the batched GPU rate recovery + HARQ combining is `raterecover_kernel`
(`ldpc5g_sch_raterecover`, sch.py)."""
import numpy as np


_ORDER = {}


def _visit_order(Ncb, k0, filler):
    """The non-filler positions of the circular buffer in the order the bit selection visits them
    from k0 (one lap), cached per geometry."""
    key = (Ncb, k0, filler.tobytes())
    o = _ORDER.get(key)
    if o is None:
        isfill = np.zeros(Ncb, bool)
        isfill[filler[(filler >= 0) & (filler < Ncb)]] = True
        cyc = (k0 + np.arange(Ncb)) % Ncb
        o = cyc[~isfill[cyc]]
        if len(_ORDER) > 256:
            _ORDER.clear()
        _ORDER[key] = o
    return o


def raterecover_ldpc(LLr_fe, Ncb, N, k0, Qm, Zc, K_apo, K):
    LLr_fe = np.asarray(LLr_fe, np.float64)
    E = LLr_fe.size
    LLr_ek = LLr_fe.reshape(E // Qm, Qm).T.reshape(E)   # bit de-interleaving (:24-27)
    max_LLR = np.max(np.abs(LLr_fe)) * 10
    filler = np.arange(K_apo, K) - 2 * Zc
    # LLR j lands in lap j // size at the (j % size)-th non-filler position visited from k0: the
    # reference's tmp_buf[rep, pos] (:34-52); its column sums (rows in order, zeros where a lap did
    # not reach) are reproduced by the same axis-0 sum over the laps
    order = _visit_order(Ncb, k0, filler)
    size = order.size
    rep_num = int(np.ceil(E / size))
    tmp = np.zeros(rep_num * size)
    tmp[:E] = LLr_ek
    s = np.sum(tmp.reshape(rep_num, size), axis=0)
    # visits per position (filler positions excluded: they are overwritten below); 0 -> 10000 (:57)
    cnt = np.full(size, float(rep_num))
    cnt[E - (rep_num - 1) * size:] -= 1.0
    cnt[cnt == 0] = 10000
    LLr_dn = np.zeros(N)
    LLr_dn[order] = s / cnt
    LLr_dn[filler] = max_LLR
    return LLr_dn
