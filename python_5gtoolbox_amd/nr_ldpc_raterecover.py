"""LDPC rate recovery (inverse of §5.4.2) — mirror of py5gphy/ldpc/nr_ldpc_raterecover.py:6-65.

Produces the decoder input LLRs: de-interleave, average repeated transmissions, 0 for
punctured bits, 10*max|LLR| on filler positions.  Per-codeblock host drop-in (the reference's
call surface); the batched GPU rate recovery + HARQ combining is `raterecover_kernel`
(`ldpc5g_sch_raterecover`, sch.py)."""
import numpy as np


def raterecover_ldpc(LLr_fe, Ncb, N, k0, Qm, Zc, K_apo, K):
    LLr_fe = np.asarray(LLr_fe, np.float64)
    E = LLr_fe.size
    LLr_ek = LLr_fe.reshape(E // Qm, Qm).T.reshape(E)
    max_LLR = np.max(np.abs(LLr_fe)) * 10
    filler = np.arange(K_apo, K) - 2 * Zc
    isfill = np.zeros(Ncb, bool)
    isfill[filler[(filler >= 0) & (filler < Ncb)]] = True
    # visit order of the circular buffer from k0; non-filler visits consume LLRs in order
    size = Ncb - filler.size
    rep_num = int(np.ceil(E / size))
    cyc = (k0 + np.arange(Ncb)) % Ncb
    keep = ~isfill[cyc]
    # number of whole/partial passes needed to consume E non-filler positions
    npass = rep_num + 1
    visit = np.tile(cyc, npass)
    take = np.tile(keep, npass)
    last = np.nonzero(take)[0][E - 1]          # index of the E-th consumed position
    visit, take = visit[:last + 1], take[:last + 1]
    rep = np.arange(visit.size) // Ncb         # pass index (row of the reference's tmp_buf)
    tmp = np.zeros((rep_num, Ncb))
    tmp[rep[take], visit[take]] = LLr_ek
    cnt = np.bincount(visit, minlength=Ncb).astype(np.float64)
    cnt[cnt == 0] = 10000
    LLr_dn = np.zeros(N)
    LLr_dn[0:Ncb] = np.sum(tmp, axis=0) / cnt
    LLr_dn[filler] = max_LLR
    return LLr_dn
