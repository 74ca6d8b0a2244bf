"""Drop-in for py5gphy/nr_pusch/nr_ulsch.py (UL-SCH encode, I_LBRM = 0) on the GPU.

    ULSCH_Crc_CodeBlockSegment(trblk, TBSize, coderateby1024) -> (cbs, Zc, bgn)  (:13-35)
    ULSCH_encoding_ratematch(cbs, Zc, bgn, Qm, G_ULSCH, num_of_layers, rv) -> g_seq (:37-70)
"""
import numpy as np

from . import _lib
from .sch import cfg_from_codeblocks, sch_config, sch_ratematch_batch, sch_segment_batch


def ULSCH_Crc_CodeBlockSegment(trblk, TBSize, coderateby1024):
    """TB CRC + base graph selection + codeblock segmentation with CRC24B (fillers -1)."""
    assert len(trblk) == TBSize
    trblk = np.asarray(trblk)
    assert (not np.any(trblk < 0)) and (not np.any(trblk > 1))
    t = _lib.require_gpu()
    # Qm / NL / rv / G do not influence segmentation; any valid values do
    cfg = sch_config(TBSize, 2, coderateby1024, 1, 0, 0, 2)
    x = _lib.to_device(np.asarray(trblk, dtype=np.int8).reshape(1, -1), "ulsch_seg")
    ck, _ = sch_segment_batch(x, cfg)
    return _lib.to_host(ck, "ulsch_seg"), cfg.Zc, cfg.bgn


def ULSCH_encoding_ratematch(cbs, Zc, bgn, Qm, G_ULSCH, num_of_layers, rv):
    """LDPC encoding + rate matching (Ncb = N) of every codeblock, then concatenation.
    Like the reference (encode_ldpc on row views), fillers of cbs at k >= 2Zc become 0."""
    t = _lib.require_gpu()
    cbs = np.asarray(cbs)
    C, K = cbs.shape
    assert K == (22 if bgn == 1 else 10) * Zc
    fill = np.nonzero(cbs[0] == -1)[0]
    K_apo = int(fill[0]) if fill.size else K
    cfg = cfg_from_codeblocks(C, K, K_apo, Zc, bgn, Qm, G_ULSCH, num_of_layers, rv)
    x = _lib.to_device(np.asarray(cbs, dtype=np.int8), "ulsch_rm")
    g = _lib.to_host(sch_ratematch_batch(x, cfg, 1)[0], "ulsch_rm")
    tail = cbs[:, 2 * Zc:]
    tail[tail == -1] = 0
    out = np.zeros(G_ULSCH, "i1")
    out[:g.size] = g
    return out
