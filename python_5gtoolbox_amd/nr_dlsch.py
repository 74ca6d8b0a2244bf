"""Drop-in for py5gphy/nr_pdsch/nr_dlsch.py — DL-SCH transport-channel encode on the GPU.

    DLSCHEncode(trblk, TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, G) -> g_seq
        (nr_dlsch.py:12-74: TB CRC, base graph, codeblock segmentation + CRC24B, LDPC encode,
        rate matching, concatenation) through ldpc5g_sch_encode; batched form
        sch.sch_encode_batch.
"""
import numpy as np

from . import _lib
from .sch import sch_config, sch_encode_batch


def DLSCHEncode(trblk, TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, G):
    """g_seq (int8, length G) of one transport block, as the reference returns it."""
    assert len(trblk) == TBSize
    trblk = np.asarray(trblk)
    assert (not np.any(trblk < 0)) and (not np.any(trblk > 1))   # crc.py:18-20
    t = _lib.require_gpu()
    cfg = sch_config(TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, G)
    x = _lib.to_device(np.asarray(trblk, dtype=np.int8).reshape(1, -1), "dlsch_enc")
    g = _lib.to_host(sch_encode_batch(x, cfg)[0], "dlsch_enc")
    out = np.zeros(G, "i1")
    out[:g.size] = g
    return out
