"""Codeblock segmentation + CRC24B (TS 38.212 §5.2.2) — mirror of
py5gphy/ldpc/nr_ldpc_cbsegment.py:7-33 (host-side caller of the encoder)."""
import numpy as np

from . import crc
from .ldpc_info import get_cbs_info


def ldpc_cbsegment(inbits, bgn):
    """cbs, Zc = ldpc_cbsegment(inbits, bgn): (C, K) int8 codeblocks, fillers = -1."""
    B = inbits.size
    assert bgn in [1, 2]
    C, cbz, L, F, K, Zc = get_cbs_info(B, bgn)
    cbs = -1 * np.ones((C, K), "i1")
    if C == 1:
        cbs[0, 0:cbz] = inbits
    else:
        for c in range(C):
            cbs[c, 0:cbz + L] = crc.nr_crc_encode(inbits[c * cbz:(c + 1) * cbz], "24B", 0)
    return cbs, Zc
