"""Drop-in for py5gphy/common/nrPRBS.py — gen_nrPRBS(c_init, N) on the GPU (ldpc5g_prbs)."""
import numpy as np

from . import _lib
from .phy import prbs_words


def gen_nrPRBS(c_init, N):
    """pseudo-random sequence of TS 38.211 5.2.1: N int8 values 0/1 (nrPRBS.py:5-25)."""
    assert N > 0
    t = _lib.require_gpu()
    w = prbs_words(t.tensor([int(c_init)], dtype=t.int64, device="cuda"), N)
    words = w[0].cpu().numpy().view(np.uint32)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:N]
    return bits.astype("i1")
