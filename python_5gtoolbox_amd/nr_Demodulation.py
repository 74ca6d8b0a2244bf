"""Drop-in for py5gphy/demodulation/nr_Demodulation.py — nrDemodulate(insymbols, modtype,
noise_var) on the GPU for QPSK / 16QAM / 64QAM / 256QAM (ldpc5g_demod_descramble without
descrambling): float32 LLRs bit-exact with the reference's piecewise max-log formulas."""
import numpy as np

from . import _lib
from .phy import QM_OF, demod_descramble


def nrDemodulate(insymbols, modtype, noise_var):
    """(hardbits, LLR) as nr_Demodulation.py:12-46 returns them."""
    insymbols = np.asarray(insymbols).reshape(-1)
    noise_var = np.asarray(noise_var).real.reshape(-1).astype("f")
    assert insymbols.size == noise_var.size
    modtype = modtype.lower()
    assert modtype in ["pi/2-bpsk", "bpsk", "qpsk", "16qam", "64qam", "256qam", "1024qam"], \
        "modulation type is incorrect"
    if modtype not in QM_OF:
        raise NotImplementedError(f"{modtype}: only QPSK..256QAM (the PDSCH data path) run on the GPU")
    t = _lib.require_gpu()
    y = t.from_numpy(np.ascontiguousarray(insymbols.astype(np.complex128)).reshape(1, -1)).cuda()
    nv = t.from_numpy(np.ascontiguousarray(noise_var).reshape(1, -1)).cuda()
    LLR = demod_descramble(y, nv, QM_OF[modtype])[0].cpu().numpy()
    hardbits = np.where(LLR > 0, 0, 1).astype(np.int64)
    return hardbits, LLR
