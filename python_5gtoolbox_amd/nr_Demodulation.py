"""Drop-in for py5gphy/demodulation/nr_Demodulation.py — nrDemodulate(insymbols, modtype,
noise_var) on the GPU for all seven modulations (ldpc5g_demod_descramble without descrambling):
LLRs bit-exact with the reference's piecewise max-log formulas, in the reference's precision —
float64 arithmetic for complex128 symbols, float32 for complex64 (numpy >= 2), float32 LLRs
except BPSK on complex128 symbols, which the reference returns as float64 (demod_bpsk.py:9)."""
import numpy as np

from . import _lib
from .phy import MOD_ID, demod_descramble


def nrDemodulate(insymbols, modtype, noise_var):
    """(hardbits, LLR) as nr_Demodulation.py:12-46 returns them."""
    insymbols = np.asarray(insymbols).reshape(-1)
    noise_var = np.asarray(noise_var).real.reshape(-1).astype("f")
    assert insymbols.size == noise_var.size
    modtype = modtype.lower()
    assert modtype in ["pi/2-bpsk", "bpsk", "qpsk", "16qam", "64qam", "256qam", "1024qam"], \
        "modulation type is incorrect"
    t = _lib.require_gpu()
    # complex64 stays complex64 (float32 arithmetic); anything else is computed as complex128
    sdt = np.complex64 if insymbols.dtype == np.complex64 else np.complex128
    y = t.from_numpy(np.ascontiguousarray(insymbols.astype(sdt)).reshape(1, -1)).cuda()
    nv = t.from_numpy(np.ascontiguousarray(noise_var).reshape(1, -1)).cuda()
    f64 = modtype == "bpsk" and sdt == np.complex128
    LLR = demod_descramble(y, nv, MOD_ID[modtype], llr_dtype=t.float64 if f64 else t.float32)
    LLR = LLR[0].cpu().numpy()
    hardbits = np.where(LLR > 0, 0, 1).astype(np.int64)
    return hardbits, LLR
