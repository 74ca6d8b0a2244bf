"""Drop-in for py5gphy/common/nrModulation.py — nrModulate(inbits, modtype) on the GPU for all seven
modulations of the reference (pi/2-BPSK, BPSK, QPSK, 16/64/256/1024QAM; ldpc5g_scramble_modulate
without scrambling), bit-exact complex64."""
import numpy as np

from . import _lib
from .phy import MOD_ID, QM_OF, scramble_modulate


def nrModulate(inbits, modtype):
    """modulation mapper of TS 38.211 5.1 (nrModulation.py:4-42)."""
    modtype = modtype.lower()
    assert modtype in ["pi/2-bpsk", "bpsk", "qpsk", "16qam", "64qam", "256qam", "1024qam"], \
        "modulation type is incorrect"
    Qm = QM_OF[modtype]
    b = np.asarray(inbits)
    assert b.size % Qm == 0, f"length of databits must be multiple of {Qm}"
    t = _lib.require_gpu()
    x = t.from_numpy(np.ascontiguousarray(b.reshape(1, -1), dtype=np.int8)).cuda()
    return scramble_modulate(x, MOD_ID[modtype])[0].cpu().numpy()
