"""Batched GPU scrambling / modulation / soft demodulation — the C-ABI
entry points ldpc5g_prbs, ldpc5g_scramble_modulate, ldpc5g_demod_descramble (include/ldpc5g.h).

    prbs_words(cinit (T,), nbits) -> (T, ceil(nbits/32)) int32 packed c(n)   (nrPRBS.py:5-25)
    scramble_modulate(bits (T, G), mod, cinit=None) -> (T, G/Qm) complex64      (nr_pdsch_process.py:17-25)
    demod_descramble(sym (T, n), noise_var (T, n), mod, cinit=None) -> (T, n*Qm) float32 LLR
                                                      (nr_Demodulation.py:12-46, nr_pdsch.py:268-274)
mod: a MOD_ID value (the order Qm for QPSK..1024QAM, 1 BPSK, -1 pi/2-BPSK).
Device tensors in and out; asynchronous on the current stream.
"""
from . import _lib

# nrModulation.py:14 / nr_Demodulation.py:29 modulation names -> ABI modulation id
MOD_ID = {"pi/2-bpsk": -1, "bpsk": 1, "qpsk": 2, "16qam": 4, "64qam": 6, "256qam": 8, "1024qam": 10}
QM_OF = {k: abs(v) for k, v in MOD_ID.items()}   # bits per symbol


def bits_per_symbol(mod):
    return abs(int(mod))


def prbs_words(cinit, nbits, out=None):
    """Packed scrambling codes: bit k of word w of row t = gen_nrPRBS(cinit[t], ...)[32w + k]."""
    t = _lib.require_gpu()
    assert cinit.dim() == 1 and cinit.dtype in (t.int32, t.int64)
    c = cinit.to(t.int32).contiguous()
    T = c.shape[0]
    nw = (int(nbits) + 31) // 32
    w = out if out is not None else t.empty((T, max(nw, 1)), dtype=t.int32, device=c.device)
    with t.cuda.device(c.device):
        _lib.check(_lib.lib().ldpc5g_prbs(_lib.ptr(c), T, int(nbits), _lib.ptr(w), w.stride(0),
                                          _lib.stream_ptr(c.device)))
    return w


def scramble_modulate(bits, mod, cinit=None, words=None, out=None):
    """bits: (T, G) int8 0/1 device tensor; mod: MOD_ID value; cinit: (T,) device tensor or None
    (no scrambling); words: precomputed prbs_words (reused across calls) instead of cinit."""
    t = _lib.require_gpu()
    assert bits.dim() == 2 and bits.dtype == t.int8 and bits.stride(1) == 1
    T, G = bits.shape
    Qm = bits_per_symbol(mod)
    w = words if words is not None else (prbs_words(cinit, G) if cinit is not None else None)
    sym = out if out is not None else t.empty((T, G // Qm), dtype=t.complex64, device=bits.device)
    with t.cuda.device(bits.device):
        _lib.check(_lib.lib().ldpc5g_scramble_modulate(
            _lib.ptr(bits), bits.stride(0), _lib.ptr(w) if w is not None else None,
            w.stride(0) if w is not None else 0, T, G, int(mod), _lib.ptr(sym), sym.stride(0),
            _lib.stream_ptr(bits.device)))
    return sym


def demod_descramble(sym, noise_var, mod, cinit=None, words=None, out=None, llr_dtype=None):
    """sym: (T, n) complex64 / complex128 device tensor, noise_var: (T, n) float32; mod: MOD_ID
    value; cinit: (T,) or None (no descrambling), or precomputed prbs `words`.  Returns (T, n*Qm)
    LLRs, float32 (llr_dtype=torch.float64 only for BPSK on complex128, demod_bpsk.py:9)."""
    t = _lib.require_gpu()
    assert sym.dim() == 2 and sym.dtype in (t.complex64, t.complex128) and sym.stride(1) == 1
    T, n = sym.shape
    Qm = bits_per_symbol(mod)
    llr_dtype = llr_dtype or t.float32
    nv = noise_var if noise_var.dtype == t.float32 and noise_var.is_contiguous() else \
        noise_var.to(t.float32).contiguous()
    assert nv.shape == (T, n)
    w = words if words is not None else (prbs_words(cinit, n * Qm) if cinit is not None else None)
    llr = out if out is not None else t.empty((T, n * Qm), dtype=llr_dtype, device=sym.device)
    assert llr.dtype in (t.float32, t.float64) and llr.shape == (T, n * Qm) and llr.stride(1) == 1
    with t.cuda.device(sym.device):
        _lib.check(_lib.lib().ldpc5g_demod_descramble(
            _lib.ptr(sym), _lib.F32 if sym.dtype == t.complex64 else _lib.F64, sym.stride(0),
            _lib.ptr(nv), nv.stride(0), _lib.ptr(w) if w is not None else None,
            w.stride(0) if w is not None else 0, T, n, int(mod), _lib.ptr(llr),
            _lib.F64 if llr.dtype == t.float64 else _lib.F32, llr.stride(0),
            _lib.stream_ptr(sym.device)))
    return llr
