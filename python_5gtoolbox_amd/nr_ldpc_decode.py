"""Drop-in for py5gphy/ldpc/nr_ldpc_decode.py, backed by the HIP min-sum decoders.

    nr_decode_ldpc(LLRin, Zc, bgn, L, algo='min-sum', alpha=1, beta=0)
        -> (blkandcrc, ck, status)                          (reference :11-49)
    decode_ldpc(LLRin, H, L, algo='min-sum', alpha=1, beta=0) -> (ck, status)   (:51-143)
    for_test_5g_ldpc_encoder(Zc, bgn, snr_db, crcpoly='24A')                     (:229-260)
    nr_decode_ldpc_batch(LLR, Zc, bgn, L, ..., schedule='flooding'|'layered')
        -> (ck[B, Nf], status[B], iters[B])                 (batched; numpy or device tensors)

Precision / parity
  * The per-codeblock drop-ins run the float64 flooding kernel: the reference's own schedule and
    arithmetic (numpy float64), so ck and status are bit-identical to the reference.
  * The batched API takes float32 LLRs by default (the bench path): flooding float32 is the same
    algorithm rounded to fp32; 'layered' is the faster row-serial schedule.
  * algo='BF' runs the GPU bit-flipping kernel (ldpc_decoder_bit_flipping.py:5-73) — bit-exact,
    ck returned as float64 like the reference; algo='BP' runs the float64 sum-product flooding
    kernel (_BP_process :145-176) — the GPU's tanh/atanh are not numpy's, so BP matches the
    reference's status and decisions to within transcendental rounding.
"""
import numpy as np

from . import _lib
from .ldpc_info import code_dims, find_iLS, match_H

SCHEDULES = {"flooding": _lib.FLOODING, "layered": _lib.LAYERED}


def _check_algo(algo):
    assert algo in ["BF", "BP", "min-sum"]


def nr_decode_ldpc_batch(LLR, Zc, bgn, L, algo="min-sum", alpha=1.0, beta=0.0,
                         schedule="flooding", full=False, out=None):
    """Decode B codeblocks of one (bgn, Zc).

    LLR: (B, N) float64 or float32 — numpy (copied to the GPU and back) or a GPU torch tensor
         (stays on the device).  N = 66Zc / 50Zc, or the full 68Zc / 52Zc when full=True.
    Returns (ck (B, Nf) int8, status (B,) bool, iters (B,) int32) of the input's kind; for
    device tensors status is uint8 and nothing is synchronised."""
    assert bgn in [1, 2]
    _check_algo(algo)
    assert schedule in SCHEDULES, f"schedule must be one of {list(SCHEDULES)}"
    t = _lib.require_gpu()
    is_np = not isinstance(LLR, t.Tensor)
    if is_np:
        a = np.asarray(LLR)
        if a.dtype != np.float32:
            a = a.astype(np.float64)
        x = t.from_numpy(np.ascontiguousarray(a)).cuda()
    else:
        x = LLR
    assert x.dim() == 2 and x.dtype in (t.float32, t.float64)
    K, N, Nf = code_dims(bgn, Zc)
    assert find_iLS(Zc) < 8
    B = x.shape[0]
    assert x.shape[1] == (Nf if full else N), f"LLR rows must hold {Nf if full else N} values"
    if x.stride(1) != 1:
        x = x.contiguous()
    dt = _lib.F64 if x.dtype == t.float64 else _lib.F32
    if out is None:
        ck = t.empty((B, Nf), dtype=t.int8, device=x.device)
        st = t.empty((B,), dtype=t.uint8, device=x.device)
        it = t.empty((B,), dtype=t.int32, device=x.device)
    else:
        ck, st, it = out
        # the C ABI trusts these buffers: wrong dtype / size / device would be out-of-bounds writes
        assert ck.dtype == t.int8 and ck.dim() == 2 and ck.shape[0] == B and ck.shape[1] >= Nf \
            and ck.stride(1) == 1, "out[0] must be int8 (B, >= Nf) with unit column stride"
        assert st.dtype == t.uint8 and it.dtype == t.int32 and st.numel() >= B and it.numel() >= B \
            and st.is_contiguous() and it.is_contiguous(), "out[1]/out[2] must be uint8/int32 (>= B,)"
        assert ck.device == x.device and st.device == x.device and it.device == x.device, \
            "outputs must live on the LLR tensor's device"
    flags = _lib.LLR_FULL if full else 0
    lib = _lib.lib()
    with t.cuda.device(x.device):
        stream = _lib.stream_ptr(x.device)
        if algo == "min-sum":
            _lib.check(lib.ldpc5g_decode_ms(
                _lib.ptr(x), dt, _lib.ptr(ck), _lib.ptr(st), _lib.ptr(it), B, bgn, Zc, int(L),
                float(alpha), float(beta), SCHEDULES[schedule], flags, x.stride(0), ck.stride(0),
                stream))
        elif algo == "BF":
            _lib.check(lib.ldpc5g_decode_bf(
                _lib.ptr(x), dt, _lib.ptr(ck), _lib.ptr(st), _lib.ptr(it), B, bgn, Zc, int(L),
                flags, x.stride(0), ck.stride(0), stream))
        else:   # BP: float64 sum-product with a per-edge message scratch
            if x.dtype != t.float64:
                x = x.double()
            n = lib.ldpc5g_bp_scratch_elems(B, bgn, Zc)
            scratch = t.empty((max(n, 1),), dtype=t.float64, device=x.device)
            _lib.check(lib.ldpc5g_decode_bp(
                _lib.ptr(x), _lib.ptr(ck), _lib.ptr(st), _lib.ptr(it), _lib.ptr(scratch), n, B,
                bgn, Zc, int(L), flags, x.stride(0), ck.stride(0), stream))
    if is_np:
        return ck.cpu().numpy(), st.cpu().numpy().astype(bool), it.cpu().numpy()
    return ck, st, it


def _decode_one(LLRin, Zc, bgn, L, algo, alpha, beta, full):
    """One codeblock through the float64 flooding kernel (the reference-exact path) with pinned
    staging: LLRs -> pinned -> device, decode into one device record (ck | status | iters), one
    D2H of that record.  Returns (ck int8 (Nf,), status bool)."""
    t = _lib.require_gpu()
    K, N, Nf = code_dims(bgn, Zc)
    n_in = Nf if full else N
    dev = t.cuda.current_device()

    def make():
        return (t.empty((1, n_in), dtype=t.float64, pin_memory=True),
                t.empty((1, n_in), dtype=t.float64, device=dev),
                t.empty((Nf + 8,), dtype=t.uint8, device=dev),
                t.empty((Nf + 8,), dtype=t.uint8, pin_memory=True))
    hin, din, drec, hrec = _lib.staging(("dec1", dev, n_in, Nf), make)
    hin.numpy()[0] = np.asarray(LLRin, np.float64).reshape(-1)
    din.copy_(hin, non_blocking=True)
    out = (drec[:Nf].view(t.int8).view(1, Nf), drec[Nf:Nf + 1], drec[Nf + 4:Nf + 8].view(t.int32))
    nr_decode_ldpc_batch(din, Zc, bgn, L, algo, alpha, beta, "flooding", full=full, out=out)
    hrec.copy_(drec, non_blocking=True)
    t.cuda.current_stream().synchronize()
    h = hrec.numpy()
    return h[:Nf].view(np.int8).copy(), bool(h[Nf])


def nr_decode_ldpc(LLRin, Zc, bgn, L, algo="min-sum", alpha=1, beta=0):
    """LDPC decode following TS 38.212 5.3.2 — drop-in for nr_ldpc_decode.nr_decode_ldpc.

    input:  LLRin: N length decoder input LLRs (log P0/P1), Zc, bgn (1/2), L: iterations,
            algo in ['BF','BP','min-sum'], alpha (normalised MS), beta (offset MS)
    output: blkandcrc = ck[0:K] (view), ck: N+2Zc hard decisions (int8), status (bool)"""
    assert bgn in [1, 2]
    assert algo in ["BF", "BP", "min-sum"]
    K, N, Nf = code_dims(bgn, Zc)
    assert N == LLRin.size
    iLS = find_iLS(Zc)
    assert iLS < 8
    _check_algo(algo)
    ck, st = _decode_one(LLRin, Zc, bgn, L, algo, alpha, beta, False)
    if algo == "BF":
        ck = ck.astype(np.float64)   # the reference's BF decisions are a float copy of LLRin
    return ck[0:K], ck, st


def decode_ldpc(LLRin, H, L, algo="min-sum", alpha=1, beta=0):
    """Drop-in for nr_ldpc_decode.decode_ldpc: LLRin holds all columns of H (punctured ones
    included).  H must be a TS 38.212 expanded matrix (getH); the GPU kernels are specialised
    to the two base graphs, other matrices raise NotImplementedError."""
    _check_algo(algo)
    M, Ncol = H.shape
    assert LLRin.size == Ncol
    m = match_H(np.asarray(H))
    if m is None:
        raise NotImplementedError("decode_ldpc: H is not a TS 38.212 base-graph expansion")
    bgn, Zc = m
    ck, st = _decode_one(LLRin, Zc, bgn, L, algo, alpha, beta, True)
    ck = ck.astype(np.float64) if algo == "BF" else ck
    return ck, st


def for_test_5g_ldpc_encoder(Zc, bgn, snr_db, crcpoly="24A"):
    """nr_ldpc_decode.py:229-260 — random K-crc bits + CRC -> GPU encode -> BPSK+AWGN -> LLR.
    Uses the global numpy RNG like the reference (seed with np.random.seed)."""
    from . import crc
    from .nr_ldpc_encode import encode_ldpc
    assert bgn in [1, 2]
    assert crcpoly in ["24A", "24B", "16"]
    K, N, _ = code_dims(bgn, Zc)
    crc_len = 24 if crcpoly in ["24A", "24B"] else 16
    inbits = np.random.randint(2, size=K - crc_len)
    blkandcrc = crc.nr_crc_encode(inbits, crcpoly)
    dn = encode_ldpc(blkandcrc, bgn)
    en = 1 - 2 * dn
    fn = en + np.random.normal(0, 10 ** (-snr_db / 20), dn.size)
    noise_power = 10 ** (-snr_db / 10)
    LLRin = 2 * fn / noise_power
    return blkandcrc, dn, LLRin
