"""Drop-in for py5gphy/ldpc/nr_ldpc_decode.py, backed by the HIP min-sum decoders.

    nr_decode_ldpc(LLRin, Zc, bgn, L, algo='min-sum', alpha=1, beta=0)
        -> (blkandcrc, ck, status)                          (reference :11-49)
    decode_ldpc(LLRin, H, L, algo='min-sum', alpha=1, beta=0) -> (ck, status)   (:51-143)
    decode_ldpc_batch(LLR, H, L, algo, alpha, beta) -> (ck[B, N], status[B], iters[B])  (any H)
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
  * decode_ldpc with a matrix that is not a TS 38.212 expansion (and nr_decode_ldpc with a
    negative offset beta, which the two-min kernels do not express) runs the float64 sparse-H
    kernel (ldpc5g_decode_sparse): the same flooding loop over a CSR/CSC of H, with the
    reference's zero-count branches written out.
"""
from collections import OrderedDict

import numpy as np

from . import _lib
from .ldpc_info import code_dims, find_iLS, match_H

SCHEDULES = {"flooding": _lib.FLOODING, "layered": _lib.LAYERED}


def _check_algo(algo):
    assert algo in ["BF", "BP", "min-sum"]


def nr_decode_ldpc_batch(LLR, Zc, bgn, L, algo="min-sum", alpha=1.0, beta=0.0,
                         schedule="flooding", full=False, out=None, rate_matched=False):
    """Decode B codeblocks of one (bgn, Zc).

    LLR: (B, N) float64 or float32 — numpy (copied to the GPU and back) or a GPU torch tensor
         (stays on the device).  N = 66Zc / 50Zc, or the full 68Zc / 52Zc when full=True.
    rate_matched: the rows come from rate recovery, so parity columns that were never transmitted
         hold +0.0 (LDPC5G_RATE_MATCHED): the min-sum kernels detect rows whose extension column
         is +0.0 in every codeblock of a workgroup and skip their null updates — same results,
         much less work at high code rates.
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
    flags = (_lib.LLR_FULL if full else 0) | (_lib.RATE_MATCHED if rate_matched else 0)
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
    """One codeblock through the float64 kernels (the reference-exact path).  min-sum: host
    buffers straight through the library (ldpc5g_decode_ms_host: per-thread pinned / device
    staging, one H2D, the launch, one D2H, one synchronisation); BF / BP through the batched
    device path.  Returns (ck int8 (Nf,), status bool)."""
    t = _lib.require_gpu()
    K, N, Nf = code_dims(bgn, Zc)
    x = np.ascontiguousarray(np.asarray(LLRin, np.float64).reshape(-1))
    if algo == "min-sum":
        ck = np.empty(Nf, np.int8)
        st = np.zeros(1, np.uint8)
        it = np.zeros(1, np.int32)
        # a last parity column of exact +0.0 (untransmitted after rate recovery, e.g. DLSCHDecode's
        # rows at high code rates) enables dead-row skipping: same results, less work
        rm = not x[-Zc:].view(np.int64).any()
        flags = (_lib.LLR_FULL if full else 0) | (_lib.RATE_MATCHED if rm else 0)
        _lib.check(_lib.lib().ldpc5g_decode_ms_host(
            x.ctypes.data, ck.ctypes.data, st.ctypes.data, it.ctypes.data, 1, bgn, Zc, int(L),
            float(alpha), float(beta), flags, _lib.stream_ptr()))
        if it[0] < 0:   # the multi-workgroup kernel gave up waiting for co-resident parts
            raise _lib.LdpcLibError("nr_decode_ldpc: the multi-workgroup decode timed out waiting for "
                                    "its workgroups to be co-resident (include/ldpc5g.h, "
                                    "ldpc5g_split_timeouts); the GPU is held by other kernels")
        return ck, bool(st[0])
    dev = t.cuda.current_device()
    n_in = Nf if full else N

    def make():
        return (t.empty((1, n_in), dtype=t.float64, pin_memory=True),
                t.empty((1, n_in), dtype=t.float64, device=dev),
                t.empty((Nf + 8,), dtype=t.uint8, device=dev),
                t.empty((Nf + 8,), dtype=t.uint8, pin_memory=True))
    hin, din, drec, hrec = _lib.staging(("dec1", dev, n_in, Nf), make)
    hin.numpy()[0] = x
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
    if algo == "min-sum" and not beta >= 0:
        # a negative offset breaks the two-min form (a zero message's neighbours would get
        # alpha * |beta|): the sparse kernel runs the reference's zero branches as written
        t = _lib.require_gpu()
        dev = t.device("cuda", t.cuda.current_device())
        g = _sparse_graph(("bg", bgn, Zc), lambda: SparseGraph.from_base_graph(bgn, Zc, dev), dev)
        full = np.concatenate([np.zeros(2 * Zc), np.asarray(LLRin, np.float64).reshape(-1)])
        ck, st = _decode_sparse_one(full, g, L, algo, alpha, beta)
        return ck[0:K], ck, st
    ck, st = _decode_one(LLRin, Zc, bgn, L, algo, alpha, beta, False)
    if algo == "BF":
        ck = ck.astype(np.float64)   # the reference's BF decisions are a float copy of LLRin
    return ck[0:K], ck, st


class SparseGraph:
    """A binary parity-check matrix as the sparse kernel reads it (include/ldpc5g.h,
    ldpc5g_decode_sparse): CSR of the rows — edges numbered row-major, columns ascending, the
    order of np.where(H[m,:] == 1) (nr_ldpc_decode.py:80-83) — and CSC of the columns — rows
    ascending (:88-91), the order Lr.sum(axis=0) adds them (:126) — as int32 device tensors."""

    def __init__(self, M, N, rows, cols, device):
        t = _lib.torch()
        rows = np.asarray(rows, np.int64)
        cols = np.asarray(cols, np.int64)
        o = np.lexsort((cols, rows))            # row-major, columns ascending
        rows, cols = rows[o], cols[o]
        self.M, self.N, self.E = int(M), int(N), int(rows.size)
        assert self.E < 2 ** 31 and self.N < 2 ** 31
        row_ptr = np.searchsorted(rows, np.arange(M + 1)).astype(np.int32)
        oc = np.lexsort((rows, cols))           # column-major, rows ascending
        col_ptr = np.searchsorted(cols[oc], np.arange(N + 1)).astype(np.int32)
        deg = np.diff(row_ptr)
        self.min_row_degree = int(deg.min()) if M else 2

        def dev(a):
            a = np.ascontiguousarray(a, np.int32)
            return t.from_numpy(a if a.size else np.zeros(1, np.int32)).to(device)
        self.row_ptr, self.col_idx = dev(row_ptr), dev(cols)
        self.col_ptr, self.col_edge, self.col_row = dev(col_ptr), dev(oc), dev(rows[oc])

    @classmethod
    def from_dense(cls, H, device):
        H = np.asarray(H)
        assert H.ndim == 2, "H must be a matrix"
        nz = H != 0
        assert bool((H[nz] == 1).all()), "decode_ldpc: H must be a 0/1 parity-check matrix"
        rows, cols = np.nonzero(nz)
        return cls(H.shape[0], H.shape[1], rows, cols, device)

    @classmethod
    def from_base_graph(cls, bgn, Zc, device):
        """The expanded TS 38.212 H of (bgn, Zc) (ldpc_info.getH) without the dense matrix."""
        from .ldpc_info import base_graph
        V = base_graph(bgn, find_iLS(Zc)).astype(np.int64)
        ii, jj = np.nonzero(V >= 0)
        m = np.arange(Zc)
        rows = (ii[:, None] * Zc + m[None, :]).ravel()
        cols = (jj[:, None] * Zc + (m[None, :] + (V[ii, jj] % Zc)[:, None]) % Zc).ravel()
        return cls(V.shape[0] * Zc, V.shape[1] * Zc, rows, cols, device)


_GRAPHS = OrderedDict()


def _sparse_graph(key, make, device):
    k = (key, str(device))
    g = _GRAPHS.get(k)
    if g is None:
        g = _GRAPHS[k] = make()
        while len(_GRAPHS) > 8:
            _GRAPHS.popitem(last=False)
    else:
        _GRAPHS.move_to_end(k)
    return g


def _dense_graph(H, device):
    H = np.ascontiguousarray(np.asarray(H))
    import hashlib
    key = ("dense", H.shape, H.dtype.str, hashlib.sha1(H.tobytes()).hexdigest())
    return _sparse_graph(key, lambda: SparseGraph.from_dense(H, device), device)


def _algo_id(algo):
    """decode_ldpc's dispatch (nr_ldpc_decode.py:65-67, :120-123): 'BF', 'BP', anything else is
    the min-sum family."""
    return {"BF": _lib.ALGO_BF, "BP": _lib.ALGO_BP}.get(algo, _lib.ALGO_MS)


def decode_ldpc_batch(LLR, H, L, algo="min-sum", alpha=1.0, beta=0.0, out=None):
    """decode_ldpc (nr_ldpc_decode.py:51-143) of B codeblocks through the sparse-H kernel.

    H: a dense 0/1 matrix (M, N) or a SparseGraph.  LLR: (B, N) float64, numpy (copied to the GPU
    and back) or a GPU torch tensor.  Returns (ck (B, N) int8, status (B,), iters (B,) int32) of
    the input's kind; iters = check-node passes run (the loop index at an early return, else L)."""
    t = _lib.require_gpu()
    is_np = not isinstance(LLR, t.Tensor)
    if is_np:
        x = t.from_numpy(np.ascontiguousarray(np.atleast_2d(np.asarray(LLR, np.float64)))).cuda()
    else:
        x = LLR if LLR.dtype == t.float64 else LLR.double()
    assert x.dim() == 2
    g = H if isinstance(H, SparseGraph) else _dense_graph(H, x.device)
    B, N = x.shape
    assert N == g.N, f"LLR rows must hold {g.N} values"
    if x.stride(1) != 1:
        x = x.contiguous()
    a = _algo_id(algo)
    if out is None:
        ck = t.empty((B, N), dtype=t.int8, device=x.device)
        st = t.empty((B,), dtype=t.uint8, device=x.device)
        it = t.empty((B,), dtype=t.int32, device=x.device)
    else:
        ck, st, it = out
        assert ck.dtype == t.int8 and ck.dim() == 2 and ck.shape[0] == B and ck.shape[1] >= N \
            and ck.stride(1) == 1 and st.dtype == t.uint8 and it.dtype == t.int32 \
            and st.numel() >= B and it.numel() >= B and st.is_contiguous() and it.is_contiguous()
    lib = _lib.lib()
    nsc = lib.ldpc5g_sparse_scratch_bytes(B, g.M, g.N, g.E, a)
    assert nsc >= 0
    scratch = t.empty((max(nsc, 1),), dtype=t.uint8, device=x.device)
    with t.cuda.device(x.device):
        _lib.check(lib.ldpc5g_decode_sparse(
            _lib.ptr(x), x.stride(0), B, g.M, g.N, g.E, _lib.ptr(g.row_ptr), _lib.ptr(g.col_idx),
            _lib.ptr(g.col_ptr), _lib.ptr(g.col_edge), _lib.ptr(g.col_row), int(L), a,
            float(alpha), float(beta), _lib.ptr(ck), ck.stride(0), _lib.ptr(st), _lib.ptr(it),
            _lib.ptr(scratch), nsc, _lib.stream_ptr(x.device)))
    if is_np:
        return ck.cpu().numpy(), st.cpu().numpy().astype(bool), it.cpu().numpy()
    return ck, st, it


def _decode_sparse_one(LLRin, g, L, algo, alpha, beta):
    ck, st, it = decode_ldpc_batch(np.asarray(LLRin, np.float64).reshape(1, -1), g, L, algo, alpha,
                                   beta)
    ck, st, it = ck[0], bool(st[0]), int(it[0])
    if _algo_id(algo) == _lib.ALGO_MS and g.min_row_degree < 2 and L > 0 and not (st and it == 0):
        # _min_sum_process on a row with < 2 edges: np.sort(...)[1] / np.min([]) (:191-194, :212)
        raise IndexError("decode_ldpc: a parity check with fewer than 2 variable nodes reached "
                         "the min-sum update (np.sort(np.abs(sel_Lq))[1] is out of bounds)")
    if _algo_id(algo) == _lib.ALGO_BF:
        ck = ck.astype(np.float64)   # the reference's BF decisions are a float copy of LLRin
    return ck, st


def decode_ldpc(LLRin, H, L, algo="min-sum", alpha=1, beta=0):
    """Drop-in for nr_ldpc_decode.decode_ldpc (:51-143): LLRin holds all columns of H (punctured
    ones included).  A TS 38.212 expansion (getH) runs the base-graph kernels; any other binary H
    runs the sparse-H kernel, float64, with the reference's semantics for 'min-sum' (alpha,
    beta), 'BP' and 'BF'."""
    H = np.asarray(H)
    M, Ncol = H.shape
    assert LLRin.size == Ncol
    a = _algo_id(algo)
    m = match_H(H)
    if m is not None and (a != _lib.ALGO_MS or beta >= 0):
        bgn, Zc = m
        name = {_lib.ALGO_BF: "BF", _lib.ALGO_BP: "BP", _lib.ALGO_MS: "min-sum"}[a]
        ck, st = _decode_one(LLRin, Zc, bgn, L, name, alpha, beta, True)
        ck = ck.astype(np.float64) if a == _lib.ALGO_BF else ck
        return ck, st
    t = _lib.require_gpu()
    dev = t.device("cuda", t.cuda.current_device())
    if m is not None:
        g = _sparse_graph(("bg",) + tuple(m), lambda: SparseGraph.from_base_graph(m[0], m[1], dev), dev)
    else:
        g = _dense_graph(H, dev)
    return _decode_sparse_one(LLRin, g, L, algo, alpha, beta)


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
