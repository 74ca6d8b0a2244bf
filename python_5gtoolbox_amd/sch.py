"""Batched GPU DL-SCH / UL-SCH chain (TS 38.212 §7.2 / §6.2) over transport blocks that share
one configuration — the C-ABI entry points ldpc5g_sch_* of include/ldpc5g.h.

    sch_config(A, Qm, coderateby1024, NL, rv, TBS_LBRM, G) -> SchCfg      (host only)
    crc_rows(bits[R, >=n], poly, nbits=None) -> rem[R] uint32             (crc.py:4-88)
    sch_encode_batch(trblk[T, A], cfg) -> g[T, E_total]                    (nr_dlsch.py:12-74)
    sch_decode_batch(llr[T, E_total], cfg, L, ...) -> SchDecodeResult      (nr_dlsch_decode.py)

Device tensors in, device tensors out, everything asynchronous on the current stream; torch only
allocates the buffers.  The per-transport-block drop-ins (nr_dlsch.DLSCHEncode,
nr_dlsch_decode.DLSCHDecode, nr_ulsch.*, nr_ulsch_decode.ULSCH_decoding) wrap these.
"""
from collections import namedtuple

from . import _lib

SchDecodeResult = namedtuple(
    "SchDecodeResult", "tb_ok tbblk llr_dn ck status iters cb_crc_ok tb_rem")


def sch_config(A, Qm, coderateby1024, NL, rv, TBS_LBRM, G):
    """Transport-block geometry (ldpc5g_sch_config).  TBS_LBRM > 0: DL-SCH limited-buffer Ncb
    (nr_dlsch.py:63-65); TBS_LBRM = 0: UL-SCH Ncb = N (nr_ulsch.py:55-58)."""
    cfg = _lib.SchCfg()
    _lib.check(_lib.lib().ldpc5g_sch_config(int(A), int(Qm), float(coderateby1024), int(NL),
                                            int(rv), int(TBS_LBRM), int(G), _lib.ctypes.byref(cfg)))
    return cfg


def cfg_from_codeblocks(C, K, K_apo, Zc, bgn, Qm, G, NL, rv, Ncb=None):
    """Configuration of ULSCH_encoding_ratematch(cbs, Zc, bgn, Qm, G_ULSCH, NL, rv)
    (nr_ulsch.py:37-70), which knows the codeblocks but not the TB size: only the codeblock and
    rate-matching fields are used by ldpc5g_sch_ratematch; A / B are made self-consistent."""
    from .nr_ldpc_ratematch import get_Er_ldpc, get_k0
    cfg = _lib.SchCfg()
    N = (66 if bgn == 1 else 50) * Zc
    Lcb = 24 if C > 1 else 0
    cbz = K_apo - Lcb
    B = C * cbz
    ltb = 24 if B - 24 > 3824 else 16
    Ncb = N if Ncb is None else Ncb
    Er = get_Er_ldpc(G, C, Qm, NL)
    E_lo, E_hi = min(Er), max(Er)
    vals = dict(A=B - ltb, B=B, tb_crc_poly=_lib.CRC_IDS["24A" if ltb == 24 else "16"], bgn=bgn,
                C=C, cbz=cbz, Lcb=Lcb, F=K - K_apo, K=K, K_apo=K_apo, Zc=Zc, N=N, Ncb=Ncb,
                k0=get_k0(Ncb, bgn, rv, Zc), Qm=Qm, NL=NL, rv=rv, E_lo=E_lo, E_hi=E_hi,
                c_switch=sum(1 for e in Er if e == E_lo) if E_lo != E_hi else C,
                G=G, E_total=sum(Er))
    for k, v in vals.items():
        setattr(cfg, k, int(v))
    return cfg


def crc_rows(bits, poly, nbits=None):
    """CRC remainders of the rows of a (R, n) int8 device tensor of 0/1 bits (ldpc5g_crc):
    nr_crc_encode's parity (crc.py:4-41, mask 0) as uint32 (int64 tensor), 0 for rows ending in
    a valid CRC (nr_crc_decode, crc.py:43-88)."""
    t = _lib.require_gpu()
    assert bits.dim() == 2 and bits.dtype == t.int8 and bits.stride(1) == 1
    n = bits.shape[1] if nbits is None else int(nbits)
    R = bits.shape[0]
    rem = t.empty((max(R, 1),), dtype=t.int32, device=bits.device)
    with t.cuda.device(bits.device):
        _lib.check(_lib.lib().ldpc5g_crc(_lib.ptr(bits), bits.stride(0), n, R,
                                         _lib.CRC_IDS[poly.upper()], _lib.ptr(rem),
                                         _lib.stream_ptr(bits.device)))
    return rem[:R].to(t.int64) & 0xFFFFFFFF


class SchWorkspace:
    """Device buffers of one batch shape (reused across calls of the bench / a TB stream)."""

    def __init__(self, cfg, T, device, dn_dtype=None):
        t = _lib.require_gpu()
        C, K, N = cfg.C, cfg.K, cfg.N
        Nf = N + 2 * cfg.Zc
        self.T = T
        self.ck = t.empty((T * C, K), dtype=t.int8, device=device)
        self.dn = t.empty((T * C, N), dtype=t.int8, device=device)
        self.tb_crc = t.empty((T,), dtype=t.int32, device=device)
        self.g = t.empty((T, max(cfg.E_total, 1)), dtype=t.int8, device=device)
        self.dec_ck = t.empty((T * C, Nf), dtype=t.int8, device=device)
        self.status = t.empty((T * C,), dtype=t.uint8, device=device)
        self.iters = t.empty((T * C,), dtype=t.int32, device=device)
        self.tbblk = t.empty((T, cfg.B), dtype=t.int8, device=device)
        self.cb_ok = t.empty((T * C,), dtype=t.uint8, device=device)
        self.tb_rem = t.empty((T,), dtype=t.int32, device=device)
        self.tb_ok = t.empty((T,), dtype=t.uint8, device=device)
        self.llr_dn = {}
        self.device = device

    def dn_buf(self, dtype, cfg):
        t = _lib.torch()
        if dtype not in self.llr_dn:
            self.llr_dn[dtype] = t.empty((self.T * cfg.C, cfg.N), dtype=dtype, device=self.device)
        return self.llr_dn[dtype]


def _dtype_id(t, dt):
    assert dt in (t.float32, t.float64), "LLRs must be float32 or float64"
    return _lib.F32 if dt == t.float32 else _lib.F64


def sch_segment_batch(trblk, cfg, ws=None):
    """TB CRC + codeblock segmentation + CRC24B of T transport blocks (ldpc5g_sch_segment):
    returns (ck (T*C, K) int8 with -1 fillers, tb_crc (T,) int32)."""
    t = _lib.require_gpu()
    assert trblk.dim() == 2 and trblk.dtype == t.int8 and trblk.stride(1) == 1
    T = trblk.shape[0]
    assert trblk.shape[1] >= cfg.A
    ws = ws or SchWorkspace(cfg, T, trblk.device)
    with t.cuda.device(trblk.device):
        _lib.check(_lib.lib().ldpc5g_sch_segment(
            _lib.ptr(trblk), trblk.stride(0), _lib.ctypes.byref(cfg), T, _lib.ptr(ws.ck),
            _lib.ptr(ws.tb_crc), _lib.stream_ptr(trblk.device)))
    return ws.ck, ws.tb_crc


def sch_ratematch_batch(ck, cfg, T, ws=None):
    """LDPC encode + rate matching + concatenation of T*C codeblocks (ldpc5g_sch_ratematch):
    ck (T*C, K) int8 -> g (T, E_total) int8."""
    t = _lib.require_gpu()
    assert ck.dim() == 2 and ck.dtype == t.int8 and ck.shape == (T * cfg.C, cfg.K) and ck.is_contiguous()
    ws = ws or SchWorkspace(cfg, T, ck.device)
    with t.cuda.device(ck.device):
        _lib.check(_lib.lib().ldpc5g_sch_ratematch(
            _lib.ptr(ck), _lib.ctypes.byref(cfg), T, _lib.ptr(ws.dn), _lib.ptr(ws.g),
            ws.g.stride(0), _lib.stream_ptr(ck.device)))
    return ws.g[:, :cfg.E_total]


def sch_encode_batch(trblk, cfg, ws=None):
    """DLSCHEncode / ULSCH encode of T transport blocks (ldpc5g_sch_encode): trblk (T, >=A) int8
    device tensor -> g (T, E_total) int8 device tensor (a view into the workspace)."""
    t = _lib.require_gpu()
    assert trblk.dim() == 2 and trblk.dtype == t.int8 and trblk.stride(1) == 1
    T = trblk.shape[0]
    assert trblk.shape[1] >= cfg.A
    ws = ws or SchWorkspace(cfg, T, trblk.device)
    with t.cuda.device(trblk.device):
        _lib.check(_lib.lib().ldpc5g_sch_encode(
            _lib.ptr(trblk), trblk.stride(0), _lib.ptr(ws.g), ws.g.stride(0),
            _lib.ctypes.byref(cfg), T, _lib.ptr(ws.ck), _lib.ptr(ws.dn), _lib.ptr(ws.tb_crc),
            _lib.stream_ptr(trblk.device)))
    return ws.g[:, :cfg.E_total]


def sch_raterecover_batch(llr, cfg, harq_in=None, dn_dtype=None, ws=None):
    """Rate recovery + HARQ combining (ldpc5g_sch_raterecover): llr (T, >=E_total) float32/64
    -> llr_dn (T*C, N) of dn_dtype (default: llr's dtype)."""
    t = _lib.require_gpu()
    assert llr.dim() == 2 and llr.stride(1) == 1
    T = llr.shape[0]
    assert llr.shape[1] >= cfg.E_total
    dn_dtype = dn_dtype or llr.dtype
    ws = ws or SchWorkspace(cfg, T, llr.device)
    out = ws.dn_buf(dn_dtype, cfg)
    if harq_in is not None:
        assert harq_in.dtype == dn_dtype and harq_in.shape == out.shape and harq_in.is_contiguous()
    with t.cuda.device(llr.device):
        _lib.check(_lib.lib().ldpc5g_sch_raterecover(
            _lib.ptr(llr), _dtype_id(t, llr.dtype), llr.stride(0), _lib.ctypes.byref(cfg), T,
            _lib.ptr(harq_in) if harq_in is not None else None, _lib.ptr(out),
            _dtype_id(t, dn_dtype), _lib.stream_ptr(llr.device)))
    return out


def sch_tb_check_batch(ck, cfg, T, ws=None):
    """TB reassembly + CB / TB CRC checks (ldpc5g_sch_tb_check) of decoded ck (T*C, >=K_apo)."""
    t = _lib.require_gpu()
    assert ck.dim() == 2 and ck.dtype == t.int8 and ck.stride(1) == 1 and ck.shape[0] == T * cfg.C
    ws = ws or SchWorkspace(cfg, T, ck.device)
    with t.cuda.device(ck.device):
        _lib.check(_lib.lib().ldpc5g_sch_tb_check(
            _lib.ptr(ck), ck.stride(0), _lib.ctypes.byref(cfg), T, _lib.ptr(ws.tbblk),
            ws.tbblk.stride(0), _lib.ptr(ws.cb_ok), _lib.ptr(ws.tb_rem), _lib.ptr(ws.tb_ok),
            _lib.stream_ptr(ck.device)))
    return ws.tb_ok, ws.tbblk, ws.cb_ok, ws.tb_rem


def sch_decode_batch(llr, cfg, L, algo="min-sum", alpha=1.0, beta=0.0, schedule="flooding",
                     harq_in=None, dn_dtype=None, ws=None):
    """DLSCHDecode / ULSCH_decoding of T transport blocks on the GPU.

    llr: (T, >=E_total) float32/64 device tensor of demodulated LLRs.  schedule 'flooding' with
    float64 (the default dn_dtype for float64 llr) is bit-exact with the reference chain;
    'layered' needs float32.  algo 'BF' / 'BP' decode through the batched decoders.
    Returns SchDecodeResult(tb_ok (T,) uint8, tbblk (T, B) int8 — TB bits then its CRC,
    llr_dn (T*C, N) — the reference's new_LLr_dns, ck, status, iters, cb_crc_ok, tb_rem)."""
    t = _lib.require_gpu()
    assert algo in ["BF", "BP", "min-sum"]
    T = llr.shape[0]
    ws = ws or SchWorkspace(cfg, T, llr.device)
    if algo == "min-sum" and not beta >= 0:
        # the reference decodes each codeblock with nr_decode_ldpc (nr_dlsch_decode.py:91,
        # nr_ulsch_decode.py:92), which keeps min-sum's literal zero branches for beta < 0
        # (nr_ldpc_decode.py:186-225): the float64 sparse flooding kernel on the base graph, as
        # nr_decode_ldpc here.  beta < 0 therefore always runs the reference's float64 flooding
        # chain: a layered schedule or a float32 dn_dtype is refused, not silently ignored.
        from .nr_ldpc_decode import SparseGraph, _sparse_graph, decode_ldpc_batch
        assert schedule == "flooding", "beta < 0 decodes with the float64 flooding sparse kernel only"
        assert dn_dtype in (None, t.float64), "beta < 0: rate recovery must be float64 (dn_dtype)"
        dn_dtype = t.float64
        llr_dn = sch_raterecover_batch(llr, cfg, harq_in, dn_dtype, ws)
        x = t.zeros((T * cfg.C, cfg.N + 2 * cfg.Zc), dtype=t.float64, device=llr.device)
        x[:, 2 * cfg.Zc:] = llr_dn   # punctured systematic columns: LLR 0 (nr_ldpc_decode.py:43)
        g = _sparse_graph(("bg", cfg.bgn, cfg.Zc),
                          lambda: SparseGraph.from_base_graph(cfg.bgn, cfg.Zc, llr.device), llr.device)
        decode_ldpc_batch(x, g, L, algo, alpha, beta, out=(ws.dec_ck, ws.status, ws.iters))
        sch_tb_check_batch(ws.dec_ck, cfg, T, ws)
    elif algo == "min-sum":
        dn_dtype = dn_dtype or (t.float32 if schedule == "layered" else llr.dtype)
        out = ws.dn_buf(dn_dtype, cfg)
        if harq_in is not None:
            assert harq_in.dtype == dn_dtype and harq_in.shape == out.shape and harq_in.is_contiguous()
        assert llr.dim() == 2 and llr.stride(1) == 1 and llr.shape[1] >= cfg.E_total
        sched = {"flooding": _lib.FLOODING, "layered": _lib.LAYERED}[schedule]
        with t.cuda.device(llr.device):
            _lib.check(_lib.lib().ldpc5g_sch_decode(
                _lib.ptr(llr), _dtype_id(t, llr.dtype), llr.stride(0), _lib.ctypes.byref(cfg), T,
                _lib.ptr(harq_in) if harq_in is not None else None, _lib.ptr(out),
                _dtype_id(t, dn_dtype), _lib.ptr(ws.dec_ck), _lib.ptr(ws.status),
                _lib.ptr(ws.iters), int(L), float(alpha), float(beta), sched, _lib.ptr(ws.tbblk),
                ws.tbblk.stride(0), _lib.ptr(ws.cb_ok), _lib.ptr(ws.tb_rem), _lib.ptr(ws.tb_ok),
                _lib.stream_ptr(llr.device)))
        llr_dn = out
    else:
        from .nr_ldpc_decode import nr_decode_ldpc_batch
        dn_dtype = dn_dtype or (t.float32 if schedule == "layered" else llr.dtype)
        llr_dn = sch_raterecover_batch(llr, cfg, harq_in, dn_dtype, ws)
        nr_decode_ldpc_batch(llr_dn, cfg.Zc, cfg.bgn, L, algo, alpha, beta, "flooding",
                             out=(ws.dec_ck, ws.status, ws.iters), rate_matched=True)
        sch_tb_check_batch(ws.dec_ck, cfg, T, ws)
    return SchDecodeResult(ws.tb_ok, ws.tbblk, llr_dn, ws.dec_ck, ws.status, ws.iters, ws.cb_ok,
                           ws.tb_rem)


# ------------------------------------------------------------ per-TB configurations (multi)
SchMultiResult = namedtuple(
    "SchMultiResult", "tb_ok tbblk llr_dn ck status iters cb_crc_ok tb_rem rows")


def multi_layout(cfgs):
    """Workspace geometry of a batch whose transport blocks each have their own configuration
    (ldpc5g_sch_multi_sizes): dict(ck, dn, dck, ncb, max_A, max_B, max_E) plus `rows`: per TB
    (first codeblock, C, dn element offset, N, decoder-ck offset, Nf) in workspace order."""
    T = len(cfgs)
    arr = (_lib.SchCfg * max(T, 1))(*cfgs)
    sizes = (_lib.ctypes.c_int64 * 7)()
    _lib.check(_lib.lib().ldpc5g_sch_multi_sizes(arr, T, sizes))
    rows, cb, dn, dck = [], 0, 0, 0
    for c in cfgs:
        nf = (68 if c.bgn == 1 else 52) * c.Zc
        rows.append((cb, c.C, dn, c.N, dck, nf))
        cb, dn, dck = cb + c.C, dn + c.C * c.N, dck + c.C * nf
    return dict(ck=sizes[0], dn=sizes[1], dck=sizes[2], ncb=sizes[3], max_A=sizes[4],
                max_B=sizes[5], max_E=sizes[6], rows=rows, arr=arr)


def sch_encode_multi(trblk, cfgs):
    """DLSCHEncode / UL-SCH encode of T transport blocks with per-TB configurations in one call
    (ldpc5g_sch_encode_multi).  trblk: (T, >= max A) int8 device tensor (TB t uses A_t bits).
    Returns g (T, max E_total) int8 (TB t's first E_total_t entries valid)."""
    t = _lib.require_gpu()
    T = len(cfgs)
    lay = multi_layout(cfgs)
    assert trblk.dim() == 2 and trblk.shape[0] == T and trblk.dtype == t.int8 and trblk.stride(1) == 1
    assert trblk.shape[1] >= lay["max_A"]
    dev = trblk.device
    g = t.empty((T, max(lay["max_E"], 1)), dtype=t.int8, device=dev)
    ck = t.empty((max(lay["ck"], 1),), dtype=t.int8, device=dev)
    dn = t.empty((max(lay["dn"], 1),), dtype=t.int8, device=dev)
    crc = t.empty((max(T, 1),), dtype=t.int32, device=dev)
    with t.cuda.device(dev):
        _lib.check(_lib.lib().ldpc5g_sch_encode_multi(
            _lib.ptr(trblk), trblk.stride(0), _lib.ptr(g), g.stride(0), lay["arr"], T,
            _lib.ptr(ck), _lib.ptr(dn), _lib.ptr(crc), _lib.stream_ptr(dev)))
    return g


def sch_raterecover_multi(llr, cfgs, harq_in=None, dn_dtype=None, out=None, lay=None):
    """Rate recovery (raterecover_ldpc, py5gphy/ldpc/nr_ldpc_raterecover.py:6-65) of T transport
    blocks with per-TB configurations in ONE launch (ldpc5g_sch_raterecover_multi).
    llr: (T, >= max E_total) float32/64 device tensor.  Returns the flat llr_dn (codeblock rows of
    N_t, TB after TB; multi_layout(cfgs)["rows"] locates them) of dn_dtype (default llr's)."""
    t = _lib.require_gpu()
    T = len(cfgs)
    lay = lay or multi_layout(cfgs)
    assert llr.dim() == 2 and llr.shape[0] == T and llr.stride(1) == 1 and llr.shape[1] >= lay["max_E"]
    dn_dtype = dn_dtype or llr.dtype
    if out is None:
        out = t.empty((max(lay["dn"], 1),), dtype=dn_dtype, device=llr.device)
    assert out.dtype == dn_dtype and out.numel() >= lay["dn"] and out.is_contiguous()
    if harq_in is not None:
        assert harq_in.dtype == dn_dtype and harq_in.numel() >= lay["dn"] and harq_in.is_contiguous()
    with t.cuda.device(llr.device):
        _lib.check(_lib.lib().ldpc5g_sch_raterecover_multi(
            _lib.ptr(llr), _dtype_id(t, llr.dtype), llr.stride(0), lay["arr"], T,
            _lib.ptr(harq_in) if harq_in is not None else None, _lib.ptr(out), _dtype_id(t, dn_dtype),
            _lib.stream_ptr(llr.device)))
    return out


class SchRaterecoverPlan:
    """sch_raterecover_multi for repeated use: the per-TB geometry is validated and copied to the
    device once (ldpc5g_sch_multi_plan); each call only launches the kernel
    (ldpc5g_sch_raterecover_multi_plan), asynchronously on the current stream."""

    def __init__(self, cfgs, device):
        t = _lib.require_gpu()
        lib = _lib.lib()
        self.lay = multi_layout(cfgs)
        self.T = len(cfgs)
        n = lib.ldpc5g_sch_multi_plan(self.lay["arr"], self.T, None, 0)
        _lib.check(int(min(n, 0)))
        self.host = t.empty((max(n, 1),), dtype=t.uint8, pin_memory=True)
        _lib.check(int(min(lib.ldpc5g_sch_multi_plan(self.lay["arr"], self.T, _lib.ptr(self.host), n), 0)))
        self.dev = self.host.to(device, non_blocking=True)

    def __call__(self, llr, out, harq_in=None):
        t = _lib.torch()
        assert llr.dim() == 2 and llr.shape[0] == self.T and llr.stride(1) == 1
        assert llr.shape[1] >= self.lay["max_E"] and out.is_contiguous() and out.numel() >= self.lay["dn"]
        if harq_in is not None:
            assert harq_in.dtype == out.dtype and harq_in.numel() >= self.lay["dn"] and harq_in.is_contiguous()
        with t.cuda.device(llr.device):
            _lib.check(_lib.lib().ldpc5g_sch_raterecover_multi_plan(
                _lib.ptr(self.dev), _lib.ptr(self.host), _lib.ptr(llr), _dtype_id(t, llr.dtype),
                llr.stride(0), _lib.ptr(harq_in) if harq_in is not None else None, _lib.ptr(out),
                _dtype_id(t, out.dtype), _lib.stream_ptr(llr.device)))
        return out


def sch_decode_multi(llr, cfgs, L, alpha=1.0, beta=0.0, schedule="flooding", harq_in=None,
                     dn_dtype=None):
    """DLSCHDecode / ULSCH_decoding of T transport blocks with per-TB configurations in one call
    (ldpc5g_sch_decode_multi): rate recovery, every codeblock decoded by the mixed-Zc decoder,
    TB reassembly and CRCs.  llr: (T, >= max E_total) float32/64 device tensor.
    Returns SchMultiResult(tb_ok (T,), tbblk (T, max B) — TB t's first B_t bits, llr_dn flat
    (the HARQ buffers new_LLr_dns of every TB, rows[t] locates them), ck flat, status, iters,
    cb_crc_ok (per codeblock), tb_rem, rows)."""
    t = _lib.require_gpu()
    T = len(cfgs)
    lay = multi_layout(cfgs)
    assert llr.dim() == 2 and llr.shape[0] == T and llr.stride(1) == 1 and llr.shape[1] >= lay["max_E"]
    dn_dtype = dn_dtype or (t.float32 if schedule == "layered" else llr.dtype)
    dev = llr.device
    llr_dn = t.empty((max(lay["dn"], 1),), dtype=dn_dtype, device=dev)
    if harq_in is not None:
        assert harq_in.dtype == dn_dtype and harq_in.numel() >= lay["dn"] and harq_in.is_contiguous()
    ck = t.empty((max(lay["dck"], 1),), dtype=t.int8, device=dev)
    n = max(lay["ncb"], 1)
    status = t.empty((n,), dtype=t.uint8, device=dev)
    iters = t.empty((n,), dtype=t.int32, device=dev)
    cb_ok = t.empty((n,), dtype=t.uint8, device=dev)
    tbblk = t.empty((T, max(lay["max_B"], 1)), dtype=t.int8, device=dev)
    tb_rem = t.empty((max(T, 1),), dtype=t.int32, device=dev)
    tb_ok = t.empty((max(T, 1),), dtype=t.uint8, device=dev)
    sched = {"flooding": _lib.FLOODING, "layered": _lib.LAYERED}[schedule]
    with t.cuda.device(dev):
        _lib.check(_lib.lib().ldpc5g_sch_decode_multi(
            _lib.ptr(llr), _dtype_id(t, llr.dtype), llr.stride(0), lay["arr"], T,
            _lib.ptr(harq_in) if harq_in is not None else None, _lib.ptr(llr_dn),
            _dtype_id(t, dn_dtype), _lib.ptr(ck), _lib.ptr(status), _lib.ptr(iters), int(L),
            float(alpha), float(beta), sched, _lib.ptr(tbblk), tbblk.stride(0), _lib.ptr(cb_ok),
            _lib.ptr(tb_rem), _lib.ptr(tb_ok), _lib.stream_ptr(dev)))
    return SchMultiResult(tb_ok[:T], tbblk, llr_dn, ck, status, iters, cb_ok, tb_rem, lay["rows"])
