"""Mixed-(bgn, Zc) batched min-sum decode (ldpc5g_decode_ms_mixed) — the shape DLSCHDecode
(py5gphy/nr_pdsch/nr_dlsch_decode.py:62-91) and ULSCH_decoding produce once their per-codeblock
loop is batched: codeblocks of different lifting sizes decoded in at most two launches."""
import numpy as np

from . import _lib
from .ldpc_info import code_dims, find_iLS


def decode_mixed(items, L, alpha=1.0, beta=0.0, schedule="flooding", rate_matched=False):
    """items: list of (bgn, Zc, llr[N]) with float32 (or all float64) LLR rows.
    rate_matched: the rows come from rate recovery (LDPC5G_RATE_MATCHED: untransmitted extension
    columns +0.0 are detected and their null row updates skipped; same results).
    Returns (list of ck int8[Nf] arrays, status bool[B], iters int32[B]) in item order."""
    t = _lib.require_gpu()
    assert schedule in ("flooding", "layered")
    B = len(items)
    f64 = all(np.asarray(l).dtype == np.float64 for _, _, l in items) and schedule == "flooding"
    dt = np.float64 if f64 else np.float32
    desc = (_lib.CbDesc * max(B, 1))()
    lo = co = 0
    rows = []
    for k, (bgn, Zc, llr) in enumerate(items):
        assert bgn in [1, 2] and find_iLS(Zc) < 8
        K, N, Nf = code_dims(bgn, Zc)
        llr = np.asarray(llr, dt)
        assert llr.size == N
        desc[k].bgn, desc[k].Zc, desc[k].llr_off, desc[k].ck_off = bgn, Zc, lo, co
        rows.append((lo, co, Nf))
        lo += N
        co += Nf
    flat = np.concatenate([np.asarray(l, dt) for _, _, l in items]) if B else np.zeros(1, dt)
    x = t.from_numpy(flat).cuda()
    ck = t.empty(max(co, 1), dtype=t.int8, device=x.device)
    st = t.empty(max(B, 1), dtype=t.uint8, device=x.device)
    it = t.empty(max(B, 1), dtype=t.int32, device=x.device)
    with t.cuda.device(x.device):
        _lib.check(_lib.lib().ldpc5g_decode_ms_mixed(
            desc, B, _lib.ptr(x), _lib.F64 if f64 else _lib.F32, _lib.ptr(ck), _lib.ptr(st),
            _lib.ptr(it), int(L), float(alpha), float(beta),
            _lib.LAYERED if schedule == "layered" else _lib.FLOODING,
            _lib.RATE_MATCHED if rate_matched else 0, _lib.stream_ptr(x.device)))
    ckh = ck.cpu().numpy()
    return ([ckh[c:c + n].copy() for _, c, n in rows], st.cpu().numpy()[:B].astype(bool),
            it.cpu().numpy()[:B])


class MixedBatch:
    """A device-resident mixed-(bgn, Zc) batch for repeated decoding (the bench's config 4):
    rows of several (bgn, Zc) groups concatenated in one flat LLR buffer, with the descriptor
    array (ldpc5g_cb_desc_t) built once.

    groups: list of (bgn, Zc, llr (n, N) device tensor), all float32 or all float64 (float64:
    flooding only, the reference's arithmetic).  flat: an existing flat buffer of that dtype
    holding exactly those rows back to back in group order (e.g. sch_raterecover_multi's output,
    whose row groups are views of it): used in place, nothing is copied."""

    def __init__(self, groups, flat=None):
        t = _lib.require_gpu()
        B = sum(g[2].shape[0] for g in groups)
        self.desc = (_lib.CbDesc * max(B, 1))()
        parts, lo, co, k = [], 0, 0, 0
        self.rows = []
        dt = groups[0][2].dtype
        assert dt in (t.float32, t.float64), "LLRs must be float32 or float64"
        self.dtype = _lib.F32 if dt == t.float32 else _lib.F64
        for bgn, Zc, llr in groups:
            assert bgn in [1, 2] and find_iLS(Zc) < 8 and llr.dtype == dt
            K, N, Nf = code_dims(bgn, Zc)
            assert llr.dim() == 2 and llr.shape[1] == N
            for _ in range(llr.shape[0]):
                d = self.desc[k]
                d.bgn, d.Zc, d.llr_off, d.ck_off = bgn, Zc, lo, co
                self.rows.append((co, Nf))
                lo += N
                co += Nf
                k += 1
            parts.append(llr.reshape(-1))
        dev = groups[0][2].device
        if flat is not None:
            assert flat.dtype == dt and flat.is_contiguous() and flat.numel() >= lo
            self.llr = flat
        else:
            self.llr = t.cat(parts).contiguous()
        self.ck = t.empty(max(co, 1), dtype=t.int8, device=dev)
        self.status = t.empty(max(B, 1), dtype=t.uint8, device=dev)
        self.iters = t.empty(max(B, 1), dtype=t.int32, device=dev)
        self.B = B
        self._plans = {}

    def _plan(self, schedule):
        """Work list for `schedule`, built on the host once (pinned) and copied to the device
        once; later decodes only launch (ldpc5g_decode_ms_mixed_plan)."""
        p = self._plans.get(schedule)
        if p is None:
            t = _lib.torch()
            lib = _lib.lib()
            sc = _lib.LAYERED if schedule == "layered" else _lib.FLOODING
            n = lib.ldpc5g_mixed_plan(self.desc, self.B, sc, None, 0)
            _lib.check(int(min(n, 0)))
            host = t.empty((max(n, 1),), dtype=t.uint8, pin_memory=True)
            _lib.check(int(min(lib.ldpc5g_mixed_plan(self.desc, self.B, sc, _lib.ptr(host), n), 0)))
            dev = host.to(self.llr.device, non_blocking=True)
            p = self._plans[schedule] = (host, dev)
        return p

    def decode(self, L, alpha=1.0, beta=0.0, schedule="layered", rate_matched=False):
        """<= 2 kernel launches on the current stream, asynchronous (no host synchronisation);
        returns the device buffers (ck flat, status (B,), iters (B,)).  rate_matched: see
        decode_mixed."""
        t = _lib.torch()
        assert schedule != "layered" or self.dtype == _lib.F32, "the layered kernel is float32"
        host, dev = self._plan(schedule)
        with t.cuda.device(self.llr.device):
            _lib.check(_lib.lib().ldpc5g_decode_ms_mixed_plan(
                _lib.ptr(dev), _lib.ptr(host), _lib.ptr(self.llr), self.dtype, _lib.ptr(self.ck),
                _lib.ptr(self.status), _lib.ptr(self.iters), int(L), float(alpha), float(beta),
                _lib.LAYERED if schedule == "layered" else _lib.FLOODING,
                _lib.RATE_MATCHED if rate_matched else 0, _lib.stream_ptr(self.llr.device)))
        return self.ck, self.status[:self.B], self.iters[:self.B]
