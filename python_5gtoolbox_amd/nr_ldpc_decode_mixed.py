"""Mixed-(bgn, Zc) batched min-sum decode (ldpc5g_decode_ms_mixed) — the shape DLSCHDecode
(py5gphy/nr_pdsch/nr_dlsch_decode.py:62-91) and ULSCH_decoding produce once their per-codeblock
loop is batched: codeblocks of different lifting sizes decoded in at most two launches."""
import numpy as np

from . import _lib
from .ldpc_info import code_dims, find_iLS


def decode_mixed(items, L, alpha=1.0, beta=0.0, schedule="flooding"):
    """items: list of (bgn, Zc, llr[N]) with float32 (or all float64) LLR rows.
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
            _lib.LAYERED if schedule == "layered" else _lib.FLOODING, 0,
            _lib.stream_ptr(x.device)))
    ckh = ck.cpu().numpy()
    return ([ckh[c:c + n].copy() for _, c, n in rows], st.cpu().numpy()[:B].astype(bool),
            it.cpu().numpy()[:B])
