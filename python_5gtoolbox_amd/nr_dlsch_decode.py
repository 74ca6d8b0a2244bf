"""Drop-in for py5gphy/nr_pdsch/nr_dlsch_decode.py — DL-SCH receive chain on the GPU.

    DLSCHDecode(LLr, TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM,
                LDPC_decoder_config, HARQ_on=False, current_LLr_dns=np.array([]))
        -> (crc_ok, tbblk, new_LLr_dns)                       (nr_dlsch_decode.py:13-110)

Rate recovery + HARQ combining, LDPC decoding of every codeblock in one batched launch, CB CRC24B
and TB CRC checks, all through ldpc5g_sch_* (the reference loops over codeblocks in Python).
algo='min-sum' runs the float64 flooding decoder (bit-exact with the reference); an extra
LDPC_decoder_config key "schedule": "layered" selects the float32 layered perf decoder.
"""
import numpy as np

from . import _lib
from .sch import SchWorkspace, sch_config, sch_decode_batch


def decode_tb(LLr, cfg, LDPC_decoder_config, HARQ_on, current_LLr_dns):
    """Shared body of DLSCHDecode / ULSCH_decoding for one transport block (host arrays).
    Host <-> device through per-thread cached pinned buffers (one H2D of the LLRs, one D2H each of
    the TB bits, the CRC flag and new_LLr_dns, one synchronisation) and a cached device workspace:
    pageable copies of the same data measured 2-4 ms per TB on the box."""
    t = _lib.require_gpu()
    dc = LDPC_decoder_config
    schedule = dc.get("schedule", "flooding")
    llr = np.asarray(LLr, np.float64).reshape(1, -1)
    G = llr.shape[1]
    dev = t.cuda.current_device()
    dn_dtype = t.float32 if schedule == "layered" else t.float64

    def make():
        return (t.empty((1, G), dtype=t.float64, pin_memory=True),
                t.empty((1, G), dtype=t.float64, device=dev),
                SchWorkspace(cfg, 1, t.device("cuda", dev), dn_dtype),
                t.empty((cfg.A + 8,), dtype=t.int8, pin_memory=True),
                t.empty((cfg.C, cfg.N), dtype=dn_dtype, pin_memory=True))
    key = ("dlsch", dev, G, cfg.A, cfg.C, cfg.N, cfg.Zc, cfg.bgn, cfg.B, cfg.K, cfg.E_total, str(dn_dtype))
    hin, x, ws, hbits, hdn = _lib.staging(key, make)
    hin.numpy()[...] = llr
    x.copy_(hin, non_blocking=True)
    harq = None
    cur = np.asarray(current_LLr_dns)
    if HARQ_on and cur.size != 0:
        assert cur.shape == (cfg.C, cfg.N)
        harq = t.from_numpy(np.ascontiguousarray(cur, np.float64)).to(x.device, dn_dtype)
    r = sch_decode_batch(x, cfg, dc["L"], dc["algo"], dc["alpha"], dc["beta"], schedule, harq,
                         dn_dtype, ws)
    hbits[:cfg.A].copy_(r.tbblk[0, :cfg.A], non_blocking=True)
    hbits[cfg.A:cfg.A + 1].copy_(r.tb_ok[:1].view(t.int8), non_blocking=True)
    hdn.copy_(r.llr_dn, non_blocking=True)
    t.cuda.current_stream().synchronize()
    b = hbits.numpy()
    return bool(b[cfg.A]), b[:cfg.A].copy(), hdn.numpy().astype(np.float64)   # astype: a copy


def DLSCHDecode(LLr, TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, LDPC_decoder_config,
                HARQ_on=False, current_LLr_dns=np.array([])):
    """DLSCH receiving processing: de-rate matching, LDPC decoder, CRC decoder."""
    G = LLr.size
    cfg = sch_config(TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, G)
    return decode_tb(LLr, cfg, LDPC_decoder_config, HARQ_on, current_LLr_dns)
