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
from .sch import sch_config, sch_decode_batch


def decode_tb(LLr, cfg, LDPC_decoder_config, HARQ_on, current_LLr_dns):
    """Shared body of DLSCHDecode / ULSCH_decoding for one transport block (host arrays)."""
    t = _lib.require_gpu()
    dc = LDPC_decoder_config
    schedule = dc.get("schedule", "flooding")
    llr = np.ascontiguousarray(np.asarray(LLr, np.float64).reshape(1, -1))
    x = t.from_numpy(llr).cuda()
    dn_dtype = t.float32 if schedule == "layered" else t.float64
    harq = None
    cur = np.asarray(current_LLr_dns)
    if HARQ_on and cur.size != 0:
        assert cur.shape == (cfg.C, cfg.N)
        harq = t.from_numpy(np.ascontiguousarray(cur, np.float64)).to(x.device, dn_dtype)
    r = sch_decode_batch(x, cfg, dc["L"], dc["algo"], dc["alpha"], dc["beta"], schedule, harq,
                         dn_dtype)
    tb_ok = bool(r.tb_ok.cpu().numpy()[0])
    tbblk = r.tbblk[0, :cfg.A].cpu().numpy().astype("i1")
    new = r.llr_dn.cpu().numpy().astype(np.float64)
    return tb_ok, tbblk, new


def DLSCHDecode(LLr, TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, LDPC_decoder_config,
                HARQ_on=False, current_LLr_dns=np.array([])):
    """DLSCH receiving processing: de-rate matching, LDPC decoder, CRC decoder."""
    G = LLr.size
    cfg = sch_config(TBSize, Qm, coderateby1024, num_of_layers, rv, TBS_LBRM, G)
    return decode_tb(LLr, cfg, LDPC_decoder_config, HARQ_on, current_LLr_dns)
