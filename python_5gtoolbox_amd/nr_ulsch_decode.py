"""Drop-in for py5gphy/nr_pusch/nr_ulsch_decode.py — UL-SCH receive chain on the GPU.

    ULSCH_decoding(g_ulsch_LLr, TBSize, coderateby1024, Qm, G_ULSCH, num_of_layers, rv,
                   LDPC_decoder_config, HARQ_on=False, current_LLr_dns=np.array([]))
        -> (crc_ok, tbblk, new_LLr_dns)                          (nr_ulsch_decode.py:13-110)
Same chain as DLSCHDecode with Ncb = N (I_LBRM = 0) and Er sized by G_ULSCH.
"""
import numpy as np

from .nr_dlsch_decode import decode_tb
from .sch import sch_config


def ULSCH_decoding(g_ulsch_LLr, TBSize, coderateby1024, Qm, G_ULSCH, num_of_layers, rv,
                   LDPC_decoder_config, HARQ_on=False, current_LLr_dns=np.array([])):
    cfg = sch_config(TBSize, Qm, coderateby1024, num_of_layers, rv, 0, G_ULSCH)
    return decode_tb(g_ulsch_LLr, cfg, LDPC_decoder_config, HARQ_on, current_LLr_dns)
