"""python_5gtoolbox_amd — MI355X-native 5G NR LDPC engine for the py5gphy/ldpc hot path.

Drop-in modules (same call surface as the reference's py5gphy.ldpc.*):
    nr_ldpc_encode.encode_ldpc(ck, bgn)
    nr_ldpc_decode.nr_decode_ldpc(LLRin, Zc, bgn, L, algo='min-sum', alpha=1, beta=0)
    nr_ldpc_decode.decode_ldpc(LLRin, H, L, algo, alpha, beta)
    ldpc_info.{get_cbs_info, find_iLS, getH, gen_ldpc_para}
Batched GPU APIs: nr_ldpc_encode.encode_ldpc_batch, nr_ldpc_decode.nr_decode_ldpc_batch,
nr_ldpc_decode_mixed.decode_mixed.  Kernels: csrc/ldpc5g.hip -> libldpc5g.so (C ABI in
include/ldpc5g.h), loaded by ctypes; torch is used for device buffers and streams only.
"""
__version__ = "0.1.0"
