"""Module-level drop-in for the reference's scripts/internal/sim_ldpc_internal.py (the BLER
harness the reference's scripts import: scripts/sim_ldpc_decoder.py:6, NMS_ldpc_search_best_alpha.py,
OMS_ldpc_search_best_beta.py, mixed_MS_ldpc_search_best_pair.py, sim_ldpc_decoder_bf.py:11):

    sys.modules["scripts.internal.sim_ldpc_internal"] = python_5gtoolbox_amd.sim_ldpc_internal

run_ldpc_simulation(Zc, bgn, crcpoly, algo_list, alpha_list, beta_list, mixed_list, L_list,
snr_db_list, filename) then runs the sweep batched on the GPU and writes the reference's pickle;
draw_ldpc_decoder_result plots it.
"""
from .sim_ldpc import draw_ldpc_decoder_result, run_ldpc_simulation, run_ldpc_simulation_fixed  # noqa: F401
