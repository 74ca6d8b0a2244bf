"""The drop-in modules expose the reference's call surface: same function names, parameter
names, order and defaults.  Compared against the reference's source via `inspect` when the
reference is present (build container); skipped elsewhere (the GPU box never has it)."""
import ast
import inspect
import os

import pytest

REF = "/root/reference/py5gphy"

PAIRS = [
    ("ldpc/nr_ldpc_encode.py", "python_5gtoolbox_amd.nr_ldpc_encode", ["encode_ldpc"]),
    ("ldpc/nr_ldpc_decode.py", "python_5gtoolbox_amd.nr_ldpc_decode",
     ["nr_decode_ldpc", "decode_ldpc", "for_test_5g_ldpc_encoder"]),
    ("ldpc/ldpc_info.py", "python_5gtoolbox_amd.ldpc_info",
     ["get_cbs_info", "find_iLS", "getH", "gen_ldpc_para"]),
    ("ldpc/nr_ldpc_cbsegment.py", "python_5gtoolbox_amd.nr_ldpc_cbsegment", ["ldpc_cbsegment"]),
    ("ldpc/nr_ldpc_ratematch.py", "python_5gtoolbox_amd.nr_ldpc_ratematch",
     ["get_Er_ldpc", "get_k0", "ratematch_ldpc"]),
    ("ldpc/nr_ldpc_raterecover.py", "python_5gtoolbox_amd.nr_ldpc_raterecover", ["raterecover_ldpc"]),
    ("crc/crc.py", "python_5gtoolbox_amd.crc", ["nr_crc_encode", "nr_crc_decode"]),
    ("nr_pdsch/nr_dlsch.py", "python_5gtoolbox_amd.nr_dlsch", ["DLSCHEncode"]),
    ("nr_pdsch/nr_dlsch_decode.py", "python_5gtoolbox_amd.nr_dlsch_decode", ["DLSCHDecode"]),
    ("nr_pusch/nr_ulsch.py", "python_5gtoolbox_amd.nr_ulsch",
     ["ULSCH_Crc_CodeBlockSegment", "ULSCH_encoding_ratematch"]),
    ("nr_pusch/nr_ulsch_decode.py", "python_5gtoolbox_amd.nr_ulsch_decode", ["ULSCH_decoding"]),
    ("common/nrPRBS.py", "python_5gtoolbox_amd.nrPRBS", ["gen_nrPRBS"]),
    ("common/nrModulation.py", "python_5gtoolbox_amd.nrModulation", ["nrModulate"]),
    ("demodulation/nr_Demodulation.py", "python_5gtoolbox_amd.nr_Demodulation", ["nrDemodulate"]),
    # the BLER harness the reference's scripts import (scripts/sim_ldpc_decoder.py:6)
    ("../scripts/internal/sim_ldpc_internal.py", "python_5gtoolbox_amd.sim_ldpc_internal",
     ["run_ldpc_simulation", "draw_ldpc_decoder_result"]),
]


def _ref_signatures(path):
    """(arg names, defaults) of each top-level def, parsed from the reference source text."""
    tree = ast.parse(open(os.path.join(REF, path)).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef):
            names = [a.arg for a in node.args.args]
            defaults = []
            for d in node.args.defaults:
                try:
                    defaults.append(ast.literal_eval(d))
                except ValueError:   # e.g. np.array([]): compared by its source text
                    defaults.append(ast.unparse(d))
            out[node.name] = (names, defaults)
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not present")
@pytest.mark.parametrize("path,mod,funcs", PAIRS)
def test_signatures_match_reference(path, mod, funcs):
    import importlib
    m = importlib.import_module(mod)
    ref = _ref_signatures(path)
    for f in funcs:
        # keyword-only extras (after `*`) are additions a reference caller never passes
        params = [p for p in inspect.signature(getattr(m, f)).parameters.values()
                  if p.kind is not p.KEYWORD_ONLY]
        names = [p.name for p in params]
        defaults = [p.default for p in params if p.default is not p.empty]
        rnames, rdefaults = ref[f]
        assert names == rnames, (f, names, rnames)
        assert len(defaults) == len(rdefaults), (f, defaults, rdefaults)
        for d, r in zip(defaults, rdefaults):
            if r == "np.array([])":
                assert getattr(d, "size", None) == 0, (f, d)
            else:
                assert d == r, (f, d, r)
