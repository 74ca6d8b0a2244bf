"""CPU tests of the DL-SCH / UL-SCH host side: ldpc5g_sch_config (pure host code in the C ABI)
against the oracle's restatement of the reference's float arithmetic (base-graph thresholds,
get_cbs_info, Nref, k0, Er), the oracle chain against the reference's own transport-block
fixtures, and argument errors.  No kernel is launched here."""
import ctypes

import numpy as np
import pytest

from conftest import GOLD, load_json
from oracle import ldpc_oracle as O
from python_5gtoolbox_amd import _lib
from python_5gtoolbox_amd.sch import cfg_from_codeblocks, sch_config


def _cases(n=400, seed=3):
    rng = np.random.default_rng(seed)
    out = [(1081512, 8, 948, 4, 0, 1081512, 8 * 4 * 36036),   # config 5 (C = 129)
           (24, 2, 100, 1, 0, 0, 200), (292, 2, 900, 1, 1, 5000, 1200),
           (3824, 4, 686, 1, 2, 20000, 9000), (3825, 4, 686, 2, 3, 0, 12000)]
    while len(out) < n:
        A = int(rng.integers(24, 400000))
        Qm = int(rng.choice([1, 2, 4, 6, 8]))
        NL = int(rng.integers(1, 5))
        R = float(rng.choice([rng.integers(30, 950), rng.uniform(30, 950)]))
        rv = int(rng.integers(0, 4))
        LBRM = int(rng.choice([0, A, int(A * rng.uniform(1, 4))]))
        G = NL * Qm * int(rng.integers(max(1, A // (NL * Qm * 2)), 3 * A // (NL * Qm) + 10))
        out.append((A, Qm, R, NL, rv, LBRM, G))
    return out


def _oracle_or_none(args):
    try:
        return O.sch_params(*args)
    except AssertionError:
        return None


@pytest.mark.parametrize("args", _cases())
def test_sch_config_matches_oracle(args):
    p = _oracle_or_none(args)
    if p is None:
        with pytest.raises(AssertionError):
            sch_config(*args)
        return
    c = sch_config(*args)
    assert (c.A, c.B, c.bgn, c.C, c.cbz, c.Lcb, c.F, c.K, c.Zc, c.N, c.Ncb, c.k0, c.K_apo) == \
        (p["A"], p["B"], p["bgn"], p["C"], p["cbz"], p["L"], p["F"], p["K"], p["Zc"], p["N"],
         p["Ncb"], p["k0"], p["K_apo"])
    assert c.tb_crc_poly == _lib.CRC_IDS[p["poly"]]
    Er = [c.E_lo if j < c.c_switch else c.E_hi for j in range(c.C)]
    assert Er == p["Er"]
    assert c.E_total == sum(p["Er"])


def test_cfg_from_codeblocks_matches_config():
    for args in _cases(60, seed=5):
        p = _oracle_or_none(args)
        if p is None:
            continue
        A, Qm, R, NL, rv, LBRM, G = args
        c = sch_config(*args)
        d = cfg_from_codeblocks(c.C, c.K, c.K_apo, c.Zc, c.bgn, Qm, G, NL, rv, Ncb=c.Ncb)
        for f in ("B", "bgn", "C", "cbz", "Lcb", "F", "K", "K_apo", "Zc", "N", "Ncb", "k0", "Qm",
                  "E_total"):
            assert getattr(c, f) == getattr(d, f), f
        assert [c.E_lo if j < c.c_switch else c.E_hi for j in range(c.C)] == \
            [d.E_lo if j < d.c_switch else d.E_hi for j in range(d.C)]


def test_sch_cfg_struct_layout():
    assert ctypes.sizeof(_lib.SchCfg) == 20 * 4 + 2 * 8


@pytest.mark.parametrize("args", [(0, 2, 500, 1, 0, 0, 100), (1000, 2, 500, 1, 4, 0, 100),
                                  (1000, 2, 500, 0, 0, 0, 100), (1000, 2, 500, 1, 0, 0, 0)])
def test_sch_config_rejects_bad_arguments(args):
    with pytest.raises(AssertionError):
        sch_config(*args)


def test_sch_entry_points_validate_before_touching_the_gpu():
    lib = _lib.lib()
    cfg = sch_config(12000, 4, 517, 1, 0, 30000, 25000)
    bad = _lib.SchCfg.from_buffer_copy(cfg)
    bad.K_apo += 1
    assert lib.ldpc5g_sch_encode(None, 12000, None, 25000, ctypes.byref(bad), 1, None, None, None,
                                 None) == _lib.ESIZE
    assert lib.ldpc5g_sch_encode(None, 12000, None, 25000, ctypes.byref(cfg), 1, None, None, None,
                                 None) == _lib.ESIZE   # null buffers
    assert lib.ldpc5g_sch_raterecover(None, 7, 25000, ctypes.byref(cfg), 1, None, None, 0,
                                      None) == _lib.ESIZE   # bad dtype
    assert lib.ldpc5g_crc(None, 10, 10, 1, 9, None, None) == _lib.ESIZE
    assert lib.ldpc5g_sch_encode(None, 0, None, 0, ctypes.byref(cfg), 0, None, None, None,
                                 None) == 0   # empty batch: nothing to do


def test_oracle_sch_encode_matches_reference_dlsch_golden():
    d = np.load(f"{GOLD}/dlsch_golden.npz")
    for i, (TBS, Qm, R, NL, rv, LBRM, G) in enumerate(d["meta"].tolist()):
        tb = np.unpackbits(d["tb"][d["tb_off"][i]:d["tb_off"][i + 1]])[:TBS].astype(np.int8)
        g = np.unpackbits(d["g"][d["g_off"][i]:d["g_off"][i + 1]])[:G].astype(np.int8)
        assert np.array_equal(O.sch_encode(tb, TBS, Qm, R, NL, rv, LBRM, G), g)


def test_oracle_sch_chain_matches_reference_sch_golden():
    """The oracle's DLSCHDecode / ULSCH_decoding restatement (rate recovery, HARQ, float64
    flooding decode, CRCs) against the reference's outputs (tests/golden/sch_golden.*)."""
    import hashlib
    cases = load_json("sch_golden.json")
    z = np.load(f"{GOLD}/sch_golden.npz")
    for n, cs in enumerate(cases):
        if cs["kind"] == "dl-encode":
            continue
        A, G = cs["TBS"], cs["G"]
        lbrm = cs["LBRM"] if cs["kind"] == "dl" else 0
        p = O.sch_params(A, cs["Qm"], cs["R"], cs["NL"], cs["rv"], lbrm, G)
        tb = np.unpackbits(z[f"trblk{n}"])[:A].astype(np.int8)
        g = np.unpackbits(z[f"g{n}"])[:G].astype(np.int8)
        assert np.array_equal(O.sch_encode(tb, A, cs["Qm"], cs["R"], cs["NL"], cs["rv"], lbrm, G), g)
        llr = z[f"llr{n}"].astype(np.float64)
        dn = O.sch_raterecover(llr, p)
        assert hashlib.sha256(dn.tobytes()).hexdigest() == cs["new_sha"]
        if cs["kind"] == "dl":   # HARQ retransmission (rv 2) combined with the first input
            p2 = O.sch_params(A, cs["Qm"], cs["R"], cs["NL"], 2, lbrm, G)
            dn2 = O.sch_raterecover(z[f"llr2_{n}"].astype(np.float64), p2, harq=dn)
            assert hashlib.sha256(dn2.tobytes()).hexdigest() == cs["new2_sha"]
        if p["Zc"] > 300:
            continue   # the float64 flooding decode of the big codeblocks runs in the GPU suite
        ck, _, _ = O.decode_flooding(dn, p["Zc"], p["bgn"], 6, 0.8, 0.0, np.float64)
        ok, blk, _ = O.sch_tb_check(ck, p)
        assert ok == cs["ok"]
        assert np.array_equal(blk, np.unpackbits(z[f"tbblk{n}"])[:A].astype(np.int8))


def test_sch_multi_sizes_host():
    """ldpc5g_sch_multi_sizes (host code) == the Python layout of a per-TB-configuration batch,
    and a bad configuration anywhere in the list is reported with its index."""
    from python_5gtoolbox_amd.sch import multi_layout
    cfgs = [sch_config(12000, 4, 517, 1, 0, 30000, 25000), sch_config(1800, 2, 308, 1, 0, 40000, 6000),
            sch_config(1081512, 8, 948, 4, 0, 1081512, 1153152)]
    lay = multi_layout(cfgs)
    assert lay["ncb"] == sum(c.C for c in cfgs)
    assert lay["ck"] == sum(c.C * c.K for c in cfgs) and lay["dn"] == sum(c.C * c.N for c in cfgs)
    assert lay["max_A"] == 1081512 and lay["max_E"] == max(c.E_total for c in cfgs)
    assert [r[0] for r in lay["rows"]] == [0, cfgs[0].C, cfgs[0].C + cfgs[1].C]
    bad = _lib.SchCfg.from_buffer_copy(cfgs[1])
    bad.K_apo += 1
    arr = (_lib.SchCfg * 3)(cfgs[0], bad, cfgs[2])
    sizes = (ctypes.c_int64 * 7)()
    assert _lib.lib().ldpc5g_sch_multi_sizes(arr, 3, sizes) == _lib.ESIZE
    assert b"cfgs[1]" in _lib.lib().ldpc5g_last_error()
