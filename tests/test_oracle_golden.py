"""CPU: pin the oracle (oracle/ldpc_oracle.py) against the reference-generated golden vectors.

Every expected value here was produced by the reference itself (tests/golden/gen_golden.py), so
these tests are what makes the oracle trustworthy as the GPU parity checker."""
import os

import numpy as np
import pytest

from conftest import GOLD, load_algo_cases, load_json, load_sparse_cases
from oracle import ldpc_oracle as O


def test_tables_structure():
    t = O.tables()
    assert t[1].shape == (8, 46, 68) and t[2].shape == (8, 42, 52)
    assert (t[1][0] >= 0).sum() == 316 and (t[2][0] >= 0).sum() == 197
    assert t[1][6, 1, 22] == 105


def test_find_ils_and_cbs_info():
    assert [O.find_iLS(z) for z in (2, 3, 5, 7, 9, 11, 13, 15, 384, 17)] == [0, 1, 2, 3, 4, 5, 6, 7, 1, 255]
    # 273 PRB 256QAM MCS27 4 layers: TBS 1,081,512 (py5gphy/nr_pdsch/dl_tbsize.py:308-317 KAT)
    C, cbz, L, F, K, Zc = O.get_cbs_info(1081512 + 24, 1)
    assert (C, L, K, Zc) == (129, 24, 8448, 384)


def test_encode_golden(encode_cases):
    assert len(encode_cases) == 204
    for bg, Zc, F, ck, dn in encode_cases:
        assert np.array_equal(O.encode(ck, bg), dn), (bg, Zc, F)


def test_encode_codewords_satisfy_H(encode_cases):
    for bg, Zc, F, ck, dn in encode_cases[::7]:
        bits = np.concatenate([np.where(ck[:2 * Zc] == -1, 1, ck[:2 * Zc]), np.where(dn == -1, 0, dn)])
        assert not O.syndrome(bits, bg, Zc).any()


def test_decode_golden_fp64(decode_cases):
    """float64 restatement == reference nr_decode_ldpc, bit for bit (ck and status)."""
    for c in decode_cases:
        if c["Zc"] == 384:
            continue
        ck, st, _ = O.decode_flooding(c["llr"][None].astype(np.float64), c["Zc"], c["bg"], c["L"],
                                      c["alpha"], c["beta"], np.float64)
        assert np.array_equal(ck[0], c["ck"]) and bool(st[0]) == c["status"], (c["kind"], c["bg"], c["Zc"])


def test_decode_golden_fp32(decode_cases):
    """The fp32 restatement (the arithmetic of the GPU fp32 flooding kernel) reproduces the
    reference's status on every fixture and its ck bit for bit whenever decoding succeeds.
    Failed decodes may end on different hard decisions: after many non-converging iterations
    fp32 rounding takes a different trajectory than numpy float64 (3 of 190 small fixtures, all
    L=32 with status False).  The float64 path is the bit-exact one."""
    diverged = 0
    for c in decode_cases:
        if c["Zc"] == 384:
            continue
        ck, st, _ = O.decode_flooding(c["llr"][None], c["Zc"], c["bg"], c["L"], c["alpha"],
                                      c["beta"], np.float32)
        assert bool(st[0]) == c["status"], (c["kind"], c["bg"], c["Zc"])
        if c["status"]:
            assert np.array_equal(ck[0], c["ck"]), (c["kind"], c["bg"], c["Zc"])
        else:
            diverged += not np.array_equal(ck[0], c["ck"])
    assert diverged <= 5


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_decode_golden_z384(decode_cases, dtype):
    big = [c for c in decode_cases if c["Zc"] == 384]
    assert len(big) == 3
    llr = np.stack([c["llr"] for c in big]).astype(dtype)
    ck, st, it = O.decode_flooding(llr, 384, 1, 8, big[0]["alpha"], 0.0, dtype)
    for k, c in enumerate(big):
        if c["alpha"] != big[0]["alpha"]:
            ck1, st1, _ = O.decode_flooding(llr[k:k + 1], 384, 1, 8, c["alpha"], 0.0, dtype)
            ck_k, st_k = ck1[0], st1[0]
        else:
            ck_k, st_k = ck[k], st[k]
        assert bool(st_k) == c["status"]
        if dtype == np.float64 or c["status"]:
            assert np.array_equal(ck_k, c["ck"])


def test_layered_agrees_at_high_snr():
    """Layered schedule (no reference counterpart) decodes the same codewords as the reference's
    flooding schedule when both converge."""
    rng = np.random.default_rng(3)
    for bg, Zc in [(1, 12), (2, 20)]:
        K = (22 if bg == 1 else 10) * Zc
        ck = rng.integers(0, 2, (40, K)).astype(np.int8)
        dn = O.encode(ck, bg)
        llr = O.bpsk_awgn_llr(dn, 2.5, rng).astype(np.float32)
        a = O.decode_layered(llr, Zc, bg, 8, 0.75, 0)
        f = O.decode_flooding(llr, Zc, bg, 8, 0.75, 0, np.float32)
        both = a[1] & f[1]
        assert both.sum() >= 35
        assert np.array_equal(a[0][both], f[0][both])
        assert (a[2][both] <= f[2][both] + 1).all()


def test_crc_golden():
    cases = load_json("crc_golden.json")
    for c in cases:
        out = O.crc_encode(np.array(c["blk"]), c["poly"], c["mask"])
        assert out.tolist() == c["out"], (c["poly"], c["mask"])
        assert O.crc_decode(out, c["poly"], c["mask"])[1] == 0


def test_ratematch_golden():
    d = np.load(os.path.join(GOLD, "ratematch_golden.npz"))
    for i, (bg, Zc, K, K_apo, N, Ncb, E, k0, Qm, rv) in enumerate(d["meta"].tolist()):
        dn = d["dn"][d["dn_off"][i]:d["dn_off"][i + 1]]
        assert O.get_k0(Ncb, bg, rv, Zc) == k0
        fe = O.ratematch(dn, Ncb, E, k0, Qm)
        assert np.array_equal(fe, d["fe"][d["fe_off"][i]:d["fe_off"][i + 1]])
        llr = d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]].astype(np.float64)
        rr = O.raterecover(llr, Ncb, N, k0, Qm, Zc, K_apo, K)
        assert np.array_equal(rr, d["rr"][d["rr_off"][i]:d["rr_off"][i + 1]])
    for c in load_json("er_golden.json"):
        assert O.get_Er(c["G"], c["C"], c["Qm"], c["NL"]) == c["Er"]


def test_dlsch_encode_chain_golden():
    """TB CRC -> BG select -> CB segmentation -> encode -> rate match (nr_dlsch.py:12-74)
    restated with the oracle reproduces the reference DLSCHEncode output."""
    import math
    d = np.load(os.path.join(GOLD, "dlsch_golden.npz"))
    for i, (TBS, Qm, R, NL, rv, LBRM, G) in enumerate(d["meta"].tolist()):
        tb = np.unpackbits(d["tb"][d["tb_off"][i]:d["tb_off"][i + 1]])[:TBS]
        g_ref = np.unpackbits(d["g"][d["g_off"][i]:d["g_off"][i + 1]])[:G]
        blk = O.crc_encode(tb, "24A" if TBS > 3824 else "16")
        bgn = 2 if (TBS <= 292 or (TBS <= 3824 and R <= 0.67 * 1024) or R <= 0.25 * 1024) else 1
        cbs, Zc = O.cbsegment(blk, bgn)
        C = cbs.shape[0]
        Er = O.get_Er(G, C, Qm, NL)
        dn = O.encode(cbs, bgn)
        out = []
        for c in range(C):
            Ncb = min(dn.shape[1], math.floor(LBRM / (C * 2 / 3)))
            k0 = O.get_k0(Ncb, bgn, rv, Zc)
            out.append(O.ratematch(dn[c], Ncb, Er[c], k0, Qm))
        assert np.array_equal(np.concatenate(out), g_ref)


@pytest.mark.parametrize("algo", ["BF", "BP"])
def test_bf_bp_golden(algo):
    """decode_bf / decode_bp restatements == reference nr_decode_ldpc(algo='BF'/'BP'), bit for
    bit (the BP restatement uses numpy's own tanh/arctanh, like the reference)."""
    fn = O.decode_bf if algo == "BF" else O.decode_bp
    for c in load_algo_cases(algo):
        ck, st, _ = fn(c["llr"][None].astype(np.float64), c["Zc"], c["bg"], c["L"])
        assert np.array_equal(ck[0], c["ck"]) and bool(st[0]) == c["status"], (c["bg"], c["Zc"])


def test_prbs_modulation_demodulation_golden():
    """prbs / modulate / demodulate restatements == the reference's gen_nrPRBS, nrModulate,
    nrDemodulate outputs (tests/golden/demod_golden.npz), bit for bit (float32 / complex64)."""
    d = np.load(os.path.join(GOLD, "demod_golden.npz"))
    for j, (cinit, N) in enumerate(d["prbs_meta"].tolist()):
        assert np.array_equal(O.prbs(cinit, N), np.unpackbits(d[f"prbs{j}"])[:N]), (cinit, N)
    for k, (Qm, n) in enumerate(d["meta"].tolist()):
        bits = np.unpackbits(d[f"bits{k}"])[:n * Qm]
        assert np.array_equal(O.modulate(bits, Qm).view(np.uint32), d[f"sym{k}"].view(np.uint32)), Qm
        llr = O.demodulate(d[f"y{k}"], d[f"nv{k}"], Qm)
        assert np.array_equal(llr.view(np.uint32), d[f"llr{k}"].view(np.uint32)), Qm


MOD_IDS = {"bpsk": 1, "pi/2-bpsk": -1, "qpsk": 2, "16qam": 4, "64qam": 6, "256qam": 8, "1024qam": 10}


def _raw(a):
    a = np.asarray(a)
    return a.view(np.uint64 if a.dtype.itemsize == 8 else np.uint32)


def test_all_modulations_golden_oracle():
    """modulate / demodulate restatements == the reference's nrModulate / nrDemodulate for all
    seven modulations (tests/golden/demod2_golden.npz), with complex128 AND complex64 symbols
    (float64 vs float32 arithmetic), raw bits compared, output dtypes included."""
    d = np.load(os.path.join(GOLD, "demod2_golden.npz"))
    mods = d["mods"].tolist()
    for k, Qm, n in d["meta"].tolist():
        mod = MOD_IDS[mods[k]]
        bits = np.unpackbits(d[f"bits{k}"])[:n * Qm]
        assert np.array_equal(_raw(O.modulate(bits, mod)), _raw(d[f"sym{k}"])), mods[k]
        for key, y in ((f"llr{k}", d[f"y{k}"]), (f"llr_c64_{k}", d[f"y{k}"].astype(np.complex64))):
            llr = O.demodulate(y, d[f"nv{k}"], mod)
            ref = d[key]
            assert llr.dtype == ref.dtype and np.array_equal(_raw(llr), _raw(ref)), (mods[k], key)


def test_config1_golden_oracle():
    """BASELINE config 1 (BG2 Zc=8, CRC24A, NMS alpha=.75, L=8): the reference's own
    for_test_5g_ldpc_encoder + nr_decode_ldpc outputs (tests/golden/config1_golden.npz) are
    reproduced by the oracle's CRC, encoder and float64 flooding decoder."""
    d = np.load(f"{GOLD}/config1_golden.npz")
    blk, dn, llr = d["blk"], d["dn"], d["llr"]
    assert np.array_equal(O.encode(blk, 2), dn)
    for i in range(blk.shape[0]):
        assert np.array_equal(O.crc_encode(blk[i, :56], "24A"), blk[i])
    ck, st, _ = O.decode_flooding(llr, 8, 2, 8, 0.75, 0.0, np.float64)
    assert np.array_equal(st.astype(np.uint8), d["status"])
    assert np.array_equal(ck, d["ck"])
    assert 0 < d["status"].sum() < d["status"].size   # both outcomes covered


def test_bler_pins_complete():
    """Every LDPC BLER value the reference published is a pin (tests/golden/bler_pins.json)."""
    pins = load_json("bler_pins.json")["pins"]
    assert len(pins) == 272 + 24 + 35
    files = {p["file"] for p in pins}
    assert "out/ldpc_decode_result_opt.pickle" in files and "out/NMS_search_alpha_ZC384_bgn1.pickle" in files
    assert "out/ldpc_decode_result_BF.pickle" in files and "out/ldpc_decode_result_all.pickle" in files
    assert {p["algo"] for p in pins} == {"min-sum", "BP", "BF"}
    # fixed-count pins: BF 200 / 2000 codeblocks below / from 4 dB (sim_ldpc_decoder_bf.py:77-80)
    bf = [p for p in pins if p["file"].endswith("_BF.pickle")]
    assert all(p["n_ref"] == (200 if p["snr"] < 4 else 2000) for p in bf)
    assert all(abs(p["bler"] * p["n_ref"] - round(p["bler"] * p["n_ref"])) < 1e-6 for p in pins if "n_ref" in p)
    assert any(p["alpha"] < 1 and p["beta"] > 0 for p in pins)      # mixed min-sum
    opt = [p["bler"] for p in pins if p["file"].endswith("_opt.pickle") and p["label"] == "NMS-alpha=0.7-L=32"]
    assert opt == [0.395, 0.135, 0.015, 0.0005, 0.0]


def test_decode_sparse_golden():
    """decode_ldpc on arbitrary binary H: the dense restatement == the reference, bit for bit,
    for min-sum (incl. negative offsets), BP and BF, incl. the bit-flipping toy H KAT shape."""
    cases, _ = load_sparse_cases()
    assert len(cases) >= 380
    for k, c in enumerate(cases):
        ck, st, _ = O.decode_sparse(c["llr"].astype(np.float64), c["H"], c["L"], c["algo"],
                                    c["alpha"], c["beta"])
        assert np.array_equal(ck[0], c["ck"]) and bool(st[0]) == c["status"], (k, c["kind"], c["algo"])


def test_decode_sparse_degree_one_row_raises():
    """_min_sum_process on a row with one edge raises (np.sort(...)[1], nr_ldpc_decode.py:191-194)
    once a check-node update runs; a zero syndrome at the first check returns before it."""
    H = np.array([[1, 1, 0], [0, 0, 1]])
    with pytest.raises(IndexError):
        O.decode_sparse(np.array([1.0, -2.0, 3.0]), H, 4)
    ck, st, it = O.decode_sparse(np.array([1.0, 2.0, 3.0]), H, 4)
    assert st[0] and it[0] == 0


def test_decode_sparse_matches_flooding_on_38212_graph():
    """On a TS 38.212 expansion the dense restatement and the edge-list flooding oracle agree."""
    rng = np.random.default_rng(3)
    for bg, Zc in ((2, 3), (1, 2)):
        H = O.getH(Zc, bg)
        K = (22 if bg == 1 else 10) * Zc
        dn = O.encode(rng.integers(0, 2, K), bg)
        llr = O.bpsk_awgn_llr(dn, 0.5, rng)
        full = np.concatenate([np.zeros(2 * Zc), llr])
        a = O.decode_sparse(full, H, 6, "min-sum", 0.8, 0.1)
        b = O.decode_flooding(llr[None], Zc, bg, 6, 0.8, 0.1)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
