"""GPU parity tests of the DL-SCH / UL-SCH chain (ldpc5g_sch_*, ldpc5g_crc) against the
reference's golden vectors and the oracle.  Run on an MI355X with `pytest -m gpu`.

Bars (all exact):
  CRC ............... remainders == the reference's CRC KATs / generated vectors (6 polynomials)
                      and the oracle on long rows crossing chunk boundaries
  encode chain ...... g == reference DLSCHEncode / ULSCH encode (incl. a config-5 TB, C = 129)
  rate recovery ..... float64 output bit-identical to raterecover_ldpc (+ HARQ combining)
  decode chain ...... (crc_ok, tbblk, sha256(new_LLr_dns)) == reference DLSCHDecode / ULSCH_decoding
  batched / layered . batch of T TBs == per-TB results; layered float32 == oracle.decode_layered
"""
import hashlib

import numpy as np
import pytest

from conftest import GOLD, load_json
from oracle import ldpc_oracle as O

pytestmark = pytest.mark.gpu

DEC = {"L": 6, "algo": "min-sum", "alpha": 0.8, "beta": 0.0}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a ROCm GPU"
    return t


@pytest.fixture(scope="module")
def sch():
    from python_5gtoolbox_amd import sch as s
    return s


@pytest.fixture(scope="module")
def gold():
    return load_json("sch_golden.json"), np.load(f"{GOLD}/sch_golden.npz")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def _bits(z, key, n):
    return np.unpackbits(z[key])[:n].astype(np.int8)


# ---------------------------------------------------------------------------------------- CRC
def test_crc_rows_vs_reference_kats(torch, sch):
    for case in load_json("crc_golden.json"):
        blk = np.array(case["blk"], np.int8)
        out = np.array(case["out"], np.int8)
        L = out.size - blk.size
        x = torch.from_numpy(blk.reshape(1, -1)).cuda()
        rem = int(sch.crc_rows(x, case["poly"]).cpu()[0])
        mask = case["mask"] & ((1 << L) - 1)
        exp = int("".join(map(str, out[blk.size:].tolist())), 2)
        assert rem ^ mask == exp, case["poly"]
        # a row ending in its own (unmasked) CRC has remainder 0
        full = np.concatenate([blk, np.array([(rem >> (L - 1 - i)) & 1 for i in range(L)], np.int8)])
        assert int(sch.crc_rows(torch.from_numpy(full.reshape(1, -1)).cuda(), case["poly"]).cpu()[0]) == 0


@pytest.mark.parametrize("n", [1, 63, 64, 65, 16383, 16384, 16385, 40000, 100003])
def test_crc_rows_long_vs_oracle(torch, sch, n):
    rng = np.random.default_rng(n)
    bits = rng.integers(0, 2, (3, n)).astype(np.int8)
    x = torch.from_numpy(bits).cuda()
    for poly in ["24A", "24B", "16", "11", "6", "24C"]:
        got = sch.crc_rows(x, poly).cpu().numpy()
        p = O._POLY[poly]
        for r in range(3):
            assert int(got[r]) == O._crc_rem(bits[r].tolist(), p, len(p)), (n, poly, r)


# ------------------------------------------------------------------------------ encode chain
def test_dlsch_encode_dropin_vs_reference(torch):
    from python_5gtoolbox_amd import nr_dlsch
    d = np.load(f"{GOLD}/dlsch_golden.npz")
    for i, (TBS, Qm, R, NL, rv, LBRM, G) in enumerate(d["meta"].tolist()):
        tb = np.unpackbits(d["tb"][d["tb_off"][i]:d["tb_off"][i + 1]])[:TBS].astype(np.int8)
        g = np.unpackbits(d["g"][d["g_off"][i]:d["g_off"][i + 1]])[:G].astype(np.int8)
        out = nr_dlsch.DLSCHEncode(tb, TBS, Qm, R, NL, rv, LBRM, G)
        assert out.dtype == np.int8 and np.array_equal(out, g), i


def test_sch_golden_encode_chains(torch, gold):
    from python_5gtoolbox_amd import nr_dlsch, nr_ulsch
    cases, z = gold
    for n, cs in enumerate(cases):
        A, G = cs["TBS"], cs["G"]
        tb = _bits(z, f"trblk{n}", A)
        g = _bits(z, f"g{n}", G)
        if cs["kind"] == "ul":
            cbs, Zc, bgn = nr_ulsch.ULSCH_Crc_CodeBlockSegment(tb, A, cs["R"])
            C, K, nfill = z[f"cbsfill{n}"].tolist()
            assert cbs.shape == (C, K) and int(np.sum(cbs[0] == -1)) == nfill
            assert np.array_equal((cbs.reshape(-1) == 1), _bits(z, f"cbs{n}", C * K).astype(bool))
            out = nr_ulsch.ULSCH_encoding_ratematch(cbs, Zc, bgn, cs["Qm"], G, cs["NL"], cs["rv"])
            assert not np.any(cbs[:, 2 * Zc:] == -1)   # encode_ldpc's in-place filler zeroing
        else:
            out = nr_dlsch.DLSCHEncode(tb, A, cs["Qm"], cs["R"], cs["NL"], cs["rv"], cs["LBRM"], G)
        assert np.array_equal(out, g), (n, cs["kind"])


def test_sch_encode_batch_vs_oracle(torch, sch):
    rng = np.random.default_rng(7)
    for args in [(24000, 6, 658, 2, 1, 100000, 40008), (300, 2, 200, 1, 3, 0, 1000),
                 (60000, 8, 900, 4, 2, 60000, 64000)]:
        A, Qm, R, NL, rv, LBRM, G = args
        cfg = sch.sch_config(*args)
        T = 5
        tb = rng.integers(0, 2, (T, A)).astype(np.int8)
        g = sch.sch_encode_batch(torch.from_numpy(tb).cuda(), cfg).cpu().numpy()
        for t in range(T):
            assert np.array_equal(g[t], O.sch_encode(tb[t], *args)[:cfg.E_total]), (args, t)


def test_ratematch_gpu_vs_oracle(torch, sch):
    """Arbitrary (Ncb, k0, E, Qm, fillers) per codeblock: GPU rate matching == the oracle's
    ratematch (pinned to ratematch_ldpc by the CPU suite's golden checks)."""
    rng = np.random.default_rng(12)
    for trial in range(12):
        bg = 1 + trial % 2
        B = int(rng.integers(100, 3000))
        try:
            C, cbz, Lc, F, K, Zc = O.get_cbs_info(B, bg)
        except AssertionError:
            continue
        K_apo = K - F
        N = (66 if bg == 1 else 50) * Zc
        Ncb = N if trial % 3 else int(rng.integers(K, N + 1))
        Qm = [1, 2, 4, 6, 8][trial % 5]
        rv = trial % 4
        E = Qm * int(rng.integers(max(1, K // (2 * Qm)), int(1.8 * N) // Qm))
        cfg = sch.cfg_from_codeblocks(1, K, K_apo, Zc, bg, Qm, E, 1, rv, Ncb=Ncb)
        ck = rng.integers(0, 2, (1, K)).astype(np.int8)
        ck[:, K_apo:] = -1
        g = sch.sch_ratematch_batch(torch.from_numpy(ck).cuda(), cfg, 1).cpu().numpy()[0]
        dn = O.encode(ck[0], bg)
        assert np.array_equal(g, O.ratematch(dn, Ncb, E, cfg.k0, Qm)), trial


# ---------------------------------------------------------------------------- rate recovery
def test_raterecover_vs_reference_golden(torch, sch):
    d = np.load(f"{GOLD}/ratematch_golden.npz")
    for i, (bg, Zc, K, K_apo, N, Ncb, E, k0, Qm, rv) in enumerate(d["meta"].tolist()):
        llr = d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]].astype(np.float64)
        rr = d["rr"][d["rr_off"][i]:d["rr_off"][i + 1]]
        cfg = sch.cfg_from_codeblocks(1, K, K_apo, Zc, bg, Qm, E, 1, rv, Ncb=Ncb)
        assert cfg.k0 == k0
        x = torch.from_numpy(llr.reshape(1, -1)).cuda()
        out = sch.sch_raterecover_batch(x, cfg, dn_dtype=torch.float64).cpu().numpy()[0]
        assert np.array_equal(out, rr), i   # bit-exact float64
        out32 = sch.sch_raterecover_batch(x.float(), cfg, dn_dtype=torch.float32).cpu().numpy()[0]
        assert np.array_equal(out32, rr.astype(np.float32)), i   # float64 result rounded once


@pytest.mark.parametrize("args", [
    (2000, 2, 500, 1, 0, 60000, 60000),     # one codeblock, E = 60000 > Ncb: repetitions, no LDS stage
    (200, 2, 300, 1, 0, 60000, 3000),       # E > Ncb with the E LLRs staged in LDS (repetitions)
    (24000, 8, 900, 1, 2, 60000, 27000),    # E = 9000 per codeblock: f32 staged in LDS, f64 not
    (8000, 4, 700, 1, 3, 60000, 4000),      # small E: staged for both input dtypes
    (3000, 6, 300, 1, 1, 60000, 6000),      # Qm = 6 (de-interleave by 6)
    (8000, 4, 700, 1, 3, 60000, 26000),     # E / (Ncb - F) = 1.04: two visits, k-major passes
    (200, 2, 300, 1, 0, 60000, 2400),       # 1.80: two visits (float64 -> float32: staged gather)
    (200, 2, 300, 1, 0, 60000, 2672),       # exactly 2.0: every rank visited twice
    (3000, 6, 300, 1, 1, 60000, 24000),     # 1.52 with Qm = 6
])
def test_raterecover_stage_paths_vs_oracle(torch, sch, args):
    """raterecover_kernel's paths — k-major passes (at most two visits per position), LDS-staged
    gather (E * sizeof(llr) <= 40 KB), global-memory gather — float32 / float64 in and out,
    T = 3 TBs, HARQ combining: == oracle.sch_raterecover
    (float64 bit-exact; float32 output = the float64 result rounded once)."""
    rng = np.random.default_rng(args[0])
    cfg = sch.sch_config(*args)
    p = O.sch_params(*args)
    T = 3
    llr = rng.normal(0, 4, (T, args[6]))
    llr[:, ::7] = 0.0
    harq = rng.normal(0, 2, (T * cfg.C, cfg.N))
    harq[:, ::5] = 0.0
    assert O.sch_params(*args)["C"] == cfg.C
    for tin in (torch.float64, torch.float32):
        x = torch.from_numpy(llr).cuda().to(tin)
        xin = x.double().cpu().numpy()
        ref = np.concatenate([O.sch_raterecover(xin[t], p) for t in range(T)])
        refh = np.where((ref == 0) | (harq == 0), ref + harq, (ref + harq) / 2.0)
        for tout in (torch.float64, torch.float32):
            out = sch.sch_raterecover_batch(x, cfg, dn_dtype=tout).cpu().numpy()
            assert np.array_equal(out, ref.astype(out.dtype)), (tin, tout)
            h = torch.from_numpy(harq).cuda().to(tout)
            hv = h.double().cpu().numpy()   # the kernel combines in float64, rounds once
            exp = np.where((ref == 0) | (hv == 0), ref + hv, (ref + hv) / 2.0).astype(out.dtype)
            outh = sch.sch_raterecover_batch(x, cfg, harq_in=h, dn_dtype=tout).cpu().numpy()
            assert np.array_equal(outh, exp), (tin, tout, "harq")
            # in place: the HARQ input is the workspace's own output row (a previous llr_dn
            # passed back with a reused workspace)
            ws = sch.SchWorkspace(cfg, T, x.device)
            buf = ws.dn_buf(tout, cfg)
            buf.copy_(h)
            outi = sch.sch_raterecover_batch(x, cfg, harq_in=buf, dn_dtype=tout, ws=ws).cpu().numpy()
            assert np.array_equal(outi, exp), (tin, tout, "harq in place")


# ------------------------------------------------------------------------------ decode chain
def test_sch_golden_decode_dropins(torch, gold):
    from python_5gtoolbox_amd import nr_dlsch_decode, nr_ulsch_decode
    cases, z = gold
    for n, cs in enumerate(cases):
        if cs["kind"] == "dl-encode":
            continue
        A, G = cs["TBS"], cs["G"]
        llr = z[f"llr{n}"].astype(np.float64)
        if cs["kind"] == "dl":
            ok, tbblk, new = nr_dlsch_decode.DLSCHDecode(llr, A, cs["Qm"], cs["R"], cs["NL"],
                                                         cs["rv"], cs["LBRM"], DEC)
        else:
            ok, tbblk, new = nr_ulsch_decode.ULSCH_decoding(llr, A, cs["R"], cs["Qm"], G, cs["NL"],
                                                            cs["rv"], DEC)
        assert ok == cs["ok"] and isinstance(ok, bool), n
        assert tbblk.dtype == np.int8 and np.array_equal(tbblk, _bits(z, f"tbblk{n}", A)), n
        assert list(new.shape) == cs["new_shape"] and _sha(new) == cs["new_sha"], n
        if cs["kind"] == "dl":   # HARQ: rv 2 retransmission combined with the first input
            llr2 = z[f"llr2_{n}"].astype(np.float64)
            ok2, tb2, new2 = nr_dlsch_decode.DLSCHDecode(llr2, A, cs["Qm"], cs["R"], cs["NL"], 2,
                                                         cs["LBRM"], DEC, True, new)
            assert ok2 == cs["ok2"] and _sha(new2) == cs["new2_sha"], n
            assert np.array_equal(tb2, _bits(z, f"tbblk2_{n}", A)), n


def test_sch_golden_decode_negative_beta(torch):
    """DLSCHDecode / ULSCH_decoding with beta < 0 (the reference's per-codeblock nr_decode_ldpc
    keeps min-sum's zero branches): reference goldens, CRC flag, TB bits, sha256 of new_LLr_dns."""
    from python_5gtoolbox_amd import nr_dlsch_decode, nr_ulsch_decode
    cases, z = load_json("sch_negbeta_golden.json"), np.load(f"{GOLD}/sch_negbeta_golden.npz")
    for n, cs in enumerate(cases):
        A, G, dec = cs["TBS"], cs["G"], cs["dec"]
        assert dec["beta"] < 0
        llr = z[f"llr{n}"].astype(np.float64)
        if cs["kind"] == "dl":
            ok, tbblk, new = nr_dlsch_decode.DLSCHDecode(llr, A, cs["Qm"], cs["R"], cs["NL"],
                                                         cs["rv"], cs["LBRM"], dec)
        else:
            ok, tbblk, new = nr_ulsch_decode.ULSCH_decoding(llr, A, cs["R"], cs["Qm"], G, cs["NL"],
                                                            cs["rv"], dec)
        assert ok == cs["ok"] and isinstance(ok, bool), n
        assert np.array_equal(tbblk, _bits(z, f"tbblk{n}", A)), n
        assert list(new.shape) == cs["new_shape"] and _sha(new) == cs["new_sha"], n


def test_sch_decode_batch_matches_per_tb_and_oracle(torch, sch):
    """T transport blocks in one call: float64 flooding == the oracle chain per TB; layered
    float32 == oracle.decode_layered on the float32-rounded rate-recovered LLRs."""
    rng = np.random.default_rng(31)
    args = (24000, 4, 700, 1, 0, 60000, 30000)
    A, Qm, R, NL, rv, LBRM, G = args
    cfg = sch.sch_config(*args)
    p = O.sch_params(*args)
    T = 6
    tb = rng.integers(0, 2, (T, A)).astype(np.int8)
    g = sch.sch_encode_batch(torch.from_numpy(tb).cuda(), cfg).cpu().numpy()
    snrs = [9.0, 9.0, 3.0, 1.0, 0.0, -2.0]
    llr = np.stack([O.bpsk_awgn_llr(g[t], snrs[t], rng) for t in range(T)])
    x = torch.from_numpy(llr).cuda()
    r = sch.sch_decode_batch(x, cfg, 5, "min-sum", 0.75, 0.0, "flooding")
    tb_ok = r.tb_ok.cpu().numpy().astype(bool)
    tbblk = r.tbblk.cpu().numpy()
    dn = r.llr_dn.cpu().numpy()
    for t in range(T):
        ref_dn = O.sch_raterecover(llr[t], p)
        assert np.array_equal(dn[t * cfg.C:(t + 1) * cfg.C], ref_dn), t
        ck, _, _ = O.decode_flooding(ref_dn, p["Zc"], p["bgn"], 5, 0.75, 0.0, np.float64)
        ok, blk, cbok = O.sch_tb_check(ck, p)
        assert tb_ok[t] == ok and np.array_equal(tbblk[t, :A], blk), t
        assert np.array_equal(r.cb_crc_ok.cpu().numpy()[t * cfg.C:(t + 1) * cfg.C].astype(bool), cbok)
    assert tb_ok[:2].all() and not tb_ok[-1]   # 9 dB decodes, -2 dB does not
    # layered float32
    r2 = sch.sch_decode_batch(x.float(), cfg, 5, "min-sum", 0.75, 0.0, "layered")
    dn32 = r2.llr_dn.cpu().numpy()
    assert dn32.dtype == np.float32
    ck, st, it = O.decode_layered(dn32, cfg.Zc, cfg.bgn, 5, 0.75, 0.0)
    assert np.array_equal(r2.ck.cpu().numpy(), ck)
    for t in range(T):
        ok, blk, _ = O.sch_tb_check(ck[t * cfg.C:(t + 1) * cfg.C], p)
        assert bool(r2.tb_ok.cpu().numpy()[t]) == ok


def test_config5_tb_stream_round_trip(torch, sch, gold):
    """Config 5 at full size: 129-codeblock TBs (273 PRB, 256QAM, 4 layers): the reference TB
    encodes bit-exactly; a stream of 8 TBs encoded on the GPU decodes back noiselessly with every
    CB and TB CRC passing (layered float32)."""
    cases, z = gold
    n = [i for i, c in enumerate(cases) if c["kind"] == "dl-encode"][0]
    cs = cases[n]
    args = (cs["TBS"], cs["Qm"], cs["R"], cs["NL"], cs["rv"], cs["LBRM"], cs["G"])
    cfg = sch.sch_config(*args)
    assert cfg.C == 129 and cfg.Zc == 384
    tb0 = _bits(z, f"trblk{n}", cs["TBS"])
    T = 8
    rng = np.random.default_rng(5)
    tb = np.concatenate([tb0[None], rng.integers(0, 2, (T - 1, cs["TBS"])).astype(np.int8)])
    xt = torch.from_numpy(tb).cuda()
    g = sch.sch_encode_batch(xt, cfg)
    assert np.array_equal(g[0].cpu().numpy(), _bits(z, f"g{n}", cs["G"]))
    llr = (1.0 - 2.0 * g.float()) * 4.0
    r = sch.sch_decode_batch(llr.contiguous(), cfg, 8, "min-sum", 0.75, 0.0, "layered")
    assert r.tb_ok.cpu().numpy().all() and r.cb_crc_ok.cpu().numpy().all()
    assert torch.equal(r.tbblk[:, :cs["TBS"]], xt)


# ------------------------------------------------------------ per-TB configurations (multi)
def _cfg_of(sch, cs, rv=None):
    lbrm = cs["LBRM"] if cs["kind"] != "ul" else 0
    return sch.sch_config(cs["TBS"], cs["Qm"], cs["R"], cs["NL"], cs["rv"] if rv is None else rv,
                          lbrm, cs["G"])


def test_sch_multi_encode_golden(torch, sch, gold):
    """Five transport blocks with five different configurations (DL with limited buffer, UL with
    Ncb = N, QPSK..256QAM, 1..4 layers, the config-5 TB of 129 codeblocks) in ONE
    ldpc5g_sch_encode_multi call == the reference's DLSCHEncode / ULSCH encode per TB."""
    cases, z = gold
    idx = [0, 2, 3, 4, 5]
    cfgs = [_cfg_of(sch, cases[n]) for n in idx]
    Amax = max(cases[n]["TBS"] for n in idx)
    tb = np.zeros((len(idx), Amax), np.int8)
    for t, n in enumerate(idx):
        tb[t, :cases[n]["TBS"]] = _bits(z, f"trblk{n}", cases[n]["TBS"])
    g = sch.sch_encode_multi(torch.from_numpy(tb).cuda(), cfgs).cpu().numpy()
    for t, n in enumerate(idx):
        assert cfgs[t].E_total == cases[n]["G"]
        assert np.array_equal(g[t, :cfgs[t].E_total], _bits(z, f"g{n}", cases[n]["G"])), n


def test_sch_multi_decode_golden(torch, sch, gold):
    """Four transport blocks with different configurations (two DL, two UL; different Zc and
    base graphs) in ONE ldpc5g_sch_decode_multi call, float64 flooding = the reference's
    DLSCHDecode / ULSCH_decoding per TB: crc_ok, TB bits and the HARQ buffer new_LLr_dns (sha256)
    bit-exact; then the two DL TBs retransmitted (rv 2) with HARQ combining in one call."""
    cases, z = gold
    idx = [0, 2, 3, 4]
    cfgs = [_cfg_of(sch, cases[n]) for n in idx]
    Emax = max(c.E_total for c in cfgs)
    llr = np.zeros((len(idx), Emax), np.float64)
    for t, n in enumerate(idx):
        llr[t, :cfgs[t].E_total] = z[f"llr{n}"].astype(np.float64)
    r = sch.sch_decode_multi(torch.from_numpy(llr).cuda(), cfgs, DEC["L"], DEC["alpha"],
                             DEC["beta"], "flooding")
    ok, tbblk, dn = r.tb_ok.cpu().numpy(), r.tbblk.cpu().numpy(), r.llr_dn.cpu().numpy()
    assert len({(c.bgn, c.Zc) for c in cfgs}) > 1
    for t, n in enumerate(idx):
        cs = cases[n]
        assert bool(ok[t]) == cs["ok"], n
        assert np.array_equal(tbblk[t, :cs["TBS"]], _bits(z, f"tbblk{n}", cs["TBS"])), n
        cb0, C, off, N, _, _ = r.rows[t]
        new = dn[off:off + C * N].reshape(C, N)
        assert list(new.shape) == cs["new_shape"] and _sha(new) == cs["new_sha"], n
    # HARQ retransmission of the DL TBs: rv 2, combined with their first-pass buffers
    dl = [0, 1]
    cfg1 = [cfgs[t] for t in dl]
    r1 = sch.sch_decode_multi(torch.from_numpy(llr[dl]).cuda(), cfg1, DEC["L"], DEC["alpha"],
                              DEC["beta"], "flooding")
    cfg2 = [_cfg_of(sch, cases[idx[t]], rv=2) for t in dl]
    E2 = max(c.E_total for c in cfg2)
    llr2 = np.zeros((len(dl), E2), np.float64)
    for k, t in enumerate(dl):
        llr2[k, :cfg2[k].E_total] = z[f"llr2_{idx[t]}"].astype(np.float64)
    r2 = sch.sch_decode_multi(torch.from_numpy(llr2).cuda(), cfg2, DEC["L"], DEC["alpha"],
                              DEC["beta"], "flooding", harq_in=r1.llr_dn)
    ok2, tb2, dn2 = r2.tb_ok.cpu().numpy(), r2.tbblk.cpu().numpy(), r2.llr_dn.cpu().numpy()
    for k, t in enumerate(dl):
        cs = cases[idx[t]]
        assert bool(ok2[k]) == cs["ok2"], idx[t]
        assert np.array_equal(tb2[k, :cs["TBS"]], _bits(z, f"tbblk2_{idx[t]}", cs["TBS"])), idx[t]
        cb0, C, off, N, _, _ = r2.rows[k]
        assert _sha(dn2[off:off + C * N].reshape(C, N)) == cs["new2_sha"], idx[t]


def test_sch_multi_layered_matches_single_config_batches(torch, sch):
    """Layered float32 through the multi chain == the single-configuration chain run per
    configuration (same codeblocks, same kernels' arithmetic): tb_ok, TB bits, iterations."""
    rng = np.random.default_rng(9)
    specs = [(24000, 4, 700, 1, 0, 60000, 30000), (3000, 2, 300, 1, 1, 10000, 9000),
             (60000, 8, 900, 2, 2, 60000, 64000)]
    cfgs = [sch.sch_config(*a) for a in specs]
    T = len(cfgs)
    Emax = max(c.E_total for c in cfgs)
    llr = np.zeros((T, Emax), np.float32)
    for t, (a, c) in enumerate(zip(specs, cfgs)):
        tb = rng.integers(0, 2, (1, a[0])).astype(np.int8)
        g = sch.sch_encode_batch(torch.from_numpy(tb).cuda(), c).cpu().numpy()[0]
        llr[t, :c.E_total] = (1 - 2 * g.astype(np.float32)) * 4 + rng.normal(0, 1.2, c.E_total)
    r = sch.sch_decode_multi(torch.from_numpy(llr).cuda(), cfgs, 8, 0.75, 0.0, "layered")
    for t, c in enumerate(cfgs):
        one = sch.sch_decode_batch(torch.from_numpy(llr[t:t + 1, :c.E_total].copy()).cuda(), c, 8,
                                   "min-sum", 0.75, 0.0, "layered")
        assert int(r.tb_ok[t]) == int(one.tb_ok[0])
        assert torch.equal(r.tbblk[t, :c.B], one.tbblk[0, :c.B])
        cb0, C, _, _, _, _ = r.rows[t]
        assert torch.equal(r.iters[cb0:cb0 + C], one.iters[:C])


def _random_sch_cases(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        A = int(rng.integers(24, 30000))
        Qm = int(rng.choice([1, 2, 4, 6, 8]))
        NL = int(rng.integers(1, 5))
        R = float(rng.choice([rng.integers(30, 950), rng.uniform(30, 950)]))
        rv = int(rng.integers(0, 4))
        LBRM = int(rng.choice([0, A, int(A * rng.uniform(1, 4))]))
        G = NL * Qm * int(rng.integers(max(1, A // (NL * Qm * 2)), 3 * A // (NL * Qm) + 10))
        try:
            O.sch_params(A, Qm, R, NL, rv, LBRM, G)
        except AssertionError:
            continue
        out.append((A, Qm, R, NL, rv, LBRM, G))
    return out


@pytest.mark.parametrize("args", _random_sch_cases(20, seed=41))
def test_sch_random_configs_chain_vs_oracle(torch, sch, args):
    """Random transport-block configurations (both base graphs, fillers, limited-buffer rate
    matching, every rv, Qm 1..8, 1-4 layers, fractional and integer R): the GPU encode chain ==
    oracle.sch_encode, and the GPU decode chain (float64 flooding, the reference-exact mode) ==
    the oracle chain — rate-recovered LLRs, hard decisions, CB CRCs, TB CRC and TB bits — for two
    TBs at different SNRs."""
    A, Qm, R, NL, rv, LBRM, G = args
    rng = np.random.default_rng(A)
    cfg = sch.sch_config(*args)
    p = O.sch_params(*args)
    T = 2
    tb = rng.integers(0, 2, (T, A)).astype(np.int8)
    g = sch.sch_encode_batch(torch.from_numpy(tb).cuda(), cfg).cpu().numpy()
    for t in range(T):
        assert np.array_equal(g[t], O.sch_encode(tb[t], *args)[:cfg.E_total]), t
    snrs = [float(rng.uniform(2.0, 6.0)), float(rng.uniform(-2.0, 1.0))]
    llr = np.stack([O.bpsk_awgn_llr(g[t], snrs[t], rng) for t in range(T)])
    r = sch.sch_decode_batch(torch.from_numpy(llr).cuda(), cfg, 4, "min-sum", 0.75, 0.0, "flooding")
    dn, ck = r.llr_dn.cpu().numpy(), r.ck.cpu().numpy()
    tb_ok, tbblk = r.tb_ok.cpu().numpy().astype(bool), r.tbblk.cpu().numpy()
    cb_ok = r.cb_crc_ok.cpu().numpy().astype(bool)
    C = cfg.C
    for t in range(T):
        ref_dn = O.sch_raterecover(llr[t], p)
        assert np.array_equal(dn[t * C:(t + 1) * C], ref_dn), t
        rck, _, _ = O.decode_flooding(ref_dn, p["Zc"], p["bgn"], 4, 0.75, 0.0, np.float64)
        assert np.array_equal(ck[t * C:(t + 1) * C], rck), t
        ok, blk, cbok = O.sch_tb_check(rck, p)
        assert tb_ok[t] == ok and np.array_equal(tbblk[t, :A], blk), t
        assert np.array_equal(cb_ok[t * C:(t + 1) * C], cbok), t


@pytest.mark.parametrize("seed", [43, 44, 45])
def test_sch_multi_random_configs_vs_oracle(torch, sch, seed):
    """Eight random per-TB configurations in ONE ldpc5g_sch_encode_multi and ONE
    ldpc5g_sch_decode_multi call (float64 flooding): every TB's rate-matched bits, rate-recovered
    LLRs, hard decisions, TB CRC flag and TB bits == the oracle chain run on that TB alone."""
    rng = np.random.default_rng(seed)
    specs = _random_sch_cases(8, seed)
    cfgs = [sch.sch_config(*a) for a in specs]
    T = len(specs)
    Amax = max(a[0] for a in specs)
    tb = np.zeros((T, Amax), np.int8)
    for t, a in enumerate(specs):
        tb[t, :a[0]] = rng.integers(0, 2, a[0])
    g = sch.sch_encode_multi(torch.from_numpy(tb).cuda(), cfgs).cpu().numpy()
    Emax = max(c.E_total for c in cfgs)
    llr = np.zeros((T, Emax), np.float64)
    for t, a in enumerate(specs):
        E = cfgs[t].E_total
        assert np.array_equal(g[t, :E], O.sch_encode(tb[t, :a[0]], *a)[:E]), t
        llr[t, :E] = O.bpsk_awgn_llr(g[t, :E], float(rng.uniform(-1.0, 6.0)), rng)
    r = sch.sch_decode_multi(torch.from_numpy(llr).cuda(), cfgs, 4, 0.75, 0.0, "flooding")
    ok, tbblk = r.tb_ok.cpu().numpy().astype(bool), r.tbblk.cpu().numpy()
    dn, ck = r.llr_dn.cpu().numpy(), r.ck.cpu().numpy()
    for t, a in enumerate(specs):
        p = O.sch_params(*a)
        cb0, C, off, N, dck, nf = r.rows[t]
        ref_dn = O.sch_raterecover(llr[t, :cfgs[t].E_total], p)
        assert np.array_equal(dn[off:off + C * N].reshape(C, N), ref_dn), t
        rck, _, _ = O.decode_flooding(ref_dn, p["Zc"], p["bgn"], 4, 0.75, 0.0, np.float64)
        assert np.array_equal(ck[dck:dck + C * nf].reshape(C, nf), rck), t
        rok, blk, _ = O.sch_tb_check(rck, p)
        assert ok[t] == rok and np.array_equal(tbblk[t, :a[0]], blk), t


@pytest.mark.parametrize("dt", ["float64", "float32"])
def test_sch_raterecover_multi_matches_per_config(torch, sch, dt):
    """ldpc5g_sch_raterecover_multi (every TB's rate recovery in ONE launch, per-TB geometry:
    the config-4 receive step) == the single-configuration rate recovery run per TB, bit for bit,
    including a HARQ-combined second call; float64 and float32 outputs.  (The single-config
    kernel is itself bit-exact vs the reference's raterecover_ldpc goldens.)"""
    rng = np.random.default_rng(17)
    specs = [(24000, 4, 700, 1, 0, 60000, 30000), (3000, 2, 300, 1, 1, 10000, 9000),
             (60000, 8, 900, 2, 2, 60000, 64000), (500, 6, 120, 1, 3, 0, 4200)]
    cfgs = [sch.sch_config(*a) for a in specs]
    # config-4 style codeblock groups too (ULSCH_encoding_ratematch geometry, no TB CRC use)
    for Zc, bg, Qm, rv in ((12, 2, 4, 1), (384, 1, 8, 3), (40, 1, 2, 0)):
        K = (22 if bg == 1 else 10) * Zc
        N = (66 if bg == 1 else 50) * Zc
        E = Qm * int(rng.integers(-(-K // Qm), int(1.6 * N) // Qm + 1))
        cfgs.append(sch.cfg_from_codeblocks(7, K, K, Zc, bg, Qm, 7 * E, 1, rv))
    T = len(cfgs)
    lay = sch.multi_layout(cfgs)
    tdt = getattr(torch, dt)
    llr = torch.zeros((T, lay["max_E"]), dtype=tdt, device="cuda")
    for t, c in enumerate(cfgs):
        llr[t, :c.E_total] = torch.from_numpy(rng.normal(0, 3, c.E_total)).to(tdt)
    flat = sch.sch_raterecover_multi(llr, cfgs, lay=lay)
    flat2 = sch.sch_raterecover_multi(llr, cfgs, harq_in=flat, lay=lay)
    plan = sch.SchRaterecoverPlan(cfgs, llr.device)   # the reusable-plan form: same bytes
    viaplan = torch.full_like(flat, float("nan"))
    assert torch.equal(plan(llr, viaplan), flat)
    for t, c in enumerate(cfgs):
        x = llr[t:t + 1, :c.E_total].contiguous()
        one = sch.sch_raterecover_batch(x, c).clone()
        _, C, off, N, _, _ = lay["rows"][t]
        assert torch.equal(flat[off:off + C * N].view(C, N), one), t
        two = sch.sch_raterecover_batch(x, c, harq_in=one.contiguous())
        assert torch.equal(flat2[off:off + C * N].view(C, N), two), t
