"""CPU tests of the product's host side: the C-ABI library loads and exports every declared
symbol, argument validation maps to the reference's AssertionError, and the host-side
reference mirrors (ldpc_info, crc, segmentation, rate matching) match the golden vectors.
No kernel is launched here (no GPU in the build container)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import GOLD, ROOT, load_json
from oracle import ldpc_oracle as O
from python_5gtoolbox_amd import _lib, crc, ldpc_info, nr_ldpc_cbsegment
from python_5gtoolbox_amd import nr_ldpc_ratematch as RM
from python_5gtoolbox_amd import nr_ldpc_raterecover as RR

HEADER = os.path.join(ROOT, "include", "ldpc5g.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc5g_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    names = declared_functions()
    assert set(names) == set(_lib.SIGNATURES), names
    for n in names:
        assert hasattr(lib, n), n
    assert lib.ldpc5g_version().startswith(b"ldpc5g")


def test_header_constants_match_binding():
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define (LDPC5G_\w+) \(?(-?\d+)\)?", src))
    assert int(consts["LDPC5G_F64"]) == _lib.F64 and int(consts["LDPC5G_F32"]) == _lib.F32
    assert int(consts["LDPC5G_FLOODING"]) == _lib.FLOODING
    assert int(consts["LDPC5G_LAYERED"]) == _lib.LAYERED
    assert int(consts["LDPC5G_LLR_FULL"]) == _lib.LLR_FULL
    assert int(consts["LDPC5G_RATE_MATCHED"]) == _lib.RATE_MATCHED
    assert (int(consts["LDPC5G_ALGO_MS"]), int(consts["LDPC5G_ALGO_BP"]),
            int(consts["LDPC5G_ALGO_BF"])) == (_lib.ALGO_MS, _lib.ALGO_BP, _lib.ALGO_BF)
    assert int(consts["LDPC5G_EBGN"]) == _lib.EBGN and int(consts["LDPC5G_EZC"]) == _lib.EZC
    assert ctypes.sizeof(_lib.CbDesc) == 24


def test_find_ils_abi_matches_reference_table():
    lib = _lib.lib()
    for z in range(1, 400):
        assert lib.ldpc5g_find_ils(z) == ldpc_info.find_iLS(z) == O.find_iLS(z)


@pytest.mark.parametrize("call,code", [
    (lambda l: l.ldpc5g_encode(None, None, 1, 3, 384, 8448, 25344, None), _lib.EBGN),
    (lambda l: l.ldpc5g_encode(None, None, 1, 1, 383, 8448, 25344, None), _lib.EZC),
    (lambda l: l.ldpc5g_encode(None, None, 1, 1, 384, 8000, 25344, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_ms(None, 0, None, None, None, 1, 1, 384, 8, 1.0, 0.0, 0, 0,
                                  25344, 26112, None), _lib.ESIZE),   # null buffers
    (lambda l: l.ldpc5g_decode_ms(None, 0, None, None, None, 1, 1, 384, 8, 1.0, 0.0, 1, 0,
                                  25344, 26112, None), _lib.ESIZE),   # layered needs F32
    (lambda l: l.ldpc5g_decode_ms(None, 1, None, None, None, 1, 2, 10, 8, 1.0, 0.0, 0, 0,
                                  499, 520, None), _lib.ESIZE),       # ldl < N
    (lambda l: l.ldpc5g_decode_ms(None, 1, None, None, None, 4, 2, 1, 8, 1.0, 0.0, 0, 0,
                                  500, 520, None), _lib.EZC),
    (lambda l: l.ldpc5g_encode(None, None, 0, 1, 384, 8448, 25344, None), 0),   # empty batch
    # sparse H: bad algo, N < 1, ldl < N, null buffers, scratch too small, empty batch
    (lambda l: l.ldpc5g_decode_sparse(None, 6, 1, 4, 6, 12, None, None, None, None, None, 8, 3,
                                      1.0, 0.0, None, 6, None, None, None, 0, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_sparse(None, 6, 1, 4, 0, 12, None, None, None, None, None, 8, 0,
                                      1.0, 0.0, None, 6, None, None, None, 0, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_sparse(None, 5, 2, 4, 6, 12, None, None, None, None, None, 8, 0,
                                      1.0, 0.0, None, 6, None, None, None, 0, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_sparse(None, 6, 1, 4, 6, 12, None, None, None, None, None, 8, 2,
                                      1.0, 0.0, None, 6, None, None, None, 0, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_sparse(None, 30000, 4, 15000, 30000, 90000, None, None, None, None,
                                      None, 8, 0, 1.0, 0.0, None, 30000, None, None, None, 100,
                                      None), _lib.ESIZE),
    (lambda l: l.ldpc5g_decode_sparse(None, 6, 0, 4, 6, 12, None, None, None, None, None, 8, 1,
                                      1.0, 0.0, None, 6, None, None, None, 0, None), 0),
])
def test_abi_validation_without_gpu(call, code):
    """Argument checks run before any HIP call and return the documented codes."""
    lib = _lib.lib()
    assert call(lib) == code
    if code:
        assert lib.ldpc5g_last_error()
        with pytest.raises(AssertionError):
            _lib.check(code)


def test_mixed_abi_validation_without_gpu():
    lib = _lib.lib()
    d = (_lib.CbDesc * 2)()
    d[0].bgn, d[0].Zc = 1, 384
    d[1].bgn, d[1].Zc = 3, 384
    dummy = ctypes.c_void_p(16)
    rc = lib.ldpc5g_decode_ms_mixed(d, 2, dummy, 1, dummy, dummy, dummy, 8, 1.0, 0.0, 0, 0, None)
    assert rc == _lib.EBGN
    d[1].bgn, d[1].Zc = 2, 7
    d[0].Zc = 385
    assert lib.ldpc5g_decode_ms_mixed(d, 2, dummy, 1, dummy, dummy, dummy, 8, 1.0, 0.0, 0, 0,
                                      None) == _lib.EZC


def test_ldpc_info_mirror():
    for B in [100, 292, 3824, 8424, 8448, 8449, 20000, 1081536]:
        for bg in (1, 2):
            try:
                ref = O.get_cbs_info(B, bg)
            except AssertionError:
                with pytest.raises(AssertionError):
                    ldpc_info.get_cbs_info(B, bg)
                continue
            assert ldpc_info.get_cbs_info(B, bg) == ref
    for bg, Zc in [(1, 2), (2, 3), (1, 13), (2, 15)]:
        H = ldpc_info.getH(Zc, bg, ldpc_info.find_iLS(Zc))
        assert np.array_equal(H, O.getH(Zc, bg))
        assert ldpc_info.match_H(H) == (bg, Zc)
        H2 = H.copy()
        H2[0, 0] ^= 1
        assert ldpc_info.match_H(H2) is None


def test_crc_mirror_golden():
    for c in load_json("crc_golden.json"):
        out = crc.nr_crc_encode(np.array(c["blk"]), c["poly"], c["mask"])
        assert out.tolist() == c["out"]
        blk, err = crc.nr_crc_decode(out, c["poly"], c["mask"])
        assert err == 0 and blk.tolist() == c["blk"]
        bad = out.copy()
        bad[len(bad) // 2] ^= 1
        assert crc.nr_crc_decode(bad, c["poly"], c["mask"])[1] == 1


def test_crc_inline_kats():
    """Known answers held inline by the reference (py5gphy/crc/crc.py:167-210)."""
    kats = [("6", [1, 1, 1, 1], 0, [1, 1, 1, 1, 0, 0, 1, 0, 1, 0]),
            ("6", [1, 0, 1, 1, 0, 1, 1, 0, 1], 45678, [1, 0, 1, 1, 0, 1, 1, 0, 1, 0, 1, 1, 1, 0, 0]),
            ("11", [1, 0, 1, 1], 12345, [1, 0, 1, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 1, 0]),
            ("24A", [0, 0, 1, 1, 0, 0, 0, 1], 45678,
             [0, 0, 1, 1, 0, 0, 0, 1, 0, 1, 0, 0, 1, 1, 1, 1, 0, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 1, 0, 1, 0, 1]),
            ("24B", [0, 0, 1, 1, 0, 0, 0, 1], 0,
             [0, 0, 1, 1, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1]),
            ("24C", [0, 0, 1, 1, 0, 0, 0, 1], 45678,
             [0, 0, 1, 1, 0, 0, 0, 1, 0, 0, 1, 0, 1, 1, 1, 0, 1, 1, 1, 0, 0, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 1])]
    for poly, blk, mask, exp in kats:
        assert crc.nr_crc_encode(np.array(blk), poly, mask).tolist() == exp
        assert O.crc_encode(np.array(blk), poly, mask).tolist() == exp


def test_ratematch_mirror_golden():
    d = np.load(os.path.join(GOLD, "ratematch_golden.npz"))
    for i, (bg, Zc, K, K_apo, N, Ncb, E, k0, Qm, rv) in enumerate(d["meta"].tolist()):
        dn = d["dn"][d["dn_off"][i]:d["dn_off"][i + 1]]
        assert RM.get_k0(Ncb, bg, rv, Zc) == k0
        assert np.array_equal(RM.ratematch_ldpc(dn, Ncb, E, k0, Qm),
                              d["fe"][d["fe_off"][i]:d["fe_off"][i + 1]])
        llr = d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]].astype(np.float64)
        assert np.array_equal(RR.raterecover_ldpc(llr, Ncb, N, k0, Qm, Zc, K_apo, K),
                              d["rr"][d["rr_off"][i]:d["rr_off"][i + 1]])
    for c in load_json("er_golden.json"):
        assert RM.get_Er_ldpc(c["G"], c["C"], c["Qm"], c["NL"]) == c["Er"]


def test_cbsegment_mirror():
    rng = np.random.default_rng(1)
    for B, bg in [(3000, 2), (30000, 1), (8448, 1), (500, 2)]:
        x = rng.integers(0, 2, B)
        a, za = nr_ldpc_cbsegment.ldpc_cbsegment(x, bg)
        b, zb = O.cbsegment(x, bg)
        assert za == zb and np.array_equal(a, b)


def test_product_fails_loudly_without_gpu():
    """No CPU fallback: the GPU entry points raise when no GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from python_5gtoolbox_amd import nr_ldpc_decode, nr_ldpc_encode
    with pytest.raises(_lib.LdpcLibError):
        nr_ldpc_encode.encode_ldpc(np.zeros(80, np.int8), 2)
    with pytest.raises(_lib.LdpcLibError):
        nr_ldpc_decode.nr_decode_ldpc(np.zeros(400), 8, 2, 8)


def test_mixed_plan_built_on_host():
    """ldpc5g_mixed_plan is pure host code: sizing call, then the plan (32-byte header: schedule,
    BG1 / BG2 workgroups, codeblock refs, the full Zc = 384 workgroups of each base graph) for 5
    BG1 Zc=384 + 3 BG2 Zc=12 codeblocks, layered (G = 2 and 64 per workgroup) and flooding (G = 1
    and 32); a work item's refs sorted by LLR offset (the kernels' 32-bit lane offsets start at its
    first codeblock)."""
    lib = _lib.lib()
    d = (_lib.CbDesc * 8)()
    for k in range(8):
        d[k].bgn, d[k].Zc = (1, 384) if k < 5 else (2, 12)
        d[k].llr_off, d[k].ck_off = 1000 * (7 - k), 2000 * k   # descending offsets
    for sched, nw1, nw2, nz1 in ((_lib.LAYERED, 3, 1, 2), (_lib.FLOODING, 5, 1, 5)):
        n = lib.ldpc5g_mixed_plan(d, 8, sched, None, 0)
        assert n == 32 + 16 * (nw1 + nw2) + 24 * 8
        buf = (ctypes.c_ubyte * n)()
        assert lib.ldpc5g_mixed_plan(d, 8, sched, buf, n) == n
        hdr = np.frombuffer(bytes(buf)[:32], np.int32)
        assert hdr[1] == sched and hdr[2] == nw1 and hdr[3] == nw2 and hdr[4] == 8
        # the BG1 Zc=384 items: a partial workgroup first, then the nz1 full ones (the Zc = 384
        # kernels' share, launched last); no BG2 Zc=384 items here
        assert hdr[5] == nz1 and hdr[6] == 0
        work = np.frombuffer(bytes(buf)[32:32 + 16 * nw1], np.int32).reshape(nw1, 4)
        assert list(work[:, 2]) == ([1, 2, 2] if sched == _lib.LAYERED else [1] * 5)
        refs = np.frombuffer(bytes(buf)[32 + 16 * (nw1 + nw2):], np.int64).reshape(8, 3)
        works = np.frombuffer(bytes(buf)[32:32 + 16 * (nw1 + nw2)], np.int32).reshape(-1, 4)
        for first, g in zip(works[:, 3], works[:, 2]):
            offs = refs[first:first + g, 0]
            assert list(offs) == sorted(offs)
        assert sorted(refs[:, 2] & 0xffffffff) == list(range(8))   # every codeblock once (out index)
    # BG2 Zc=384 codeblocks are counted for the frame kernel too
    d2 = (_lib.CbDesc * 2)()
    for k in range(2):
        d2[k].bgn, d2[k].Zc, d2[k].llr_off, d2[k].ck_off = 2, 384, 20000 * k, 20000 * k
    n = lib.ldpc5g_mixed_plan(d2, 2, _lib.FLOODING, None, 0)
    buf = (ctypes.c_ubyte * n)()
    assert lib.ldpc5g_mixed_plan(d2, 2, _lib.FLOODING, buf, n) == n
    assert np.frombuffer(bytes(buf)[:32], np.int32)[6] == 2
    # rows of one work item more than 4 GiB apart: refused
    d2[1].bgn, d2[1].Zc = 1, 12
    d2[0].bgn, d2[0].Zc = 1, 12
    d2[1].llr_off = 1 << 30
    assert lib.ldpc5g_mixed_plan(d2, 2, _lib.LAYERED, None, 0) == _lib.ESIZE
    d[3].Zc = 383
    assert lib.ldpc5g_mixed_plan(d, 8, _lib.LAYERED, None, 0) == _lib.EZC
    assert lib.ldpc5g_decode_ms_mixed_plan(None, None, None, 1, None, None, None, 8, 1.0, 0.0,
                                           _lib.LAYERED, 0, None) == _lib.ESIZE


def test_sch_multi_plan_rows_largest_first():
    """ldpc5g_sch_multi_plan (pure host code): header, per-TB geometry, then one row reference
    (TB, codeblock) per codeblock row — every row exactly once, ordered by the elements the row
    moves (E + N) descending, so the rate-recovery launch's big rows start first."""
    from python_5gtoolbox_amd import sch
    cfgs = [sch.sch_config(*a) for a in ((8000, 4, 700, 1, 3, 60000, 26000), (200, 2, 300, 1, 0, 60000, 2400),
                                          (24000, 8, 900, 1, 2, 60000, 27000), (3000, 6, 300, 1, 1, 60000, 24000))]
    lay = sch.multi_layout(cfgs)
    lib = _lib.lib()
    n = lib.ldpc5g_sch_multi_plan(lay["arr"], len(cfgs), None, 0)
    assert n > 24
    buf = (ctypes.c_ubyte * n)()
    assert lib.ldpc5g_sch_multi_plan(lay["arr"], len(cfgs), buf, n) == n
    hdr = np.frombuffer(bytes(buf)[:16], np.int32)
    nrows = sum(c.C for c in cfgs)
    assert hdr[0] == 0x4c505253 and hdr[1] == len(cfgs) and hdr[2] == nrows
    assert hdr[3] == max(max(c.E_lo, c.E_hi) for c in cfgs)
    refs = np.frombuffer(bytes(buf)[n - 8 * nrows:], np.int32).reshape(nrows, 2)
    assert sorted(map(tuple, refs.tolist())) == [(t, c) for t, cf in enumerate(cfgs) for c in range(cf.C)]

    def work(t, c):
        cf = cfgs[t]
        return (cf.E_lo if c < cf.c_switch else cf.E_hi) + cf.N
    w = [work(t, c) for t, c in refs]
    assert w == sorted(w, reverse=True)


@pytest.mark.parametrize("call,code", [
    (lambda l: l.ldpc5g_pack_records(None, 10, 2, 10, None, None, None, 1, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_unpack_records(None, 8, 2, 10, None, 10, None, None, 0, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_pack_records(None, 10, 0, 10, None, None, None, 2, None), 0),
    (lambda l: l.ldpc5g_scramble_modulate(None, 10, None, 0, 1, 10, 3, None, 10, None), _lib.ESIZE),
    (lambda l: l.ldpc5g_demod_descramble(None, 1, 10, None, 10, None, 0, 1, 10, 2, None, 0, 20,
                                         None), _lib.ESIZE),   # float64 LLRs need BPSK + c128
    (lambda l: l.ldpc5g_demod_descramble(None, 0, 10, None, 10, None, 0, 1, 10, 1, None, 0, 10,
                                         None), _lib.ESIZE),   # null buffers
])
def test_pack_and_phy_validation_without_gpu(call, code):
    assert call(_lib.lib()) == code


def test_sparse_scratch_sizing():
    """LDS when the per-codeblock working set fits 156 KB, else (N + E) doubles per codeblock
    (soft) / 5N + M bytes rounded to 16 (BF) of caller scratch; -1 on bad arguments."""
    lib = _lib.lib()
    assert lib.ldpc5g_sparse_scratch_bytes(10, 4, 6, 12, _lib.ALGO_MS) == 0
    assert lib.ldpc5g_sparse_scratch_bytes(3, 8000, 16000, 48000, _lib.ALGO_MS) == 3 * 64000 * 8
    assert lib.ldpc5g_sparse_scratch_bytes(3, 8000, 16000, 48000, _lib.ALGO_BF) == 0
    assert lib.ldpc5g_sparse_scratch_bytes(2, 40000, 80000, 9, _lib.ALGO_BF) == 2 * 440000
    assert lib.ldpc5g_sparse_scratch_bytes(1, 4, 0, 12, _lib.ALGO_MS) == -1
    assert lib.ldpc5g_sparse_scratch_bytes(1, 4, 6, 12, 7) == -1


def test_sim_harness_result_file_and_plot(tmp_path):
    """Host side of the sim_ldpc_internal drop-in (no GPU): the result file is the reference's
    pickle [sim_config, labels, bler lists] (scripts/internal/sim_ldpc_internal.py:89-91, plain
    containers), and draw_ldpc_decoder_result (:93-117) plots a synthetic sweep to a file."""
    import pickle
    from python_5gtoolbox_amd import sim_ldpc, sim_ldpc_internal
    cfg, flags = {"Zc": 12, "bgn": 1}, ["NMS-alpha=0.7-L=32", "mixed-MS-[alpha,beta]=[0.8,0.3]-L=32"]
    res = [[0.395, 0.135, 0.015, 0.0005, 0.0], [0.275, 0.065, 0.00375, 0.0015, 0.0]]
    snrs = [-1.0, -0.5, 0.0, 0.5, 1.0]
    f = tmp_path / "r.pickle"
    sim_ldpc._dump(str(f), None, cfg, flags, res, [[[1000, 1]] * 5] * 2, snrs, "flooding")

    class NoGlobals(pickle.Unpickler):
        def find_class(self, module, name):
            raise AssertionError((module, name))
    with open(f, "rb") as fh:
        assert NoGlobals(fh).load() == [cfg, flags, res]
    png = tmp_path / "r.png"
    sim_ldpc_internal.draw_ldpc_decoder_result(snrs, cfg, flags, res, str(png))
    assert png.read_bytes()[:4] == b"\x89PNG"


def test_staging_cache_bounded():
    """The drop-ins' per-thread staging cache (_lib.staging) keeps at most STAGING_MAX entries,
    least recently used evicted: a sweep over many TB configurations cannot grow it without
    bound."""
    from python_5gtoolbox_amd import _lib
    made = []
    for i in range(3 * _lib.STAGING_MAX):
        _lib.staging(("sweep", i), lambda: made.append(1) or object())
        assert _lib.staging_entries() <= _lib.STAGING_MAX
    assert len(made) == 3 * _lib.STAGING_MAX
    last = ("sweep", 3 * _lib.STAGING_MAX - 1)
    n = len(made)
    _lib.staging(last, lambda: made.append(1) or object())   # cached: not rebuilt
    assert len(made) == n
