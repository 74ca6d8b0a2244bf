"""GPU edge cases: empty batches through every batched entry point, the largest lifting size at a
16384-codeblock batch for both base graphs (size-independent property: every encoded codeword
satisfies all checks, so noise-free LLRs decode with status 1 within one iteration), and the
smallest lifting sizes."""
import numpy as np
import pytest

from oracle import ldpc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a ROCm GPU"
    return t


def test_empty_codec_batches(torch):
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    for bg, kb, nb in ((1, 22, 66), (2, 10, 50)):
        dn = E.encode_ldpc_batch(torch.empty((0, kb * 384), dtype=torch.int8, device="cuda"), bg)
        assert tuple(dn.shape) == (0, nb * 384)
        dn_np = E.encode_ldpc_batch(np.zeros((0, kb * 64), np.int8), bg)
        assert dn_np.shape == (0, nb * 64) and dn_np.dtype == np.int8
        for schedule in ("flooding", "layered"):
            ck, st, it = D.nr_decode_ldpc_batch(torch.empty((0, nb * 384), device="cuda"), 384, bg,
                                                8, "min-sum", 0.75, 0.0, schedule)
            torch.cuda.synchronize()
            assert tuple(ck.shape) == (0, (nb + 2) * 384) and st.numel() == 0 and it.numel() == 0


def test_empty_phy_batches(torch):
    from python_5gtoolbox_amd import phy
    for Qm in (2, 8):
        sym = phy.scramble_modulate(torch.empty((0, 64 * Qm), dtype=torch.int8, device="cuda"), Qm,
                                    torch.empty((0,), dtype=torch.int64, device="cuda"))
        assert sym.shape[0] == 0
        llr = phy.demod_descramble(torch.empty((0, 64), dtype=torch.complex64, device="cuda"),
                                   torch.empty((0, 64), dtype=torch.float32, device="cuda"), Qm,
                                   torch.empty((0,), dtype=torch.int64, device="cuda"))
        torch.cuda.synchronize()
        assert tuple(llr.shape) == (0, 64 * Qm)


@pytest.mark.parametrize("bg", [1, 2])
def test_max_lifting_size_large_batch_codewords(torch, bg):
    """16384 codeblocks at Zc = 384: GPU encode, then noise-free LLRs (+-10) through the float32
    flooding decoder with L = 1.  The first 2Zc (punctured) bits enter with LLR 0, i.e. as hard
    decision 0, so a codeblock stops at the iteration-0 syndrome check exactly when those bits
    are all 0; every other one needs the single iteration, after which all checks hold: status 1
    everywhere and the hard decisions equal (ck, dn)."""
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    B, Zc = 16384, 384
    kb = 22 if bg == 1 else 10
    g = torch.Generator(device="cuda")
    g.manual_seed(100 + bg)
    ck = torch.randint(0, 2, (B, kb * Zc), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, bg)
    llr = 10.0 * (1 - 2 * dn.float())
    out, st, it = D.nr_decode_ldpc_batch(llr, Zc, bg, 1, "min-sum", 1.0, 0.0, "flooding")
    torch.cuda.synchronize()
    assert int(st.sum()) == B
    assert torch.equal(it.long(), ck[:, :2 * Zc].any(dim=1).long())
    assert torch.equal(out[:, :kb * Zc], ck) and torch.equal(out[:, 2 * Zc:], dn)
    # spot-check a few codewords against the oracle encoder (bit-exact)
    idx = [0, B // 2, B - 1]
    ref = O.encode(ck[idx].cpu().numpy(), bg)
    assert np.array_equal(dn[idx].cpu().numpy(), ref)


@pytest.mark.parametrize("bg", [1, 2])
def test_smallest_lifting_sizes_batch_vs_oracle(torch, bg):
    """Zc = 2, 3, 4, 5 (the lifting sets' smallest members): batched encode bit-exact with the
    oracle, layered decode of AWGN LLRs bit-exact (ck, status, iters)."""
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    rng = np.random.default_rng(bg)
    kb = 22 if bg == 1 else 10
    for Zc in (2, 3, 4, 5):
        ck = rng.integers(0, 2, (37, kb * Zc)).astype(np.int8)
        dn = E.encode_ldpc_batch(ck, bg)
        ref = O.encode(ck, bg)
        assert np.array_equal(dn, ref), Zc
        llr = O.bpsk_awgn_llr(ref, 1.0, rng).astype(np.float32)
        out, st, it = D.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, "layered")
        r = O.decode_layered(llr, Zc, bg, 8, 0.75, 0.0)
        assert np.array_equal(np.asarray(out), r[0]) and np.array_equal(np.asarray(st), r[1]) \
            and np.array_equal(np.asarray(it), r[2]), Zc


@pytest.mark.parametrize("bg,Zc,B", [(1, 384, 3), (2, 176, 5), (1, 64, 13), (2, 8, 97), (1, 352, 1)])
@pytest.mark.parametrize("schedule", ["layered", "flooding"])
def test_batch_tail_slots_vs_oracle(torch, bg, Zc, B, schedule):
    """Batches with B > G and B % G != 0 (G = codeblocks per workgroup) leave workgroup slots past
    the end of the batch: those threads must neither decode nor read past the caller's rows.  The
    LLRs sit in their own exactly-sized device tensor (a padded copy's tail is poisoned with NaN, so
    a read past the batch that leaked into a real slot would change its result), and every output
    is compared with the oracle (batch-tail row pointers)."""
    from python_5gtoolbox_amd import nr_ldpc_decode as D
    rng = np.random.default_rng(Zc * 13 + B)
    K = (22 if bg == 1 else 10) * Zc
    ck = rng.integers(0, 2, (B, K)).astype(np.int8)
    dn = O.encode(ck, bg)
    snr = rng.uniform(-1.0, 2.0, (B, 1))
    llr = (2 * ((1 - 2 * dn) + rng.normal(size=dn.shape) * 10 ** (-snr / 20)) /
           10 ** (-snr / 10)).astype(np.float32)
    pad = torch.full((B + 4, llr.shape[1]), float("nan"), device="cuda")
    pad[:B] = torch.from_numpy(llr).cuda()
    exact = pad[:B].clone()
    for x in (exact, pad[:B]):
        got = D.nr_decode_ldpc_batch(x, Zc, bg, 10, "min-sum", 0.75, 0.0, schedule)
        got = [g.cpu().numpy() for g in got]
        ref = (O.decode_layered(llr, Zc, bg, 10, 0.75, 0.0) if schedule == "layered"
               else O.decode_flooding(llr, Zc, bg, 10, 0.75, 0.0, np.float32))
        assert np.array_equal(got[0], ref[0])
        assert np.array_equal(got[1].astype(bool), ref[1].astype(bool))
        assert np.array_equal(got[2], ref[2])
