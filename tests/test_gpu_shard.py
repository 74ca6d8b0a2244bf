"""GPU side of the multi-GPU path: the gather-record kernels
(ldpc5g_pack_records / ldpc5g_unpack_records) against np.packbits, and the sharded codeblock / TB
decode entry points at world size 1 (every HIP step of the N-rank path, without the collective;
the collective itself is covered by tests/test_shard.py with gloo at world size 2)."""
import numpy as np
import pytest

from oracle import ldpc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a ROCm GPU"
    return t


@pytest.mark.parametrize("nbits,offset", [(8448, 0), (130, 0), (1, 0), (1081536, 0), (77, 3)])
def test_pack_unpack_records_vs_numpy(torch, nbits, offset):
    from python_5gtoolbox_amd.shard import pack_records, record_bytes, unpack_records
    rng = np.random.default_rng(nbits)
    R = 5 if nbits > 100000 else 37
    full = rng.integers(0, 2, (R, nbits + offset + 5)).astype(np.int8)
    bits = torch.from_numpy(full).cuda()[:, offset:offset + nbits]   # unaligned rows when offset
    st = torch.from_numpy(rng.integers(0, 2, R).astype(np.uint8)).cuda()
    it = torch.from_numpy(rng.integers(-5, 1 << 30, R).astype(np.int32)).cuda()
    rec = pack_records(bits, nbits, st, it).cpu().numpy()
    assert rec.shape == (R, record_bytes(nbits))
    nb = (nbits + 7) // 8
    assert np.array_equal(rec[:, :nb], np.packbits(full[:, offset:offset + nbits].astype(np.uint8), axis=1))
    assert np.array_equal(rec[:, nb], st.cpu().numpy())
    assert np.array_equal(np.ascontiguousarray(rec[:, nb + 1:]).view("<i4")[:, 0], it.cpu().numpy())
    # unpack into strided views (every 2nd row), as the TB gather does
    back = torch.full((2 * R, nbits), 7, dtype=torch.int8, device="cuda")
    st2 = torch.full((2 * R,), 9, dtype=torch.uint8, device="cuda")
    it2 = torch.full((2 * R,), 9, dtype=torch.int32, device="cuda")
    unpack_records(torch.from_numpy(rec).cuda(), R, nbits, bits=back[1::2], status=st2[1::2],
                   iters=it2[1::2])
    assert np.array_equal(back[1::2].cpu().numpy(), full[:, offset:offset + nbits])
    assert (back[0::2].cpu().numpy() == 7).all()
    assert np.array_equal(st2[1::2].cpu().numpy(), st.cpu().numpy()) and (st2[0::2].cpu().numpy() == 9).all()
    assert np.array_equal(it2[1::2].cpu().numpy(), it.cpu().numpy())


@pytest.mark.parametrize("schedule,dtype", [("layered", np.float32), ("flooding", np.float64)])
def test_sharded_codeblock_decode_world1(torch, schedule, dtype):
    """decode_codeblocks_sharded on one GPU: decode -> pack records -> unpack == the plain batched
    decode (info bits, status, iterations); float64 flooding (the default schedule, the
    reference's arithmetic) also == the oracle's float64 decode_ldpc."""
    from python_5gtoolbox_amd.nr_ldpc_decode import nr_decode_ldpc_batch
    from python_5gtoolbox_amd.shard import decode_codeblocks_sharded
    rng = np.random.default_rng(1)
    bg, Zc, B = 1, 384, 64
    ck = rng.integers(0, 2, (B, 22 * Zc)).astype(np.int8)
    x = O.bpsk_awgn_llr(O.encode(ck, bg), 0.5, rng).astype(dtype)
    llr = torch.from_numpy(x).cuda()
    timing = {}
    info, st, it = decode_codeblocks_sharded(llr, Zc, bg, 8, 0.75, 0.0, schedule, timing=timing)
    rck, rst, rit = nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, schedule)
    assert torch.equal(info, rck[:, :22 * Zc]) and torch.equal(st, rst) and torch.equal(it, rit)
    assert timing["gather_bytes"] == B * (1056 + 5)
    if dtype == np.float64:
        oc, os_, oi = O.decode_flooding(x[:8], Zc, bg, 8, 0.75, 0.0, np.float64)
        assert np.array_equal(info[:8].cpu().numpy(), oc[:, :22 * Zc])
        assert np.array_equal(st[:8].cpu().numpy().astype(bool), os_) and np.array_equal(it[:8].cpu().numpy(), oi)


@pytest.mark.parametrize("schedule", ["layered", "flooding"])
def test_sharded_tb_decode_world1(torch, schedule):
    """decode_tbs_sharded on one GPU over a 3-TB DL-SCH batch: the gathered (crc_ok, tbblk) equal
    sch_decode_batch's and carry the transmitted bits (flooding: float64 rate recovery + float64
    flooding, DLSCHDecode's arithmetic)."""
    from python_5gtoolbox_amd import sch
    from python_5gtoolbox_amd.shard import decode_tbs_sharded
    A, Qm, R, NL, rv, G = 30000, 2, 500, 1, 0, 2 * 40000
    cfg = sch.sch_config(A, Qm, R, NL, rv, A, G)
    g = torch.Generator(device="cuda")
    g.manual_seed(2)
    tb = torch.randint(0, 2, (3, A), dtype=torch.int8, device="cuda", generator=g)
    bits = sch.sch_encode_batch(tb, cfg).contiguous()
    llr = (8.0 * (1 - 2 * bits.float())).contiguous()
    dn = torch.float64 if schedule == "flooding" else None
    ok, tbblk = decode_tbs_sharded(llr, cfg, 8, "min-sum", 0.75, 0.0, schedule, dn_dtype=dn)
    r = sch.sch_decode_batch(llr, cfg, 8, "min-sum", 0.75, 0.0, schedule, dn_dtype=dn)
    assert r.llr_dn.dtype == (torch.float64 if schedule == "flooding" else torch.float32)
    assert torch.equal(ok, r.tb_ok) and torch.equal(tbblk, r.tbblk)
    assert ok.cpu().numpy().all() and torch.equal(tbblk[:, :A], tb)
