"""CPU (gloo, world_size 2 and 3) tests of the multi-GPU sharding/gather logic.

The per-rank decode here is the oracle injected as `decode_fn` (test infrastructure); on the
GPU box the same code path runs the HIP decoder over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from python_5gtoolbox_amd.shard import shard_bounds, shard_round_robin


def test_sharded_defaults_are_the_reference_schedule():
    """Both sharded entry points decode in the reference's schedule unless asked otherwise
    (float64 flooding for float64 LLRs: nr_ldpc_decode.py:51-143, nr_dlsch_decode.py:62-106)."""
    import inspect
    from python_5gtoolbox_amd.shard import decode_codeblocks_sharded, decode_tbs_sharded
    for f in (decode_codeblocks_sharded, decode_tbs_sharded):
        assert inspect.signature(f).parameters["schedule"].default == "flooding"
    assert inspect.signature(decode_tbs_sharded).parameters["dn_dtype"].default is None


def test_shard_bounds_cover_exactly():
    for n in [0, 1, 7, 4096, 4097]:
        for w in [1, 2, 3, 8]:
            got = [shard_bounds(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [hi - lo for lo, hi in got]
            assert max(sizes) - min(sizes) <= 1
    assert shard_round_robin(10, 1, 4) == [1, 5, 9]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def np_pack(bits, nbits, status=None, iters=None, out=None):
    """Test double of shard.pack_records (the HIP kernel) for CPU tensors: same record layout."""
    b = bits[:, :nbits].numpy().astype(np.uint8)
    parts = [np.packbits(b, axis=1)]
    if status is not None:
        parts.append(status.numpy().astype(np.uint8)[:, None])
    if iters is not None:
        parts.append(iters.numpy().astype("<i4").view(np.uint8).reshape(-1, 4))
    rec = np.concatenate(parts, axis=1)
    out[:rec.shape[0], :rec.shape[1]] = torch.from_numpy(rec)
    return out


def np_unpack(rec, R, nbits, bits=None, status=None, iters=None):
    """Test double of shard.unpack_records for CPU tensors."""
    r = rec[:R].numpy()
    nb = (nbits + 7) // 8
    if bits is not None:
        bits.copy_(torch.from_numpy(np.unpackbits(r[:, :nb], axis=1)[:, :nbits].astype(np.int8)))
    o = nb
    if status is not None:
        status.copy_(torch.from_numpy(r[:, o].copy()))
        o += 1
    if iters is not None:
        iters.copy_(torch.from_numpy(np.ascontiguousarray(r[:, o:o + 4]).view("<i4")[:, 0].copy()))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import ldpc_oracle as O
        from python_5gtoolbox_amd.shard import decode_codeblocks_sharded, decode_tbs_sharded
        from python_5gtoolbox_amd.shard import shard_bounds, shard_round_robin
        bg, Zc, B = 2, 13, 11                     # K = 130: not a multiple of 8 (padded bytes)
        rng = np.random.default_rng(5)           # same data on every rank (the "full batch")
        ck = rng.integers(0, 2, (B, 10 * Zc)).astype(np.int8)
        llr = O.bpsk_awgn_llr(O.encode(ck, bg), 1.0, rng).astype(np.float32)

        def dec(x):
            c, s, i = O.decode_layered(x.numpy(), Zc, bg, 8, 0.75, 0.0)
            return torch.from_numpy(c), torch.from_numpy(s.astype(np.uint8)), torch.from_numpy(i)

        timing = {}
        res = decode_codeblocks_sharded(torch.from_numpy(llr), Zc, bg, 8, 0.75, 0.0,
                                        decode_fn=dec, pack_fn=np_pack, unpack_fn=np_unpack,
                                        timing=timing)
        # the reference's precision: float64 LLRs through float64 flooding (the default schedule)
        llr64 = llr.astype(np.float64) * 1.37

        def dec64(x):
            assert x.dtype == torch.float64
            c, s, i = O.decode_flooding(x.numpy(), Zc, bg, 8, 0.75, 0.0, np.float64)
            return torch.from_numpy(c), torch.from_numpy(s.astype(np.uint8)), torch.from_numpy(i)
        res64 = decode_codeblocks_sharded(torch.from_numpy(llr64), Zc, bg, 8, 0.75, 0.0,
                                          decode_fn=dec64, pack_fn=np_pack, unpack_fn=np_unpack)
        # transport blocks round robin: TB i decodes to bits i, i+1, ... and CRC flag i % 2 == 0
        T, nb = 5, 37

        def tb_dec(x):
            idx = x[:, 0].long()
            bits = ((idx[:, None] + torch.arange(nb)[None, :]) % 2).to(torch.int8)
            return (idx % 2 == 0).to(torch.uint8), bits
        tb_llr = torch.arange(T, dtype=torch.float32)[:, None].repeat(1, 3)
        tb = decode_tbs_sharded(tb_llr, {"B": nb}, 8, decode_fn=tb_dec, pack_fn=np_pack,
                                unpack_fn=np_unpack)
        exp_bits = (np.arange(T)[:, None] + np.arange(nb)[None, :]) % 2
        ok = True
        # this rank's rows passed explicitly (T_total / n_total): same results, gathered to the
        # LAST rank; a row count that differs from the rank's assignment is refused
        mine = shard_round_robin(T, rank, world)
        tb2 = decode_tbs_sharded(tb_llr[mine], {"B": nb}, 8, T_total=T, decode_fn=tb_dec,
                                 pack_fn=np_pack, unpack_fn=np_unpack, dst=world - 1)
        if rank == world - 1:
            ok &= tb2[0].tolist() == [1, 0, 1, 0, 1] and np.array_equal(tb2[1].numpy(), exp_bits)
        else:
            ok &= tb2 is None
        lo, hi = shard_bounds(B, rank, world)
        try:
            extra = np.concatenate([llr[lo:hi], llr[:1]])      # one row too many on every rank
            decode_codeblocks_sharded(torch.from_numpy(extra), Zc, bg, 8, n_total=B,
                                      decode_fn=dec, pack_fn=np_pack, unpack_fn=np_unpack)
            ok = False
        except AssertionError:
            pass
        if world == 3:
            # a sub-group {1, 2}: dst is a rank within it (group rank 0 = global rank 1)
            sub = dist.new_group([1, 2])
            if rank in (1, 2):
                tb3 = decode_tbs_sharded(tb_llr, {"B": nb}, 8, decode_fn=tb_dec, pack_fn=np_pack,
                                         unpack_fn=np_unpack, group=sub, dst=0)
                if rank == 1:
                    ok &= tb3[0].tolist() == [1, 0, 1, 0, 1] and np.array_equal(tb3[1].numpy(), exp_bits)
                else:
                    ok &= tb3 is None
        if rank == 0:
            fc, fs, fi = O.decode_flooding(llr64, Zc, bg, 8, 0.75, 0.0, np.float64)
            ok &= (np.array_equal(res64[0].numpy(), fc[:, :10 * Zc])
                   and np.array_equal(res64[1].numpy().astype(bool), fs)
                   and np.array_equal(res64[2].numpy(), fi))
            rc, rs, ri = O.decode_layered(llr, Zc, bg, 8, 0.75, 0.0)
            ok &= (np.array_equal(res[0].numpy(), rc[:, :10 * Zc])
                   and np.array_equal(res[1].numpy().astype(bool), rs)
                   and np.array_equal(res[2].numpy(), ri)
                   and tb[0].tolist() == [1, 0, 1, 0, 1]
                   and np.array_equal(tb[1].numpy(), exp_bits)
                   and timing["gather_bytes"] == world * -(-B // world) * (17 + 5))
        else:
            ok &= res is None and tb is None and res64 is None
        q.put(bool(ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_decode_gloo(world):
    """world 2: even / uneven codeblock shards; world 3: 11 codeblocks as 4/4/3, 5 TBs as 2/2/1
    round robin, gathers to rank 0, to the last rank, and within a sub-group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(results), results
