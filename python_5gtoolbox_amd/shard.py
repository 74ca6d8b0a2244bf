"""Multi-GPU sharding: one process per GPU, work split with no collective on the data path, one
gather of packed results to rank 0 at the end (BASELINE.json north_star: "RCCL only for the final
gather").

The reference decodes codeblocks one at a time in a Python loop (py5gphy/nr_pdsch/
nr_dlsch_decode.py:62-103); codeblocks are independent until the transport-block CRC (:106), so
the batch axis shards with no exchange:
  * codeblocks (configs 2-4): contiguous row ranges (shard_bounds);
  * transport blocks (config 5): whole TBs round robin (shard_round_robin), so every TB's CRC
    stays rank-local.
Each rank packs its results on its GPU into gather records (ldpc5g_pack_records: np.packbits
order, plus status / iteration fields — 1061 B per BG1 Zc=384 codeblock instead of 8448 B of
info bytes), and ONE dist.gather (RCCL over xGMI; gloo in the CPU tests) brings every rank's
record block to rank `dst`, which unpacks them on its GPU in shard order.

torch.distributed and torch tensors are plumbing (device buffers, the collective); the packing
and unpacking are HIP kernels.  Tests on CPU (gloo, no GPU) inject `decode_fn` / `pack_fn` /
`unpack_fn` (numpy) — the product path requires the GPU.
"""
import time

from . import _lib


def shard_bounds(n, rank, world):
    """Contiguous [lo, hi) range of n items owned by `rank` (the first n % world ranks get one
    extra item)."""
    assert 0 <= rank < world
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_round_robin(n, rank, world):
    """Item indices owned by `rank` under round-robin assignment (whole transport blocks)."""
    return list(range(rank, n, world))


def record_bytes(nbits, status=True, iters=True):
    """Bytes of one gather record (include/ldpc5g.h ldpc5g_pack_records)."""
    return (nbits + 7) // 8 + (1 if status else 0) + (4 if iters else 0)


def pack_records(bits, nbits, status=None, iters=None, out=None):
    """bits (R, >= nbits) int8 device tensor (+ status (R,) uint8, iters (R,) int32) -> records
    (R, record_bytes) uint8 on the same device (`out` may have more rows: only R are written)."""
    t = _lib.require_gpu()
    R = bits.shape[0]
    rb = record_bytes(nbits, status is not None, iters is not None)
    rec = out if out is not None else t.empty((R, rb), dtype=t.uint8, device=bits.device)
    assert rec.dtype == t.uint8 and rec.shape[0] >= R and rec.shape[1] >= rb and rec.stride(1) == 1
    assert bits.dtype == t.int8 and bits.stride(1) == 1 and bits.shape[1] >= nbits
    with t.cuda.device(bits.device):
        for r0 in range(0, max(R, 1), 65535):   # grid.y limit
            n = min(65535, R - r0)
            if n <= 0:
                break
            _lib.check(_lib.lib().ldpc5g_pack_records(
                _lib.ptr(bits[r0:]), bits.stride(0), n, int(nbits),
                _lib.ptr(status[r0:]) if status is not None else None,
                _lib.ptr(iters[r0:]) if iters is not None else None,
                _lib.ptr(rec[r0:]), rec.stride(0), _lib.stream_ptr(bits.device)))
    return rec


def unpack_records(rec, R, nbits, bits=None, status=None, iters=None):
    """Inverse of pack_records into the given device tensors (any may be None; bits rows and the
    1-D status / iters may be strided views, e.g. every world-th TB)."""
    t = _lib.require_gpu()
    fs = (status if status is not None else iters).stride(0) if (status is not None or iters is not None) else 1
    assert iters is None or status is None or iters.stride(0) == status.stride(0)
    assert bits is None or (bits.dtype == t.int8 and bits.stride(1) == 1)
    with t.cuda.device(rec.device):
        for r0 in range(0, max(R, 1), 65535):
            n = min(65535, R - r0)
            if n <= 0:
                break
            _lib.check(_lib.lib().ldpc5g_unpack_records(
                _lib.ptr(rec[r0:]), rec.stride(0), n, int(nbits),
                _lib.ptr(bits[r0:]) if bits is not None else None,
                bits.stride(0) if bits is not None else 0,
                _lib.ptr(status[r0:]) if status is not None else None,
                _lib.ptr(iters[r0:]) if iters is not None else None, fs,
                _lib.stream_ptr(rec.device)))


def gather_record_blocks(torch, dist, rec, counts, rank, world, dst=0, group=None):
    """ONE dist.gather of every rank's record block (padded to the largest shard) to `dst`.
    rank, world and dst are ranks WITHIN `group` (group_dst: the rank that allocates the gather
    list is the one that receives, whatever group is passed).
    rec: (m, rb) uint8 with m = max(counts) rows, this rank's counts[rank] first.  Returns on dst
    the (world, m, rb) buffer (rank r's records in [r, :counts[r]]), None elsewhere."""
    assert rec.shape[0] >= max(counts)
    assert 0 <= dst < world
    buf = torch.empty((world,) + tuple(rec.shape), dtype=rec.dtype, device=rec.device) \
        if rank == dst else None
    dist.gather(rec, gather_list=list(buf.unbind(0)) if buf is not None else None,
                group=group, group_dst=dst)
    return buf


def _world(group):
    import torch.distributed as dist
    if dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def decode_codeblocks_sharded(llr, Zc, bgn, L, alpha=1.0, beta=0.0, schedule="flooding",
                              n_total=None, decode_fn=None, pack_fn=None, unpack_fn=None,
                              group=None, dst=0, timing=None):
    """Decode this rank's shard of a codeblock batch and gather the results to rank `dst`.

    llr: this rank's (n_local, N) LLR rows (device tensor), or the full (n_total, N) batch, in
         which case the rank slices its own range.
    schedule: "flooding" (default) decodes in the reference's schedule — with float64 LLRs its
         arithmetic too, bit-identical to nr_decode_ldpc (nr_ldpc_decode.py:11-143); "layered" is
         the float32 perf kernel.
    Returns on rank dst: (info bits (n_total, K) int8, status (n_total,) uint8,
    iters (n_total,) int32) on dst's device; None on other ranks.  `timing` (dict) receives
    decode_s / gather_s measured on this rank (synchronised wall clock)."""
    import torch
    import torch.distributed as dist
    from .ldpc_info import code_dims
    world, rank = _world(group)
    K, N, Nf = code_dims(bgn, Zc)
    if n_total is None:
        n_total = llr.shape[0]
        lo, hi = shard_bounds(n_total, rank, world)
        llr = llr[lo:hi]
    else:   # the caller's rows must be exactly this rank's shard_bounds range
        lo, hi = shard_bounds(n_total, rank, world)
        assert llr.shape[0] == hi - lo, \
            f"rank {rank}: {llr.shape[0]} LLR rows, shard_bounds({n_total}) assigns {hi - lo}"
    if decode_fn is None:
        from .nr_ldpc_decode import nr_decode_ldpc_batch

        def decode_fn(x):
            return nr_decode_ldpc_batch(x, Zc, bgn, L, "min-sum", alpha, beta, schedule)
    pack_fn = pack_fn or pack_records
    unpack_fn = unpack_fn or unpack_records
    sync = torch.cuda.synchronize if llr.is_cuda else (lambda: None)
    t0 = time.perf_counter()
    ck, st, it = decode_fn(llr)
    sync()
    t1 = time.perf_counter()
    counts = [hi - lo for lo, hi in (shard_bounds(n_total, r, world) for r in range(world))]
    assert ck.shape[0] == counts[rank] and st.shape[0] == counts[rank] and it.shape[0] == counts[rank]
    rb = record_bytes(K)
    rec = torch.empty((max(counts + [1]), rb), dtype=torch.uint8, device=llr.device)
    pack_fn(ck, K, st.to(torch.uint8), it.to(torch.int32), out=rec)
    if world == 1:
        buf, counts = rec.unsqueeze(0), [ck.shape[0]]
    else:
        buf = gather_record_blocks(torch, dist, rec, counts, rank, world, dst, group)
    out = None
    if buf is not None:
        info = torch.empty((n_total, K), dtype=torch.int8, device=buf.device)
        status = torch.empty((n_total,), dtype=torch.uint8, device=buf.device)
        iters = torch.empty((n_total,), dtype=torch.int32, device=buf.device)
        lo = 0
        for r, c in enumerate(counts):
            unpack_fn(buf[r], c, K, bits=info[lo:lo + c], status=status[lo:lo + c],
                      iters=iters[lo:lo + c])
            lo += c
        out = (info, status, iters)
    sync()
    if timing is not None:
        timing.update(decode_s=t1 - t0, gather_s=time.perf_counter() - t1,
                      gather_bytes=rb * max(counts) * world)
    return out


def decode_tbs_sharded(llr, cfg, L, algo="min-sum", alpha=1.0, beta=0.0, schedule="flooding",
                       T_total=None, decode_fn=None, pack_fn=None, unpack_fn=None, group=None,
                       dst=0, timing=None, dn_dtype=None):
    """Config 5 shape: whole transport blocks round robin across ranks (every TB's CRC stays
    rank-local), each rank running the GPU DL-SCH receive chain (sch_decode_batch: rate recovery,
    LDPC decode, CB / TB CRCs) on its TBs; (tb_ok, tbblk) records gathered to `dst`.

    llr: this rank's (T_local, G) LLR rows in round-robin order (TB rank, rank + world, ...), or
         the full (T_total, G) batch (then the rank takes its TBs).
    schedule: "flooding" (default: float64 rate recovery and decoding for float64 LLRs, or with
         dn_dtype float64 — DLSCHDecode's arithmetic) or "layered" (float32 perf kernel).
    dn_dtype: the rate-recovered rows' dtype (sch_decode_batch; None: float32 for layered, the
         LLRs' dtype for flooding).
    Returns on dst: (tb_ok (T_total,) uint8, tbblk (T_total, B) int8 — TB bits then CRC) in TB
    order; None elsewhere."""
    import torch
    import torch.distributed as dist
    world, rank = _world(group)
    mine_idx = None
    if T_total is None:
        T_total = llr.shape[0]
        mine_idx = shard_round_robin(T_total, rank, world)
        llr = llr[mine_idx[0]::world] if mine_idx else llr[:0]
    else:   # the caller's rows must be exactly this rank's round-robin TBs
        n_mine = len(shard_round_robin(T_total, rank, world))
        assert llr.shape[0] == n_mine, \
            f"rank {rank}: {llr.shape[0]} TB rows, round robin over {T_total} assigns {n_mine}"
    if decode_fn is None:
        from .sch import sch_decode_batch

        def decode_fn(x):
            r = sch_decode_batch(x, cfg, L, algo, alpha, beta, schedule, dn_dtype=dn_dtype)
            return r.tb_ok, r.tbblk
    pack_fn = pack_fn or pack_records
    unpack_fn = unpack_fn or unpack_records
    sync = torch.cuda.synchronize if llr.is_cuda else (lambda: None)
    nb = int(cfg.B) if hasattr(cfg, "B") else int(cfg["B"])
    t0 = time.perf_counter()
    tb_ok, tbblk = decode_fn(llr)
    sync()
    t1 = time.perf_counter()
    counts = [len(shard_round_robin(T_total, r, world)) for r in range(world)]
    assert tb_ok.shape[0] == counts[rank] and tbblk.shape[0] == counts[rank]
    rb = record_bytes(nb, iters=False)
    rec = torch.empty((max(counts + [1]), rb), dtype=torch.uint8, device=llr.device)
    pack_fn(tbblk, nb, tb_ok.to(torch.uint8), None, out=rec)
    if world == 1:
        buf = rec.unsqueeze(0)
    else:
        buf = gather_record_blocks(torch, dist, rec, counts, rank, world, dst, group)
    out = None
    if buf is not None:
        ok = torch.empty((T_total,), dtype=torch.uint8, device=buf.device)
        bits = torch.empty((T_total, nb), dtype=torch.int8, device=buf.device)
        for r, c in enumerate(counts):   # rank r holds TBs r, r + world, ...: strided rows
            unpack_fn(buf[r], c, nb, bits=bits[r::world], status=ok[r::world])
        out = (ok, bits)
    sync()
    if timing is not None:
        timing.update(decode_s=t1 - t0, gather_s=time.perf_counter() - t1,
                      gather_bytes=rb * max(counts) * world)
    return out
