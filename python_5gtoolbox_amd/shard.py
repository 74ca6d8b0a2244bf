"""Multi-GPU codeblock sharding: one process per GPU, codeblocks split into contiguous ranges,
no collective on the data path, one gather of the decoded bits to rank 0 at the end.

The reference decodes codeblocks one at a time in a Python loop (py5gphy/nr_pdsch/
nr_dlsch_decode.py:62-103); codeblocks are independent until the transport-block CRC (:106),
so the batch axis shards with no exchange.  Transport blocks (config 5) shard whole, round
robin, so each TB's CRC stays rank-local.

torch.distributed is plumbing here: backend "nccl" (= RCCL over xGMI) on the GPU box, "gloo"
in the CPU tests.  The per-rank decode is the HIP batch decoder unless a test passes its own
`decode_fn`.
"""
import numpy as np


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


def _gather_rows(torch, dist, local, n_total, world, group):
    """all_gather of variable-length row blocks (padded to the largest shard) -> (n_total, ...)
    on every rank; rank order = shard order."""
    counts = [shard_bounds(n_total, r, world) for r in range(world)]
    m = max(hi - lo for lo, hi in counts)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:hi - lo] for b, (lo, hi) in zip(bufs, counts)], dim=0)


def decode_codeblocks_sharded(llr, Zc, bgn, L, alpha=1.0, beta=0.0, schedule="layered",
                              n_total=None, decode_fn=None, group=None, dst=0):
    """Decode this rank's shard of a codeblock batch and gather the results to rank `dst`.

    llr: this rank's (n_local, N) LLR rows (torch tensor on this rank's device), or the full
         (n_total, N) batch, in which case the rank slices its own range.
    Returns on rank dst: (info bits (n_total, K) int8, status (n_total,) uint8,
    iters (n_total,) int32); None on other ranks."""
    import torch
    import torch.distributed as dist
    from .ldpc_info import code_dims
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    K, N, Nf = code_dims(bgn, Zc)
    if n_total is None:
        n_total = llr.shape[0]
        lo, hi = shard_bounds(n_total, rank, world)
        llr = llr[lo:hi]
    if decode_fn is None:
        from .nr_ldpc_decode import nr_decode_ldpc_batch

        def decode_fn(x):
            return nr_decode_ldpc_batch(x, Zc, bgn, L, "min-sum", alpha, beta, schedule)
    ck, st, it = decode_fn(llr)
    info = ck[:, :K].contiguous()
    st = st.to(torch.uint8)
    it = it.to(torch.int32)
    if world == 1:
        return info, st, it
    g_info = _gather_rows(torch, dist, info, n_total, world, group)
    g_st = _gather_rows(torch, dist, st, n_total, world, group)
    g_it = _gather_rows(torch, dist, it, n_total, world, group)
    if rank != dst:
        return None
    return g_info, g_st, g_it


def decode_tbs_sharded(tbs, decode_tb, group=None, dst=0):
    """Config 5 shape: whole transport blocks round robin across ranks.  decode_tb(tb) ->
    (crc_ok, tb_bits) runs the full per-TB chain (rate recovery, decode, CRCs) locally; the
    (crc_ok, bits) results are gathered to rank dst as Python objects."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mine = {i: decode_tb(tbs[i]) for i in shard_round_robin(len(tbs), rank, world)}
    if world == 1:
        return [mine[i] for i in range(len(tbs))]
    parts = [None] * world
    dist.all_gather_object(parts, {i: (bool(ok), np.asarray(b, np.int8)) for i, (ok, b) in mine.items()},
                           group=group)
    if rank != dst:
        return None
    merged = {}
    for p in parts:
        merged.update(p)
    return [merged[i] for i in range(len(tbs))]
