"""Multi-GPU sharding of one block.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank
r owns the byte range [begin_r, end_r) of the block -- i.e. candidate positions
(begin_r, end_r] -- and reads up to YR_MAX_ATOM_LENGTH bytes before begin_r as
warm-up (libyara's trie is at most 4 deep, limits.h:68), so no data-path
exchange is needed.  The only collective is the final gather of the per-rank
candidate lists to rank 0; concatenated in rank order they are exactly the
full block's ascending candidate stream.
"""
import torch
import torch.distributed as dist

# halo kept in front of a shard: >= YR_MAX_ATOM_LENGTH (4) and a multiple of 16
# so the shard's first byte stays 16-byte aligned for the scan kernel
HALO = 16


def shard_bounds(n: int, world: int, rank: int, align: int = 1 << 20):
    """Byte range [begin, end) of `rank`: equal `align`-multiple slices, the
    last rank takes the remainder (and therefore position n)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    if align % 16:
        raise ValueError("align must be a multiple of 16")
    per = (n // world) // align * align
    begin = rank * per
    end = n if rank == world - 1 else begin + per
    return begin, end


def local_window(begin: int, end: int):
    """(first byte a rank must hold, byte offset of its shard inside it)."""
    halo = min(HALO, begin)
    return begin - halo, halo


def gather_positions(local: torch.Tensor, group=None, dst: int = 0):
    """Gather every rank's ascending int64 candidate positions to `dst`.

    all_gather of the counts, then one padded gather (payloads are KB-MB, far
    below what the xGMI links move per microsecond).  Returns the rank-ordered
    concatenation on `dst`, None elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if dist.get_backend(group) == "gloo":
        local = local.cpu()                  # gloo collectives run on host tensors
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    counts_t = torch.empty(world, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(counts_t, n, group=group)
    counts = counts_t.tolist()               # one host sync for all ranks' counts
    width = max(max(counts), 1)
    if local.numel() == width:
        padded = local.contiguous()
    else:
        padded = torch.empty((width,), dtype=torch.int64, device=local.device)
        padded[:local.numel()] = local
        padded[local.numel():] = -1
    global _GATHER_OK
    if _GATHER_OK:
        bufs = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
        try:
            dist.gather(padded, bufs, dst=dst, group=group)
        except RuntimeError:   # a backend without gather: every rank takes the same branch
            _GATHER_OK = False
    if not _GATHER_OK:
        flat = torch.empty(world * width, dtype=torch.int64, device=local.device)
        dist.all_gather_into_tensor(flat, padded, group=group)
        bufs = list(flat.view(world, width))
    if rank != dst:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


_GATHER_OK = True
