"""Multi-GPU sharding of one block.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank
r owns the byte range [begin_r, end_r) of the block -- i.e. candidate positions
(begin_r, end_r] (rank 0 also position 0) -- and holds a WINDOW of the block
around it in HBM:

  * candidates only: 4 bytes before begin_r (libyara's trie is at most 4 deep,
    limits.h:68, so the walk restarts exactly there);
  * verification-complete (the default): the tables' verify halos
    (yr_amd_tables_info: max backtrack + YR_RE_SCAN_LIMIT before, max(
    YR_RE_SCAN_LIMIT, 2 x longest string) after), so yr_amd_verify_device
    decides every verify call of the rank's candidates exactly as on the whole
    block (literal comparisons, regexp scans of up to 4096 bytes each way,
    limits.h:162-163).

yr_amd_scan_window addresses the window by block positions, so candidates and
records come out block-global.  No data-path exchange; the only collective is
the final gather to rank 0 of either the candidate lists or the pre-verified
{offset, pool index} records (every verify call that can have an effect, the
rest dropped on the device), concatenated in rank order = exactly the whole
block's stream.
"""
import torch
import torch.distributed as dist

WARMUP = 4        # YR_MAX_ATOM_LENGTH


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


def shard_window(n: int, begin: int, end: int, halo_before: int = WARMUP, halo_after: int = 0):
    """[lo, hi): the bytes of the block a rank holds for the shard [begin, end):
    halo_before bytes in front (lo rounded down to 16 for the kernels'
    alignment), halo_after behind, clipped to the block."""
    if not 0 <= begin <= end <= n:
        raise ValueError("bad shard")
    lo = max(0, begin - max(halo_before, WARMUP)) // 16 * 16
    hi = min(n, end + halo_after)
    return lo, hi


def tables_halos(tables):
    """(halo_before, halo_after) a verification-complete shard needs
    (yr_amd_tables_get_info)."""
    info = tables.info()
    return int(info["verify_halo_before"]), int(info["verify_halo_after"])


def _gather_backend(group):
    """Gather strategy, chosen from the backend up front (every rank takes the
    same branch, so no rank is left waiting in a collective another abandoned):
    nccl (RCCL) and gloo implement gather; anything else all-gathers."""
    return "gather" if dist.get_backend(group) in ("nccl", "gloo") else "all_gather"


def gather_rows(local: torch.Tensor, group=None, dst: int = 0, split: bool = False,
                error: str = None):
    """Gather every rank's int64 rows [m_r, w] to `dst`: all_gather of the
    counts, one padded gather (payloads are KB-MB, far below what the xGMI
    links move per microsecond).  Returns the rank-ordered concatenation on
    `dst` (with ``split``: the list of every rank's rows), None elsewhere.

    ``error``: this rank's input is bad.  The rank still enters the counts
    all-gather, with a count of -1, so EVERY rank learns of it there and
    raises ValueError together -- none is left waiting in the payload gather."""
    if local.dim() != 2 or local.dtype not in (torch.int64, torch.int32):
        raise ValueError("rows must be a 2-d int64 or int32 tensor")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if dist.get_backend(group) == "gloo":
        local = local.cpu()                  # gloo collectives run on host tensors
    w = local.shape[1]
    n = torch.tensor([-1 if error else local.shape[0]], dtype=torch.int64, device=local.device)
    counts_t = torch.empty(world, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(counts_t, n, group=group)
    counts = counts_t.tolist()               # one host sync for all ranks' counts
    if min(counts) < 0:
        bad = [r for r, c in enumerate(counts) if c < 0]
        raise ValueError(error if error else "rank(s) %s reported bad input to the gather" % bad)
    width = max(max(counts), 1)
    if local.shape[0] == width:
        padded = local.contiguous()
    else:
        padded = torch.full((width, w), -1, dtype=local.dtype, device=local.device)
        padded[:local.shape[0]] = local
    if _gather_backend(group) == "gather":
        bufs = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
        dist.gather(padded, bufs, dst=dst, group=group)
    else:
        flat = torch.empty((world * width, w), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(flat, padded, group=group)
        bufs = list(flat.view(world, width, w))
    if rank != dst:
        return None
    if split:
        return [b[:c] for b, c in zip(bufs, counts)]
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def gather_positions(local: torch.Tensor, group=None, dst: int = 0, begins=None, end=None):
    """Gather every rank's ascending int64 candidate positions to `dst`.

    With ``begins`` (every rank's shard begin) and ``end`` (the block size, the
    last rank's end) each rank sends its positions as 32-bit offsets from its
    own base -- half the bytes over the links -- and `dst` restores them.  Rank
    r's positions lie in (begin_r, end_r] (rank 0: [0, end_0]), so the base is
    begin_r + 1 (rank 0: 0) and a shard of at most 2^32 positions fits.  If any
    shard is larger, every rank takes the int64 gather instead (the decision is
    made from the arguments alone, so all ranks take the same branch)."""
    if begins is None:
        out = gather_rows(local.reshape(-1, 1).to(torch.int64), group, dst)
        return None if out is None else out.reshape(-1)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(begins) != world:
        raise ValueError("one shard begin per rank")
    if end is None:
        raise ValueError("gather_positions(begins=...) needs the block size (end)")
    ends = list(begins[1:]) + [end]
    bases = [0] + [b + 1 for b in begins[1:]]
    # positions of rank r: [bases[r], ends[r]] -- offsets up to ends[r] - bases[r]
    if any(e - b > 0xFFFFFFFF for b, e in zip(bases, ends)):
        out = gather_rows(local.reshape(-1, 1).to(torch.int64), group, dst)
        return None if out is None else out.reshape(-1)
    loc = local.to(torch.int64)
    error = None
    if loc.numel() and (int(loc.min()) < bases[rank] or int(loc.max()) > ends[rank]):
        # raised inside gather_rows, on every rank at once (a rank raising
        # here alone would leave the others waiting in the collective)
        error = "rank %d: positions outside its shard [%d, %d]" % (rank, bases[rank], ends[rank])
    off = (loc - bases[rank]).to(torch.int32)   # (wraps past 2^31; restored below)
    rows = gather_rows(off.reshape(-1, 1), group, dst, split=True, error=error)
    if rows is None:
        return None
    return torch.cat([(part.reshape(-1).to(torch.int64) & 0xFFFFFFFF) + bases[r]
                      for r, part in enumerate(rows)])


def records_to_rows(d_records: int, count: int, device) -> torch.Tensor:
    """Device yr_amd_verify_rec[count] -> int64 rows [count, 2] = {offset,
    pool index} (the record's 32-bit candidate index is local to the shard's
    stream and dropped)."""
    from ._hip import memcpy
    rows = torch.empty((max(count, 1), 2), dtype=torch.int64, device=device)
    memcpy(rows.data_ptr(), d_records, count * 16, 3)      # D2D, 16 B per record
    rows = rows[:count]
    rows[:, 1] &= 0xFFFFFFFF
    return rows
