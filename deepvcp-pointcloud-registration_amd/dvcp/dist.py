"""Multi-GPU layout: one process per GPU, cloud pairs sharded, no data-path collective.

Pairs are independent in eval mode, so a global batch of P pairs is split
into contiguous per-rank shards and every rank runs the full hot path on its shard.  The only
collective is one all_gather of the per-pair results (R 9 + t 3 fp64) at the end -- a few KB,
latency-bound over xGMI (backend "nccl" = RCCL on ROCm), or gloo on CPU for tests.
"""
import torch
import torch.distributed as dist


def shard(total, rank, world):
    """Contiguous [start, end) of `total` pairs for `rank` (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack_results(R, t):
    """(B, 3, 3), (B, 3, 1) -> (B, 12) fp64 rows."""
    return torch.cat([R.reshape(-1, 9), t.reshape(-1, 3)], 1).double()


def gather_results(rows, world=None):
    """all_gather per-rank (B_r, 12) result rows into the global (sum B_r, 12), rank order.
    Shards may differ in size by one, so rows are padded to the max and trimmed."""
    world = world or (dist.get_world_size() if dist.is_initialized() else 1)
    if world == 1:
        return rows
    n = torch.tensor([rows.shape[0]], device=rows.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s) for s in sizes))
    pad = torch.zeros(m, rows.shape[1], dtype=rows.dtype, device=rows.device)
    pad[: rows.shape[0]] = rows
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(s)] for b, s in zip(bufs, sizes)])


def max_over_ranks(seconds, device):
    """The job's time is its slowest rank's."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
