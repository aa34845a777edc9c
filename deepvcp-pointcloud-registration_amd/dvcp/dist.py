"""Multi-GPU layout: one process per GPU, cloud pairs sharded, no data-path collective.

Pairs are independent in eval mode, so a global batch of P pairs is split
into contiguous per-rank shards and every rank runs the full hot path on its shard.  The only
collective is one all_gather of the per-pair results (R 9 + t 3 fp64) at the end -- a few KB,
latency-bound over xGMI (backend "nccl" = RCCL on ROCm), or gloo on CPU for tests.
"""
import torch
import torch.distributed as dist

# bench.py's synthetic data: lane L's global batch is make_pairs(P, N, seed=LANE_SEED0 + LANE_STRIDE * L)
LANE_SEED0, LANE_STRIDE = 1234, 104729


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


class ShardPlan:
    """What every rank of a sharded run uses (bench.py), chosen so that rank r's rows equal rows
    [lo, hi) of a single-process run of the same global batch, bit for bit:

    * data: in-flight lane L's global batch of P = pairs_per_rank x world pairs is one
      ``make_pairs(P, N, seed(L))`` draw on every rank; each rank takes its ``shard``;
    * weights: the same seed on every rank, and the weighting layer's calibration
      (``synthetic.condition_weights``) runs on ``calibration_src`` -- global pair 0 of lane 0, whose
      points do not depend on P (make_pairs draws every source cloud before any pose) -- so the
      model is the same whatever the world size and whichever rank holds pair 0;
    * FPS starts: every rank draws the seven start vectors for the whole global batch from the
      same CPU generator state (``starts``), in the reference's order, and keeps its columns.
      Every rank makes the same draws in the same order, so step i's starts are the global
      batch's whatever the world size.
    (The round-4 bench calibrated on each rank's own shard and seeded the starts with 1 + rank,
    so an N-GPU run used N different models and could not be checked against one GPU.)"""

    def __init__(self, pairs_per_rank, world=1, rank=0):
        self.pairs_per_rank, self.world, self.rank = int(pairs_per_rank), int(world), int(rank)
        self.total = self.pairs_per_rank * self.world
        self.lo, self.hi = shard(self.total, self.rank, self.world)

    @staticmethod
    def lane_seed(lane):
        return LANE_SEED0 + LANE_STRIDE * int(lane)

    def lane_pairs(self, lane, n_points, make_pairs):
        """(src, tgt, R, t) of this rank's shard of lane ``lane``'s global batch (CPU tensors)."""
        full = make_pairs(self.total, n_points, seed=self.lane_seed(lane))
        return tuple(x[self.lo:self.hi].contiguous() for x in full)

    def calibration_src(self, n_points, make_pairs):
        """(1, C, N) source cloud of global pair 0 of lane 0: the same on every rank and world size."""
        return make_pairs(1, n_points, seed=self.lane_seed(0))[0]

    def starts(self, model, n_points):
        """This rank's columns of the global batch's seven FPS start vectors (call on every rank
        for every step, in the same order)."""
        return model.draw_starts(self.total, n_points, n_points)[:, self.lo:self.hi].contiguous()
