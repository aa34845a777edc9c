"""The N>1 layout on CPU: 2 gloo ranks shard the pairs, run the pose solve on their shard and
all_gather the results; the gathered rows must equal a single-process run bit for bit, and the
job time is the max over ranks."""
import os
import socket

import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle as O
    from dvcp import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    P = 7
    x = torch.rand(P, 64, 3, generator=g, dtype=torch.float64)
    y = (x + 0.01 * torch.randn(P, 64, 3, generator=g, dtype=torch.float64)).float()
    Rt = torch.eye(3, dtype=torch.float64).expand(P, 3, 3)
    tt = torch.zeros(P, 3, 1, dtype=torch.float64)
    a, b = D.shard(P, rank, world)
    _, R, t = O.deepVCP_loss(x[a:b], y[a:b], Rt[a:b], tt[a:b], 0.5)
    rows = D.gather_results(D.pack_results(R, t), world)
    tmax = D.max_over_ranks(float(rank + 1), torch.device("cpu"))
    if rank == 0:
        q.put((rows, tmax))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather():
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import oracle as O
    from dvcp import dist as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rows, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(0)
    P = 7
    x = torch.rand(P, 64, 3, generator=g, dtype=torch.float64)
    y = (x + 0.01 * torch.randn(P, 64, 3, generator=g, dtype=torch.float64)).float()
    _, R, t = O.deepVCP_loss(x, y, torch.eye(3, dtype=torch.float64).expand(P, 3, 3),
                             torch.zeros(P, 3, 1, dtype=torch.float64), 0.5)
    want = D.pack_results(R, t)
    assert rows.shape == want.shape
    torch.testing.assert_close(rows, want, rtol=0, atol=1e-12)
    assert tmax == 2.0


def test_shard_covers_everything():
    from dvcp import dist as D
    for total in (0, 1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            spans = [D.shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1


# ---- bench.py's sharded workload (dvcp.dist.ShardPlan) -------------------------------------
# A sharded run must compute, on every rank, rows [lo, hi) of what one process computes for the
# same global batch: same data shard, same weights, same FPS starts.  Small C3-like sizes so the
# oracle (the CPU restatement; no GPU here) runs each pair in about a second.
_PN, _PK, _PNPT, _PSTEPS = 1024, 32, 256, 2   # K >= the key-point group's 32 neighbours


def _plan_model(plan):
    """bench.py's model construction on CPU: seed 0, randomised BN, weighting layer calibrated on
    the plan's calibration cloud (the oracle's FE stands in for FE1.run, with the three FPS starts
    FE1.run would draw)."""
    import oracle as O
    import dvcp
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn
    torch.manual_seed(0)
    model = dvcp.DeepVCP(use_normal=False, K=_PK, r=1.0, s=0.4, fe_npoint=_PNPT).eval()
    randomize_bn(model)
    cal = plan.calibration_src(_PN, make_pairs)
    st = [torch.randint(0, n, (1,), dtype=torch.long) for n in (_PN, _PNPT, _PNPT)]
    ref = O.DeepVCP(use_normal=False, K=_PK, r=1.0, s=0.4, fe_npoint=_PNPT).eval()
    ref.load_state_dict(model.state_dict())
    with torch.no_grad(), O.fps_starts(st):
        _, feats = ref.FE1(cal)
    condition_weights(model, feats=feats)
    torch.manual_seed(1)
    return model


def _plan_rows(plan):
    """(steps, pairs of this rank, 12) oracle rows of bench.py's step loop (two lanes alternating)."""
    import oracle as O
    from dvcp import dist as D
    from dvcp.synthetic import make_pairs
    model = _plan_model(plan)
    ref = O.DeepVCP(use_normal=False, K=_PK, r=1.0, s=0.4, fe_npoint=_PNPT).eval()
    ref.load_state_dict(model.state_dict())
    lanes = [plan.lane_pairs(lane, _PN, make_pairs) for lane in range(2)]
    out = []
    for i in range(_PSTEPS):
        src, tgt, R, t = lanes[i % 2]
        starts = plan.starts(model, _PN)
        with torch.no_grad(), O.fps_starts(list(starts)):
            kp, vcp = ref(src, tgt, R, torch.zeros(1, 3))
            _, Rp, tp = O.deepVCP_loss(kp, vcp, R, t, 0.5)
        out.append(D.pack_results(Rp, tp))
    return torch.stack(out)


def _plan_worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import torch.distributed as dist

    from dvcp import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = D.ShardPlan(2, world, rank)
        rows = _plan_rows(plan)                                     # (steps, 2, 12)
        flat = D.gather_results(rows.reshape(-1, 12), world)        # rank order
        if rank == 0:
            q.put(flat.reshape(world, _PSTEPS, 2, 12).permute(1, 0, 2, 3).reshape(_PSTEPS, 2 * world, 12))
        dist.barrier()
    except Exception:
        import traceback
        q.put(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def test_shard_plan_inputs_are_rank_independent():
    """Data shards, FPS starts and the calibration cloud of a world-2 plan are exactly the world-1
    plan's for the same global batch, split by rank (no oracle run needed)."""
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dvcp
    from dvcp import dist as D
    from dvcp.synthetic import make_pairs
    whole = D.ShardPlan(4, 1, 0)
    parts = [D.ShardPlan(2, 2, r) for r in range(2)]
    for lane in range(3):
        w = whole.lane_pairs(lane, 512, make_pairs)
        ps = [p.lane_pairs(lane, 512, make_pairs) for p in parts]
        for k in range(4):
            assert torch.equal(w[k], torch.cat([p[k] for p in ps]))
    assert all(torch.equal(whole.calibration_src(512, make_pairs), p.calibration_src(512, make_pairs)) for p in parts)
    # the calibration cloud is global pair 0's source whatever the global batch size
    assert torch.equal(whole.calibration_src(512, make_pairs), make_pairs(8, 512, seed=D.ShardPlan.lane_seed(0))[0][:1])
    model = dvcp.DeepVCP(use_normal=False, K=16, r=1.0, s=0.4, fe_npoint=256)
    torch.manual_seed(1)
    sw = [whole.starts(model, 512) for _ in range(3)]
    got = []
    for p in parts:
        torch.manual_seed(1)
        got.append([p.starts(model, 512) for _ in range(3)])
    for i in range(3):
        assert torch.equal(sw[i], torch.cat([g[i] for g in got], 1))


def test_bench_plan_world2_rows_equal_world1():
    """bench.py's sharded workload at world 2 (gloo) gives, pair for pair, the rows of a world-1 run
    of the same global batch: weights conditioned identically on every rank, FPS starts drawn for
    the global batch -- computed here by the oracle (round 4's bench calibrated per shard and
    seeded the starts by rank, so its ranks ran different models)."""
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    from dvcp import dist as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rows2 = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert not isinstance(rows2, str), rows2
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    rows1 = _plan_rows(D.ShardPlan(4, 1, 0))
    assert rows1.shape == rows2.shape == (_PSTEPS, 4, 12)
    assert torch.equal(rows1, rows2)
