"""The sharded HIP path with two ranks on one GPU: each rank runs dvcp.DeepVCP +
deepVCP_loss on its dvcp.dist.shard of a C3-shaped batch (N = 16384, K = 64, r = 2.0, s = 0.4,
FE npoint 10000) and the per-pair rows are all_gathered with dvcp.dist.gather_results (gloo, so
both ranks can share cuda:0; the 8-GPU RCCL run is the driver's).  The gathered rows must equal a
single-process run of the whole batch bit for bit, and the job time is the max over ranks."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

P_TOTAL, N, K, R_, S_ = 6, 16384, 64, 2.0, 0.4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model_and_data():
    import dvcp
    from dvcp.synthetic import make_pairs
    src, tgt, R_gt, t_gt = make_pairs(P_TOTAL, N, seed=4242)
    torch.manual_seed(0)
    model = dvcp.DeepVCP(use_normal=False, K=K, r=R_, s=S_).eval()
    torch.manual_seed(1)
    starts = model.draw_starts(P_TOTAL, N, N)   # one draw for the global batch, sharded below
    return model, (src, tgt, R_gt, t_gt), starts


def _run(model, data, starts, dev):
    import dvcp
    from dvcp import dist as D
    src, tgt, R_gt, t_gt = (x.to(dev) for x in data)
    with torch.no_grad():
        kp, vcp = model(src, tgt, R_gt, torch.zeros(1, 3), starts=starts)
        _, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt, t_gt, 0.5)
    return D.pack_results(R, t)


def _worker(rank, world, port, q):
    import sys
    import time
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import torch.distributed as dist

    from dvcp import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        model, data, starts = _model_and_data()
        model.to(dev)
        a, b = D.shard(P_TOTAL, rank, world)
        dist.barrier()
        t0 = time.perf_counter()
        rows = _run(model, tuple(x[a:b] for x in data), starts[:, a:b], dev)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        gathered = D.gather_results(rows.cpu(), world)
        tmax = D.max_over_ranks(elapsed, torch.device("cpu"))
        if rank == 0:
            q.put((gathered, tmax, elapsed))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_equal_single_process(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        rows, tmax, t0 = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    model, data, starts = _model_and_data()
    want = _run(model.to(cuda), data, starts, cuda).cpu()
    assert rows.shape == want.shape == (P_TOTAL, 12)
    assert torch.equal(rows, want), float((rows - want).abs().max())
    assert tmax >= t0
