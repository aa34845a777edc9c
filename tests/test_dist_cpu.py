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
