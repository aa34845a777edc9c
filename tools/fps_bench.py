"""FPS micro-benchmark at the C3 shapes: 16 clouds (8 pairs) of 16384 points -> 10000 centres
(sa1), then those centres -> 10000 (sa2 / sa3: a full FPS order; serial and paired).  Prints ms per call
(CUDA events, median of 5) and a checksum of the indices (identical across builds: FPS is exact)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    from dvcp import ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(8, 16384, seed=1234)
    xyz = torch.cat([src, tgt]).to(dev).contiguous()  # (16, 3, N)
    B = xyz.shape[0]
    start = torch.zeros(B, dtype=torch.long, device=dev)
    _, c1 = ops.fps(xyz, 10000, start, pdim=2)
    for name, pts in (("sa1", xyz), ("sa2", c1.contiguous())):
        for _ in range(2):
            i, _ = ops.fps(pts, 10000, start, pdim=2)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            i, _ = ops.fps(pts, 10000, start, pdim=2)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"{name}: {statistics.median(ts):.4f} ms/call (min {min(ts):.4f})  idx checksum {int(i.sum())}",
              flush=True)
    # layers 2 + 3: two serial launches against the paired launch, start3 at 0, N/4, N/2, N - 1
    c1 = c1.contiguous()
    N = c1.shape[2]
    for s3v in (0, N // 4, N // 2, N - 1):
        s3 = torch.full((B,), s3v, dtype=torch.long, device=dev)
        res = {}
        for mode in ("serial", "pair"):
            def run():
                if mode == "pair":
                    return ops.fps_pair(c1, start, s3, pdim=2)[2]
                _, c2 = ops.fps(c1, N, start, pdim=2)
                return ops.fps(c2, N, s3, pdim=2)[0]
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                i3 = run()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[mode] = (statistics.median(ts), int(i3.sum()))
        print(f"sa2+sa3 start3={s3v}: serial {res['serial'][0]:.4f} ms, pair {res['pair'][0]:.4f} ms  "
              f"idx3 checksum {res['serial'][1]} / {res['pair'][1]}", flush=True)


if __name__ == "__main__":
    main()
