"""Split-select FPS micro-benchmark (round 6): C3's FE chain -- 16 clouds of 16384 points -> 10000
centres (sa1), then those 10000 -> 10000 (sa2 / sa3) -- with 1, 2, 4 and 8 workgroups per cloud.
Prints ms per launch (HIP events, median of 5) and whether the indices equal the one-workgroup
kernel's (FPS is exact: they must).

    python tools/fps_parts_bench.py [--parts 1,2,4,8] [--reps 5]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), min(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dvcp import _lib, ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(8, 16384, seed=1234)
    xyz = torch.cat([src, tgt]).to(dev).contiguous()  # (16, 3, N)
    B = xyz.shape[0]
    start = torch.randint(0, 16384, (B,), generator=torch.Generator().manual_seed(7)).to(dev)
    _, c1 = ops.fps(xyz, 10000, start, pdim=2, parts=1)
    c1 = c1.contiguous()
    s2 = torch.randint(0, 10000, (B,), generator=torch.Generator().manual_seed(8)).to(dev)
    ref = {"sa1": ops.fps(xyz, 10000, start, pdim=2, parts=1)[0], "sa2": ops.fps(c1, 10000, s2, pdim=2, parts=1)[0]}
    for parts in [int(p) for p in a.parts.split(",")]:
        for name, pts, st in (("sa1 16384->10000", xyz, start), ("sa2 10000->10000", c1, s2)):
            med, mn, out = timed(lambda: ops.fps(pts, 10000, st, pdim=2, parts=parts)[0], a.reps)
            same = torch.equal(out, ref[name[:3]])
            print(f"parts {parts}  {name}: {med:.4f} ms/launch (min {mn:.4f})  equal to 1 WG: {same}", flush=True)
    _lib.check_device_flags(block=True)


if __name__ == "__main__":
    main()
