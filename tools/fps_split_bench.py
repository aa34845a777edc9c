"""Split-FPS micro-benchmark at the C5 shape: 4 clouds (2 pairs) of 65536 points -> 10000 centres.
Prints ms per dvcp_fps call (CUDA events, median of 3) and an index checksum."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    from dvcp import ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(2, 65536, seed=1234)
    xyz = torch.cat([src, tgt]).to(dev).contiguous()
    start = torch.zeros(xyz.shape[0], dtype=torch.long, device=dev)
    i, _ = ops.fps(xyz, 10000, start, pdim=2)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        i, _ = ops.fps(xyz, 10000, start, pdim=2)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"split fps 65536 -> 10000 x{xyz.shape[0]}: {statistics.median(ts):.3f} ms/call  idx checksum {int(i.sum())}",
          flush=True)


if __name__ == "__main__":
    main()
