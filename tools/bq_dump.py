"""Dump the ball-query count output for the three C3 layers (diagnostic builds put per-wave
figures there) to gpurun_out/<tag>.pt."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    tag = sys.argv[1]
    from dvcp import ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(8, 16384, seed=1234)
    xyz = torch.cat([src, tgt]).to(dev)
    if xyz.shape[1] == 3:
        xyz = xyz.transpose(1, 2)
    xyz = xyz[..., :3].contiguous()
    idx, _ = ops.fps(xyz, 10000, torch.zeros(16, dtype=torch.int64, device=dev), pdim=1)
    c1 = torch.gather(xyz, 1, idx.unsqueeze(-1).expand(-1, -1, 3)).contiguous()
    out = {"c1": c1.cpu(), "xyz": xyz.cpu()}
    for name, pts, ctr, r, ns in [("sa1", xyz, c1, 0.1, 256), ("sa2", c1, c1, 0.2, 128), ("sa3", c1, c1, 0.4, 64)]:
        for _ in range(3):
            cnt, _, _ = ops.ball_query(pts, ctr, r, ns)
        torch.cuda.synchronize()
        out[name] = cnt.cpu()
    torch.save(out, os.path.join(os.path.dirname(__file__), "..", "gpurun_out", tag + ".pt"))


if __name__ == "__main__":
    main()
