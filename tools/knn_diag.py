"""kNN per-wave diagnostics from a DVCP_KNN_DIAG build (dvcp/libdvcp_hip_D.so copied over the
in-tree library by tools/gpu_r3_knndiag.sh): on the C3 shape of tools/knn_bench.py, each wave's
lane-0 row carries [tiles scanned, tiles with an active lane, merges, appends (all lanes), clk,
clk in merges, tiles in the cloud].  Prints their distribution.  Diagnostics only."""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    from dvcp import ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(8, 16384, seed=1234)
    g = torch.Generator().manual_seed(0)
    sel = torch.stack([torch.randperm(16384, generator=g)[:10000] for _ in range(8)])
    ref = torch.gather(tgt, 2, sel.unsqueeze(1).expand(-1, 3, -1)).to(dev).contiguous()
    kp = torch.gather(src, 2, sel[:, :64].unsqueeze(1).expand(-1, 3, -1)).permute(0, 2, 1)
    ax = torch.arange(-2.0, 2.0001, 0.4)
    off = torch.tensor(list(itertools.product(ax.tolist(), repeat=3)), dtype=torch.float32)
    qry = (kp[:, :, None, :] + off[None, None]).reshape(8, -1, 3).to(dev).contiguous()
    dist, idx, _ = ops.knn(ref, qry, 32, ref_pdim=2, qry_pdim=1, want_idx64=False, method="tiled")
    torch.cuda.synchronize()
    d = dist.cpu().numpy().reshape(-1, 32)
    rows = d[d[:, 31] == -12345.0][:, :7]
    names = ["scanned", "active", "merges", "appends", "clk", "merge_clk", "skip_clk"]
    print(f"waves {len(rows)}")
    for i, n in enumerate(names):
        v = rows[:, i]
        print(f"{n:10s} mean {v.mean():12.1f}  p50 {np.percentile(v, 50):12.1f}  p90 {np.percentile(v, 90):12.1f}  "
              f"max {v.max():12.1f}  sum {v.sum():14.1f}")
    print(f"merge share of wave clk {rows[:, 5].sum() / rows[:, 4].sum():.3f}")
    print(f"skipped-tile share of wave clk {rows[:, 6].sum() / rows[:, 4].sum():.3f}, "
          f"clk per skipped tile {rows[:, 6].sum() / (rows[:, 0].sum() - rows[:, 1].sum()):.1f}")
    print(f"appends per active tile per lane {rows[:, 3].sum() / rows[:, 1].sum() / 64:.3f}")
    # by distance of the wave's first query from the cloud centre
    q = qry.cpu().numpy().reshape(-1, 3)
    print("clk of the slowest 1% of waves", np.percentile(rows[:, 4], 99), "median", np.percentile(rows[:, 4], 50))


if __name__ == "__main__":
    main()
