"""CPG phase clocks from a DVCP_CPG_DIAG build (pass its path with --lib): wave 0 of each workgroup
records the shader clock at the phase boundaries of cpg_kernel (load the target block; per
8-channel quarter: zero the images, build the cost pieces, conv1 MFMA; conv1 output; conv2; conv3 +
softmax + weighted mean) on the C3 shape (8 x 64 key points, G = 11).  Diagnostics only."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    a = ap.parse_args()
    from dvcp import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import dvcp
    from dvcp import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    B, K, G = 8, 64, 11
    C = G ** 3
    cpg = dvcp.cpg().eval().to(dev)
    src = torch.randn(B, K, 32, generator=g).to(dev)
    tgt = torch.randn(B, K, C, 32, generator=g).to(dev)
    cand = torch.randn(B, K, C, 3, generator=g).to(dev)
    for _ in range(3):
        v, w = ops.cpg(src, tgt.permute(0, 1, 3, 2), cand, G, cpg.packed_params(), want_weight=True)
    torch.cuda.synchronize()
    d = w.reshape(B * K, C)[:, :17].cpu().numpy().astype(np.float64)
    names = ["load"] + [f"q{q} {x}" for q in range(4) for x in ("zero", "build", "mfma")] + ["out1", "conv2", "rest", "total"]
    for i, n in enumerate(names):
        col = d[:, i]
        print(f"{n:12s} mean {col.mean():10.0f}  p50 {np.percentile(col, 50):10.0f}  p90 {np.percentile(col, 90):10.0f}")


if __name__ == "__main__":
    main()
