"""Paired-FPS diagnostics (build with -DDVCP_FPS_PAIR_DIAG=3): per cloud, layer 3's count of
re-ranked (tied) rounds and the gated-recomputation flag, at the C3 layer-2 shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepvcp-pointcloud-registration_amd"))


def main():
    from dvcp import _lib, ops
    from dvcp.synthetic import make_pairs
    dev = torch.device("cuda", 0)
    src, tgt, _, _ = make_pairs(8, 16384, seed=1234)
    xyz = torch.cat([src, tgt]).to(dev).contiguous()
    B = xyz.shape[0]
    _, c1 = ops.fps(xyz, 10000, torch.zeros(B, dtype=torch.long, device=dev), pdim=2)
    c1 = c1.contiguous()
    N = c1.shape[2]
    for s3v in (0, N - 1):
        s2 = torch.zeros(B, dtype=torch.long, device=dev)
        s3 = torch.full((B,), s3v, dtype=torch.long, device=dev)
        i2 = torch.empty(B, N, dtype=torch.long, device=dev)
        i3 = torch.empty_like(i2)
        c2 = torch.empty(B, 3, N, device=dev)
        c3 = torch.empty_like(c2)
        ws = torch.empty(int(_lib.load().dvcp_fps_pair_workspace_bytes(B, N)) // 4, dtype=torch.int32, device=dev)
        _lib.call("dvcp_fps_pair", 0, _lib.ptr(c1), 3 * N, N, 1, B, N, _lib.ptr(s2), _lib.ptr(s3), _lib.ptr(i2),
                  _lib.ptr(c2), _lib.ptr(i3), _lib.ptr(c3), _lib.ptr(ws), _lib.stream())
        torch.cuda.synchronize()
        sl = ws[1:1 + B].tolist()
        print(f"start3={s3v}: re-ranked rounds per cloud {[v & 0xFF for v in sl]}  their clocks (x1024) "
              f"{[(v >> 8) & 0xFFFFFF for v in sl]}  flags {ws[1 + B:1 + 2 * B].tolist()}", flush=True)


if __name__ == "__main__":
    main()
