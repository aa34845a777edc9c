"""FPS latency probe: ms per launch and us per serial step across cloud sizes (diagnostics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepvcp-pointcloud-registration_amd"))
import torch  # noqa: E402

from dvcp import ops  # noqa: E402


def run(B, N, npoint, reps=3):
    g = torch.Generator().manual_seed(0)
    xyz = (torch.rand(B, 3, N, generator=g) * 2 - 1).cuda()
    start = torch.zeros(B, dtype=torch.int64).cuda()
    ops.fps(xyz, npoint, start, pdim=2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        idx, _ = ops.fps(xyz, npoint, start, pdim=2)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, idx


if __name__ == "__main__":
    tag = os.environ.get("DVCP_FPS_NOPRUNE", "0")
    for B, N, npoint in [(16, 1024, 10000), (16, 4096, 10000), (16, 10000, 10000), (16, 16384, 10000),
                         (16, 16384, 1000), (1, 16384, 10000), (64, 16384, 10000)]:
        ms, idx = run(B, N, npoint)
        print(f"noprune={tag} B={B:3d} N={N:6d} npoint={npoint:6d}: {ms:8.3f} ms/launch  {ms * 1e3 / npoint:6.3f} us/step",
              flush=True)
