"""Timeline of one single-batch C3 step (the bench's latency measurement), kernel by kernel.

Diagnostic for the serial chain: every library launch carries HIP events (``_lib.EVENT_LOG``) on
the stream it runs on; offsets are taken from one event recorded on the lane stream before the
step.  Prints each launch's start / end / duration and the idle gaps of the union of busy
intervals (host issue, torch glue kernels and waits show up as gaps).

    python tools/latency_timeline.py [--parts 0 8] [--reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepvcp-pointcloud-registration_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "24")

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--parts", type=int, nargs="+", default=[0, 8])
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--npoints", type=int, default=16384)
    p.add_argument("--K", type=int, default=64)
    p.add_argument("--cprofile", action="store_true", help="host profile of one step (cProfile, tottime)")
    p.add_argument("--serial-fe", action="store_true",
                   help="run the extractor's side-stream work on the lane stream (FPS launches alone)")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import dvcp
    from dvcp import _lib
    from dvcp import dist as D
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn

    B, N = args.batch, args.npoints
    plan = D.ShardPlan(B, 1, 0)
    torch.manual_seed(0)
    model = dvcp.DeepVCP(use_normal=False, K=args.K, r=2.0, s=0.4).eval().to(dev)
    src, tgt, R, t = (x.to(dev) for x in plan.lane_pairs(0, N, make_pairs))
    randomize_bn(model)
    with torch.no_grad():
        _, calib, _ = model.FE1.run(plan.calibration_src(N, make_pairs).to(dev))
    condition_weights(model, feats=calib)
    t_init = torch.zeros(1, 3)
    lane = torch.cuda.Stream(device=dev)
    if args.serial_fe:
        model._side_stream = lambda d: torch.cuda.current_stream(d)

    host = []   # (label, perf_counter) of the step's host issue
    from dvcp import ops
    _fps = ops.fps

    def fps_timed(*a, **k):
        host.append(("fps enter", time.perf_counter()))
        r = _fps(*a, **k)
        host.append(("fps return", time.perf_counter()))
        return r
    ops.fps = fps_timed

    def step(base=None):
        starts = plan.starts(model, N)
        host.clear()
        with torch.no_grad(), torch.cuda.stream(lane):
            if base is not None:
                base.record()
            host.append(("base", time.perf_counter()))
            kp, vcp = model(src, tgt, R, t_init, starts=starts)
            loss, Rp, tp = dvcp.deepVCP_loss(kp, vcp, R, t, 0.5)
            dvcp.registration_errors(Rp, tp, R, t)
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            host.append(("end", time.perf_counter()))
        return end

    for parts in args.parts:
        model.FE1.fps_parts = parts or None
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        for rep in range(args.reps):
            base = torch.cuda.Event(enable_timing=True)
            _lib.EVENT_LOG = []
            end = step(base)
            torch.cuda.synchronize()
            log, _lib.EVENT_LOG = _lib.EVENT_LOG, None
            total = base.elapsed_time(end)
            rows = sorted((base.elapsed_time(e0), base.elapsed_time(e1), name) for name, e0, e1, _ in log)
            print(f"== parts={parts} rep={rep}: step {total:.3f} ms (base -> end event on the lane)")
            print("  host issue (ms after base): " + ", ".join(f"{lb} {(t1 - host[0][1]) * 1e3:.3f}" for lb, t1 in host))
            busy_end, idle = 0.0, []
            for s0, s1, name in rows:
                if s0 > busy_end + 0.005:
                    idle.append((busy_end, s0))
                busy_end = max(busy_end, s1)
                if rep == args.reps - 1:
                    print(f"  {s0:8.3f} {s1:8.3f} {s1 - s0:7.3f}  {name}")
            if total > busy_end + 0.005:
                idle.append((busy_end, total))
            print(f"  idle gaps > 5 us: {sum(b - a for a, b in idle):.3f} ms in {len(idle)}: "
                  + ", ".join(f"{a:.2f}+{b - a:.3f}" for a, b in idle[:24]))
        if args.cprofile:
            import cProfile
            import pstats
            torch.cuda.synchronize()
            prof = cProfile.Profile()
            prof.enable()
            step()
            prof.disable()
            torch.cuda.synchronize()
            pstats.Stats(prof).sort_stats("tottime").print_stats(30)
    model.FE1.fps_parts = None


if __name__ == "__main__":
    main()
