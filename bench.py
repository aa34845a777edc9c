#!/usr/bin/env python3
"""DeepVCP registration hot path benchmark (BASELINE.json metric, config C3 / C4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU, RCCL)

One step = DeepVCP.forward + deepVCP_loss (the two-pass pose solve) over one batch of
synthetic KITTI-like pairs (B pairs per GPU, N=16384 points, K=64 key points, candidate grid
r=2.0 / s=0.4 -> C=1331), inputs resident in HBM, eval mode, random-init weights
(torch.manual_seed(0)).  Pairs are independent, so ranks shard the pairs with no data-path
collective ("weak" scaling); the per-pair (R, t) are all-gathered over RCCL once at the end of
the timed region.  Rank 0 prints one JSON line.  At N=1 the CPU oracle (REF-R restated in
torch CPU ops) is timed on the same pairs with the same weights and FPS starts (median of
--cpu-pairs), and its R, t are compared with the GPU's.

Roofline fields: ``roofline`` is the dominant entry point's (largest device
time per step) executed work against the fp32 / HBM peak with its PMC counters; ``fps_roofline``
is the FPS chain against its measured step floor and the fp32 VALU peak; ``step_roofline`` and
``stages`` are SURVEY.md 8(d)'s per-stage ceilings on executed work from one batch in flight;
``live_launch_ms`` are per-launch durations over the timed region (batches in flight contend, so
they exceed the isolated ones).
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepvcp-pointcloud-registration_amd"))

# Hardware queues per process (read when HIP initialises, so set before torch touches the GPU).
# Each in-flight batch drives two streams (the FPS chain and its side stream); with HIP's default
# of 4 queues, streams that share a queue serialise behind each other's multi-millisecond FPS
# launches.  8 measured +13% over 4.  With the round-2 kernels, 10 batches in flight on 24 queues
# measured ~1510 pairs/s against ~1413 for 8 on 16 (same box, 3 alternating reps each; 12 batches
# drop to ~1260: profiles/round2/r2s_inflight_sweep*.log), so that is the default.  --hw-queues
# overrides.
def _hw_queues(argv):
    for i, a in enumerate(argv):
        if a == "--hw-queues" and i + 1 < len(argv):
            return argv[i + 1]
        if a.startswith("--hw-queues="):
            return a.split("=", 1)[1]
    return "24"


os.environ["GPU_MAX_HW_QUEUES"] = _hw_queues(sys.argv)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_FP32_TFLOPS = 157.3   # fp32 vector = fp32 MFMA dense rate
PEAK_BF16_TFLOPS = 16 * PEAK_FP32_TFLOPS   # bf16 MFMA dense rate (the SA layer 2's split pieces)
PEAK_HBM_GBS = 8000.0
N_CU = 256
# flops counted per unit of the distance-scan kernels (dvcp/ops.py): one (query, point) evaluation =
# 3 sub + 3 mul + 2 add + 1 compare = 9; SURVEY.md 8(d) prices it at ~8 (no compare), i.e. 8/9 of
# the reported achieved rate
FLOP_CONVENTION = {
    "dvcp_knn_tiled": "9 flop per (query, reference point) pair of the reference's brute-force graph: 3 sub, "
                      "3 mul, 2 add, 1 compare (SURVEY 8(d) counts ~8 without the compare: x 8/9)",
    "dvcp_ball_query_ws": "9 flop per (centre, point) pair of the reference's dense graph (as the kNN)",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--config", choices=["c3", "c5"], default="c3",
                   help="c3: BASELINE's headline (8 pairs x 16384 points, K=64); c5: the stress config "
                        "(65536 points, K=256, 2 pairs per batch, fp16 features, no CPU baseline)")
    p.add_argument("--batch", type=int, default=None, help="pairs per GPU (c3: 8, c5: 2)")
    p.add_argument("--feat-dtype", choices=["f32", "f16"], default=None,
                   help="target feature-table storage (c3: f32 = the reference's; c5: f16, BASELINE's "
                        "'fp16 features')")
    p.add_argument("--npoints", type=int, default=None)
    p.add_argument("--K", type=int, default=None)
    p.add_argument("--r", type=float, default=2.0)
    p.add_argument("--s", type=float, default=0.4)
    p.add_argument("--inflight", type=int, default=10,
                   help="independent batches in flight (one stream each); 1 = strictly serial steps")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--graphs", choices=["on", "off"], default="off",
                   help="replay each lane's step as a captured HIP graph (dvcp.graphs.CapturedStep) instead of "
                        "issuing it eagerly, one Python + ctypes call per kernel.  Off by default: on this ROCm the "
                        "replay ran the FPS chain and the side stream's tables one after the other (single-batch "
                        "latency 13.4 -> 22.3 ms, 2278 -> 2034 pairs/s; profiles/round6/r6k_*)")
    p.add_argument("--lane-priority", choices=["default", "high"], default="default",
                   help="stream priority of the in-flight batches' lanes (FPS chain + head)")
    p.add_argument("--hw-queues", type=int, default=24, help="GPU_MAX_HW_QUEUES for this process (<= 32)")
    p.add_argument("--stage-report", action="store_true", help="print the per-kernel table to stderr")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="skip the eager pass that times every launch at the run's concurrency (live_launch_ms); "
                        "the timed region never carries per-launch events")
    p.add_argument("--iso-steps", type=int, default=3,
                   help="steps timed per kernel with one batch in flight (stage roofline)")
    p.add_argument("--cpu-pairs", type=int, default=3,
                   help="C3 pairs timed for the CPU baseline (median, SURVEY 8(d)); one pair is ~20 s on 16 host threads")
    p.add_argument("--fps-parts-latency", type=int, default=8, choices=[0, 2, 4, 8],
                   help="also time the single-batch latency with the FPS select rounds split over this many "
                        "workgroups per cloud (DeepVCP(fps_parts=...); 0: skip)")
    p.add_argument("--dfe", choices=["collapsed", "literal"], default="collapsed",
                   help="target DFE: fc3.fc2.fc1 collapsed into one 32x35 map (dvcp_dfe_tgt, default) or the three "
                        "layers chained as written (dvcp_dfe_tgt_literal, SURVEY App. A.3 Q14)")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="process group for world > 1: nccl (= RCCL, one rank per GPU) or gloo (rehearsal: "
                        "several ranks may share a GPU)")
    p.add_argument("--rows-out", default=None,
                   help="rank 0 writes the gathered per-pair rows (steps x global batch, 14 fp64: R, t, rotation "
                        "and translation error) to this .pt file: a sharded run's rows equal a one-GPU run's of "
                        "the same global batch (dvcp.dist.ShardPlan)")
    p.add_argument("--detail-json", default=None,
                   help="also write the full record (per-stage roofline, live launch times) to this file; it "
                        "always goes to stderr as one 'bench-detail' JSON line")
    a = p.parse_args()
    c5 = a.config == "c5"
    a.batch = a.batch if a.batch is not None else (2 if c5 else 8)
    a.npoints = a.npoints if a.npoints is not None else (65536 if c5 else 16384)
    a.K = a.K if a.K is not None else (256 if c5 else 64)
    a.feat_dtype = a.feat_dtype or ("f16" if c5 else "f32")
    if c5:
        a.no_cpu_baseline = True   # minutes per pair on the host: not a bounded sample
    return a


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; --dist-backend gloo lets a rehearsal put several ranks on one GPU
    # (device index LOCAL_RANK mod the visible count; device_count does not initialise HIP)
    dev_idx = local % max(1, torch.cuda.device_count())
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)

    import dvcp
    from dvcp import _lib
    from dvcp import dist as D
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn

    B, N, K, r, s = args.batch, args.npoints, args.K, args.r, args.s
    P = max(1, args.inflight)
    # rank-independent by construction (dvcp.dist.ShardPlan): every rank draws each lane's global
    # batch and keeps its shard, builds the same model, and draws the global batch's FPS starts
    plan = D.ShardPlan(B, world, rank)
    torch.manual_seed(0)
    model = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s,
                         feat_dtype=torch.float16 if args.feat_dtype == "f16" else torch.float32,
                         dfe_literal=args.dfe == "literal").eval().to(dev)
    batches = [tuple(x.to(dev) for x in plan.lane_pairs(lane, N, make_pairs)) for lane in range(P)]
    src, tgt, R_gt, t_gt = batches[0]
    # random init, conditioned so key-point scores are separated beyond fp32 noise (the default
    # init's scores are 0.62 +- 1e-4): BN stats randomised, WL calibrated on global pair 0's
    # features -- the same cloud on every rank and at every world size
    randomize_bn(model)
    with torch.no_grad():
        _, calib, _ = model.FE1.run(plan.calibration_src(N, make_pairs).to(dev))
    condition_weights(model, feats=calib)
    t_init = torch.zeros(1, 3)
    torch.manual_seed(1)
    # lane streams (each batch's FPS chain and head); --lane-priority high puts them above the
    # extractor's side streams (the set-abstraction tables), which keep the default priority
    lanes = [torch.cuda.Stream(device=dev, priority=-1 if args.lane_priority == "high" else 0) for _ in range(P)]

    def rows(Rp, tp, rot, trans):
        # per pair: R (9), t (3), rotation error (deg), translation error -> (B, 14)
        return torch.cat([Rp.reshape(B, 9), tp.reshape(B, 3), rot.reshape(B, 1), trans.reshape(B, 1)], 1)

    def step_eager(lane=0):
        """One pass over one batch: DeepVCP.forward + deepVCP_loss, issued on the lane's stream."""
        b_src, b_tgt, b_R, b_t = batches[lane]
        starts = plan.starts(model, N)   # this rank's columns of the global batch's draw
        with torch.no_grad(), torch.cuda.stream(lanes[lane]):
            kp, vcp = model(b_src, b_tgt, b_R, t_init, starts=starts)
            loss, Rp, tp = dvcp.deepVCP_loss(kp, vcp, b_R, b_t, 0.5)
            rot, trans = dvcp.registration_errors(Rp, tp, b_R, b_t)  # train.py:112-120 harness
            return rows(Rp, tp, rot, trans)

    graphs = None

    def step_graph(lane=0):
        """The same step replayed from the lane's captured graph (dvcp.graphs.CapturedStep): one
        host call for the whole dependency graph; the rows are copied out on the lane's stream."""
        starts = plan.starts(model, N)
        out = graphs[lane].replay(starts)
        with torch.cuda.stream(lanes[lane]):
            return rows(*out)

    def step(lane=0):
        return step_graph(lane) if graphs is not None else step_eager(lane)

    if args.graphs == "on":
        # one captured graph per lane (after an eager warm-up inside CapturedStep)
        from dvcp.graphs import CapturedStep
        graphs = [CapturedStep(model, *batches[ln], alpha=0.5, stream=lanes[ln], starts=plan.starts(model, N))
                  for ln in range(P)]
    # warmup, and the single-batch latency (strictly serial steps on one stream)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t_lat = time.perf_counter()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    latency_ms = (time.perf_counter() - t_lat) / 2 * 1e3
    for lane in range(1, P):
        step(lane)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    _lib.EVENT_LOG = None   # (per-kernel events: a separate eager pass after the timed region)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [step(i % P) for i in range(args.steps)]
    t_issue = time.perf_counter() - t0  # host time to issue every step (no sync inside)
    cur = torch.cuda.current_stream(dev)
    for ln in lanes:
        cur.wait_stream(ln)
    res = torch.cat(outs)   # (steps * B, 14)
    if world > 1 and args.dist_backend == "gloo":
        res = res.cpu()   # gloo gathers host tensors (rehearsal only; RCCL gathers in HBM)
    res = D.gather_results(res, world)      # the one collective: RCCL all_gather of the rows
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    log = []
    if world > 1:
        dist.barrier()
    elapsed = D.max_over_ranks(elapsed, dev if args.dist_backend == "nccl" else torch.device("cpu"))

    # ---- per-kernel HIP-event timing (events on the stream each kernel is launched on) --------
    # (1) live over the timed region, the batches in flight: per-launch durations under contention
    #     (graph replays carry no per-kernel events: then an eager pass of the same steps after it)
    #     The timed region itself carries no per-kernel events (two HIP events per launch were about
    #     half of its host issue time); this eager pass of the same steps at the same concurrency
    #     times every launch.
    if not args.no_kernel_events:
        graphs_keep, graphs = graphs, None
        _lib.EVENT_LOG = []
        for i in range(args.steps):
            step(i % P)
        torch.cuda.synchronize()
        log, _lib.EVENT_LOG = _lib.EVENT_LOG, None
        graphs = graphs_keep
    live = _per_kernel(log)
    # (2) isolated: the same step with one batch in flight (a few steps on lane 0, after the timed
    #     region), for the per-stage roofline; (3) the FPS step floor probe
    _lib.EVENT_LOG = []
    for _ in range(args.iso_steps):
        step_eager(0)
        torch.cuda.synchronize()
    iso, _lib.EVENT_LOG = _per_kernel(_lib.EVENT_LOG), None
    floor_us = fps_step_floor_us(dev)
    # the single-batch latency with the split-select FPS (opt-in at C3: it shortens a lone batch's
    # chain, but with batches in flight its CU time costs pairs/s), same batch and model
    lat_split = None
    if args.fps_parts_latency and args.config == "c3":
        model.FE1.fps_parts = args.fps_parts_latency
        for _ in range(2):
            step_eager()
        torch.cuda.synchronize()
        t_ls = time.perf_counter()
        for _ in range(2):
            step_eager()
        torch.cuda.synchronize()
        lat_split = {"parts": args.fps_parts_latency, "ms": round((time.perf_counter() - t_ls) / 2 * 1e3, 3)}
        model.FE1.fps_parts = None
    ms_step = elapsed / args.steps * 1e3
    S = model.FE1.sa1.npoint
    C = int((2 * r) / s + 1) ** 3
    stages, step_roof = stage_roofline(iso, args.iso_steps, ms_step)
    pmc = _pmc(args.config)   # profiles/pmc_summary.json (C3) / pmc_summary_c5.json (C5)
    roofline = dominant_roofline(live, iso, stages, pmc)
    fps_roof = fps_roofline(live, iso, floor_us, pmc)
    roofline["by_kernel_time"] = kernel_time_dominant(iso, stages, fps_roof)
    res_cpu = res.cpu()
    if rank == 0 and args.rows_out:
        # gathered in rank order (each rank: steps x B rows) -> (steps, global batch, 14)
        by_step = res_cpu.reshape(world, args.steps, B, 14).permute(1, 0, 2, 3).reshape(args.steps, B * world, 14)
        torch.save({"rows": by_step.contiguous(), "global_batch": B * world, "steps": args.steps, "world": world,
                    "columns": "R (9), t (3), rotation error deg, translation error"}, args.rows_out)
    reg_err = {"rot_deg_mean": float(res_cpu[:, 12].mean()), "rot_deg_max": float(res_cpu[:, 12].max()),
               "trans_mean": float(res_cpu[:, 13].mean()), "trans_max": float(res_cpu[:, 13].max()),
               "pairs": int(res_cpu.shape[0]),
               "note": "vs ground truth (train.py:112-120 metric), random-init weights, R_init = R_gt as train.py:105 passes it"}
    pairs = B * world * args.steps
    value = pairs / elapsed
    c5 = args.config == "c5"
    out = {
        "metric": (f"pairs/sec (full DeepVCP forward) at N=65536, K=256 (C5 stress, {args.feat_dtype} features)" if c5 else
                   "pairs/sec (full DeepVCP forward) at N=16384, K=64; rot/trans error vs ref"),
        "value": round(value, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": ("C5: synthetic 65536-point pairs, K=256, DeepVCP.forward + deepVCP_loss (eval), "
                                f"{args.feat_dtype} target feature table (dvcp_dfe_tgt_f16 for f16)" if c5 else
                                "C3: KITTI-like synthetic pairs, DeepVCP.forward + deepVCP_loss (eval)"),
                   "pairs_per_gpu": B, "global_batch": B * world, "n_points": N, "K": K, "r": r, "s": s,
                   "candidates": C, "fe_npoint": S, "parallelism": f"pairs sharded x{world}, all_gather(R,t)",
                   "inflight_batches": P, "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                   # what the headline runs where it regroups the reference's arithmetic
                   "dfe": ("literal: fc1, fc2, fc3 chained as written (dvcp_dfe_tgt_literal)" if args.dfe == "literal" else
                           "collapsed: fc3.fc2.fc1 as one 32x35 map formed in fp64, rounded once (SURVEY App. A.3 "
                           "Q14 deviation; --dfe literal runs the chain)") if args.feat_dtype == "f32" else
                          "collapsed, fp16 feature table (dvcp_dfe_tgt_f16)",
                   "sa_layer1": "per-point split: W1f.f + b1 once per point, W1x.(p - c) per grouped row (exact in "
                                "real arithmetic; held to the fp32 bars)",
                   "fps": _fps_parts_label(N, model.FE1.fps_parts),
                   "issue": ("each lane's step replayed from a captured HIP graph (dvcp.graphs.CapturedStep)"
                             if args.graphs == "on" else "eager: one Python + ctypes call per kernel")},
        "latency_ms_single_batch": round(latency_ms, 3),
        "latency_ms_single_batch_split_fps": lat_split,
        "host_issue_ms_per_step": round(t_issue / args.steps * 1e3, 3),
        "registration_error_vs_gt": reg_err,
        "roofline": roofline,
        "fps_roofline": fps_roof,
        "step_roofline": step_roof,
        "stages": stages,
        "live_launch_ms": {k: round(v["ms"] / v["n"], 4) for k, v in sorted(live.items(), key=lambda kv: -kv[1]["ms"])},
    }
    # HBM fraction of the whole step (north_star asks for it; the path is compute/latency bound)
    out["hbm_fraction_step"] = round(sum(v["bytes"] for v in iso.values()) / args.iso_steps /
                                     (elapsed / args.steps) / (PEAK_HBM_GBS * 1e9), 6)
    out["hbm_fraction_note"] = ("algorithmic bytes of every stage (one batch in flight) over ms_per_step x 8 TB/s; "
                                "the path is compute/latency bound, so this is structurally small")

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["parity"] = cpu_baseline(model, src, tgt, R_gt, t_gt, dev, args.cpu_pairs)
    if rank == 0:
        if args.stage_report:
            for k, v in stages.items():
                print(f"{k:28s} {v}", file=sys.stderr)
            print(json.dumps(step_roof), file=sys.stderr)
        # the full record to stderr (and --detail-json); stdout gets ONE compact headline line that
        # a log tail keeps whole (value, latency, roofline, cpu_baseline, parity, errors)
        print("bench-detail " + json.dumps(out), file=sys.stderr, flush=True)
        if args.detail_json:
            with open(args.detail_json, "w") as fh:
                json.dump(out, fh, indent=1)
        print(json.dumps(headline(out)), flush=True)
    if world > 1:
        dist.destroy_process_group()


HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config", "latency_ms_single_batch",
                 "latency_ms_single_batch_split_fps", "roofline", "cpu_baseline", "parity", "registration_error_vs_gt")


def _fps_parts_label(N, forced=None):
    """The FE chain's FPS layers (N -> 10000, then 10000 -> 10000 twice): workgroups per cloud."""
    from dvcp import ops
    p1, p2 = (forced, forced) if forced else (ops.fps_parts(N), ops.fps_parts(10000))
    if p1 == p2:
        return f"select rounds on {p1} workgroup(s) per cloud"
    return f"select rounds on {p1} workgroups per cloud (layer 1, {N} points), {p2} (layers 2, 3)"


def headline(out):
    """The stdout line: the contract's fields plus latency, roofline, cpu_baseline, parity and the
    registration error, each trimmed of its long notes; the FPS chain and the step roofline as
    one-number summaries (the full objects are in the stderr 'bench-detail' line)."""
    h = {k: out[k] for k in HEADLINE_KEYS if k in out}
    h["roofline"] = {k: v for k, v in out["roofline"].items() if k not in ("note", "pmc", "work_basis")}
    if out["roofline"].get("pmc"):
        h["roofline"]["pmc"] = {k: v for k, v in out["roofline"]["pmc"].items() if k != "note"}
    if "cpu_baseline" in out:
        h["cpu_baseline"] = {k: out["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind", "sample", "cpu_model")}
    if "parity" in out:
        h["parity"] = {k: v for k, v in out["parity"].items() if not k.endswith("_note")}
    if "registration_error_vs_gt" in out:
        h["registration_error_vs_gt"] = {k: v for k, v in out["registration_error_vs_gt"].items() if k != "note"}
    fr = out.get("fps_roofline") or {}
    h["fps"] = {k: fr.get(k) for k in ("us_per_centre", "step_floor_us", "frac_of_step_floor", "avg_launch_ms_isolated")}
    h["step_roofline_frac"] = out["step_roofline"]["achieved_frac"]
    h["hbm_fraction_step"] = out["hbm_fraction_step"]
    return h


def _per_kernel(log):
    """EVENT_LOG -> {entry point: {n, ms, cu_ms, flops, bytes, exec_flops, mfma_flops, wgs, steps}}
    (sums; cu_ms: each launch's duration x the CU share of its grid, so an entry point whose launches
    differ in grid size -- C5's 65536-point FPS layer on 8 workgroups per cloud, its 10000-point
    layers on one -- gets a time-weighted share).  Executed work given as a callable (the SA tables'
    real ball-query hit counts) is evaluated here, after the timed region."""
    out = {}
    for name, e0, e1, w in log:
        d = out.setdefault(name, {"n": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "exec_flops": 0.0,
                                  "mfma_flops": 0.0, "bf16_alg": 0.0, "bf16_hw": 0.0, "exec_known": True,
                                  "wgs": None, "steps": 0, "cu_ms": 0.0})
        d["n"] += 1
        ms = e0.elapsed_time(e1)
        d["ms"] += ms
        w = tuple(w or ()) + (None,) * 5
        d["cu_ms"] += ms * (min(1.0, w[3] / N_CU) if w[3] else 1.0)
        d["flops"] += w[0] or 0.0
        d["bytes"] += w[1] or 0.0
        ex = w[2]
        if callable(ex):
            ex = ex()
        if ex is None:
            d["exec_known"] = False
        else:
            ex = (ex,) if isinstance(ex, (int, float)) else tuple(ex)
            tot, mf, b_alg, b_hw = ex + (0.0,) * (4 - len(ex))
            d["exec_flops"] += tot
            d["mfma_flops"] += mf
            d["bf16_alg"] += b_alg
            d["bf16_hw"] += b_hw
        if w[3] is not None:
            d["wgs"] = w[3]
            d["steps"] += w[4]
    return out


def fps_step_floor_us(dev, steps=20000):
    """Measured floor of one FPS step: dvcp_fps_step_floor (a 512-thread workgroup running the
    chain's per-step DPP argmax + LDS slot + barrier + slot reduction with no point work)."""
    from dvcp import _lib
    out = torch.empty(16, dtype=torch.float32, device=dev)
    st = _lib.stream()
    _lib.call("dvcp_fps_step_floor", 1000, 16, _lib.ptr(out), st)   # warm-up
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.call("dvcp_fps_step_floor", steps, 16, _lib.ptr(out), st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def stage_roofline(iso, iso_steps, ms_step):
    """SURVEY.md 8(d) per stage, on the work each kernel EXECUTES.

    For every entry point (one batch in flight, ``--iso-steps`` steps): its device time = measured
    duration x the share of the 256 CUs its grid can occupy (the FPS chain: one workgroup per
    cloud, 16/256), and its ceiling = max(algorithmic bytes / 8 TB/s, work / 157.3 TF/s) in
    full-chip time, where work = the flops the kernels execute when the entry point counts them
    (the SA tables from the ball query's real hit counts, the DFE's MFMA count) and the
    reference-graph flops otherwise (ball query, kNN, FPS: an upper bound of what their pruned
    scans execute).  frac_of_ceiling = ceiling / device time.  The step roofline is the sum of
    the ceilings over ``ms_per_step`` (measured with the default batches in flight)."""
    stages, ideal_dev, meas_dev = {}, 0.0, 0.0
    for k, v in sorted(iso.items(), key=lambda kv: -kv[1]["ms"]):
        ms = v["ms"] / iso_steps
        share = v["cu_ms"] / v["ms"] if v["ms"] > 0 else 1.0
        dev_ms = ms * share
        t_byte = v["bytes"] / iso_steps / (PEAK_HBM_GBS * 1e9) * 1e3
        t_ref = v["flops"] / iso_steps / (PEAK_FP32_TFLOPS * 1e12) * 1e3
        known = v["exec_known"] and v["exec_flops"] > 0
        # executed work at its pipe's peak: the bf16 pieces of the SA layer 2 at the bf16 MFMA rate
        t_exec = ((v["exec_flops"] - v["bf16_alg"]) / (PEAK_FP32_TFLOPS * 1e12)
                  + v["bf16_hw"] / (PEAK_BF16_TFLOPS * 1e12)) / iso_steps * 1e3 if known else None
        t_work = t_exec if known else t_ref
        ceil, bound = (t_work, "fp32") if t_work >= t_byte else (t_byte, "hbm")
        if bound == "fp32" and known and v["mfma_flops"] > 0.5 * v["exec_flops"]:
            bound = "mfma"
        ideal_dev += ceil
        meas_dev += dev_ms
        st = {"launches_per_step": round(v["n"] / iso_steps, 2), "isolated_ms_per_step": round(ms, 4),
              "cu_share": round(share, 4), "device_ms_per_step": round(dev_ms, 4),
              "ceiling_ms_per_step": round(ceil, 4), "bound": bound,
              "work_basis": "executed" if known else "reference graph (upper bound of the executed work)",
              "frac_of_ceiling": round(ceil / dev_ms, 4) if dev_ms > 0 else None,
              "ref_graph_gflop": round(v["flops"] / iso_steps / 1e9, 3),
              "executed_gflop": round(v["exec_flops"] / iso_steps / 1e9, 3) if known else None,
              "mfma_gflop": round(v["mfma_flops"] / iso_steps / 1e9, 3) if known else None,
              # rate over the CUs the grid occupies (work / (duration x share of the chip))
              "tflops": round((v["exec_flops"] if known else v["flops"]) / (v["ms"] * 1e-3) / share / 1e12, 3)
              if v["ms"] > 0 and (known or v["flops"]) else None}
        if st["frac_of_ceiling"] is not None and st["frac_of_ceiling"] > 1.0:
            st["ceiling_note"] = "ceiling above the measured time: the counted work exceeds what the kernel runs"
        stages[k] = st
    roof = {"formula": "sum_s max(bytes_s / 8 TB/s, executed flops_s / 157.3 TF/s (the SA layer 2's bf16 split "
                       "pieces at 2516.8 TF/s)) / ms_per_step; "
                       "stages without an executed count use their reference-graph flops",
            "ceiling_device_ms_per_step": round(ideal_dev, 4), "measured_device_ms_per_step_isolated": round(meas_dev, 4),
            "ms_per_step": round(ms_step, 4), "achieved_frac": round(ideal_dev / ms_step, 4),
            "isolated_frac": round(ideal_dev / meas_dev, 4) if meas_dev else None,
            "note": "stage times from one batch in flight (bench --iso-steps); ms_per_step with the default "
                    "batches in flight; device time = duration x CU share of the grid"}
    return stages, roof


def dominant_roofline(live, iso, stages, pmc):
    """The JSON ``roofline``: the entry point with the largest device time per step (what bounds
    pairs/s), its executed work per average isolated launch against the fp32 peak (157.3 TF/s:
    the fp32 MFMA and fp32 VALU rates are equal on gfx950) or HBM, and its PMC counters
    (profiles/pmc_summary.json: HBM bytes per launch, MFMA / VALU busy)."""
    name = max(stages, key=lambda k: stages[k]["device_ms_per_step"])
    v, st = iso[name], stages[name]
    known = v["exec_known"] and v["exec_flops"] > 0
    flops = v["exec_flops"] if known else v["flops"]
    launch_ms = v["ms"] / v["n"]
    share = st["cu_share"]
    if st["bound"] == "hbm":
        achieved, peak, unit = v["bytes"] / v["n"] / (launch_ms * 1e-3) / 1e9, PEAK_HBM_GBS, "GB/s"
    else:
        # the peak of this kernel's pipe mix: fp32 work at 157.3 TF/s, the bf16 pieces of the SA
        # layer 2 (6 bf16 products per fp32-equivalent product) at the bf16 MFMA rate
        t_peak = (flops - v["bf16_alg"]) / PEAK_FP32_TFLOPS + v["bf16_hw"] / PEAK_BF16_TFLOPS if known else None
        peak_eff = flops / t_peak if t_peak else PEAK_FP32_TFLOPS
        achieved, peak, unit = flops / v["n"] / (launch_ms * 1e-3) / 1e12, peak_eff * share, "TFLOP/s"
    w = live.get(name)
    p = pmc.get(name, {})
    return {"bound": {"mfma": "mfma", "fp32": "valu", "hbm": "hbm"}[st["bound"]],
            "bound_note": "the stage's own bound: mfma (matrix cores), valu (fp32 vector ALU; on gfx950 its peak "
                          "equals the fp32 MFMA rate, 157.3 TF/s) or hbm",
            "flop_convention": FLOP_CONVENTION.get(name, "executed flops as counted by dvcp/ops.py"),
            "kernel": name, "achieved": round(achieved, 3), "peak": round(peak, 3), "unit": unit,
            "frac": round(achieved / peak, 4),
            "frac_survey_8flop": round(achieved / peak * 8 / 9, 4) if name in FLOP_CONVENTION else None,
            "traffic": p.get("hbm_bytes_per_launch"),
            "work_basis": st["work_basis"], "flops_per_launch": flops / v["n"],
            "algorithmic_bytes_per_launch": v["bytes"] / v["n"],
            "avg_launch_ms_isolated": round(launch_ms, 4),
            "avg_launch_ms_live": round(w["ms"] / w["n"], 4) if w else None,
            "pmc": {k: p[k] for k in ("mfma_util", "valu_busy", "valu_util_lanes", "note") if k in p} or None,
            "note": "dominant = largest device time per step (duration x CU share), one batch in flight; "
                    "achieved = executed flops (reference-graph flops if not counted) per launch / average "
                    "isolated launch time; peak = fp32 157.3 TF/s x the grid's CU share (fp32 MFMA = fp32 "
                    "VALU rate on gfx950; for the SA tables the fp32-equivalent rate of their pipe mix: the "
                    "layer-2 split pieces at the 2516.8 TF/s bf16 MFMA rate, 6 per fp32-equivalent product) "
                    "or 8 TB/s; traffic = PMC HBM bytes per launch"}


FPS_ENTRIES = ("dvcp_fps_parts", "dvcp_fps_ws")   # ops.fps's entry point (ABI 4), and its predecessor


def kernel_time_dominant(iso, stages, fps_roof):
    """The entry point with the largest kernel time per step (rocprof's ranking: the FPS chain at C3,
    16 clouds on a fraction of the chip), beside ``roofline``'s device-share-dominant one: its
    reference-graph rate against the fp32 peak of the whole chip and of the CUs its grid occupies,
    and, for the FPS, its time per centre against the measured step floor."""
    name = max(iso, key=lambda k: iso[k]["ms"])
    v, st = iso[name], stages[name]
    tot = sum(x["ms"] for x in iso.values())
    rec = {"kernel": name, "share_of_kernel_time": round(v["ms"] / tot, 4),
           "avg_launch_ms_isolated": round(v["ms"] / v["n"], 4)}
    if fps_roof and name == fps_roof["kernel"]:
        rec.update({"bound": "latency (serial chain)", "unit": "TFLOP/s", "achieved": fps_roof["tflops_ref_graph"],
                    "peak": PEAK_FP32_TFLOPS, "frac": fps_roof["frac_of_fp32_peak_chip"],
                    "frac_own_cus": fps_roof["frac_of_fp32_peak_own_cus"], "cu_share": st["cu_share"],
                    "traffic": fps_roof["traffic"], "us_per_centre": fps_roof["us_per_centre"],
                    "step_floor_us": fps_roof["step_floor_us"], "frac_of_step_floor": fps_roof["frac_of_step_floor"],
                    "flop_convention": "9 flop per point-update of the reference graph (npoint x N per cloud); "
                                       "SURVEY 8(d)'s 8 flop: x 8/9"})
    else:
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12
        rec.update({"bound": st["bound"], "unit": "TFLOP/s", "achieved": round(tf, 3), "peak": PEAK_FP32_TFLOPS,
                    "frac": round(tf / PEAK_FP32_TFLOPS, 4), "cu_share": st["cu_share"]})
    return rec


def fps_roofline(live, iso, floor_us, pmc):
    """FPS is a serial chain of npoint dependent argmax steps per cloud, one workgroup per cloud:
    reported against the measured step floor of its synchronisation (dvcp_fps_step_floor, us per
    centre) AND against the fp32 VALU peak, both of the whole chip and of the 16 CUs a C3 batch's
    16 clouds occupy (reference-graph flops: 9 per point-update, npoint x N per cloud)."""
    name = next((n for n in FPS_ENTRIES if n in iso), None)
    if name is None:
        return None
    v, w = iso[name], live.get(name)
    us_iso = v["ms"] * 1e3 / v["steps"]
    us_live = w["ms"] * 1e3 / w["steps"] if w and w["steps"] else None
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12
    share = v["cu_ms"] / v["ms"]
    return {"kernel": name, "us_per_centre": round(us_iso, 4), "step_floor_us": round(floor_us, 4),
            "frac_of_step_floor": round(floor_us / us_iso, 4),
            "tflops_ref_graph": round(tf, 3), "frac_of_fp32_peak_chip": round(tf / PEAK_FP32_TFLOPS, 4),
            "frac_of_fp32_peak_own_cus": round(tf / (PEAK_FP32_TFLOPS * share), 4),
            "avg_launch_ms_isolated": round(v["ms"] / v["n"], 4),
            "avg_launch_ms_live": round(w["ms"] / w["n"], 4) if w else None,
            "us_per_centre_live": round(us_live, 4) if us_live else None,
            "traffic": pmc.get(name, {}).get("hbm_bytes_per_launch"),
            "algorithmic_bytes_per_launch": v["bytes"] / v["n"],
            "note": "frac_of_step_floor: the select kernel certifies several centres per round, so it can pass "
                    "1; the fp32 fractions count the reference graph's 9 flop per point-update"}


def _pmc(config="c3"):
    """The PMC summary of this configuration (tools/gpu_pmc.sh, one batch in flight):
    profiles/pmc_summary.json (C3) or profiles/pmc_summary_c5.json (C5); {} if absent."""
    name = "pmc_summary.json" if config == "c3" else f"pmc_summary_{config}.json"
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except Exception:
        return {}


def _cpu_topology():
    """(model name, physical cores, logical CPUs) from lscpu."""
    info = {}
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except Exception:
        pass
    try:
        phys = int(info["Core(s) per socket"]) * int(info["Socket(s)"])
    except Exception:
        phys = None
    return info.get("Model name", platform.processor() or ""), phys, os.cpu_count()


def cpu_baseline(model, src, tgt, R_gt, t_gt, dev, n_pairs):
    """Time the CPU oracle (REF-R in torch CPU ops) on the bench's C3 pairs, same
    weights and FPS starts: one warm-up forward on a small pair (oneDNN / allocator warm-up), then
    the median of ``n_pairs`` full-size pairs, one pair per forward (B = 1, eval, no_grad).
    Threads: the physical cores this process may use, capped by the box's CPU share per GPU
    (OMP_NUM_THREADS, 16 on the GPU pool), stated in the result."""
    import oracle as O
    import dvcp
    from dvcp.synthetic import make_pairs
    cpu_model, phys, logical = _cpu_topology()
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (logical or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    threads = max(1, min(avail, phys or avail, share))
    torch.set_num_threads(threads)
    ref = O.DeepVCP(use_normal=False, K=model.K, r=model.r, s=model.s).eval()
    ref.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    N = src.shape[2]
    n_pairs = max(1, min(n_pairs, src.shape[0]))
    with torch.no_grad():   # warm-up: a small pair through the same ops
        ws, wt, wR, _ = make_pairs(1, 2048, seed=4321)
        small = O.DeepVCP(use_normal=False, K=model.K, r=model.r, s=model.s, fe_npoint=512).eval()
        small.load_state_dict(ref.state_dict())
        small(ws, wt, wR, torch.zeros(1, 3))
    secs, parity = [], None
    for b in range(n_pairs):
        starts = model.draw_starts(1, N, N)
        sl = slice(b, b + 1)
        s0, g0, R0, t0 = src[sl].cpu(), tgt[sl].cpu(), R_gt[sl].cpu(), t_gt[sl].cpu()
        t_start = time.perf_counter()
        with torch.no_grad(), O.fps_starts(list(starts)):
            kpo, vcpo = ref(s0, g0, R0, torch.zeros(1, 3))
            _, Ro, to = O.deepVCP_loss(kpo, vcpo, R0, t0, 0.5)
        secs.append(time.perf_counter() - t_start)
        if b == 0:   # the GPU's result for the same pair and starts
            with torch.no_grad():
                kp, vcp = model(src[sl], tgt[sl], R_gt[sl], torch.zeros(1, 3), starts=starts)
                _, Rg, tg = dvcp.deepVCP_loss(kp, vcp, R_gt[sl], t_gt[sl], 0.5)
            rot_vs_ref, trans_vs_ref = dvcp.registration_errors(Rg, tg, Ro.to(dev), to.to(dev))
            parity = {"R_maxabs_vs_ref": float((Rg.cpu() - Ro).abs().max()),
                      "t_maxabs_vs_ref": float((tg.cpu() - to).abs().max()),
                      "rot_err_deg_vs_ref": float(rot_vs_ref.max()), "trans_err_vs_ref": float(trans_vs_ref.max()),
                      "rot_trans_err_note": "train.py:112-120 metric between the GPU pose and the oracle pose; "
                                            "PairwiseDistance's eps contributes sqrt(3)*1e-6 at exact agreement",
                      "vcp_maxabs_vs_ref": float((vcp.cpu() - vcpo).abs().max()),
                      "keypts_equal": bool(torch.equal(kp.cpu(), kpo)),
                      "keypts_same_set": bool(torch.equal(torch.sort(kp.cpu().reshape(-1, 3), 0).values,
                                                          torch.sort(kpo.reshape(-1, 3), 0).values))}
    med = sorted(secs)[len(secs) // 2]
    base = {"value": round(1.0 / med, 5), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"median of {len(secs)} C3 pairs (N=16384, K=64, r=2.0, one pair per forward) after a "
                      f"small warm-up pair; oracle/ref_r.py torch CPU ops; per pair "
                      f"{', '.join(f'{x:.1f}' for x in secs)} s",
            "cpu_model": cpu_model, "physical_cores": phys, "os_cpu_count": logical,
            "threads_note": "physical cores available to the process, capped at the box's CPU share per GPU "
                            "(OMP_NUM_THREADS)"}
    return base, parity


if __name__ == "__main__":
    main()
