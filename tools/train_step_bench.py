"""Training step throughput at C3 (train.py:96-125): the head with the feature extractor frozen,
(--train-fe) the whole model with the extractor trainable in frozen-BN mode (FE1.eval()), or
(--train-fe --bn-train) train.py's own setting: model.train(), FE1's BatchNorms on batch
statistics.

One step = model(src, tgt, R_gt, t_init) with autograd on the head -> deepVCP_loss -> backward
-> Adam step, on one batch of synthetic KITTI-like pairs (8 x 16384 points, K=64, r=2.0, s=0.4).
Prints one JSON line: pairs/s, ms/step and the per-entry-point HIP-event times of the backward
kernels (and the forward's) over the timed steps.

    python tools/train_step_bench.py [--steps 10 --warmup 2] [--prefetch P]

--prefetch P: the frozen feature extractor of the next P batches runs ahead on P streams
(DeepVCP.extract_features) while the current batch's head trains (DeepVCP.forward_head); the
head steps themselves stay in order on the default stream, as the optimizer requires.
"""
import collections
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# prefetch lanes each drive two streams (bench.py's reasoning): 16 hardware queues, read when HIP
# initialises (P=3: 496 pairs/s at HIP's default of 4, 512 at 16)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, os.path.join(ROOT, "deepvcp-pointcloud-registration_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--npoints", type=int, default=16384)
    ap.add_argument("--prefetch", type=int, default=0)
    ap.add_argument("--train-fe", action="store_true",
                    help="train FE1 too (frozen-BN: eval-mode BatchNorm, trainable parameters); no prefetch")
    ap.add_argument("--bn-train", action="store_true",
                    help="with --train-fe: FE1 in training mode (batch-statistics BatchNorm, as model.train())")
    args = ap.parse_args()
    if args.bn_train and not args.train_fe:
        ap.error("--bn-train needs --train-fe")
    if args.train_fe and args.prefetch:
        ap.error("--train-fe trains the extractor, so its forward cannot run ahead (--prefetch 0)")
    import dvcp
    from dvcp import _lib
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = dvcp.DeepVCP(use_normal=False, K=64, r=2.0, s=0.4).to(dev)
    src, tgt, R_gt, t_gt = [t.to(dev) for t in make_pairs(args.batch, args.npoints, seed=1234)]
    randomize_bn(model)
    model.FE1.eval()
    with torch.no_grad():
        _, calib, _ = model.FE1.run(src)
    condition_weights(model, feats=calib)
    model.FE1.requires_grad_(args.train_fe)
    if args.bn_train:
        model.FE1.train()
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    t_init = torch.zeros(1, 3)

    P = args.prefetch
    lanes = [torch.cuda.Stream(device=dev) for _ in range(max(P, 1))]
    batches = [(src, tgt, R_gt, t_gt)]
    for i in range(1, max(P, 1)):
        batches.append(tuple(t.to(dev) for t in make_pairs(args.batch, args.npoints, seed=1234 + 7919 * i)))
    main = torch.cuda.current_stream(dev)
    pending = collections.deque()
    issued = [0]

    def issue():
        i = issued[0]
        issued[0] += 1
        lane = lanes[i % len(lanes)]
        lane.wait_stream(main)
        b = batches[i % len(batches)]
        with torch.no_grad(), torch.cuda.stream(lane):
            f = model.extract_features(b[0], b[1])
            ev = torch.cuda.Event()
            ev.record(lane)
        pending.append((f, ev, b))

    def step():
        if P == 0:
            kp, vcp = model(src, tgt, R_gt, t_init)
            Rg, tg = R_gt, t_gt
        else:
            while len(pending) < P:
                issue()
            f, ev, (_, _, Rg, tg) = pending.popleft()
            main.wait_event(ev)
            for t in f.values():
                t.record_stream(main)
            kp, vcp = model.forward_head(f, Rg)
        opt.zero_grad()
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, Rg, tg, 0.5)
        loss.backward()
        opt.step()
        if P:
            issue()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _lib.EVENT_LOG = []
    t0 = time.perf_counter()
    losses = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    log, _lib.EVENT_LOG = _lib.EVENT_LOG, None
    per = {}
    for name, e0, e1, _ in log:
        per.setdefault(name, []).append(e0.elapsed_time(e1))
    stages = {k: {"launches": len(v), "avg_ms": round(sum(v) / len(v), 4),
                  "total_ms_per_step": round(sum(v) / args.steps, 4)}
              for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}
    print(json.dumps({
        "metric": ("training steps (forward + deepVCP_loss + backward + Adam), whole model in training mode "
                   "(FE1 batch-statistics BN)" if args.bn_train else
                   "training steps (forward + deepVCP_loss + backward + Adam), FE trainable with frozen BN"
                   if args.train_fe else "head-training steps (forward + deepVCP_loss + backward + Adam), FE frozen"),
        "prefetch": P,
        "value": round(args.batch * args.steps / dt, 3), "unit": "pairs/s",
        "ms_per_step": round(1e3 * dt / args.steps, 3), "steps": args.steps, "warmup": args.warmup,
        "config": {"pairs": args.batch, "n_points": args.npoints, "K": 64, "r": 2.0, "s": 0.4},
        "loss_first_last": [float(losses[0].detach()), float(losses[-1].detach())],
        "stages": stages}))


if __name__ == "__main__":
    main()
