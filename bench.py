"""Benchmark: the Stage-4 uncertainty-guided training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Workload (BASELINE.json configs[1], weak-scaled for N > 1): per GPU a batch of
16 synthetic 3x256x256 images ~N(0,1) with Bernoulli(0.5) masks; one step =
UncertaintyGuidedProgressiveTrainer.train_step at stage 4 =
PGUNet4 train forward + PGUNet3 eval forward at 128^2 for the uncertainty map +
uncertainty-weighted BCE + backward + RCCL gradient all-reduce (N > 1) +
RMSprop + Dice/accuracy, with one host synchronisation per step (as the
trainer does).  Random-init weights of the reference architecture, fp32.

Prints ONE JSON line (rank 0).  `roofline` is measured live: every conv launch of
every 5th step inside the timed region (--roofline-every) is bracketed by HIP events
on the launching stream; achieved = algorithmic FLOPs / kernel time for the dominant
kernel.  `cpu_baseline` times the CPU oracle (oracle/ref_cpu.py: the
reference's torch CPU ops, same order) on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

METRIC = "images/sec Stage-4 256×256 bs16 fwd+bwd at 1/2/4/8 MI355X; Dice vs ref"
FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 16 * FP32_PEAK_TFLOPS  # dense bf16 MFMA = 16x the f32 rate (same guide)
X6_PRODUCTS = 6  # split-bf16: 6 bf16 MFMA products per fp32-accurate multiply-add
UG_STEP_GFLOP = 225.2866  # per image, SURVEY.md §8d


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-every", type=int, default=5,
                    help="bracket the conv launches of every E-th timed step with HIP events "
                         "(1 = every step; each event pair costs ~3 us of GPU time)")
    ap.add_argument("--secondary-steps", type=int, default=5,
                    help="steps of the secondary line (S4 fwd+bwd without the uncertainty "
                         "map, SURVEY.md 8d); 0 = skip")
    ap.add_argument("--conv-math", choices=("x6", "bf16", "f32"), default="x6",
                    help="conv arithmetic: x6 = fp32-accurate split-bf16 (configs[1], default); "
                         "bf16 = bf16 operands, fp32 accumulation (configs[2] arithmetic)")
    ap.add_argument("--workload", choices=("seg", "herlev"), default="seg",
                    help="seg: the Stage-4 UG segmentation step (BASELINE metric, default); "
                         "herlev: the Herlev Stage-4 classifier UG step (BASELINE configs[3])")
    ap.add_argument("--classes", type=int, default=7, help="Herlev classes (--workload herlev)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the training step from a captured hipGraph (trainer.enable_graphs; "
                         "single process; the sampled roofline steps still run eagerly)")
    return ap.parse_args()


def cpu_cores():
    """Physical cores this process can use: the affinity mask's cores (logical CPUs / SMT
    width), capped by the cgroup CPU quota (a container's share of the host)."""
    logical = len(os.sched_getaffinity(0))
    try:
        sib = open("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list").read().strip()
        smt = 0
        for part in sib.split(","):
            a, _, b = part.partition("-")
            smt += int(b) - int(a) + 1 if b else 1
    except (OSError, ValueError):
        smt = 1
    cores = max(1, logical // max(smt, 1))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            cores = min(cores, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return cores


def cpu_baseline(batch, res, steps, thread_counts):
    """Time the CPU oracle's UG step (the reference's torch CPU ops, same order) on this
    host: for each thread count, 1 warm-up step then the median of `steps` timed steps
    (SURVEY.md §8d protocol).  Progress goes to stderr (a long silent phase reads as hung)."""
    import torch
    from oracle import detgen as G
    from oracle import ref_cpu as O
    cur0 = G.make_state(O.state_spec(4, 3, 1), 0)
    prev = G.make_state(O.state_spec(3, 3, 1), 1)
    x = G.randn(1, (batch, 3, res, res), "x")
    t = G.bernoulli(2, (batch, 1, res, res), 0.5, "t")
    rates = {}
    for threads in thread_counts:
        torch.set_num_threads(threads)
        cur = {k: v.clone() for k, v in cur0.items()}
        sq = {k: torch.zeros_like(v) for k, v in cur.items()
              if v.is_floating_point() and not O._is_buffer(k)}
        O.ug_train_step(4, cur, prev, x, t, sq, 1e-4)  # warm-up
        times = []
        for i in range(steps):
            t0 = time.perf_counter()
            O.ug_train_step(4, cur, prev, x, t, sq, 1e-4)
            times.append(time.perf_counter() - t0)
            print(f"cpu baseline: {threads} threads, step {i + 1}/{steps}: {times[-1]:.2f} s",
                  file=sys.stderr, flush=True)
        times.sort()
        rates[threads] = round(batch / times[len(times) // 2], 4)
    top = max(thread_counts)
    return {"value": rates[top], "unit": "images/sec", "cores": top, "kind": "port",
            "by_cores": {str(k): v for k, v in rates.items()},
            "sample": f"oracle UG step (bs{batch} {res}^2: S4 fwd+bwd + S3 U-map + RMSprop), "
                      f"torch CPU fp32, median of {steps} steps after 1 warm-up, at "
                      f"{' and '.join(str(k) for k in thread_counts)} threads (= physical cores)"}


def herlev_gflop(res):
    """Algorithmic GFLOP per image of the Herlev UG step (at 256^2 the
    Stage-4 encoder fwd+bwd is 80.18 GF, the Stage-3 prediction at 128^2 19.44 GF; the
    encoder scales with the pixel count, the Stage-3 input is always 128^2)."""
    return 80.18 * (res / 256) ** 2 + 19.44


def cpu_baseline_herlev(batch, res, steps, thread_counts, classes):
    """The CPU oracle's Herlev UG step (oracle.ref_cpu.herlev_train_step: the reference's
    torch CPU ops -- model, dropout, Stage-3 prediction, UG CE, torch.optim.Adam), same
    protocol as cpu_baseline."""
    import torch
    from oracle import detgen as G
    from oracle import ref_cpu as O
    spec4 = O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, classes)
    spec3 = O.state_spec(3, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, classes)
    cur0, prev = G.make_state(spec4, 0), G.make_state(spec3, 1)
    x = G.randn(1, (batch, 3, res, res), "x")
    y = G.randint(2, (batch,), classes, "y")
    cw = torch.linspace(0.5, 2.0, classes)
    rates = {}
    for threads in thread_counts:
        torch.set_num_threads(threads)
        cur = {k: v.clone() for k, v in cur0.items()}
        params = [v.requires_grad_(True) for k, v in cur.items()
                  if v.is_floating_point() and not O._is_buffer(k)]
        opt = torch.optim.Adam(params, lr=1e-4, weight_decay=1e-4)
        O.herlev_train_step(cur, prev, x, y, opt, num_classes=classes, class_weights=cw)
        times = []
        for i in range(steps):
            t0 = time.perf_counter()
            O.herlev_train_step(cur, prev, x, y, opt, num_classes=classes, class_weights=cw)
            times.append(time.perf_counter() - t0)
            print(f"cpu baseline (herlev): {threads} threads, step {i + 1}/{steps}: "
                  f"{times[-1]:.2f} s", file=sys.stderr, flush=True)
        times.sort()
        rates[threads] = round(batch / times[len(times) // 2], 4)
    top = max(thread_counts)
    return {"value": rates[top], "unit": "images/sec", "cores": top, "kind": "port",
            "by_cores": {str(k): v for k, v in rates.items()},
            "sample": f"oracle Herlev UG step (bs{batch} {res}^2, {classes} classes: S4 classifier "
                      f"fwd+bwd with dropout + S3 prediction at 128^2 + UG CE + Adam), torch CPU "
                      f"fp32, median of {steps} steps after 1 warm-up, at "
                      f"{' and '.join(str(k) for k in thread_counts)} threads (= physical cores)"}


def roofline_from(timer, steps, every, math):
    """(roofline, kernels) of the live-timed conv launches: the dominant kernel's
    algorithmic FLOPs / its HIP-event time, against the peak of the arithmetic it runs."""
    summ = timer.summary()
    sampled = len(range(0, steps, every))
    kernels = {k: {"launches": v["launches"], "ms_per_step": round(v["ms"] / sampled, 3),
                   "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2)}
               for k, v in summ.items()}
    dom = max(summ, key=lambda k: summ[k]["ms"])
    d = summ[dom]
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    peak = {"x6": BF16_PEAK_TFLOPS / X6_PRODUCTS, "bf16": BF16_PEAK_TFLOPS}.get(
        math, FP32_PEAK_TFLOPS)
    traffic, src = pmc_traffic(dom, bf16=math == "bf16")
    roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2),
            "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_source": src,
            "arithmetic": {"x6": "split-bf16 x6: fp32-accurate products from 6 bf16 MFMAs; "
                                 "peak = dense bf16 MFMA peak / 6",
                           "bf16": "bf16 operands, fp32 accumulation: dense bf16 MFMA peak"
                           }.get(math, "fp32 MFMA"),
            "flops_per_launch": round(d["flops"] / d["launches"]),
            "avg_launch_ms": round(d["ms"] / d["launches"], 4),
            "timed_steps": f"{sampled} of {steps} (every {every})"}
    return roof, kernels


def pmc_traffic(family, bf16=False):
    """HBM bytes per launch of a kernel family from the newest committed PMC summary of
    the same arithmetic (profiles/*_pmc.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 read correction; the bf16 runs'
    summaries carry "bf16" in their name); None when absent."""
    # newest = last by name (r1c < r1d < ...): a checkout gives every file the same mtime
    files = sorted((p for p in (ROOT / "profiles").glob("*_pmc.json") if ("bf16" in p.name) == bf16),
                   key=lambda p: p.name)
    if not files:
        return None, None
    rows = json.load(open(files[-1]))
    sel = [r for k, r in rows.items() if k.split("<")[0].split("::")[-1].startswith(family + "_")
           or k.split("<")[0].split("::")[-1] == family + "_kernel"]
    calls = sum(r["calls"] for r in sel)
    if not calls:
        return None, None
    return round(sum(r["calls"] * r["hbm_bytes"] for r in sel) / calls), f"profiles/{files[-1].name}"


def main():
    args = parse()
    args.roofline_every = max(1, args.roofline_every)
    if args.workload == "herlev":
        return main_herlev(args)
    import torch
    import torch.distributed as dist
    import ugpg
    from ugpg import ops
    from ugpg.dist import init_from_env, max_over_ranks, sync_batchnorm_enabled
    from ugpg.trainer import MetricsReadback

    ops.set_conv_math(args.conv_math)
    # UGPG_DIST_BACKEND / UGPG_BENCH_DEVICE: rehearsal of the N-rank path on one GPU
    # (gloo, every rank on device 0); the driver's runs use RCCL, one GPU per rank
    rank, world = init_from_env(os.environ.get("UGPG_DIST_BACKEND", "nccl"))
    local = int(os.environ.get("UGPG_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but world size {world}", file=sys.stderr)

    torch.manual_seed(1234)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
    tr.current_stage = 4
    tr.current_model = tr.models[4]
    tr.setup_optimizer(4)  # (the trainer constructor already made the replicas equal)
    B, R = args.batch, args.res
    # --res other than 256: the U map comes from Stage 3 at half the resolution, as in the
    # reference's 128 -> 256 schedule
    tr.stage_configs[4]["resolution"], tr.stage_configs[3]["resolution"] = R, R // 2
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(B, 3, R, R, generator=g).to(dev)
    t = (torch.rand(B, 1, R, R, generator=g) < 0.5).float().to(dev)
    tr.current_model.train()
    tr.models[3].eval()
    if args.graph:
        if world > 1:
            raise SystemExit("--graph: single process only")
        tr.enable_graphs()

    def run(n, timer=None):
        # the trainer's epoch loop: step k's metrics are read back (pinned copy +
        # event) after step k+1 has been enqueued, so the GPU never waits on Python.
        # `timer`: the live roofline's HIP events bracket every conv launch of the steps
        # k = 0, E, 2E, ... (E = --roofline-every): an event pair costs ~3 us of GPU time
        # per launch (2.5 % of the step when every step is bracketed), the sample does not
        pending, last = None, None
        for k in range(n):
            ops.TIMER = timer if timer is not None and k % args.roofline_every == 0 else None
            cur = MetricsReadback(tr.train_step(x, t, 4))
            if pending is not None:
                last = pending.values()
            pending = cur
        return pending.values() if pending is not None else last

    last = run(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = None if args.no_roofline else ops.KernelTimer()
    t0 = time.perf_counter()
    last = run(args.steps, timer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.TIMER = None
    elapsed = max_over_ranks(elapsed, dev)
    ms = 1000 * elapsed / args.steps
    value = world * B * args.steps / elapsed

    # secondary line (after the timed region): the pure S4 fwd+bwd step without the
    # uncertainty map = forward + BCE(pos_weight) + backward + all-reduce + RMSprop
    secondary = None
    if args.secondary_steps > 0:
        from ugpg.dist import allreduce_gradients, overlapped_allreduce
        from ugpg.loss import weighted_loss_tensors

        def step_plain():
            mbuf = torch.zeros(8, dtype=torch.float32, device=dev)
            tr.optimizer.zero_grad()
            out = tr.current_model(x)
            final, _ = weighted_loss_tensors(tr.base_criterion, out, t, None, 1.0, out=mbuf[0:2])
            with overlapped_allreduce():
                final.backward()
            tr.optimizer.grad_scale = allreduce_gradients(
                [p for g in tr.optimizer.param_groups for p in g["params"]])
            tr.optimizer.step()
            return mbuf.tolist()

        step_plain()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.secondary_steps):
            step_plain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el2 = max_over_ranks(time.perf_counter() - t1, dev)
        secondary = {"metric": "images/sec Stage-4 256x256 bs16 fwd+bwd without uncertainty map",
                     "value": round(world * B * args.secondary_steps / el2, 3),
                     "ms_per_step": round(1000 * el2 / args.secondary_steps, 3),
                     "steps": args.secondary_steps}

    roof, kernels = (None, None) if timer is None else \
        roofline_from(timer, args.steps, args.roofline_every, ops.conv_math())
    # the step's whole-FLOP rate against the peak of the arithmetic the convs run
    step_peak = {"x6": BF16_PEAK_TFLOPS / X6_PRODUCTS, "bf16": BF16_PEAK_TFLOPS}.get(
        args.conv_math, FP32_PEAK_TFLOPS)

    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if args.conv_math == "bf16" else "fp32",
        "data": "synthetic (x~N(0,1), masks~Bernoulli(0.5); random-init weights)",
        "config": {"workload": "Stage-4 uncertainty-guided train step: PGUNet4 fwd+bwd 256^2 + "
                               "PGUNet3 eval fwd 128^2 (U-map) + weighted BCE + RMSprop",
                   "per_gpu_batch": B, "global_batch": B * world, "resolution": R,
                   "parallelism": f"dp{world}",
                   "batchnorm": "sync (global batch)" if sync_batchnorm_enabled() else "local (per rank)",
                   "execution": ("hipGraph replay of the whole step (eager on the sampled roofline steps)"
                                 if args.graph else "eager launches"),
                   "baseline_config": ("BASELINE.json configs[2] arithmetic (bf16 conv operands, "
                                       "fp32 accumulation, bf16 activation storage)" if args.conv_math == "bf16"
                                       else "BASELINE.json configs[1]")},
        "step_roofline": {"gflop_per_image": UG_STEP_GFLOP,
                          "achieved_tflops_per_gpu": round(value / world * UG_STEP_GFLOP / 1e3, 2),
                          "peak_tflops": round(step_peak, 1),
                          "frac": round(value / world * UG_STEP_GFLOP / 1e3 / step_peak, 4)},
        "roofline": roof,
        "kernels": kernels,
        "last_step_metrics": {"loss": last[0], "base_loss": last[1], "dice": last[2],
                              "unc_mean": last[5], "unc_std": last[6]},
        "cpu_baseline": None,
        "secondary": secondary,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        phys = cpu_cores()
        counts = sorted({phys, min(8, phys)})
        result["cpu_baseline"] = cpu_baseline(B, R, args.cpu_steps, counts)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_herlev(args):
    """BASELINE.json configs[3]: the Herlev Stage-4 classifier uncertainty-guided training
    step (Herlev/train_herlev.py:298-325 with the UG forward pass :216-296) on one GPU:
    ugpg's HerlevTrainer.train_step = PGUNet4 encoder + classifier fwd/bwd (dropout
    active) + the Stage-3 classifier's eval prediction at 128^2 + UG CE + Adam.  bs16
    synthetic N(0,1) images at --res (224 = the reference's Stage-4 resolution, 256 =
    BASELINE's), labels ~ U{0..K-1}, random-init weights, fp32 (split-bf16 convs)."""
    import torch
    import ugpg  # noqa: F401
    from ugpg import ops
    from ugpg.dist import init_from_env, max_over_ranks
    from ugpg.herlev import HerlevTrainer
    ops.set_conv_math(args.conv_math)
    rank, world = init_from_env(os.environ.get("UGPG_DIST_BACKEND", "nccl"))
    local = int(os.environ.get("UGPG_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(1234)
    K, B, R = args.classes, args.batch, args.res
    tr = HerlevTrainer({"device": dev, "epochs_per_stage": 1, "num_classes": K,
                        "class_weights": torch.linspace(0.5, 2.0, K).tolist(),
                        "uncertainty_alpha": 1.0, "weight_decay": 1e-4, "stage4_resolution": R})
    tr.setup_optimizer_scheduler(4)
    tr.models[4].train()
    tr.models[3].eval()
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(B, 3, R, R, generator=g).to(dev)
    y = torch.randint(0, K, (B,), generator=g).to(dev)

    def run(n, timer=None):
        last = None
        for k in range(n):
            ops.TIMER = timer if timer is not None and k % args.roofline_every == 0 else None
            out = tr.train_step(x, y, 4)
            if last is not None:
                last.tolist()  # the trainer's per-batch host read, one step behind
            last = out
        return last.tolist()

    run(args.warmup)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    timer = None if args.no_roofline else ops.KernelTimer()
    t0 = time.perf_counter()
    last = run(args.steps, timer)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ops.TIMER = None
    value = world * B * args.steps / elapsed
    gf = herlev_gflop(R)
    roof, kernels = (None, None) if timer is None else \
        roofline_from(timer, args.steps, args.roofline_every, ops.conv_math())
    result = {
        "metric": f"images/sec Herlev Stage-4 classifier UG train step {R}x{R} bs{B}",
        "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if args.conv_math == "bf16" else "fp32",
        "data": "synthetic (x~N(0,1), labels~U{0..K-1}; random-init weights)",
        "config": {"workload": "Herlev Stage-4 classifier UG train step: PGUNet4 encoder + "
                               "classifier fwd+bwd (dropout) + PGUNet3 classifier eval at 128^2 "
                               "+ uncertainty-weighted CE + Adam",
                   "per_gpu_batch": B, "global_batch": B * world, "resolution": R,
                   "classes": K, "parallelism": f"dp{world}",
                   "baseline_config": "BASELINE.json configs[3]"},
        "step_roofline": {"gflop_per_image": round(gf, 3),
                          "achieved_tflops_per_gpu": round(value / world * gf / 1e3, 2)},
        "roofline": roof, "kernels": kernels,
        "last_step_metrics": {"loss": last[0], "base_loss": last[1], "w_mean": last[2],
                              "w_std": last[3]},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        phys = cpu_cores()
        result["cpu_baseline"] = cpu_baseline_herlev(B, R, args.cpu_steps,
                                                     sorted({phys, min(8, phys)}), K)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
