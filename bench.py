#!/usr/bin/env python3
"""UP-Retinex hot-path benchmark (BASELINE.json metric: images/s at 512x512 bs=32).

One step = one MultiScaleUP_Retinex forward over one resident batch of 32
synthetic 512x512 images per GPU (configs[1]: random-init plain model, fp32;
--precision fp16 --variant preact_aspp gives configs[2]).  Multi-GPU: one
process per GPU.  `--gpus N` (N > 1) run directly makes this process a pure
launcher (it never touches the GPU): it starts `torch.distributed.run` with N
ranks on 127.0.0.1 and exits with its code; run under torch.distributed.run
(WORLD_SIZE set) it is one rank.  Each rank processes its own 32-image shard
with no data-path collective (weak scaling); `--collect` adds the final
collect of SURVEY §8e inside the timed region (one RCCL all_gather_into_tensor
of the fp16 enhanced images per step).  Barrier + synchronize bracket the
timed region and rank 0 reports the max over ranks.  `--dry-run` replaces the
GPU work by a small CPU step over gloo (tests the launcher / rank plumbing on
a machine without a GPU).

Extra objects on the JSON line:
  roofline      the conv kernel family (CONV_KERNELS below, ~97% of device time), timed live with HIP events around every
                launch of the last timed step on the model's stream
                (upr_model_profile); traffic from rocprofv3 FETCH_SIZE/WRITE_SIZE
                child passes run before this process touches the GPU;
                --ceilings adds the fractions against measured MFMA / HBM rates
  cpu_baseline  the CPU oracle forward (oracle/net.py, torch-CPU fp32) on the
                host cores, rank 0 only: the full timed batch in one forward
                when a one-image warm-up predicts <= 30 s, else a bounded sample
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "retinex-image-enhancement_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

PEAK_TFLOPS = {"fp32": 157.3, "fp16": 2516.6}   # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
REF_GFLOP_PER_IMG = {"plain": 105.6, "preact_aspp": 123.4}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--precision", choices=["fp32", "fp16"], default="fp32")
    ap.add_argument("--variant", choices=["plain", "preact_aspp"], default="plain")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline budget (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-launch HIP events")
    ap.add_argument("--breakdown", action="store_true", help="print per-layer stats to stderr")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--ceilings", action="store_true",
                    help="after the timed steps, measure the chip's reachable fp16 MFMA and HBM-copy rates "
                         "(upr/calib.py, ~5 s) and report the roofline fractions against them as well")
    ap.add_argument("--train", action="store_true",
                    help="configs[4]: one training step (fwd + TotalLoss + bwd + clip + Adam) per step, "
                         "bs=8 512x512 plain model (batch/size overridable)")
    ap.add_argument("--collect", action="store_true",
                    help="time the final collect too: all_gather_into_tensor of the fp16 enhanced images (RCCL)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks run a small CPU step through the same launch / barrier / report path")
    ap.add_argument("--amp", action="store_true",
                    help="with --train: the reference's AMP branch (GradScaler: scaled backward, unscale_, "
                         "skip on inf/nan, scale update); arithmetic stays fp32")
    return ap.parse_args()


def cpu_baseline(sd, pre, aspp, size, budget_s, batch):
    """Oracle forward on host cores.  After a one-image warm-up, the full
    `batch` (the timed GPU workload's shape) runs as one forward
    when the warm-up predicts it fits in max(budget, 30 s); otherwise single
    images until the budget is spent."""
    from oracle import net as onet  # checker / baseline only
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    x = torch.rand(1, 3, size, size, generator=torch.Generator().manual_seed(99))
    with torch.no_grad():
        t0 = time.perf_counter()
        onet.forward(sd, x, pre, aspp)  # warm-up
        t1 = time.perf_counter() - t0
        if t1 * batch <= max(budget_s, 30.0):
            xb = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(99))
            t0 = time.perf_counter()
            onet.forward(sd, xb, pre, aspp)
            el = time.perf_counter() - t0
            return {"value": batch / el, "unit": "images/s", "cores": threads, "kind": "port",
                    "sample": f"one {batch}x3x{size}x{size} fp32 forward of oracle/net.py (torch-CPU, the full "
                              f"timed batch) after a 1-image warm-up, {el:.1f}s"}
        n, t0 = 0, time.perf_counter()
        while True:
            onet.forward(sd, x, pre, aspp)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 64:
                break
    return {"value": n / el, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} x 1x3x{size}x{size} fp32 forwards of oracle/net.py (torch-CPU), {el:.1f}s"}


def parity_vs_cpu(sd, pre, aspp, x, outs, precision):
    """Per-pixel max |d| of image 0 of the last timed step's outputs against the
    CPU oracle (oracle/net.py, fp32) on the same input (the fp16 run's input is
    the fp16-rounded image, widened to fp32 for the oracle)."""
    from oracle import net as onet  # checker only
    with torch.no_grad():
        ref = onet.forward(sd, x[:1].float().cpu(), pre, aspp)
    names = ("enhanced", "reflectance", "illumination")
    d = {n: (o[:1].float().cpu() - r).abs().max().item() for n, o, r in zip(names, outs, ref)}
    if precision == "fp16":  # reflectance x/(I+1e-6) is unbounded: relative to max(1, max|R|) as in the tests
        d["reflectance"] /= max(1.0, ref[1].abs().max().item())
    tol = 1e-3  # fp32: north_star; fp16: tests/test_gpu_bn_parity.py FP16_TOL
    return {"max_abs_diff": d, "tol": tol, "pass": all(v <= tol for v in d.values()),
            "sample": "image 0 of the last timed batch vs oracle/net.py fp32 on host cores"}


# every kernel launch_conv dispatches to (the bench's conv family = the executor's GEMM ops)
CONV_KERNELS = ("conv_halo_kernel", "conv_igemm_kernel", "conv_wide_kernel", "conv_wide32_kernel",
                "conv_stream_kernel", "conv_stream_fam_kernel", "conv_ring_kernel", "conv_ring32_kernel",
                "conv_hwide_kernel", "conv_hwide3_kernel", "conv_t2_kernel", "conv_t2_f32_kernel")


def pmc_traffic(args):
    """HBM bytes of the conv kernels per forward from rocprofv3 PMC counters.

    Runs BEFORE this process touches the GPU: two child passes of this script
    (one forward of warm-up + one timed) under `rocprofv3 --pmc FETCH_SIZE` and
    `--pmc WRITE_SIZE` (separate passes: they do not fit one pass on gfx950).
    FETCH_SIZE (KB) reports half the bytes of wide coalesced reads on gfx950, so
    it is doubled (MI355X_MICROARCH.md, HBM section).  Returns None on failure."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None
    out = {}
    base = [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "1", "--cpu-seconds", "0",
            "--no-profile", "--no-traffic", "--batch", str(args.batch), "--size", str(args.size),
            "--precision", args.precision, "--variant", args.variant]
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="upr_pmc_", dir="/tmp")
        cmd = [exe, "--pmc", ctr, "--kernel-trace", "-T", "-d", d, "-o", "p", "--output-format", "csv", "--"] + base
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=300, check=True)
            path = None
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        path = os.path.join(root, f)
            if path is None:
                return None
            tot, n = 0.0, 0
            with open(path) as f:
                for r in csv.DictReader(f):
                    if r["Counter_Name"] == ctr and any(k in r["Kernel_Name"] for k in CONV_KERNELS):
                        tot += float(r["Counter_Value"])
                        n += 1
            out[ctr] = (tot, n)
        except Exception:
            return None
        finally:
            shutil.rmtree(d, ignore_errors=True)
    fetch_kb, n_launch = out["FETCH_SIZE"]
    write_kb, _ = out["WRITE_SIZE"]
    if n_launch == 0:
        return None
    per_fwd = (2.0 * fetch_kb + write_kb) * 1024.0 / 2.0  # 2 forwards (1 warm-up + 1 timed)
    return {"bytes_per_launch": per_fwd / (n_launch / 2.0), "bytes_per_forward": per_fwd,
            "read_bytes_per_forward": 2.0 * fetch_kb * 1024.0 / 2.0, "write_bytes_per_forward": write_kb * 1024.0 / 2.0,
            "launches_per_forward": n_launch / 2.0}


def launch_ranks(args):
    """`--gpus N` without WORLD_SIZE: this process is only the launcher and never
    initialises the GPU.  It runs torch.distributed.run with N ranks (one per
    GPU, rendezvous on 127.0.0.1) over this same script and exits with its code;
    rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    """(world, rank, device) of this process; initialises the process group
    (RCCL over xGMI on the GPU, gloo for --dry-run) when WORLD_SIZE > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            torch.distributed.init_process_group("gloo")
        return world, rank, torch.device("cpu")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    return world, rank, dev


def sync(world, dev):
    if world > 1:
        torch.distributed.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def max_over_ranks(world, dev, seconds):
    if world == 1:
        return seconds
    t = torch.tensor([seconds], device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return t.item()


def dry_run(args):
    """The launcher / rank / barrier / max-over-ranks / report path with a small
    CPU step in place of the forward (CPU test of --gpus N, gloo)."""
    world, rank, dev = dist_setup(args)
    torch.manual_seed(rank)
    a = torch.rand(256, 256)
    for _ in range(args.warmup):
        a = torch.tanh(a @ a.T / 256)
    sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = torch.tanh(a @ a.T / 256)
    sync(world, dev)
    elapsed = max_over_ranks(world, dev, time.perf_counter() - t0)
    ranks = [None] * world
    if world > 1:
        torch.distributed.all_gather_object(ranks, (rank, os.getpid()))
    else:
        ranks = [(rank, os.getpid())]
    if rank == 0:
        print(json.dumps({"metric": "dry run (no GPU work)", "value": world * args.steps / elapsed, "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1000.0 * elapsed / args.steps, "ranks": ranks, "data": "none"}))
    if world > 1:
        torch.distributed.destroy_process_group()


TRAIN_GFLOP_PER_IMG = 668.0  # model fwd+bwd + VGG19 fwd x2 + dgrad, 512x512


def cpu_train_baseline(sd, size, budget_s):
    """Oracle training step (oracle/train.py, torch-CPU fp32) on 1 image until the budget is spent."""
    from oracle import train as otrain
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    vgg = otrain.vgg19_state(1234)
    x = torch.rand(1, 3, size, size, generator=torch.Generator().manual_seed(98))
    n, t0 = 0, time.perf_counter()
    while True:
        sdc = {k: v.clone() for k, v in sd.items()}
        otrain.train_step(sdc, vgg, x, False, False)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 16:
            break
    return {"value": n / el, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} x 1x3x{size}x{size} training steps of oracle/train.py (torch-CPU autograd), {el:.1f}s"}


def train_main(args):
    world, rank, dev = dist_setup(args)
    from models.model import UP_Retinex
    from losses.loss import TotalLoss
    from trainers.train import make_optimizer, train_step
    B = args.batch if args.batch != 32 else 8
    S = args.size
    torch.manual_seed(0)
    model = UP_Retinex(use_preact=args.variant == "preact_aspp", use_aspp=args.variant == "preact_aspp")
    sd_cpu = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev).train()
    crit = TotalLoss(use_freq_loss=True).to(dev)
    opt = make_optimizer(model, lr=1e-4, weight_decay=1e-5)
    x = torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(2 + rank)).to(dev)
    from upr.dist import allreduce_grads
    scaler = None
    if args.amp:
        from trainers.train import GradScaler
        scaler = GradScaler()

    def tstep():
        if world == 1:
            return train_step(model, x, crit, opt, scaler=scaler, use_amp=args.amp)
        return train_step(model, x, crit, opt, scaler=scaler, use_amp=args.amp,
                          grad_hook=lambda: allreduce_grads(opt))

    for _ in range(args.warmup):
        tstep()
    sync(world, dev)
    t0 = time.perf_counter()
    d = None
    for _ in range(args.steps):
        _, d = tstep()
    sync(world, dev)
    elapsed = max_over_ranks(world, dev, time.perf_counter() - t0)
    imgs = world * B * args.steps
    gf = TRAIN_GFLOP_PER_IMG * (S / 512.0) ** 2
    achieved = gf * B * args.steps / elapsed / 1e3
    out = {
        "metric": f"train images/sec at {S}x{S} bs={B} (UP-Retinex fwd + TotalLoss + bwd + clip + Adam)",
        "value": imgs / elapsed, "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "f16 convs under autocast (fp32 accumulate; fp16-operand weight gradients; fp32 BN / loss / Adam)" if args.amp else "f32",
        "data": "synthetic torch.rand inputs, random-init weights (seed 0), seeded random-init VGG19 (seed 1234)",
        "config": {"workload": f"configs[4]: bs={B}/GPU {S}x{S} {args.variant} train step"
                               + (" AMP: autocast (fp16 MFMA convs) + GradScaler" if args.amp else " (fp32)"),
                   "global_batch": world * B, "image_size": S, "variant": args.variant,
                   "parallelism": f"data-parallel x{world} (per-rank shard"
                                  + (", RCCL all-reduce of the flat gradient buffer)" if world > 1 else ")")},
        "last_loss": d,
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
                     "frac": achieved / PEAK_TFLOPS["fp32"], "traffic": None,
                     "kernel": "whole training step (algorithmic 668 GF/img at 512^2 over step time)"},
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_train_baseline(sd_cpu, S, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


def _cfg_index(args):
    """BASELINE.json configs[] entry a forward run corresponds to."""
    if args.size == 1024 and args.variant == "preact_aspp":
        return 3  # bs=256 1024^2 over 8 GPUs = 32 per GPU
    return 1 if args.precision == "fp32" and args.variant == "plain" else 2


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        return dry_run(args)
    if args.train:
        return train_main(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    traffic = None
    if world == 1 and not args.no_traffic and not any(k.startswith("ROCPROF") for k in os.environ):
        traffic = pmc_traffic(args)  # child processes, before this process initialises the GPU
    world, rank, dev = dist_setup(args)

    from models.model import UP_Retinex
    pre = aspp = args.variant == "preact_aspp"
    torch.manual_seed(0)
    model = UP_Retinex(use_preact=pre, use_aspp=aspp).eval()
    sd_cpu = {k: v.clone() for k, v in model.state_dict().items()}
    dt = torch.float16 if args.precision == "fp16" else torch.float32
    model = model.to(dev)
    if args.precision == "fp16":
        model = model.half()
    B, S = args.batch, args.size
    g = torch.Generator().manual_seed(1 + rank)
    x = torch.rand(B, 3, S, S, generator=g).to(dev, dt)

    collect = None
    if args.collect:
        from upr.dist import gather_shards
        collect = gather_shards

    gathered = [None]

    def step():
        with torch.no_grad():
            out = model(x)
            if collect is not None:  # SURVEY §8e final collect: fp16 enhanced images of every rank
                gathered[0] = collect(out[0].half(), world * B)
            return out

    last = [None]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    handle = next(iter(model.__dict__["_upr_cache"].values()))[1]

    # The per-launch HIP events of the roofline are recorded in the LAST timed
    # step only (a sample inside the timed region): events around every launch
    # of every step cost ~5% of the fp16 step (two event packets per launch).
    sync(world, dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1 and not args.no_profile:
            handle.profile(True)
        last[0] = step()
    sync(world, dev)
    elapsed = time.perf_counter() - t0
    stats = handle.profile_read() if not args.no_profile else []
    handle.profile(False)
    elapsed = max_over_ranks(world, dev, elapsed)

    total_imgs = world * B * args.steps
    out = {
        "metric": f"images/sec at {S}x{S} bs={B} per GPU (UP-Retinex forward)",
        "value": total_imgs / elapsed,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "f16 (fp32 accumulate)",
        "data": "synthetic torch.rand inputs, random-init weights (torch.manual_seed(0))",
        "config": {"workload": f"configs[{_cfg_index(args)}]: bs={B}/GPU {S}x{S} "
                               f"{args.variant} forward, {args.precision}",
                   "global_batch": world * B, "image_size": S, "variant": args.variant,
                   "parallelism": f"batch-shard x{world} " + (
                       "(+ timed final collect: RCCL all_gather_into_tensor of fp16 enhanced)" if args.collect
                       else "(no data-path collective)")},
    }
    if stats:
        gemm = [s for s in stats if s["kind"] == "conv_igemm"]
        g_ms = sum(s["ms"] for s in gemm)
        g_calls = sum(s["calls"] for s in gemm)
        g_flops = sum(s["flops"] for s in gemm)
        g_bytes = sum(s["bytes"] for s in gemm)
        all_ms = sum(s["ms"] for s in stats)
        achieved = g_flops / (g_ms * 1e-3) / 1e12 if g_ms > 0 else 0.0
        peak = PEAK_TFLOPS[args.precision]
        # per-layer roofline: each conv launch is bounded by max(flops / MFMA
        # peak, algorithmic bytes / HBM peak); layer_frac = sum of those bounds
        # over the measured conv time (1.0 = every conv at its own roofline)
        t_roof = sum(max(s["flops"] / (peak * 1e12), s["bytes"] / (PEAK_HBM_GBS * 1e9)) for s in gemm)
        n_hbm = sum(1 for s in gemm if s["bytes"] / (PEAK_HBM_GBS * 1e9) > s["flops"] / (peak * 1e12))
        out["roofline"] = {
            "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "traffic_unit": "bytes per conv launch (rocprofv3 FETCH_SIZE*2 + WRITE_SIZE)",
            "traffic_per_img_GB": traffic["bytes_per_forward"] / B / 1e9 if traffic else None,
            "alg_bytes_per_launch": g_bytes / max(g_calls, 1),
            "kernel": "conv family: " + "/".join(k[:-7] for k in CONV_KERNELS) + " (all conv launches of the step)",
            "profiled_steps": 1,
            "launches_per_step": g_calls,
            "avg_launch_us": 1000.0 * g_ms / max(g_calls, 1),
            "gemm_gflop_per_img": g_flops / B / 1e9,
            "gemm_alg_GB_per_img": g_bytes / B / 1e9,
            "gemm_share_of_device_time": g_ms / all_ms if all_ms else None,
            "layer_roofline_frac": (t_roof * 1e3) / g_ms if g_ms > 0 else None,
            "layer_roofline_note": f"sum over conv launches of max(flops/MFMA peak, alg bytes/HBM peak) / measured; "
                                   f"{n_hbm} of {len(gemm)} conv ops are HBM-bound at {args.precision}",
            "ref_equiv_tflops": REF_GFLOP_PER_IMG[args.variant] * (S / 512) ** 2 * total_imgs / world / elapsed / 1e3,
        }
        if args.ceilings:
            from upr.calib import measure
            cz = measure(dev)
            # fp32 MFMA: MI355X_MICROARCH.md's measured 155 TF (99% of nominal), not re-measured here
            mf = cz["mfma_f16_TF"] if args.precision == "fp16" else 155.0
            # HBM: the better of this run's copy kernel and the guide's measured float4 copy (6.29 TB/s)
            hb = max(cz["hbm_copy_TBps"] * 1e3, 6290.0)
            t_meas = sum(max(s["flops"] / (mf * 1e12), s["bytes"] / (hb * 1e9)) for s in gemm)
            out["roofline"]["measured_ceilings"] = {
                "mfma_TFLOPs": mf, "hbm_GBs": hb, "detail": cz,
                "frac_vs_measured_mfma": achieved / mf,
                "layer_roofline_frac_vs_measured": (t_meas * 1e3) / g_ms if g_ms > 0 else None,
                "note": "fp16: best of 1/2 waves per SIMD of back-to-back 16x16x32 MFMAs on random register "
                        "operands after 2 s of load (DVFS-settled clock), measured in this process right after the timed "
                        "steps; HBM: max(this run's best 16-B/lane copy of 1 GiB, read + write, and "
                        "MI355X_MICROARCH.md's measured 6.29 TB/s float4 copy)"}
        if args.breakdown and rank == 0:
            for s in stats:
                tf = s["flops"] / (s["ms"] * 1e-3) / 1e12 if s["ms"] else 0
                gbs = s["bytes"] / (s["ms"] * 1e-3) / 1e9 if s["ms"] else 0
                print(f"{s['name']:44s} {s['kind']:10s} {s['ms'] / max(s['calls'], 1):9.3f} ms "
                      f"{tf:8.1f} TF/s {gbs:8.1f} GB/s", file=sys.stderr)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(sd_cpu, pre, aspp, S, args.cpu_seconds, B)
        out["parity"] = parity_vs_cpu(sd_cpu, pre, aspp, x, last[0], args.precision)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
