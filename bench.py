#!/usr/bin/env python3
"""Throughput benchmark: D+G training iterations per second on synthetic images.

Workload (BASELINE.json configs[1]): RaSGAN (--loss_D 6) DCGAN 128x128, h=128, batch 64
per GPU, fp32 (weak scaling: global batch = 64 * n_gpus).  One "step" = one reference
iteration (GLI:560-714): D step (D(real), G(z) no-grad, D(fake), head, backward, Adam)
+ G step (G(z), D(fake), fresh real batch D(x), head, backward, Adam).  Inputs are
resident in HBM (a 1024-image synthetic set; batches gathered on the device, z drawn
on the device).

Prints ONE JSON line (rank 0).  Extra fields:
  roofline     -- the dominant kernel (the fp32-MFMA implicit-GEMM conv): algorithmic
                  FLOPs / its HIP-event-timed duration over the timed region, against
                  the fp32 MFMA peak (157.3 TFLOP/s);
  cpu_baseline -- the oracle (CPU restatement of the reference step, torch CPU fp32) on
                  a bounded sample of the same workload on this host (rank 0, N=1).
Launch: python bench.py [--gpus N --steps K --warmup W]; N>1 under torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train images/sec (D+G step) RaLSGAN DCGAN 64²/256² at 1/2/4/8 GPU; MFMA util"
FP32_MFMA_PEAK = 157.3e12  # MI355X_MICROARCH.md: Peak FP32 (matrix) = vector peak

WORKLOADS = {
    # name: (loss_D, image_size, batch per GPU, h)
    "C2": (6, 128, 64, 128),   # BASELINE configs[1]: RaSGAN DCGAN 128x128 batch 64, one MI355X
    "C1": (7, 64, 32, 128),    # configs[0] shape (RaLSGAN 64x64 B32) on the GPU
    "C3": (7, 256, 32, 128),   # configs[2] per-GPU shard: RaLSGAN 256x256, 32 per GPU
    "C3h32": (7, 256, 32, 32),
    "C5": (8, 128, 32, 128),   # spectral RaHinge 128x128 (spectral flag set below)
}


def conv_flops_per_iteration(t):
    """9 F_D + 4 F_G - 2 d0 - g0; F = forward conv FLOPs (2*MACs)."""
    def layer_flops(net, x_shape):
        out, h = [], torch.zeros(x_shape, device="meta")
        for layer in net._plan:
            c = layer.conv
            geom = layer.spec.geom
            if layer.in_view is not None:
                h = torch.zeros((h.shape[0],) + tuple(layer.in_view), device="meta")
            B, cin, H, W = h.shape
            w = c.w if hasattr(c, "w") else c.weight
            if layer.w_view is not None:
                w = w.view(*layer.w_view)
            cout = w.shape[1] if geom.transposed else w.shape[0]
            Ho, Wo = geom.out_hw(H, W)
            pix = H * W if geom.transposed else Ho * Wo
            out.append(2.0 * B * cin * cout * geom.k * geom.k * pix)
            h = torch.zeros((B, cout, Ho, Wo), device="meta")
            if layer.out_view is not None:
                h = torch.zeros((B,) + tuple(layer.out_view), device="meta")
        return out
    p = t.p
    fg = layer_flops(t.G, (t.B, p.z_size, 1, 1))
    fd = layer_flops(t.D, (t.B, p.n_colors, p.image_size, p.image_size))
    return 9 * sum(fd) + 4 * sum(fg) - 2 * fd[0] - fg[0]


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "round1_c2_pmc_traffic.json")


def pmc_traffic(workload, symbol):
    """HBM-side bytes per launch of `symbol` from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.sh on this bench command: FETCH_SIZE x2 + WRITE_SIZE), or None."""
    if workload != "C2" or not os.path.exists(PMC_TRAFFIC):
        return None, None
    with open(PMC_TRAFFIC) as f:
        d = json.load(f)
    ent = d.get(symbol)
    if ent is None:
        return None, None
    return ent["bytes_per_launch"], os.path.relpath(PMC_TRAFFIC, ROOT)


def cpu_baseline(loss_D, size, batch, h, spectral, seconds_hint):
    """Oracle (CPU restatement, pinned to the reference) on this host: bounded sample."""
    from oracle.reference_cpu import Trainer as OracleTrainer, make_param, synthetic_images
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    p = make_param(loss_D=loss_D, image_size=size, batch_size=batch, G_h_size=h, D_h_size=h, seed=1, cuda=False,
                   print_every=10 ** 9, spectral=spectral)
    t = OracleTrainer(p, synthetic_images(256, size))
    t.iteration(1)  # warm-up (i=1: skips the i=0 sample-image forward)
    n, t0 = 0, time.perf_counter()
    while True:
        t.iteration(2 + n)
        n += 1
        el = time.perf_counter() - t0
        if el > seconds_hint or n >= 5:
            break
    return {"value": batch * n / el, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} timed + 1 warm-up oracle iterations of the same workload (B={batch}, {size}^2, h={h}), "
                      f"torch {torch.__version__} CPU fp32, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--sync-bn", action="store_true",
                    help="SyncBN over ranks (default: per-shard BN = the reference's DataParallel)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RGAN_BENCH_BACKEND=gloo + more ranks than GPUs: rehearsal of the N>1 path on one GPU
    backend = os.environ.get("RGAN_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    from relativisticgan_amd import dp, kernels as K
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        dp.setup(sync_bn=args.sync_bn)
    loss_D, size, bpg, h = WORKLOADS[args.workload]
    spectral = args.workload == "C5"
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg * world, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=spectral, rgan_rng="device")
    images = synthetic_images(1024, size, device="cuda")
    t = Trainer(p, images)
    flops_iter = conv_flops_per_iteration(t)

    for i in range(args.warmup):
        t.iteration(i + 1)
    t.flush()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    K.profile_begin(capacity=200 * args.steps + 64)
    t0 = time.perf_counter()
    for i in range(args.steps):
        t.iteration(args.warmup + 1 + i)
    t.flush()  # the last G step (deferred under DP) is inside the timed region
    barrier()
    elapsed = time.perf_counter() - t0
    prof = K.profile_end()
    if world > 1:
        e = torch.tensor([elapsed], device="cuda")
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    imgs = bpg * world * args.steps
    value = imgs / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    # dominant kernel = the conv kernel symbol with the most time (HIP events around each
    # launch on its stream); the whole conv family is reported beside it
    gemm_ms, gemm_flops = prof["ms"], prof["flops"]
    top = max(prof["kernels"], key=lambda k: k["ms"])
    achieved = top["flops"] / (top["ms"] / 1000.0)
    traffic, traffic_src = pmc_traffic(args.workload, top["name"])
    roofline = {"bound": "mfma", "achieved": achieved / 1e12, "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
                "frac": achieved / FP32_MFMA_PEAK, "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": traffic_src, "kernel": top["name"], "launches": top["launches"],
                "avg_launch_us": 1000.0 * top["ms"] / top["launches"],
                "flops_per_launch": top["flops"] / top["launches"],
                "conv_family": {"achieved": gemm_flops / (gemm_ms / 1000.0) / 1e12, "launches": prof["launches"],
                                "ms_per_step": gemm_ms / args.steps,
                                "frac": gemm_flops / (gemm_ms / 1000.0) / FP32_MFMA_PEAK,
                                "kernels": prof["kernels"]}}
    out = {
        "metric": METRIC, "value": value, "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": f"{args.workload}: loss_D {loss_D} DCGAN arch0 {size}x{size}, h={h}, "
                               f"batch {bpg}/GPU{', spectral D' if spectral else ''}",
                   "loss_D": loss_D, "image_size": size, "batch_per_gpu": bpg, "global_batch": bpg * world,
                   "G_h_size": h, "D_h_size": h, "parallelism": f"dp{world}",
                   "batchnorm": "SyncBN" if args.sync_bn else "per-shard (reference DataParallel)"},
        "step_mfma_util": flops_iter * args.steps / elapsed / (world * FP32_MFMA_PEAK),
        "conv_tflop_per_step": flops_iter / 1e12,
        "roofline": roofline,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(loss_D, size, bpg, h, spectral, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
