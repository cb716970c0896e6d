#!/usr/bin/env python3
"""Throughput benchmark: D+G training iterations per second on synthetic images.

Workload (BASELINE.json metric "RaLSGAN DCGAN 64^2/256^2", configs[2]'s per-GPU shard):
RaLSGAN (--loss_D 7) DCGAN 256x256, h=128 (the reference default, GLI:24-25), batch 32
per GPU, fp32 (weak scaling: global batch = 32 * n_gpus; 8 GPUs = configs[2]'s global
batch 256).  One "step" = one reference iteration (GLI:560-714): D step (D(real), G(z)
no-grad, D(fake), head, backward, Adam) + G step (G(z), D(fake), fresh real batch D(x),
head, backward, Adam).  Inputs are resident in HBM (a 1024-image synthetic set; batches
gathered on the device, z drawn on the device).  On one GPU the line also carries the
64^2 half of the metric (C1: RaLSGAN 64^2, B=32, h=128 = configs[0]'s shape) and
configs[1] (C2: RaSGAN 128^2, B=64) under ``extra_workloads``.

Prints ONE JSON line (rank 0).  Extra fields:
  roofline     -- the dominant kernel (the fp32-MFMA implicit-GEMM conv): algorithmic
                  FLOPs / its HIP-event-timed duration over the timed region, against
                  the fp32 MFMA peak (157.3 TFLOP/s);
  fp32_emulated_bf16x6 -- (N=1) the same workload again with the forward / data-gradient
                  conv GEMMs on the bf16x6 fp32 emulation (rgan_set_gemm_emulation): its
                  throughput and roofline, priced against the bf16 MFMA peak / 6 products;
  cpu_baseline -- the oracle (CPU restatement of the reference step, torch CPU fp32) on
                  a bounded sample of the same workload on this host (rank 0, N=1); C1's
                  own (>= 5 timed iterations) under extra_workloads.C1;
  dp_path_n1   -- (N=1) the workload (and C1) run exactly as each rank of an N>1 run does
                  (launch mode of the data-parallel path: eager above 50M parameters,
                  piecewise graphs below): the like-for-like baseline of the scaling runs.
Launch: python bench.py [--gpus N --steps K --warmup W].  N>1: either under
``torch.distributed.run --nproc-per-node N`` (WORLD_SIZE must equal N), or plain
``python bench.py --gpus N``, which starts the N ranks itself (torch.distributed.run as a
child process, before anything touches the GPU) and relays rank 0's line (the
reference's --n_gpu N, GLI:40, 393-394, 455-456).
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
from relativisticgan_amd.perf import FP32_MFMA_PEAK, conv_flops_per_iteration  # noqa: E402
BF16_MFMA_PEAK = 2.5e15    # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
EMU_PRODUCTS = 6           # bf16 MFMA products per emulated fp32 product (bf16x6)


def kernel_peak(symbol):
    """fp32-equivalent FLOP/s ceiling of a conv kernel symbol: the fp32 MFMA peak, or for the
    bf16x6 emulation the dense bf16 MFMA peak shared by its six products."""
    return BF16_MFMA_PEAK / EMU_PRODUCTS if "bf16x6" in symbol else FP32_MFMA_PEAK

WORKLOADS = {
    # name: (loss_D, image_size, batch per GPU, h)
    "C2": (6, 128, 64, 128),   # BASELINE configs[1]: RaSGAN DCGAN 128x128 batch 64, one MI355X
    "C1": (7, 64, 32, 128),    # configs[0] shape (RaLSGAN 64x64 B32) on the GPU
    "C3": (7, 256, 32, 128),   # configs[2] per-GPU shard: RaLSGAN 256x256, 32 per GPU
    "C3h32": (7, 256, 32, 32),
    "C5": (8, 128, 32, 128),   # spectral RaHinge 128x128 (spectral flag set below)
    "C4": (3, 32, 32, 128),    # configs[3]: WGAN-GP standard CNN (arch 1, 32x32 only: GLI:246,313)
    "C4p": (3, 64, 32, 128),   # configs[3] at 64x64 on DCGAN arch 0 (SURVEY C4')
}
ARCH = {"C4": 1}
DEFAULT_WORKLOAD = "C3"
EXTRA_WORKLOADS = ("C1", "C2")


def pmc_traffic(workload, symbol):
    """HBM-side bytes per launch of `symbol` from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.sh on this bench command: FETCH_SIZE x2 + WRITE_SIZE), or None.
    The newest round's file for the workload wins."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"round*_{workload.lower()}_pmc_traffic.json")),
                   key=lambda f: int(os.path.basename(f).split("_")[0][5:]))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    ent = d.get(symbol)
    if ent is None:
        return None, None
    return ent["bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def host_cpus():
    """The CPUs this process may use: affinity mask, cgroup CPU quota (the lease's share
    on the GPU box), and the machine's model / physical cores (lscpu's fields from
    /proc/cpuinfo)."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model, cores = None, set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo").read().splitlines() + [""]:
            if not line.strip():
                if cur.get("processor") is not None and int(cur["processor"]) in aff:
                    cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    model = model or cur.get("model name")
                cur = {}
                continue
            k, _, v = line.partition(":")
            cur[k.strip()] = v.strip()
    except OSError:
        pass
    usable = len(aff) if quota is None else max(1, min(len(aff), int(quota)))
    return {"threads": usable, "affinity_cpus": len(aff), "cgroup_cpu_quota": quota,
            "physical_cores_in_affinity": len(cores) or None, "model": model}


def cpu_baseline(loss_D, size, batch, h, spectral, seconds_hint, arch=0, min_iters=1):
    """Oracle (CPU restatement, pinned bitwise to the reference) on this host's CPUs:
    every CPU the process is allowed (affinity, capped by the cgroup quota), 1 warm-up
    iteration, then timed iterations until ~seconds_hint of CPU work or 5 iterations
    (at least ``min_iters``)."""
    from oracle.reference_cpu import Trainer as OracleTrainer, make_param, synthetic_images
    cpus = host_cpus()
    threads = cpus["threads"]
    torch.set_num_threads(threads)
    p = make_param(loss_D=loss_D, image_size=size, batch_size=batch, G_h_size=h, D_h_size=h, seed=1, cuda=False,
                   print_every=10 ** 9, spectral=spectral, arch=arch)
    t = OracleTrainer(p, synthetic_images(256, size))
    t.iteration(1)  # warm-up (i=1: skips the i=0 sample-image forward)
    n, t0 = 0, time.perf_counter()
    while True:
        t.iteration(2 + n)
        n += 1
        el = time.perf_counter() - t0
        if (el > seconds_hint and n >= min_iters) or n >= max(5, min_iters):
            break
    return {"value": batch * n / el, "unit": "images/s", "cores": threads, "kind": "port",
            "cpu": cpus, "s_per_iter": el / n,
            "sample": f"{n} timed + 1 warm-up oracle iterations of the same workload (B={batch}, {size}^2, h={h}), "
                      f"torch {torch.__version__} CPU fp32, {threads} threads on {cpus['model']}"}


def emu_parity_evidence():
    """The bf16x6 variant's qualification: the full-size BASELINE configs'
    teacher-forced GPU-vs-reference parity run with rgan_set_gemm_emulation(1) -- the committed
    audit's compact summary (profiles/round*_parity_summary.json, tests/test_parity_gpu.py
    ``-bf16x6`` cases): tensors passed directly / against the mask-forced fp64 step, envelope
    uses (0 = fp32-accurate), and the fp32 run's counts beside them."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*_parity_summary.json")),
                   key=lambda f: int(os.path.basename(f).split("_")[0][5:]))
    if not files:
        return None
    with open(files[-1]) as fh:
        d = json.load(fh)
    out = {"source": os.path.relpath(files[-1], ROOT), "configs": {}}
    for name, e in d["configs"].items():
        if not name.endswith("-bf16x6"):
            continue
        base = d["configs"].get(name[:-len("-bf16x6")], {})
        out["configs"][name[:-len("-bf16x6")]] = {
            "tensors": e["tensors"], "direct": e["direct"], "forced": e.get("forced", 0), "envelope": e["envelope"],
            "failed": e.get("FAIL") or 0, "fp32_direct": base.get("direct"), "fp32_forced": base.get("forced")}
    return out


def restatement_check():
    """the oracle timed against the unmodified reference script on the same host
    (tests/golden/time_reference.py, run in the build container -- the reference does not
    travel to the GPU box): the committed result files, oracle / reference seconds per
    iteration within +-10 %."""
    import glob
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "round*_cpu_reference_vs_oracle_*.json"))):
        with open(f) as fh:
            d = json.load(fh)
        out.append({k: d.get(k) for k in ("config", "threads", "reference_s_per_iter", "oracle_s_per_iter",
                                           "oracle_over_reference", "within_10pct")}
                   | {"source": os.path.relpath(f, ROOT)})
    return out


def run_workload(name, steps, warmup, world, args, K, emu=False, dp_path=False, host_rng=False):
    """Train `steps` timed iterations of workload `name` (after `warmup`); returns the
    measurement (max over ranks).  emu: forward / data-gradient GEMMs on bf16x6.  dp_path:
    run one process in the launch mode every rank of an N > 1 run uses (eager above 50M
    parameters, piecewise graphs below; batched D pass as at N = 1) -- the like-for-like
    N = 1 baseline of the scaling runs.  host_rng: batches and z drawn on the host in the reference's order (numpy choice,
    torch CPU generator, seed 1: SURVEY §8(d) -- the oracle's exact draws), eager launches
    (a graph replay would repeat its capture's draws)."""
    prev_emu = K.set_gemm_emulation(emu)
    try:
        return _run_workload(name, steps, warmup, world, args, K, dp_path, host_rng)
    finally:
        K.set_gemm_emulation(prev_emu)


def _run_workload(name, steps, warmup, world, args, K, dp_path=False, host_rng=False):
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    loss_D, size, bpg, h = WORKLOADS[name]
    spectral = name == "C5"
    bd = {"auto": None, "on": True, "off": False}[args.batch_d]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg * world, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=spectral, rgan_rng="host" if host_rng else "device",
                   arch=ARCH.get(name, 0), rgan_batch_D=bd)
    images = synthetic_images(1024, size, device="cuda")
    t = Trainer(p, images)
    flops_iter = conv_flops_per_iteration(t)

    # launch mode: "graph" = one iteration captured as a HIP graph (one process);
    # "piecewise" = the iteration captured as HIP graphs cut at its collectives, which run
    # eagerly between the replays (dp.PiecewiseGraph); "eager".  auto: graph for one
    # process; under DP piecewise for small (launch-bound) models, eager for large ones,
    # whose gradient buckets all-reduce overlapped with the backward (a captured backward
    # cannot launch them mid-way)
    n_params = sum(q.numel() for q in list(t.G.parameters()) + list(t.D.parameters()))
    from relativisticgan_amd import dp as _dpm
    multi = world > 1 or dp_path or _dpm.active()
    if host_rng:
        mode = "eager"
    elif args.graph == "auto":
        mode = ("piecewise" if n_params < 50e6 else "eager") if multi else "graph"
    elif args.graph == "on":
        mode = "piecewise" if multi else "graph"
    else:
        mode = args.graph if args.graph == "piecewise" else "eager"
    use_graph = mode in ("graph", "piecewise")
    # graph mode runs every iteration on one side stream: autograd's per-parameter
    # AccumulateGrad nodes keep the stream of the first backward, and the captured backward
    # must accumulate on the capturing stream
    side = torch.cuda.Stream() if use_graph else torch.cuda.current_stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for i in range(warmup):
            t.iteration(i + 1)
        t.flush()
    torch.cuda.current_stream().wait_stream(side)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    it = warmup + 1
    if use_graph:
        # One iteration captured as a HIP graph and replayed: the same kernels, launches and
        # state updates (Adam's device step counter, the device RNG's philox offsets), without
        # the ~10-20 us of Python + ctypes per launch that leaves a small model's step
        # launch-bound.
        if mode == "piecewise":
            from relativisticgan_amd import dp as _dp
            t.defer_G = False
            graph = _dp.PiecewiseGraph(side).capture(lambda: t.iteration(it))
        else:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                t.iteration(it)
        t.graph_captured = True  # host mirrors (Adam step, LR) freeze from here: no checkpoints
        it += 1
        graph_segments = getattr(graph, "n_segments", 1)
        graph.replay()  # one untimed replay
        barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            graph.replay()
        barrier()
        elapsed = time.perf_counter() - t0
        # per-kernel HIP events cannot be read out of graph replays: the kernel statistics
        # of the roofline come from eager iterations of the same step, right after
        nprof = max(3, min(steps, 10))
        K.profile_begin(capacity=400 * nprof + 64)
        with torch.cuda.stream(side):
            for i in range(nprof):
                t.iteration(it + i)
            t.flush()
        torch.cuda.current_stream().wait_stream(side)
        barrier()
        prof = K.profile_end()
        prof["steps"] = nprof
        del graph
    else:
        graph_segments = 0
        barrier()
        K.profile_begin(capacity=400 * steps + 64)
        t0 = time.perf_counter()
        for i in range(steps):
            t.iteration(it + i)
        t.flush()  # the last G step (deferred under DP) is inside the timed region
        barrier()
        elapsed = time.perf_counter() - t0
        prof = K.profile_end()
        prof["steps"] = steps
    if world > 1:
        e = torch.tensor([elapsed], device="cuda")
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    res = {"name": name, "loss_D": loss_D, "size": size, "bpg": bpg, "h": h, "spectral": spectral,
           "arch": ARCH.get(name, 0), "batch_D": t.batch_D, "elapsed": elapsed, "steps": steps, "mode": mode,
           "segments": graph_segments,
           "value": bpg * world * steps / elapsed, "ms_per_step": 1000.0 * elapsed / steps,
           "flops_iter": flops_iter, "prof": prof, "graph": use_graph}
    del t, images
    torch.cuda.empty_cache()
    return res


def roofline_of(res, workload):
    """Dominant kernel = the conv kernel symbol with the most time (HIP events around each
    launch on its stream); the whole conv family is reported beside it."""
    prof, steps = res["prof"], res["prof"]["steps"]
    gemm_ms, gemm_flops = prof["ms"], prof["flops"]
    top = max(prof["kernels"], key=lambda k: k["ms"])
    achieved = top["flops"] / (top["ms"] / 1000.0)
    peak = kernel_peak(top["name"])
    traffic, traffic_src = pmc_traffic(workload, top["name"])
    # conv family ceiling: each kernel's time at its own peak
    fam_floor_s = sum(k["flops"] / kernel_peak(k["name"]) for k in prof["kernels"])
    return {"bound": "mfma", "achieved": achieved / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s",
            "frac": achieved / peak, "traffic": traffic, "traffic_unit": "bytes/launch",
            "traffic_source": traffic_src, "kernel": top["name"], "launches": top["launches"],
            "avg_launch_us": 1000.0 * top["ms"] / top["launches"],
            "flops_per_launch": top["flops"] / top["launches"],
            "conv_family": {"achieved": gemm_flops / (gemm_ms / 1000.0) / 1e12, "launches": prof["launches"],
                            "ms_per_step": gemm_ms / steps,
                            "frac": fam_floor_s / (gemm_ms / 1000.0),
                            "kernels": prof["kernels"]}}


HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: HBM3E peak (spec)


def hbm_kernels(name, K, reps=10):
    """achieved HBM GB/s of the HBM-bound kernels of the step (BatchNorm
    apply / backward, the one-launch small-layer BN backward, Adam, activation backward) at
    the workload's own layer shapes: algorithmic bytes per launch (BN apply
    8 B/elem, BN backward 8 + 12 B/elem, Adam 28 B/param, act' 12 B/elem) / the launch's
    average duration (torch.cuda.Event pairs on the launch stream, reps launches after 2)."""
    loss_D, size, bpg, h = WORKLOADS[name]
    if ARCH.get(name, 0) != 0:
        return None
    torch.manual_seed(0)
    dev = "cuda"
    B2 = 2 * bpg  # the batched D pass: both calls' halves in one launch
    c_big, hw_big = 2 * h, size // 4  # D's first BatchNorm layer (the largest)
    c_small = h * (size // 8)  # D's last BatchNorm layer (4 x 4): h * S / 8 channels

    def nhwc(B, C, H):
        return K.empty_nhwc(B, C, H, H, dev).normal_()

    def timed(fn):
        for _ in range(2):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1000.0  # us

    out = []

    def add(kernel, shape, nbytes, us):
        gbs = nbytes / us / 1e3
        out.append({"kernel": kernel, "shape": shape, "bytes_per_launch": nbytes, "us": us, "GB_s": gbs,
                    "frac_of_hbm_peak": gbs * 1e9 / HBM_PEAK})

    y = nhwc(B2, c_big, hw_big)
    C = c_big
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    stats = torch.cat([torch.randn(2, C, device=dev), torch.rand(2, C, device=dev) + 0.5], 1)
    a = torch.empty_like(y)
    n = y.numel()
    add("bn_apply_segments (normalise + LeakyReLU)", list(y.shape), 8 * n,
        timed(lambda: K.bn_apply_segments(y, stats, gamma, beta, "lrelu", 0.2, out=a)))
    da = torch.randn_like(y)
    dy = torch.empty_like(y)
    add("bn_backward_segments (sums + merge + apply, act')", list(y.shape), 20 * n,
        timed(lambda: K.bn_backward_segments(da, y, stats, gamma, beta, "lrelu", 0.2, True, True, dy)))
    add("act_backward (LeakyReLU')", list(y.shape), 12 * n, timed(lambda: K.act_backward(da, a, "lrelu", 0.2)))
    ys = nhwc(B2, c_small, 4)
    Cs = c_small
    gs, bs = torch.rand(Cs, device=dev) + 0.5, torch.randn(Cs, device=dev)
    sts = torch.cat([torch.randn(2, Cs, device=dev), torch.rand(2, Cs, device=dev) + 0.5], 1)
    das, dys = torch.randn_like(ys), torch.empty_like(ys)
    add("bn_bwd_small (4x4 layer under D's dense head, one launch)", list(ys.shape), 20 * ys.numel(),
        timed(lambda: K.bn_backward_segments(das, ys, sts, gs, bs, "lrelu", 0.2, True, True, dys)))
    # Adam over a D-sized parameter set (the conv weights of the workload's D)
    shapes, cin, s = [], 3, size
    cout = h
    while s > 4:
        shapes.append((cout, cin, 4, 4))
        cin, cout, s = cout, cout * 2, s // 2
    shapes.append((1, cin, 4, 4))
    ps = [torch.randn(sh, device=dev) * 0.02 for sh in shapes]
    gs_ = [torch.randn_like(p) for p in ps]
    ms, vs = [torch.zeros_like(p) for p in ps], [torch.zeros_like(p) for p in ps]
    hyper = torch.tensor([1e-4, 0.5, 0.999, 1e-8, 0.0, 0, 0, 0], dtype=torch.float64, device=dev)
    step = torch.zeros(1, device=dev)
    npar = sum(p.numel() for p in ps)
    add("adam (multi-tensor, D's conv weights)", [npar], 28 * npar, timed(lambda: K.adam(ps, gs_, ms, vs, hyper, step)))
    del y, a, da, dy, ys, das, dys, ps, gs_, ms, vs
    torch.cuda.empty_cache()
    return {"peak_GB_s": HBM_PEAK / 1e9, "note": "algorithmic bytes (SURVEY §8(d)) / HIP-event launch time",
            "kernels": out}


def describe(res):
    arch = "arch1 (standard CNN)" if res["arch"] == 1 else "arch0"
    return (f"{res['name']}: loss_D {res['loss_D']} DCGAN {arch} {res['size']}x{res['size']}, h={res['h']}, "
            f"batch {res['bpg']}/GPU{', spectral D' if res['spectral'] else ''}"
            f"{', gradient penalty' if res['loss_D'] == 3 else ''}")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, backend):
    """``python bench.py --gpus N`` without a launcher: run this script as N ranks under
    ``torch.distributed.run`` in a CHILD process (this process has not initialised the GPU
    and never replaces itself), stream the ranks' output through, and return the launcher's
    exit status (non-zero if any rank failed).  Rank 0 prints the JSON line."""
    import subprocess
    if backend == "nccl":
        have = torch.cuda.device_count()  # counts devices without initialising HIP (this image)
        if have < n:
            print(f"bench.py: --gpus {n} over RCCL but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env["RGAN_BENCH_LAUNCHER"] = "bench.py --gpus (torch.distributed.run child)"
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD, choices=sorted(WORKLOADS))
    ap.add_argument("--extra", default=",".join(EXTRA_WORKLOADS),
                    help="comma-separated workloads also measured on one GPU (extra_workloads); '' = none")
    ap.add_argument("--batch-d", default="auto", choices=("auto", "on", "off"),
                    help="D(x), D(x_fake) as one batched pass (auto = on, also under DP; off = the "
                         "reference's separate D(x) / D(x_fake) calls)")
    ap.add_argument("--graph", default="auto", choices=("auto", "on", "off", "piecewise"),
                    help="time replays of one iteration captured as a HIP graph (one process) or as graphs "
                         "cut at the collectives (piecewise, DP); auto: graph at N=1, under DP piecewise "
                         "below 50M parameters (launch-bound), else eager (bucket all-reduce overlapped)")
    ap.add_argument("--no-emu-extra", action="store_true",
                    help="skip the N=1 re-run of the workload with the bf16x6 fp32-emulated GEMMs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dp-path", action="store_true",
                    help="skip the N=1 runs of the data-parallel launch mode (dp_path_n1)")
    ap.add_argument("--no-host-draws", action="store_true",
                    help="skip the N=1 eager run with the reference's host-side draws (host_draws_n1)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-hbm", action="store_true", help="skip the HBM-bound kernels' GB/s table (hbm_kernels)")
    ap.add_argument("--sync-bn", action="store_true",
                    help="SyncBN over ranks (default: per-shard BN = the reference's DataParallel)")
    ap.add_argument("--force-dp", action="store_true",
                    help="run the data-parallel path (process group, distributed heads, gradient buckets on "
                         "the second communicator) even with one rank: a one-GPU rehearsal of the N > 1 "
                         "collectives over RCCL (RGAN_BENCH_BACKEND, default nccl)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus}: need at least one GPU")
    # RGAN_BENCH_BACKEND=gloo + more ranks than GPUs: rehearsal of the N>1 path on one GPU
    backend = os.environ.get("RGAN_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: this process never touches the GPU; it starts the
        # N ranks and relays their output
        sys.exit(launch_ranks(args.gpus, backend))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # the reference's --n_gpu N is N devices under one data_parallel (GLI:40, 455-456);
        # here one process per GPU: a mismatch would time the wrong job
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch with "
                         f"torch.distributed.run --nproc-per-node {args.gpus}, or without a launcher "
                         "(bench.py starts the ranks itself)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    from relativisticgan_amd import dp, kernels as K
    distributed = world > 1 or args.force_dp
    if distributed:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        dp.setup(sync_bn=args.sync_bn, force=args.force_dp)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    pg = ({"backend": str(torch.distributed.get_backend()), "world_size": torch.distributed.get_world_size(),
           "launcher": os.environ.get("RGAN_BENCH_LAUNCHER", "external (torch.distributed.run)")}
          if distributed else None)
    res = run_workload(args.workload, args.steps, args.warmup, world, args, K)
    emu_res = None
    if world == 1 and not args.no_emu_extra:
        emu_res = run_workload(args.workload, args.steps, min(args.warmup, 5), world, args, K, emu=True)
    extras, dp_paths, host_draws = {}, {}, {}
    if world == 1:
        for name in [w for w in args.extra.split(",") if w and w != args.workload]:
            r = run_workload(name, args.steps, min(args.warmup, 5), world, args, K)
            extras[name] = {"workload": describe(r), "value": r["value"], "unit": "images/s",
                            "ms_per_step": r["ms_per_step"], "steps": r["steps"], "hip_graph": r["graph"],
                            "step_mfma_util": r["flops_iter"] / (r["ms_per_step"] / 1000.0) / FP32_MFMA_PEAK,
                            "roofline": {k: v for k, v in roofline_of(r, name).items() if k != "conv_family"}}
            if name == "C1" and not args.no_cpu_baseline:
                extras[name]["cpu_baseline"] = cpu_baseline(r["loss_D"], r["size"], r["bpg"], r["h"], r["spectral"],
                                                            args.cpu_seconds, arch=r["arch"], min_iters=5)
        if not args.no_dp_path:
            for name in [args.workload] + [w for w in ("C1",) if w in args.extra.split(",")]:
                r = run_workload(name, args.steps, min(args.warmup, 5), world, args, K, dp_path=True)
                dp_paths[name] = {"value": r["value"], "unit": "images/s", "ms_per_step": r["ms_per_step"],
                                  "steps": r["steps"], "batched_D_step": r["batch_D"], "launch_mode": r["mode"]}
        if not args.no_host_draws:
            for name in [args.workload] + [w for w in ("C1",) if w in args.extra.split(",")]:
                r = run_workload(name, args.steps, min(args.warmup, 5), world, args, K, host_rng=True)
                host_draws[name] = {"value": r["value"], "unit": "images/s", "ms_per_step": r["ms_per_step"],
                                    "steps": r["steps"], "launch_mode": r["mode"],
                                    "draws": "host: numpy.random.choice batches + torch CPU z, seed 1, "
                                             "the reference's order (SURVEY §8(d)); H2D per draw"}
    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    out = {
        "metric": METRIC, "value": res["value"], "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (1024 seeded images resident in HBM; batches / z drawn on the device -- "
                "host_draws_n1: the reference's host draws)",
        "config": {"workload": describe(res), "loss_D": res["loss_D"], "image_size": res["size"],
                   "batch_per_gpu": res["bpg"], "global_batch": res["bpg"] * world, "G_h_size": res["h"],
                   "D_h_size": res["h"], "arch": res["arch"], "parallelism": f"dp{world}",
                   "batched_D_step": res["batch_D"], "hip_graph": res["graph"], "launch_mode": res["mode"],
                   "graph_segments": res["segments"],
                   "batchnorm": "SyncBN" if args.sync_bn else "per-shard (reference DataParallel)",
                   "forced_dp": bool(args.force_dp), "process_group": pg},
        "step_mfma_util": res["flops_iter"] * args.steps / res["elapsed"] / (world * FP32_MFMA_PEAK),
        "conv_tflop_per_step": res["flops_iter"] / 1e12,
        "roofline": roofline_of(res, args.workload),
    }
    if extras:
        out["extra_workloads"] = extras
    if dp_paths:
        # what each rank of the N > 1 runs executes (separate D passes, eager), on one GPU:
        # the like-for-like N = 1 baseline for the scaling efficiency of `value` at N > 1
        out["dp_path_n1"] = dp_paths
    if host_draws:
        # `value` draws on the device (Philox, csrc/sampling.hip) so that the iteration can be
        # replayed as a HIP graph; this is the same workload with the oracle's own host draws
        out["host_draws_n1"] = host_draws
    if emu_res is not None:
        out["fp32_emulated_bf16x6"] = {
            "value": emu_res["value"], "unit": "images/s", "ms_per_step": emu_res["ms_per_step"],
            "steps": emu_res["steps"], "hip_graph": emu_res["graph"],
            "gemm_arith": "forward / data-gradient conv GEMMs: fp32 operands split exactly into 3 bf16 "
                          "pieces, 6 bf16 MFMA products accumulated in fp32 (weight gradients: fp32 MFMA)",
            "roofline": roofline_of(emu_res, args.workload),
            "parity": emu_parity_evidence()}
    if world == 1 and not args.no_hbm:
        out["hbm_kernels"] = hbm_kernels(args.workload, K)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(res["loss_D"], res["size"], res["bpg"], res["h"], res["spectral"],
                                           args.cpu_seconds, arch=res["arch"])
        out["cpu_baseline"]["restatement_check"] = restatement_check()
    print(json.dumps(out), flush=True)
    if distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
