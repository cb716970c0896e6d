"""bench.py's driver contract on the GPU box: the N=1 JSON line, and the N>1 path (torchrun,
one process per rank, max-over-ranks timing) rehearsed with 2 and 4 gloo ranks on the one GPU
(RGAN_BENCH_BACKEND=gloo: RCCL refuses two ranks on one device).  Small workload (C1),
few steps: this checks the code path and the line's keys, not the numbers."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline"}


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_bench_one_gpu_line():
    r = subprocess.run([sys.executable, "bench.py", "--workload", "C1", "--extra=", "--no-emu-extra",
                        "--no-cpu-baseline", "--steps", "3", "--warmup", "1"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["dtype"] == "fp32"
    assert d["config"]["parallelism"] == "dp1" and d["config"]["global_batch"] == 32
    rf = d["roofline"]
    assert rf["bound"] == "mfma" and 0 < rf["frac"] < 1 and rf["peak"] == 157.3
    # the N > 1 launch mode on one GPU (the scaling runs' like-for-like baseline)
    dpp = d["dp_path_n1"]["C1"]
    assert dpp["value"] > 0 and dpp["batched_D_step"] is True and dpp["launch_mode"] == "piecewise"
    # the same workload on the reference's host draws (eager)
    hd = d["host_draws_n1"]["C1"]
    assert hd["value"] > 0 and hd["launch_mode"] == "eager"


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multi_rank_rehearsal(world):
    env = _env()
    env["RGAN_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(29613 + world), "bench.py", "--gpus",
                        str(world), "--workload", "C1", "--extra=", "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)  # rank 0 only prints
    assert KEYS <= set(d)
    assert d["n_gpus"] == world and d["config"]["parallelism"] == f"dp{world}"
    assert d["config"]["global_batch"] == 32 * world
    # C1 (24M parameters) under DP: HIP graphs cut at the collectives
    assert d["config"]["batched_D_step"] is True and d["config"]["launch_mode"] == "piecewise"
    assert d["config"]["graph_segments"] > 4
    assert "cpu_baseline" not in d and d["value"] > 0


def test_bench_headline_two_rank_rehearsal():
    """The headline C3 shard (366M parameters) under DP: eager launches with the gradient
    buckets all-reduced asynchronously from the backward's hooks (gloo here, RCCL on the node)."""
    env = _env()
    env["RGAN_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29640", "bench.py", "--gpus", "2",
                        "--workload", "C3", "--extra=", "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 64 and d["config"]["launch_mode"] == "eager"
    # one batched D(x) / D(x_fake) pass under DP too (round 6), as at N = 1
    assert d["config"]["batched_D_step"] is True
    assert d["value"] > 0


def test_bench_gpus_flag_spawns_the_ranks():
    """The driver's plain `python bench.py --gpus N` (no launcher): bench.py starts the N ranks
    itself (torch.distributed.run as a child process) and relays rank 0's line, which records
    the process group the ranks actually formed.  Two gloo ranks on the one GPU."""
    env = _env()
    env["RGAN_BENCH_BACKEND"] = "gloo"
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--workload", "C1", "--extra=", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 64
    pg = d["config"]["process_group"]
    assert pg["world_size"] == 2 and pg["backend"] == "gloo" and pg["launcher"].startswith("bench.py --gpus")
    assert d["value"] > 0


@pytest.mark.parametrize("workload,mode", [("C1", "piecewise"), ("C3", "eager")])
def test_bench_forced_dp_over_rccl_one_rank(workload, mode):
    """The driver's N > 1 command shape with ONE rank over RCCL and the data-parallel path
    forced on (``--force-dp``): process group on nccl, distributed heads, gradient buckets on
    the second communicator, piecewise graphs (C1) / eager overlapped buckets (C3) -- the
    collectives the scaling runs use, on the real backend."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29652", "bench.py", "--gpus", "1",
                        "--force-dp", "--workload", workload, "--extra=", "--steps", "2", "--warmup", "1",
                        "--no-emu-extra", "--no-cpu-baseline", "--no-dp-path", "--no-host-draws", "--no-hbm"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["config"]["forced_dp"] is True and d["config"]["launch_mode"] == mode
    assert d["value"] > 0


def test_bench_configs2_job_shape_eight_ranks():
    """BASELINE configs[2]'s job shape -- RaLSGAN 256^2, 8 ranks x 32 = batch 256, h = z = 128 --
    through the driver's own command (plain `bench.py --gpus 8`, which starts the ranks), the
    8 ranks sharing the one GPU over gloo (RCCL needs one device per rank): every rank builds
    the 366M-parameter nets, runs the batched D pass and the bucketed gradient SUM all-reduce of
    both nets, and rank 0 reports the 8-rank line (run r6f: 2.8 s per step on the shared GPU)."""
    env = _env()
    env["RGAN_BENCH_BACKEND"] = "gloo"
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--workload", "C3", "--extra=", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["config"]["global_batch"] == 256
    assert d["config"]["image_size"] == 256 and d["config"]["G_h_size"] == 128 and d["config"]["batched_D_step"]
    assert d["config"]["process_group"]["world_size"] == 8 and d["value"] > 0
