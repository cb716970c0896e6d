"""bench.py's rank-count guards, on the CPU (nothing here reaches a GPU call).

* ``--gpus N`` under a launcher whose WORLD_SIZE differs fails loudly (it would time the
  wrong job), as train.py refuses a mismatched --n_gpu (GLI:40, 455-456);
* plain ``--gpus N`` (no WORLD_SIZE) starts the ranks itself; over RCCL it first checks that
  N devices are visible -- this container has none, so it must refuse before launching.
The launch itself (two gloo ranks on one GPU) is tests/test_bench_gpu.py.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env_over):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=120)


def test_world_size_mismatch_fails():
    r = _bench(["--gpus", "2"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=4" in r.stderr
    r = _bench(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_gpus_flag_without_devices_refuses_before_launch():
    r = _bench(["--gpus", "2"], RGAN_BENCH_BACKEND="nccl")
    assert r.returncode == 2
    assert "--gpus 2 over RCCL but only 0 GPU(s) visible" in r.stderr


def test_gpus_must_be_positive():
    r = _bench(["--gpus", "0"])
    assert r.returncode != 0 and "at least one GPU" in r.stderr
