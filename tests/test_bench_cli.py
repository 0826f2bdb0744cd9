"""bench.py's launch contract on CPU: a multi-GPU request
never turns into a silent one-GPU line.

* `--gpus N` without a launcher (WORLD_SIZE unset) takes the one-process path
  (zrt_multi_*), which needs N visible GPUs: with fewer it exits 2 and says so;
* a launcher whose WORLD_SIZE differs from --gpus is refused the same way;
* `--devices 0,0` (the one-GPU rehearsal of the one-process path) needs GPU 0.

No kernel runs here (this container has no GPU); the GPU rehearsal is
tests/test_gpu_runtime.py::test_bench_one_process_rehearsal.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def _visible_gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_visible_gpus() >= 2, reason="needs a box with fewer than 2 GPUs")
def test_gpus_2_without_enough_devices_fails_loudly():
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode == 2, r.stderr
    assert "visible" in r.stderr and "--gpus 2" in r.stderr
    assert not any(line.startswith("{") for line in r.stdout.splitlines()), "a bench line was printed"


def test_world_size_mismatch_fails_loudly():
    r = run_bench(["--gpus", "4", "--steps", "1", "--warmup", "0"],
                  {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=2" in r.stderr
    assert not any(line.startswith("{") for line in r.stdout.splitlines())


@pytest.mark.skipif(_visible_gpus() >= 1, reason="CPU-only check")
def test_rehearsal_devices_need_a_gpu():
    r = run_bench(["--devices", "0,0", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, r.stderr
    assert "0 visible" in r.stderr


def test_bad_device_list_refused():
    r = run_bench(["--devices", "0,-1"])
    assert r.returncode == 2 and "non-negative" in r.stderr
