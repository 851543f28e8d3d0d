"""bench.py's `--gpus N` contract: an unaided `--gpus N > 1`
starts N ranks itself, a launcher's WORLD_SIZE must agree with --gpus, and the
parent decides this before anything touches the GPU.  CPU only."""
import importlib.util
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_check_world_decisions():
    b = _bench()
    assert b.check_world(1, {}) == "run"
    assert b.check_world(8, {}) == "launch"
    assert b.check_world(2, {"WORLD_SIZE": "2"}) == "run"
    assert b.check_world(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit):
        b.check_world(8, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        b.check_world(1, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        b.check_world(0, {})


def test_launch_command_passes_every_flag():
    b = _bench()
    argv = ["--gpus", "4", "--steps", "20", "--warmup", "5", "--no-large"]
    cmd = b.launch_command(argv, 4, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    k = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[k + 1:] == argv


def _run_bench(args, env_extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=300)


def test_mismatched_world_size_exits_nonzero():
    r = _run_bench(["--gpus", "8"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 8" in r.stderr
    assert r.stdout == ""


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs a host with fewer than 2 GPUs")
def test_unaided_multi_gpu_without_devices_refuses():
    r = _run_bench(["--gpus", "2"], {})
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert r.stdout == ""
