"""bench.py's multi-rank launcher (the contract's ``python bench.py --gpus N``), on the CPU.

* ``--gpus N`` without a torch.distributed environment starts N ranks itself, as a child
  torch.distributed.run on 127.0.0.1 (the parent never touches the GPU); ``--check-launch`` makes
  the ranks join a gloo process group, assert its size and print the n_gpus line;
* under torch.distributed.run (WORLD_SIZE set, as the driver launches it) ``--gpus`` must equal
  WORLD_SIZE, else the run stops before any work.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True, timeout=240)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == n and line["gpus_requested"] == n and line["backend"] == "gloo"


def test_single_rank_default():
    r = _run(["--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _line(r.stdout)["n_gpus"] == 1


def test_world_size_mismatch_stops():
    r = _run(["--gpus", "3", "--check-launch"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_resolve_world():
    assert bench.resolve_world(None, {}) == 1
    assert bench.resolve_world(4, {}) == 4
    assert bench.resolve_world(None, {"WORLD_SIZE": "8"}) == 8
    assert bench.resolve_world(8, {"WORLD_SIZE": "8"}) == 8
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "1"})


def test_launch_command_shape():
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-5:] == [os.path.abspath(BENCH), "--gpus", "8", "--steps", "5"]
