"""World >= 2 paths in the GPU gate: the rank workers of tests/mp/ under torch.distributed.run, all
ranks on the one MI355X over gloo (RCCL refuses two ranks on one device; the driver's 8-GPU bench
runs them over RCCL, one rank per GPU).

* row-sharded config-4 step (engine/sharded.py, rows form) at 2 and 4 ranks vs the unsharded step
  and the single-GPU LightGCN_ID (lightgcn.py:134-177 arithmetic): losses rel 1e-5, gradients
  1e-4 * max, replicated item tables bit-identical across ranks after 3 Adam steps;
* HealthRec data parallelism at 2 ranks: row-exchanged gradients == the dense mean (1e-6 * max),
  identical on every rank; GraphedDPStep == the eager data-parallel step (losses rel 1e-4).
"""
import os
import re
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks(script, world, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "mp", script)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    out = r.stdout + r.stderr
    # one verdict per rank; the ranks share stdout, so two lines can land interleaved on one line:
    # take every "[rank k/world] ... PASS|FAIL" span, not whole lines
    verdicts = re.findall(r"\[rank \d+/\d+\].*?(?:PASS|FAIL)", out)
    assert r.returncode == 0, out[-4000:]
    ranks = sorted(set(re.findall(r"\[rank (\d+)/\d+\]", " ".join(verdicts))))
    assert len(verdicts) == world and len(ranks) == world and all(v.endswith("PASS") for v in verdicts), \
        out[-4000:]
    return verdicts


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_rows_form_ranks(cuda, world):
    v = _ranks("sharded_worker.py", world)
    print("\n".join(v))


@pytest.mark.gpu
def test_healthrec_graphed_dp_two_ranks(cuda):
    v = _ranks("dp_worker.py", 2)
    print("\n".join(v))
