"""Multi-rank runs fail fast instead of hanging (bench.py --gpus 8 on the driver's node): the
engine's process groups carry an explicit collective timeout (FR_PG_TIMEOUT_S), and the row-sharded
rows form cross-checks |S| across ranks before the |S|-row collectives (engine/sharded.py).
gloo, world 4, on the CPU."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mp", "failfast_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(mode, world=4, timeout_s=5, limit=90):
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(world):
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(r), FR_PG_TIMEOUT_S=str(timeout_s), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, WORKER, mode], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    codes, took = [], []
    try:
        for p in procs:
            p.wait(timeout=max(1.0, limit - (time.time() - t0)))
            codes.append(p.returncode)
            took.append(time.time() - t0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return codes, took, [p.stdout.read() for p in procs]


def test_agreeing_counts_pass():
    codes, _, out = _run("ok")
    assert codes == [0, 0, 0, 0], out


def test_count_mismatch_raises_on_every_rank():
    codes, took, out = _run("mismatch")
    assert codes == [3, 3, 3, 3], out
    assert all("disagree" in o for o in out), out
    assert max(took) < 60, took


def test_missing_rank_times_out():
    codes, took, out = _run("hang", timeout_s=5)
    assert codes[:3] == [3, 3, 3], out  # the ranks that joined the collective raise ...
    assert max(took[:3]) < 5 + 40, took  # ... within the process group's timeout (plus start-up)
