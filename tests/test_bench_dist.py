"""CPU tests of bench.py's own multi-rank launcher (`--gpus N` without torchrun): a rank that dies
must end the whole run with a non-zero exit within seconds -- its peers, blocked in a collective the
dead rank never joins, are stopped by the launcher instead of waiting for the collective timeout.
DKG_BENCH_FAIL_RANK (bench.fault_rehearsal) injects the failure after the gloo process group is up;
no GPU is touched."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(fail_rank, gpus=2):
    env = dict(os.environ, DKG_BENCH_FAIL_RANK=str(fail_rank))
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend", "gloo",
                        "--dist-timeout", "300"], env=env, capture_output=True, text=True, timeout=240)
    return p, time.time() - t0


def test_failed_rank_ends_the_run_fast():
    p, dt = _run(1)
    assert p.returncode != 0, p.stderr[-2000:]
    assert "rank 1 exited with 1" in p.stderr, p.stderr[-2000:]
    # far below the 300-s collective timeout: the launcher stopped rank 0 out of its barrier
    assert dt < 60, dt
    assert p.stdout == ""  # no result line from a failed run


def test_failed_rank_zero_of_three():
    p, dt = _run(0, gpus=3)
    assert p.returncode != 0 and dt < 60, (p.returncode, dt, p.stderr[-2000:])


def test_all_ranks_succeed():
    p, dt = _run(-1)
    assert p.returncode == 0, p.stderr[-2000:]
