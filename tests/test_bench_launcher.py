"""bench.py's multi-rank launcher (``--gpus N`` without torchrun) must fail
fast: the driver's one-shot 8-GPU run records nothing useful if one dead rank
leaves the others waiting in a collective until an outer time limit.  CPU
only: the failure is injected at rank start-up (SEM_BENCH_INJECT), before
any GPU call, and the surviving ranks block as if waiting on the lost peer."""
import os
import subprocess
import sys
import time

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(inject, deadline, n=3):
    env = dict(os.environ, SEM_BENCH_INJECT=inject)
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    pr = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--deadline", str(deadline)],
                        env=env, capture_output=True, text=True, timeout=120)
    return pr, time.monotonic() - t0


def test_rank_failure_stops_all_ranks_promptly():
    pr, dt = _run("fail:1", deadline=100)
    assert pr.returncode != 0
    assert "rank 1 exited with status 3" in pr.stderr
    assert dt < 40, dt  # the blocked ranks were killed, not waited for


def test_deadline_stops_a_hung_run():
    pr, dt = _run("fail:99", deadline=8, n=2)  # nobody fails, everybody blocks
    assert pr.returncode == 124
    assert "deadline" in pr.stderr
    assert dt < 40, dt
