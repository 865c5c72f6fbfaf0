#!/usr/bin/env python
"""One parameterised runner for the GPU calls (replaces round 3's per-call
tools/archive/r03/gpu_*.sh scripts).

  python tools/gpu_steps.py OUTDIR "label|timeout_s|command" ["label|timeout_s|command" ...]

Each step runs as a child process in its own session (never exec'd over
this process; this process never touches the GPU), with stdout to
OUTDIR/label.out and stderr to OUTDIR/label.err, under its own time limit
(SIGTERM, then SIGKILL 10 s later).  The first step that fails, aborts,
faults or times out ends the call: nothing after it starts.  A bench JSON
line on a step's stdout is summarised on this process's stdout.
TMPDIR is /tmp for every step (rocprofv3).  The command is split with shlex
(no shell; leading VAR=value words set the step's environment): put the
program itself right after rocprofv3's `--`.
"""
import json
import os
import shlex
import signal
import subprocess
import sys
import time


def summarise(path):
    try:
        with open(path) as f:
            lines = [ln for ln in f.read().strip().splitlines() if ln.startswith("{")]
        d = json.loads(lines[-1])
    except Exception:
        return None
    if "value" in d and "config" in d:
        c, r = d["config"], d.get("roofline", {})
        q = c.get("kernel_ms_quartiles")
        return ("value %.4g ms/step %.4f kernel q %s frac %s parity %s plan %s" % (
            d["value"], d["ms_per_step"], [round(x, 4) for x in q] if q else None,
            round(r["frac"], 3) if "frac" in r else None,
            d.get("parity", {}).get("rel_l2"), c.get("scatter_plan", {}).get("plan")))
    if "mode" in d and "step" in d:
        return ("step wall %.4f ms ev %.4f interior %s side %s exposed %s host %s single %s" % (
            d["step"]["wall_ms_per_step"], d["step"]["event_ms_avg"],
            d["interior_alone"] and round(d["interior_alone"]["event_ms_avg"], 4),
            d["side_chain_alone"] and round(d["side_chain_alone"]["event_ms_avg"], 4),
            d["exposed_beyond_interior_ms"] and round(d["exposed_beyond_interior_ms"], 4),
            {k: round(v, 1) for k, v in d["host"].items()},
            d["single_gpu_whole_mesh"] and round(d["single_gpu_whole_mesh"]["wall_ms_per_step"],
                                                 4)))
    return json.dumps(d)[:300]


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp", PYTHONUNBUFFERED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for spec in sys.argv[2:]:
        label, tmo, cmd = spec.split("|", 2)
        tmo = float(tmo)
        so, se = os.path.join(out, label + ".out"), os.path.join(out, label + ".err")
        t0 = time.time()
        with open(so, "w") as fo, open(se, "w") as fe:
            argv, step_env = shlex.split(cmd), dict(env)
            while argv and "=" in argv[0] and not argv[0].startswith(("-", "/", ".")):
                k, v = argv.pop(0).split("=", 1)  # leading VAR=value: environment
                step_env[k] = v
            pr = subprocess.Popen(argv, stdout=fo, stderr=fe, env=step_env,
                                  start_new_session=True)
            rc = None
            while rc is None:
                try:
                    rc = pr.wait(timeout=5)
                except subprocess.TimeoutExpired:
                    if time.time() - t0 > tmo:
                        os.killpg(pr.pid, signal.SIGTERM)
                        try:
                            pr.wait(timeout=10)
                        except subprocess.TimeoutExpired:
                            os.killpg(pr.pid, signal.SIGKILL)
                            pr.wait()
                        rc = 124
        dt = time.time() - t0
        print("step %s rc=%s %.1fs" % (label, rc, dt), flush=True)
        s = summarise(so)
        if s:
            print("  " + s, flush=True)
        else:
            with open(so) as f:
                tail = f.read().strip().splitlines()[-2:]
            for ln in tail:
                print("  " + ln[:300], flush=True)
        if rc != 0:
            with open(se) as f:
                for ln in f.read().strip().splitlines()[-8:]:
                    print("  ! " + ln[:300], flush=True)
            print("stopping: step %s failed (rc=%s)" % (label, rc), flush=True)
            return rc if rc > 0 else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
