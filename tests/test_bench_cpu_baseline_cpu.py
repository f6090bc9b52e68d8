"""bench.py's CPU-baseline leg on the CPU (`--cpu-baseline-only`, the leg the bench line carries as
`cpu_baseline`): the fields the line promises, and the run-budget guard that stops after the last timed
iteration that fits and states the shortfall in `deviation`.  Tiny samples (batch 2) so each run takes
seconds; the leg itself is the oracle iteration of past_acc.py:194-212 (bench.py cpu_baseline)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("OMP_NUM_THREADS", "4")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--cpu-baseline-only", *args], capture_output=True,
                       text=True, env=env, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_cpu_baseline_fields():
    cb = _run("--cpu-batch", "2", "--cpu-iters", "2", "--cpu-warm-batch", "2")
    assert cb["kind"] == "port" and cb["unit"] == "samples/s" and cb["value"] > 0
    assert cb["batch"] == 2 and cb["timed_iterations"] == 2 and cb["cores"] >= 1
    assert cb["seconds_per_iteration"] > 0 and "oracle/fusion_oracle.py" in cb["sample"]
    assert "deviation" not in cb
    assert abs(cb["value"] - 2 / cb["seconds_per_iteration"]) / cb["value"] < 0.05


def test_cpu_baseline_budget_guard_states_the_shortfall():
    # the bench line's leg (bench.py main: cpu_baseline(..., args.cpu_budget)) with a budget the warm-up
    # has already spent: the first timed iteration still runs (a baseline needs one), the second would end
    # past the budget, so the leg stops there and says so.  (--cpu-baseline-only, the separate cross-check
    # run, times every iteration it is asked for.)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("OMP_NUM_THREADS", "4")
    code = ("import json, sys; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench.cpu_baseline('prigumbel', 2, 3, 2, 1.0)))" % str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    cb = json.loads(r.stdout.strip().splitlines()[-1])
    assert cb["timed_iterations"] == 1 and cb["batch"] == 2
    assert "deviation" in cb and "1 of 3 timed iterations" in cb["deviation"]
