"""bench.py's one-line JSON contract at N = 1 on the GPU (a short run, no CPU leg): every field the driver
and the judge read -- the headline metric of BASELINE.json, whole-job samples/s, the roofline object of the
dominant kernel (algorithmic FLOPs / live launch time against the dense bf16 peak, PMC traffic), and the
HBM-bound kernels in GB/s."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_bench_line_contract():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--steps", "10", "--warmup", "2",
                        "--no-cpu-baseline"], capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.loads((ROOT / "BASELINE.json").read_text())
    assert d["metric"] == base["metric"]
    assert d["unit"] == "samples/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["n_gpus"] == 1 and d["steps"] == 10 and d["warmup"] == 2
    assert d["dtype"] == "bf16" and d["data"] == "synthetic" and d["vs_baseline"] is None
    assert d["config"]["global_batch"] == 256 and d["config"]["workload"]
    # whole-job throughput consistent with the step time
    assert d["value"] > 1000 and abs(d["value"] - 256 / (d["ms_per_step"] * 1e-3)) / d["value"] < 0.02
    rf = d["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 2500.0
    assert 0 < rf["frac"] < 1 and abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 1e-3
    assert abs(rf["flops_per_launch"] / (rf["avg_ms"] * 1e-3) / 1e12 - rf["achieved"]) / rf["achieved"] < 0.01
    assert rf["traffic"] is None or rf["traffic"] > 0
    hk = d["hbm_kernels"]
    assert set(hk) == {"fusion_fwd", "fusion_bwd", "cross_entropy", "ln_fwd768", "adam"}
    for t, e in hk.items():
        assert e["unit"] == "GB/s" and e["peak"] == 8000.0 and 0 < e["frac"] < 1, (t, e)
        calc = e["alg_bytes_per_launch"] / (e["avg_us"] * 1e-6) / 1e9     # the line rounds GB/s to 0.1
        assert abs(calc - e["achieved"]) <= max(0.01 * e["achieved"], 0.06), (t, calc, e["achieved"])
