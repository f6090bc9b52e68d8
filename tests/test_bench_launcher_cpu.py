"""bench.py's multi-GPU contract on the CPU: `--gpus N` outside a launcher
starts N fresh ranks through torch.distributed.run, a WORLD_SIZE / --gpus mismatch exits 2, and the
reported world size is the process group's (gloo world-2 selftest)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                        "MASTER_PORT")}
    e.update(kw)
    return e


def test_gpus_two_launches_two_ranks():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--selftest", "--master-port", "29611"],
                       capture_output=True, text=True, env=_env(OMP_NUM_THREADS="1"), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["world_size"] == 2 and lines[0]["allreduce"] == 2.0
    assert lines[0]["backend"] == "gloo"


def test_world_size_mismatch_exits_2():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--selftest"], capture_output=True,
                       text=True, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_single_rank_selftest():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--selftest"], capture_output=True, text=True,
                       env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["world_size"] == 1
