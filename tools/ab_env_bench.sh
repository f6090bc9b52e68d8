#!/bin/bash
# Interleaved step A/B of environment settings on bench.py (one process per setting and round).
# usage (on the box, repo root): bash tools/ab_env_bench.sh <tag> <rounds> "<NAME=VALUE or none> ..." [bench args]
set -o pipefail
TAG=$1 ROUNDS=$2 SETS=$3; shift 3
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for r in $(seq 1 $ROUNDS); do
  for v in $SETS; do
    envs=""; [ $v != none ] && envs=$v
    echo "== $v $r" >> $O/${TAG}_bench_ab.log
    env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" >> $O/${TAG}_bench_ab.log 2>&1 || exit 1
  done
done
python3 - "$O/${TAG}_bench_ab.log" <<'PY'
import json, re, sys, collections
cur, res = None, collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+) \d+", line)
    if m: cur = m.group(1); continue
    if line.startswith("{"):
        res[cur].append(json.loads(line)["ms_per_step"])
for k, v in res.items():
    v = sorted(v)
    print(f"{k:24s} median {v[len(v) // 2]:.3f} ms/step  all {v}")
PY
