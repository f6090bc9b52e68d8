#!/bin/bash
# Interleaved A/B of ab/libbase.so against the in-tree library on one box: bit identity of the GEMM
# epilogues (tools/epi_bits.py), GEMM shapes, then bench steps, each in alternating rounds.
# usage (on the box, repo root): bash tools/ab_round.sh <tag> <reps> [gemm shape names...]
set -o pipefail
TAG=${1:-ab}
REPS=${2:-3}
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$O/${TAG}_ab.log
NEW=${NEWLIB:-}          # the "new" arm: the in-tree library, or NEWLIB (a variant build under ab/)
: > $L
run() {   # run <label> <lib or ""> <seconds> <cmd...>
  local label=$1 lib=$2 t=$3; shift 3
  echo "== $label" >> $L
  EEGF_LIB=$lib timeout -k 10 $t "$@" >> $L 2>&1
}
run "base bits" ab/libbase.so 120 python -u tools/epi_bits.py || exit 1
run "new bits" "$NEW" 120 python -u tools/epi_bits.py || exit 1
if [ $# -gt 2 ]; then
  for rep in $(seq $REPS); do
    run "base gemm $rep" ab/libbase.so 200 python -u tools/gemm_bench.py "${@:3}" || exit 1
    run "new gemm $rep" "$NEW" 200 python -u tools/gemm_bench.py "${@:3}" || exit 1
  done
fi
if [ -n "$WGRAD" ]; then
  for rep in $(seq $REPS); do
    run "base wgrad $rep" ab/libbase.so 200 python -u tools/wgrad_probe.py || exit 1
    run "new wgrad $rep" "$NEW" 200 python -u tools/wgrad_probe.py || exit 1
  done
fi
if [ -n "$ATTN" ]; then
  for rep in $(seq $REPS); do
    run "base attn $rep" ab/libbase.so 200 python -u tools/attn_bench.py --nobits || exit 1
    run "new attn $rep" "$NEW" 200 python -u tools/attn_bench.py --nobits || exit 1
  done
fi
for rep in $(seq $REPS); do
  run "base bench $rep" ab/libbase.so 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit 1
  run "new bench $rep" "$NEW" 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit 1
done
python - "$L" > $O/${TAG}_ab_summary.log <<'EOF'
import json, re, sys
from collections import defaultdict
cur, bits, ms, gem = None, defaultdict(list), defaultdict(list), defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("== "):
        cur = line[3:].split()[0]
        continue
    if line.startswith(("fwd ", "dgrad ", "wgrad ", "attn ")):
        bits[cur].append(line.strip())
    elif line.startswith("{"):
        try:
            ms[cur].append(json.loads(line)["ms_per_step"])
        except Exception:
            pass
    else:
        m = re.match(r"(\S+)\s+M=\s*\d+ N=\s*\d+ K=\s*\d+\s+eegf\s+([\d.]+) us", line)
        if m:
            gem[(cur, m.group(1))].append(float(m.group(2)))
        m = re.match(r"(attn_\w+) B=\d+ L=\d+ p=\S+ bits=(\d):\s+([\d.]+) us", line)
        if m:
            gem[(cur, m.group(1) + ("+bits" if m.group(2) == "1" else ""))].append(float(m.group(3)))
        m = re.match(r"(\S+_wgrad)\s+\S+\s+with bias grad\s+([\d.]+) us\s+plain\s+([\d.]+) us", line)
        if m:
            gem[(cur, m.group(1) + "+bias")].append(float(m.group(2)))
            gem[(cur, m.group(1))].append(float(m.group(3)))
print("bits identical:", bits["base"] == bits["new"] and len(bits["base"]) > 0)
for a, b in zip(bits["base"], bits["new"]):
    if a != b:
        print("  DIFF", a, "|", b)
for (who, shape), v in sorted(gem.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print(f"{shape:20s} {who:5s} median {sorted(v)[len(v)//2]:8.1f} us  all {v}")
for who, v in ms.items():
    print(f"bench {who:5s} median {sorted(v)[len(v)//2]:.3f} ms/step  all {v}")
EOF
cat $O/${TAG}_ab_summary.log
echo "[ab_round] done"
