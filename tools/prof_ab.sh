#!/bin/bash
# rocprofv3 kernel stats of the bench step for ab/libbase.so and the in-tree library (one box), then the
# per-kernel comparison (tools/prof_cmp.py).  usage (on the box, repo root): bash tools/prof_ab.sh <tag>
set -o pipefail
TAG=${1:-pab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for arm in base new; do
  lib=""; [ $arm = base ] && lib=$R/ab/libbase.so
  EEGF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${TAG}_$arm -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probe > $O/${TAG}_$arm.log 2>&1 || exit 1
done
cd $R
python3 tools/prof_cmp.py $O/${TAG}_base $O/${TAG}_new 8 > $O/${TAG}_cmp.log 2>&1
cat $O/${TAG}_cmp.log | head -60
