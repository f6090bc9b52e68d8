#!/bin/bash
# PMC evidence for the bench workload: three counter passes (SQ mix + clocks, FETCH_SIZE, WRITE_SIZE),
# each its own rocprofv3 run, then the per-kernel table (tools/pmc_table.py -> profiles/).
# usage (on the box, from the repo root): bash tools/pmc_round.sh <tag>
set -o pipefail
TAG=${1:-r2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe"
cd /tmp && export TMPDIR=/tmp
pass() { local n=$1; shift; echo "[pmc] $n"; timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $O/${TAG}_pmc_$n -o run --output-format csv -- $B > $O/${TAG}_pmc_$n.log 2>&1; local rc=$?; echo "[pmc] $n rc=$rc"; return $rc; }
pass sq SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
cd $R
python3 tools/pmc_table.py $TAG 3 $O/${TAG}_pmc_sq $O/${TAG}_pmc_fetch $O/${TAG}_pmc_write > $O/${TAG}_pmc_table.log 2>&1 || exit 1
cp profiles/${TAG}_pmc_table.md profiles/pmc_${TAG}.json $O/
echo "[pmc] done"
