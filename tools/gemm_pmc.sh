#!/bin/bash
# Stall breakdown of one GEMM shape (tools/gemm_one.py), ours vs hipBLASLt: three counter passes per
# variant (SQ issue / VMEM-LDS queues / TA), then tools/kpmc.py.
# usage (on the box, repo root): bash tools/gemm_pmc.sh <tag> <shape> "<variant ...>"   (variant: -1 or torch)
set -o pipefail
TAG=$1 SHAPE=$2 VARS=$3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  vn=${v/-/m}
  pass() { local n=$1; shift; echo "[pmc] $vn $n"; timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d $O/${TAG}_${vn}_$n -o run --output-format csv -- python3 $R/tools/gemm_one.py $SHAPE $v 20 > $O/${TAG}_${vn}_$n.log 2>&1; local rc=$?; echo "[pmc] $vn $n rc=$rc"; return $rc; }
  pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
  pass b SQ_WAVE_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  pass c TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE || exit 1
done
cd $R
for v in $VARS; do
  vn=${v/-/m}
  echo "== $vn" >> $O/${TAG}_pmc.txt
  python3 tools/kpmc.py Cijk,gemm4 $O/${TAG}_${vn}_a $O/${TAG}_${vn}_b $O/${TAG}_${vn}_c >> $O/${TAG}_pmc.txt 2>&1
done
echo "[pmc] done"
