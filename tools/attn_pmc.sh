#!/bin/bash
# stall / issue breakdown of the L = 256 attention kernels (tools/attn_bench.py at p = 0 and 0.1,
# regenerated masks): three SQ counter passes, then tools/kpmc.py.  usage: bash tools/attn_pmc.sh <tag>
set -o pipefail
TAG=${1:-attn}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
pass() { local n=$1; shift; echo "[pmc] $n"; timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d $O/${TAG}_$n -o run --output-format csv -- python3 $R/tools/attn_bench.py 0 0.1 --nobits > $O/${TAG}_$n.log 2>&1; local rc=$?; echo "[pmc] $n rc=$rc"; return $rc; }
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit 1
pass b SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit 1
pass c SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
cd $R && python3 tools/kpmc.py attn_fwd256,attn_bwd256 $O/${TAG}_a $O/${TAG}_b $O/${TAG}_c > $O/${TAG}_pmc.txt 2>&1
echo "[pmc] done"
