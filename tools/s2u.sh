cd $GRAFT_REPO_ROOT
O=gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 8 0; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $GRAFT_REPO_ROOT/$O/s2u_pmc_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/gemm_one.py sq4k $v 10 > $GRAFT_REPO_ROOT/$O/s2u_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_WAVES -d $GRAFT_REPO_ROOT/$O/s2u_pmc2_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/gemm_one.py sq4k $v 10 > $GRAFT_REPO_ROOT/$O/s2u2_$v.log 2>&1 || exit 1
done
echo done
