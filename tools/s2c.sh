cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 > $O/s2c_attn.log 2>&1 && EEGF_ATTN256=0 timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 >> $O/s2c_attn.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/$O/s2c_pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py 0.1 > $GRAFT_REPO_ROOT/$O/s2c_pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$O/s2c_pmc2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py 0.1 > $GRAFT_REPO_ROOT/$O/s2c_pmc2.log 2>&1 || exit 1
echo done
