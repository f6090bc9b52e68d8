cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/dbg_acs.py 4096 768 2304 > gpurun_out/s3c.log 2>&1 || exit 1
echo done
