cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/dbg_acs2.py > gpurun_out/s3d.log 2>&1 || exit 1
echo done
