cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/s3e_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/s3e_bench.json 2> $O/s3e_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/s3e_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/s3e_prof.log 2>&1 || exit 1
echo done
