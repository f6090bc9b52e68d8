# round-end evidence: PMC traffic of the roofline kernel, kernel stats, then the full bench line
cd $GRAFT_REPO_ROOT
O=gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/s3f_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/s3f_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/s3f_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/s3f_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s3f_stats -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $R/$O/s3f_stats.log 2>&1 || exit 1
cd $R
python3 tools/parse_prof.py r1s3 $O/s3f_stats $O/s3f_fetch $O/s3f_write --steps 6 > $O/s3f_parse.log 2>&1 || exit 1
cp profiles/traffic.json profiles/r1s3_kernel_stats.md $O/ 
timeout -k 10 600 python -u bench.py > $O/s3f_bench.json 2> $O/s3f_bench.err || exit 1
echo done
