set -o pipefail
O=gpurun_out; export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in cur sprio; do
    lib=""; [ $v = sprio ] && lib=ab/libsprio.so
    echo "== $v $r" >> $O/r4zh_attn.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/attn_bench.py --nobits >> $O/r4zh_attn.log 2>&1 || exit 1
  done
done
for r in 1 2 3; do
  for v in cur sprio; do
    lib=""; [ $v = sprio ] && lib=ab/libsprio.so
    echo "== $v $r" >> $O/r4zh_bench.log
    EEGF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 >> $O/r4zh_bench.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/r4zh_attn.log; grep -h "==\|ms_per_step" $O/r4zh_bench.log | sed 's/.*"ms_per_step": \([0-9.]*\).*/ms \1/'
