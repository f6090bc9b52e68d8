#!/bin/bash
# attention dropout renumbering + forward rewrite: attention / dropout / varlen / determinism tests,
# then interleaved attn_bench base (ab/libbase.so) / new, then the step A/B
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_parity_gpu.py tests/test_determinism_gpu.py tests/test_varlen_gpu.py tests/test_dpsgd_gpu.py -q --timeout 200 --timeout-method thread > $O/r3m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r3m_tests.log; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v attn $rep" >> $O/r3m_ab.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 --nobits >> $O/r3m_ab.log 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v bench $rep" >> $O/r3m_ab.log
    EEGF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 >> $O/r3m_ab.log 2>&1 || exit 1
  done
done
echo done
