#!/bin/bash
# One GPU session: parity tests, GEMM schedule A/B, bench line, rocprofv3 kernel stats.
# usage (on the box, from the repo root): bash tools/gpu_round.sh <tag> [steps...]
set -o pipefail
TAG=${1:-r1}
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { local name=$1; shift; echo "[gpu_round] $name" >&2; "$@"; local rc=$?; echo "[gpu_round] $name rc=$rc" >&2; return $rc; }
# pytest exit 1 = some test failed (no fault): keep going; anything else (timeout 124/137, abort 134,
# segfault 139, interrupted 2) ends the session
tstep() { step "$@"; local rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
for s in "${@:2}"; do
  case $s in
    newtests) tstep newtests timeout -k 10 600 python -u -m pytest tests/test_fixtures_gpu.py tests/test_production_gpu.py -v --timeout 240 --timeout-method thread > $O/${TAG}_new_tests.log 2>&1 || exit 1 ;;
    prof16) (cd /tmp && export TMPDIR=/tmp && step prof16 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/${TAG}_prof16 -o run -- python3 -m pytest $GRAFT_REPO_ROOT/tests/test_production_gpu.py -x -q -k "b16 and not priconcat and not True" --timeout 240 > $GRAFT_REPO_ROOT/$O/${TAG}_prof16.log 2>&1) || exit 1 ;;
    tests) tstep tests timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || exit 1 ;;
    gemm8tests) EEGF_GEMM8=4 step gemm8tests timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/${TAG}_gemm8_tests.log 2>&1 || exit 1 ;;
    gemmab) step gemmab timeout -k 10 300 python -u tools/gemm_bench.py --ab > $O/${TAG}_gemm_ab.log 2>&1 || exit 1 ;;
    attn) step attn timeout -k 10 120 python -u tools/attn_bench.py > $O/${TAG}_attn.log 2>&1 && EEGF_ATTN256=0 step attn0 timeout -k 10 120 python -u tools/attn_bench.py >> $O/${TAG}_attn.log 2>&1 || exit 1 ;;
    attntests) step attntests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/${TAG}_attn_tests.log 2>&1 || exit 1 ;;
    gemm) step gemm timeout -k 10 300 python -u tools/gemm_bench.py > $O/${TAG}_gemm.log 2>&1 || exit 1 ;;
    bench) step bench timeout -k 10 580 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 1 ;;
    prof) (cd /tmp && export TMPDIR=/tmp && step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/${TAG}_prof.log 2>&1) || exit 1 ;;
    profnp) (cd /tmp && export TMPDIR=/tmp && step profnp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/${TAG}_profnp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probe > $GRAFT_REPO_ROOT/$O/${TAG}_profnp.log 2>&1) || exit 1 ;;
    c5) step c5 timeout -k 10 600 python -u bench.py --batch 512 --eps-sweep 0.1,1,3,5,10 --feawei 2048 --steps 4 --warmup 2 --no-cpu-baseline > $O/${TAG}_c5.json 2> $O/${TAG}_c5.err || exit 1 ;;
    priconcat) step priconcat timeout -k 10 300 python -u bench.py --variant priconcat --no-cpu-baseline > $O/${TAG}_priconcat.json 2> $O/${TAG}_priconcat.err || exit 1 ;;
    b512) step b512 timeout -k 10 300 python -u bench.py --batch 512 --no-cpu-baseline > $O/${TAG}_b512.json 2> $O/${TAG}_b512.err || exit 1 ;;
    pmc) step pmc bash tools/pmc_round.sh $TAG || exit 1 ;;
    cpub256) step cpub256 timeout -k 10 1080 python -u bench.py --cpu-baseline-only --cpu-batch 256 --cpu-iters 3 --cpu-warm-batch 16 --cpu-baseline-out $O/cpu_baseline_b256.json > $O/${TAG}_cpub256.json 2> $O/${TAG}_cpub256.err || exit 1 ;;
    layer11) tstep layer11 timeout -k 10 300 python -u -m pytest tests/test_attn_layer11_gpu.py -x -v -s --timeout 240 --timeout-method thread > $O/${TAG}_layer11.log 2>&1 || exit 1 ;;
    smoke) step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit 1 ;;
  esac
done
echo "[gpu_round] done"
