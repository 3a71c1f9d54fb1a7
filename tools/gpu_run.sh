#!/bin/bash
# Runs on the GPU box (via gpurun): GPU tests, bench, rocprofv3 kernel stats.
# Stops at the first fault / abort / segfault / timeout (rc not in {0,1}).
# Usage: tools/gpu_run.sh [tag] [steps] [pytest-args...]
TAG=${1:-r02}
STEPS=${2:-20}
shift 2 2>/dev/null
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method thread "$@" \
    > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $OUT/pytest_gpu_$TAG.log
ok $rc || exit $rc

timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -3 $OUT/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-host-path --no-sweep --no-algos --no-config4 \
    > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $OUT/prof_$TAG.log
exit $rc
