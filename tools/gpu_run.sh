#!/bin/bash
# Runs on the GPU box (via gpurun): GPU tests, bench, rocprofv3 kernel stats.
# Stops at the first fault / abort / segfault / timeout (rc not in {0,1}).
# Usage: tools/gpu_run.sh [tag] [steps]
TAG=${1:-r01}
STEPS=${2:-20}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu_$TAG.log
ok $rc || exit $rc

timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-host-path > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof_$TAG.log
find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -3
exit $rc
