#!/bin/bash
# GPU box: segment-walk engine parity tests, then timing sweeps of the
# segment size / warm-up (tools/walk_bench.py).  Stops at the first failure.
TAG=${1:-walk}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -m gpu -v -x --timeout 240 --timeout-method thread \
    > $OUT/pytest_walk_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_walk_$TAG.log
[ $rc -eq 0 ] || exit $rc
for W in ${WALKS:-default 15,4 16,8 15,16}; do
    if [ $W = default ]; then unset CHUNKFS_AMD_WALK; else export CHUNKFS_AMD_WALK=$W; fi
    timeout -k 10 120 python -u tools/walk_bench.py >> $OUT/walk_bench_$TAG.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "walk_bench $W rc=$rc"; tail -5 $OUT/walk_bench_$TAG.log; exit $rc; }
done
cat $OUT/walk_bench_$TAG.log
