#!/bin/bash
# Bounded first GPU run of pipeline 2 (run on the GPU box via gpurun):
#   stage tests (scan records vs pipeline 1, links vs the CPU model), then the
#   full parity suite with pipeline 2, then the SHA-256 / index / C++ tests,
#   then a pipeline-2 bench and its rocprof kernel stats.
# Each GPU step has its own time limit; the script stops at the first fault,
# abort or timeout (exit status other than 0/1).
TAG=${1:-r02a}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }

CHUNKFS_AMD_TEST_PIPELINE2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline2.py -m gpu -v -x \
    --timeout 120 --timeout-method thread -k "stage" > $OUT/p2_stage_$TAG.log 2>&1
rc=$?; echo "stage rc=$rc"; tail -20 $OUT/p2_stage_$TAG.log; ok $rc || exit $rc

CHUNKFS_AMD_TEST_PIPELINE2=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline2.py -m gpu -v \
    --timeout 300 --timeout-method thread > $OUT/p2_parity_$TAG.log 2>&1
rc=$?; echo "p2 parity rc=$rc"; tail -20 $OUT/p2_parity_$TAG.log; ok $rc || exit $rc

timeout -k 10 600 python -u -m pytest tests/test_gpu_sha256.py tests/test_gpu_index.py tests/test_cpp_mirror.py \
    -m gpu -v -rxX --timeout 300 --timeout-method thread > $OUT/new_kernels_$TAG.log 2>&1
rc=$?; echo "sha/index/cpp rc=$rc"; tail -20 $OUT/new_kernels_$TAG.log; ok $rc || exit $rc

CHUNKFS_AMD_PIPELINE=2 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --hash > $OUT/bench_p2_$TAG.json 2> $OUT/bench_p2_$TAG.err
rc=$?; echo "bench p2 rc=$rc"; cat $OUT/bench_p2_$TAG.json; tail -5 $OUT/bench_p2_$TAG.err; [ $rc -eq 0 ] || exit $rc

CHUNKFS_AMD_PIPELINE=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p2_$TAG -o run \
    -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-host-path > $OUT/prof_p2_$TAG.log 2>&1
rc=$?; echo "rocprof p2 rc=$rc"
exit $rc
