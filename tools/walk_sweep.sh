#!/bin/bash
# Walk-engine segment / warm-up sweep at config 5's avg 64 KiB and the bench
# sizes (CHUNKFS_AMD_WALK="seg_log2,warm_over_avg"; read at handle creation).
# Usage: tools/walk_sweep.sh TAG "setting ..."
TAG=${1:-wsweep}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for w in "$@"; do
  for sz in "16384 65536 524288" "4096 8192 16384"; do
    CHUNKFS_AMD_WALK=$w timeout -k 10 120 python -u tools/walk_bench.py 1073741824 $sz > $OUT/w_${w/,/_}_${sz// /_}.log 2>&1 || exit 1
    echo "== walk $w sizes $sz"; grep GiB $OUT/w_${w/,/_}_${sz// /_}.log
  done
done
