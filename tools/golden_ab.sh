#!/bin/bash
# golden_repro.py (small path) per library (diagnostics).
mkdir -p gpurun_out
T=${1:-r06gr}; R=${2:-40}; shift 2
for v in "$@"; do
  n=$(basename $(dirname $v)); [ $v = main ] && n=main
  if [ $v = main ]; then L=""; else L="CHUNKFS_AMD_LIB=$v"; fi
  env $L timeout -k 10 300 python3 -u tools/golden_repro.py $R > gpurun_out/${T}_${n}.log 2>&1 || exit 1
  echo "$n: $(grep -v amdgpu.ids gpurun_out/${T}_${n}.log | tail -3 | tr '\n' ' ')"
done
