#!/bin/bash
# Scan-kernel timing modes (CHUNKFS_AMD_DIAG bits 8-9: 256 = loads and
# transposes only, 512 = hashing only; results meaningless) beside the real
# scan, plus the ubench reference rows.  Usage: tools/scan_modes.sh TAG
TAG=${1:-modes}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BENCH="bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 --no-parity"
for m in 0 256 512; do
  CHUNKFS_AMD_DIAG=$m timeout -k 10 120 python -u $BENCH > $OUT/bench_$m.json 2> $OUT/bench_$m.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$m.json')); print('diag $m scan_ms', round(d['phase_ms']['scan'],4))"
done
