#!/bin/bash
# Time every experiment build under _exp/ (tools/build_variants.py): FastCDC
# parity of a 1 GiB stream vs the oracle plus scan / resolve / step times.
# Usage: tools/scan_variants.sh TAG [variant ...]
TAG=${1:-var}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
VARS=${@:-$(ls _exp)}
for v in $VARS; do
  CHUNKFS_AMD_LIB=_exp/$v/lib.so timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 \
      --no-host-path --no-sweep --no-algos --no-config4 > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -3 $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); p=d['phase_ms']; print('$v'.ljust(10), 'value', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'scan', round(p['scan'],4), 'resolve', round(p['resolve'],4), 'parity', d.get('parity_vs_oracle'))"
done
