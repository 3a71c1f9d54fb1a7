#!/bin/bash
# Host-visible release of the resolve's output: mismatch count of the tail
# sweep (tools/tails_repro.py) and the headline, per library (diagnostics).
mkdir -p gpurun_out
T=${1:-r06hr}; shift
for v in "$@"; do
  n=$(basename $(dirname $v)); [ $v = main ] && n=main
  if [ $v = main ]; then L=""; else L="CHUNKFS_AMD_LIB=$v"; fi
  env $L timeout -k 10 400 python3 -u tools/tails_repro.py 60 > gpurun_out/${T}_${n}_tails.log 2>&1 || exit 1
  echo "$n $(tail -1 gpurun_out/${T}_${n}_tails.log)"
  env $L timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 --no-config5 > gpurun_out/${T}_${n}.json 2> gpurun_out/${T}_${n}.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f ms/step sustained %.4f sync %.4f alone %.4f' % (d['ms_per_step'], d['sustained']['ms_per_step'], d['latency_sync']['median_ms'], d['phase_ms']['scan_alone']))" gpurun_out/${T}_${n}.json $n
done
