#!/bin/bash
# Bench lines (headline + sweep + parity) of experiment builds against the
# in-tree library, interleaved: tools/lib_ab.sh TAG REPS LIB... (diagnostics;
# "main" = the in-tree library).
mkdir -p gpurun_out
T=$1; REPS=$2; shift 2
H="--cpu-seconds 0 --no-host-path --no-algos --no-config4 --no-config5"
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    n=$(basename $(dirname $v)); [ $v = main ] && n=main
    f=gpurun_out/${T}_${n}_$rep.json
    if [ $v = main ]; then env -u CHUNKFS_AMD_LIB timeout -k 10 300 python3 -u bench.py $H > $f 2> ${f%.json}.err || exit 1
    else CHUNKFS_AMD_LIB=$v timeout -k 10 300 python3 -u bench.py $H > $f 2> ${f%.json}.err || exit 1; fi
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
sw={k:(round(v['ms_per_step'],4), v['parity_vs_oracle']) for k,v in d['sweep'].items() if isinstance(v,dict)}
print(sys.argv[2], 'rep', sys.argv[3], '%.4f ms/step' % d['ms_per_step'], 'alone %.4f' % d['phase_ms']['scan_alone'], 'sync %.4f' % d['latency_sync']['median_ms'], 'parity', d.get('parity_vs_oracle'), sw)" $f $n $rep
  done
done
