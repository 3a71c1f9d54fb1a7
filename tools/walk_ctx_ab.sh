#!/bin/bash
# Async walk lines (tools/leg.py algos) with 2 / 3 / 4 contexts (diagnostics).
mkdir -p gpurun_out
T=${1:-r06wc}
for rep in 1 2; do for k in 2 3 4; do
  CHUNKFS_AMD_WALK_CTX=$k timeout -k 10 300 python3 -u tools/leg.py algos --cpu-seconds 0 --no-parity > gpurun_out/${T}_c${k}_$rep.json 2> gpurun_out/${T}_c${k}_$rep.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('ctx', sys.argv[2], ' '.join('%s %.0f (%.3f)' % (k, v['GiBps'], v['frac_of_hbm']) for k,v in d.items()))" gpurun_out/${T}_c${k}_$rep.json $k
done; done
