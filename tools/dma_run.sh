#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/ubdma
timeout -k 10 120 ./_build/ubench_dma > gpurun_out/ubdma/sweep.txt 2>&1 || exit $?
cat gpurun_out/ubdma/sweep.txt
for v in 8,1,2,0 8,1,2,1; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_dma --output-format csv -d gpurun_out/ubdma/pmc_$v -o p -- ./_build/ubench_dma $v > gpurun_out/ubdma/pmc_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/ubdma/pmc_$v -name "*counter_collection.csv" | head -1)
  python3 -c "
import csv,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if r['Counter_Name']=='FETCH_SIZE']
print('$v FETCH_SIZE per launch (KB):', [round(x) for x in v[:4]], 'x2/2^30 =', 2*v[-1]*1024/2**30)
"
done
