#!/bin/bash
# SQ counters of the DMA scan kernel (bench) and of the DMA ubench (8,1,2,1),
# one counter set per rocprofv3 pass.
OUT=gpurun_out/${1:-pmc_dma}
mkdir -p $OUT
export TMPDIR=/tmp
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_LDS"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex scan_dma --output-format csv -d $OUT/b$i -o p -- \
     python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --no-host-path --no-algos --no-sweep --no-config4 > $OUT/b$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-include-regex k_dma --output-format csv -d $OUT/u$i -o p -- ./_build/ubench_dma 8,1,2,1 > $OUT/u$i.log 2>&1 || exit $?
done
for d in $OUT/b1 $OUT/b2 $OUT/u1 $OUT/u2; do f=$(find $d -name "*counter_collection.csv" | head -1); echo "== $d"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"  {k:24s} mean/launch {sum(v)/len(v):.4g}")
PY
done
