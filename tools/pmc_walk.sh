#!/bin/bash
# PMC passes on the segment-walk engine's kernels (separate rocprofv3 runs,
# counters only, MI355X_MICROARCH.md), over tools/walk_bench.py.
# Usage: tools/pmc_walk.sh TAG [kernel-regex] [algos]
TAG=${1:-r03}
KRE=${2:-"bits_kernel|wwalk_kernel"}
export WB_ALGOS=${3:-rabin,ultra}
OUT=gpurun_out/pmcw_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$name -o p -- python3 tools/walk_bench.py > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD || exit 1
run sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
for d in $OUT/*/; do f=$(find $d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && echo "== $d" && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r.get("Kernel_Name")[:45], r.get("Counter_Name"))].append(float(r.get("Counter_Value", 0)))
for k, v in sorted(agg.items()):
    print(f"{k[0]:45s} {k[1]:22s} n={len(v)} mean={sum(v)/len(v):.4g}")
PY
done
exit 0
