#!/bin/bash
# PMC passes for one kernel (separate rocprofv3 runs, counters only).
# Usage: tools/pmc_kernel.sh TAG KERNEL_REGEX
TAG=${1:-r02}
KRE=${2:-chain_kernel}
OUT=gpurun_out/pmck_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$name -o p -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-host-path \
      --no-sweep > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD || exit 1
run b SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE || exit 1
for d in $OUT/*/; do f=$(find $d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && echo "== $d" && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r.get("Kernel_Name")[:40], r.get("Counter_Name"))].append(float(r.get("Counter_Value", 0)))
for k, v in sorted(agg.items()):
    print(f"{k[0]} {k[1]}: n={len(v)} mean={sum(v)/len(v):.4g}")
PY
done
exit 0
