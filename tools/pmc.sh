#!/bin/bash
# PMC passes on the scan kernel (separate rocprofv3 runs, counters only, as
# MI355X_MICROARCH.md prescribes).  Usage: tools/pmc.sh TAG [kernel-regex]
TAG=${1:-r02}
KRE=${2:-p3::.*scan_kernel}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...  (kernel regex: $RKRE, default $KRE)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "${RKRE:-$KRE}" --output-format csv \
      -d $OUT/$name -o p -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --no-host-path --no-algos \
      --no-sweep --no-config4 --no-config5 > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit 1
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run sq3 SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT64 SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES || exit 1
run fetch FETCH_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
# calibration: the same counter on the bench's bare read of the stream (read_kernel,
# the achievable-bandwidth reference), so the scan's ratio can be read against it
RKRE="read_kernel" run fetch_read FETCH_SIZE || exit 1
for d in $OUT/*/; do f=$(find $d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && echo "== $d" && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, v in agg.items():
    print(f"{k}: n={len(v)} mean={sum(v)/len(v):.4g} min={min(v):.4g} max={max(v):.4g}")
PY
done
f=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 tools/traffic_json.py "$f" $OUT/traffic.json 1073741824
f=$(find $OUT/fetch_read -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 tools/traffic_json.py "$f" $OUT/traffic_read.json 1073741824 read_kernel
exit 0
