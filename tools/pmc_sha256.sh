#!/bin/bash
# SHA-256 fingerprint kernel against its VALU roofline: kernel time and the
# VALU instruction count of the same command (separate rocprofv3 runs:
# kernel trace, then one counters-only pass).  Usage: tools/pmc_sha256.sh TAG
TAG=${1:-r02}
OUT=gpurun_out/sha_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --hash --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-host-path --no-sweep"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- $CMD \
    > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-include-regex sha256 \
    --output-format csv -d $OUT/pmc -o p -- $CMD > $OUT/pmc.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
grep -h sha256 $(find $OUT/trace -name "*kernel_stats.csv") | head -3
f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k}: n={len(v)} mean={sum(v)/len(v):.6g}")
PY
cat gpurun_out/sha_$TAG/trace.log | tail -1 | cut -c1-2000 > $OUT/bench_line.json
exit 0
