#!/bin/bash
# Scan-kernel iteration on the GPU box: FastCDC parity tests, a short bench
# (no extras), the kernel statistics and one PMC pass (LDS / VALU counters).
# Usage: tools/scan_exp.sh TAG
TAG=${1:-exp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py -x -q --timeout 200 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
BENCH="bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4"
timeout -k 10 200 python -u $BENCH > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('value', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'scan frac', round(d['roofline']['frac'],4), d['phase_ms'], 'parity', d.get('parity_vs_oracle'))"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $BENCH --no-parity \
    > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 $f | head -8
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    --kernel-include-regex scan_kernel --output-format csv -d $OUT/pmc -o p -- python3 $BENCH --no-parity --steps 3 > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"
f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, v in sorted(agg.items()):
    print(f"{k}: mean={sum(v)/len(v):.4g}")
PY
exit $rc
