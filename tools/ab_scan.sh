#!/bin/bash
# FastCDC parity tests, then the bench line with the default scan and with the
# register-staged scan (CHUNKFS_AMD_DIAG=1024) for A/B.  Usage: tools/ab_scan.sh TAG
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
Q="--cpu-seconds 0 --no-host-path --no-algos --no-sweep --no-config4"
for v in dma reg dma reg; do
  if [ $v = reg ]; then export CHUNKFS_AMD_DIAG=1024; else unset CHUNKFS_AMD_DIAG; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 $Q > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit $?
  python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', round(d['value'],1), 'scan_ms', round(d['roofline']['kernel_ms'],4), 'frac', round(d['roofline']['frac'],3), 'resolve', round(d['phase_ms']['resolve'],4), 'parity', d.get('parity_vs_oracle'))"
done
unset CHUNKFS_AMD_DIAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity $Q > $OUT/prof.log 2>&1 || exit $?
grep -h scan $OUT/prof/run_kernel_stats.csv | cut -c1-200
