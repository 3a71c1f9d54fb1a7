# SeqCDC walk after a change: seq parity tests, then per-kernel times of the
# shipped build and of variant builds given as arguments (_exp/<name>/lib.so).
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py -k "${TESTK:-seq or walk_rules}" > gpurun_out/t_y.log 2>&1
rc=$?; tail -2 gpurun_out/t_y.log; [ $rc -eq 0 ] || exit $rc
# WALKS="17,16 18,12": also the shipped build with those CHUNKFS_AMD_WALK overrides
for v in base "$@" $(for w in $WALKS; do echo w$w; done); do
  lib=""; walk=""
  case $v in base) ;; w*) walk=${v#w} ;; *) lib=_exp/$v/lib.so ;; esac
  CHUNKFS_AMD_LIB=$lib CHUNKFS_AMD_WALK=$walk WB_ALGOS=${WB_ALGOS:-seq} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_y_$v -o run -- python3 tools/walk_bench.py > gpurun_out/prof_y_$v.log 2>&1 || exit 1
  grep -E "^(seq|rabin|ultra|leap) " gpurun_out/prof_y_$v.log
  python3 - $v <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/prof_y_{sys.argv[1]}/run_kernel_stats.csv')))
print(sys.argv[1], [(r['Name'].split('(')[0].split('::')[-1], int(r['Calls']), round(float(r['AverageNs'])/1e3, 1)) for r in rows if float(r['TotalDurationNs']) > 60000 and 'fill' not in r['Name']])
PY
done
# per-phase / per-round walk timings of the shipped build (CHUNKFS_AMD_WALKDIAG)
[ -n "$DIAG" ] && CHUNKFS_AMD_WALKDIAG=1 WB_ALGOS=$DIAG timeout -k 10 120 python3 tools/walk_bench.py 2>&1 | grep -E "walkdiag|^(seq|rabin|ultra|leap) " | tail -24
exit 0
