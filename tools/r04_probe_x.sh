# SeqCDC wave walk timing experiments: the shipped build vs variant builds
# without bitmap loads / without jumps (results differ; timing only), and
# segment size / warm-up overrides (CHUNKFS_AMD_WALK=seg_log2,warm_over_avg).
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py -k seq > gpurun_out/t_x.log 2>&1
rc=$?; tail -2 gpurun_out/t_x.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib walk
  CHUNKFS_AMD_LIB=$2 CHUNKFS_AMD_WALK=$3 WB_ALGOS=seq timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x_$1 -o run -- python3 tools/walk_bench.py > gpurun_out/prof_x_$1.log 2>&1 || exit 1
  grep "^seq" gpurun_out/prof_x_$1.log
  python3 - $1 <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/prof_x_{sys.argv[1]}/run_kernel_stats.csv')))
print(sys.argv[1], {r['Name'].split('::')[-1][:18]: (int(r['Calls']), round(float(r['AverageNs'])/1e3, 1)) for r in rows if 'walk' in r['Name'] and float(r['TotalDurationNs']) > 100000})
PY
}
run base "" "" && run noload _exp/noload/lib.so "" && run nojump _exp/nojump/lib.so "" && run both _exp/both/lib.so "" \
 && run s19w16 "" 19,16 && run s20w16 "" 20,16 && run s19w12 "" 19,12 && run s20w24 "" 20,24
