# Walk engine after a change: walk parity tests, then walk_bench (1 GiB) with
# per-kernel stats for the bitmap rules.
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk.py tests/test_gpu_configs.py > gpurun_out/t_w.log 2>&1
rc=$?; tail -3 gpurun_out/t_w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/walk_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
WB_ALGOS=${WB_ALGOS:-seq,ultra} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w -o run -- python3 tools/walk_bench.py > gpurun_out/prof_w.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_w/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
