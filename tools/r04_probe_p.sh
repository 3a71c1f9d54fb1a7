export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk.py -k "rabin" > gpurun_out/t_p.log 2>&1
rc=$?; tail -3 gpurun_out/t_p.log; [ $rc -eq 0 ] || exit $rc
WB_ALGOS=rabin timeout -k 10 300 python -u tools/walk_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
WB_ALGOS=rabin timeout -k 10 300 python -u tools/walk_bench.py 1073741824 2048 4096 8192 2>&1 | grep -v amdgpu.ids || exit 1
WB_ALGOS=rabin timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p -o run -- python3 tools/walk_bench.py > gpurun_out/prof_p.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/prof_p/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:5]:
    print(f"{float(r['AverageNs'])/1e3:10.1f} us avg x{r['Calls']:>4}  {r['Name'][:100]}")
PY
