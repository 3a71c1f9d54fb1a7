export TMPDIR=/tmp
timeout -k 10 300 python -u tools/walk_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_o -o run -- python3 tools/walk_bench.py > gpurun_out/prof_o.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/prof_o/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us avg x{r['Calls']:>4}  {r['Name'][:100]}")
PY
