export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py tests/test_gpu_configs.py > gpurun_out/t_v.log 2>&1
rc=$?; tail -3 gpurun_out/t_v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-host-path --no-algos --no-config4 > gpurun_out/b_v.json 2> gpurun_out/b_v.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/b_v.json')); print(d['value'], d['ms_per_step'], d['phase_ms'], d['parity_vs_oracle'], {k:(round(v['GiBps']),v['parity_vs_oracle']) for k,v in d['sweep'].items()})"
CHUNKFS_AMD_DIAG=128 timeout -k 10 120 python -u tools/fast_probe.py 3 --no-parity 2>&1 | grep -v amdgpu.ids | tail -3
