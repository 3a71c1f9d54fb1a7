# Round-5 probe: host placement + config-5 full-size tests, the host path with
# NUMA placement on/off (same box, interleaved), the config-5 leg with whole-stream parity.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r05n}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hostpath.py tests/test_gpu_small.py "tests/test_gpu_configs.py::test_config5_full_gib_stream_avg64k" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
HP="--steps 5 --warmup 2 --cpu-seconds 0 --no-sweep --no-algos --no-config4 --no-config5"
for r in 1 2; do for nm in 1 0; do
  CHUNKFS_AMD_COPY_NUMA=$nm timeout -k 10 300 python3 -u bench.py $HP > gpurun_out/${T}_hp_numa${nm}_$r.json 2> gpurun_out/${T}_hp_numa${nm}_$r.err
  rc=$?; echo "numa=$nm rep=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_hp_numa${nm}_$r.json').read().splitlines()[-1]); h=d['host_path']; c=h['chunk_data_1MiB_calls']; print(json.dumps(h.get('numa')), round(c['us_per_call'],2), round(c['GiBps']/c['cpu_oracle_same_loop_GiBps'],3), round(h['write_stream_1MiB_segments']['GiBps'],2), round(h['GiBps'],2))"
done; done
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err
rc=$?; echo "c5 rc=$rc"; python3 -c "import json; d=json.loads(open('gpurun_out/${T}_c5.json').read().splitlines()[-1]); print(json.dumps(d['summary'].get('config5')))"; exit $rc
