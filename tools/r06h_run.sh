mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_walk.py tests/test_gpu_configs.py tests/test_gpu_hostpath.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r06h_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for f in 1 0; do
  CHUNKFS_AMD_WALK_FUSED=$f timeout -k 10 300 python3 -u tools/leg.py algos > gpurun_out/r06h_algos_f${f}_$rep.json 2> gpurun_out/r06h_algos_f${f}_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06h_algos_f${f}_$rep.json')); print('fused=$f', {k: (round(v['GiBps'],1), round(v['frac_of_hbm'],4), v['parity_vs_oracle']) for k,v in d.items()})"
done; done
echo done
