mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sha256.py tests/test_gpu_index.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06f_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r06f_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -k 10 300 python3 -u tools/leg.py config3 > gpurun_out/r06f_c3_${v}_$rep.json 2> gpurun_out/r06f_c3_${v}_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06f_c3_${v}_$rep.json')); print('$v', round(d['gpu_GiBps'],1), {k: round(x,3) for k,x in d['gpu_phase_ms'].items()}, round(d['sha256_GiBps'],1), d['dedup_ratio_equal'], d['chunks_bit_exact'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06f -o run -- python3 tools/leg.py config3 > gpurun_out/prof_r06f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex sha256 --output-format csv -d gpurun_out/pmc_r06f -o p -- python3 tools/leg.py config3 > gpurun_out/pmc_r06f.log 2>&1 || exit 1
echo done
