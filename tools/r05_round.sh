# Round-5 combined probe (one gpurun call): FastCDC parity + async tests, resolve
# timings, pipelined steps; Rabin parity and the bitmap-pass variants.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r05}
bash tools/r05_probe.sh $T || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py tests/test_gpu_configs.py tests/test_gpu_parity_hooks.py -k "rabin or Rabin or config3 or poly" > gpurun_out/${T}_rabin_pytest.log 2>&1
rc=$?; echo "rabin tests"; tail -2 gpurun_out/${T}_rabin_pytest.log; [ $rc -eq 0 ] || exit $rc
WB_ALGOS=rabin timeout -k 10 120 python3 -u tools/walk_bench.py > gpurun_out/${T}_rabin_skew.log 2>&1; rc=$?; echo "rabin skew"; grep -v amdgpu gpurun_out/${T}_rabin_skew.log | tail -3; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS}; do
  CHUNKFS_AMD_LIB=_exp/$v/lib.so WB_ALGOS=rabin timeout -k 10 120 python3 -u tools/walk_bench.py > gpurun_out/${T}_rabin_$v.log 2>&1; rc=$?; echo "rabin $v"; grep -v amdgpu gpurun_out/${T}_rabin_$v.log | tail -3; [ $rc -eq 0 ] || exit $rc
done
