# Round-5 probe: FastCDC parity subset + async tests, resolve timings, pipelined steps.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r05}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py tests/test_gpu_async.py > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for d in ${DIAGS:-0 128}; do
  timeout -k 10 120 python3 -u tools/diag_resolve.py $d > gpurun_out/${T}_d$d.log 2>&1; rc=$?; echo "DIAG $d"; tail -2 gpurun_out/${T}_d$d.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 180 python3 -u tools/pipe_probe.py 20 > gpurun_out/${T}_pipe.log 2>&1; rc=$?; cat gpurun_out/${T}_pipe.log | grep -v amdgpu.ids; exit $rc
