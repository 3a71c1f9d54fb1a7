export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_small.py tests/test_gpu_hostpath.py tests/test_gpu_parity.py > gpurun_out/t_u.log 2>&1
rc=$?; tail -3 gpurun_out/t_u.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/small_stamps.py 1048576 2>&1 | grep -v amdgpu.ids | tail -6 || exit 1
for i in 1 2; do timeout -k 10 300 python -u tools/hostpath_leg.py 2>&1 | grep -v amdgpu.ids | head -1 | cut -c1-200 || exit 1; done
