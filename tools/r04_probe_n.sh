export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk.py tests/test_gpu_configs.py > gpurun_out/t_n.log 2>&1
rc=$?; tail -3 gpurun_out/t_n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lowent_lines.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/walk_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
