export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_small.py tests/test_gpu_hostpath.py > gpurun_out/t_m.log 2>&1
rc=$?; tail -3 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/small_stamps.py 1048576 2>&1 | grep -v amdgpu.ids || exit 1
for v in 1 0 1 0; do echo "== CHUNKFS_AMD_SMALL_FEED=$v"; CHUNKFS_AMD_SMALL_FEED=$v timeout -k 10 120 python -u tools/host_probe.py 1048576 1060000 || exit 1; done
