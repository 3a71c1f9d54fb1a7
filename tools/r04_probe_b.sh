export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_small.py tests/test_gpu_parity_hooks.py tests/test_gpu_hostpath.py > gpurun_out/t_small.log 2>&1
rc=$?; tail -5 gpurun_out/t_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/small_stamps.py 1048576 1060000 4194304 || exit 1
for v in "" "CHUNKFS_AMD_SMALL_ZC=0" "CHUNKFS_AMD_SMALL=0"; do echo "== $v"; env $v timeout -k 10 120 python -u tools/host_probe.py 1048576 1060000 4194304 || exit 1; done
