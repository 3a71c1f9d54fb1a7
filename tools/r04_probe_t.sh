export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_small.py tests/test_gpu_hostpath.py > gpurun_out/t_t.log 2>&1
rc=$?; tail -3 gpurun_out/t_t.log; [ $rc -eq 0 ] || exit $rc
for cfg in "CHUNKFS_AMD_SMALL_FEED=1" "CHUNKFS_AMD_SMALL_FEED=1 CHUNKFS_AMD_SMALL_FEED_POOL=0" "CHUNKFS_AMD_SMALL_FEED=0" "CHUNKFS_AMD_SMALL_FEED=1"; do
  echo "== $cfg"; env $cfg timeout -k 10 300 python -u tools/hostpath_leg.py 2>&1 | grep -v amdgpu.ids | head -1 | cut -c1-200 || exit 1
done
for g in 0 500; do echo "== gap $g"; timeout -k 10 120 python -u tools/host_probe.py --gap-us $g 1048576 || exit 1; done
