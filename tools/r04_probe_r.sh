export TMPDIR=/tmp
timeout -k 10 300 python -u tools/hostpath_leg.py 2>&1 | grep -v amdgpu.ids || exit 1
CHUNKFS_AMD_SMALL_FEED=0 timeout -k 10 300 python -u tools/hostpath_leg.py 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
