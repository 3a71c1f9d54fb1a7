export TMPDIR=/tmp
timeout -k 10 120 python -u tools/small_stamps.py 1048576 2>&1 | grep -v amdgpu.ids || exit 1
