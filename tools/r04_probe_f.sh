export TMPDIR=/tmp
timeout -k 10 120 python -u tools/small_stamps.py 1048576 1060000 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python -u tools/host_probe.py 1048576 1060000 4194304 || exit 1
