export TMPDIR=/tmp
for v in 1 0; do echo "== CHUNKFS_AMD_SMALL_FEED=$v"; CHUNKFS_AMD_SMALL_FEED=$v timeout -k 10 120 python -u tools/host_probe.py 1048576 1060000 4194304 || exit 1; done
for sp in 0 1000; do echo "== COPY_SPIN_US=$sp"; CHUNKFS_AMD_COPY_SPIN_US=$sp timeout -k 10 120 python -u tools/host_probe.py 1048576 || exit 1; done
