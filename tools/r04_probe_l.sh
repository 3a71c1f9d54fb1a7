export TMPDIR=/tmp
for v in 1 2 0 1 2 0; do echo "== CHUNKFS_AMD_SMALL_FEED=$v"; CHUNKFS_AMD_SMALL_FEED=$v timeout -k 10 120 python -u tools/host_probe.py 1048576 || exit 1; done
for t in 1 2 8; do echo "== COPY_THREADS=$t"; CHUNKFS_AMD_COPY_THREADS=$t timeout -k 10 120 python -u tools/host_probe.py 1048576 || exit 1; done
