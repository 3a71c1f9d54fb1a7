# Per-call latency of the 1 MiB host path against the copy pool's thread count.
export TMPDIR=/tmp
for r in 1 2; do
for t in 2 4 6 8 12; do
  echo -n "threads $t: "
  CHUNKFS_AMD_COPY_THREADS=$t timeout -k 10 60 python3 tools/host_probe.py 1048576 2>&1 | grep "n=" || exit 1
done
done
