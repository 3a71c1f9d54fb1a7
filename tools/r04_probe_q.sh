export TMPDIR=/tmp
for g in 0 500; do for pool in 0 1; do echo "== gap $g us, feed pool $pool"; CHUNKFS_AMD_SMALL_FEED_POOL=$pool timeout -k 10 120 python -u tools/host_probe.py --gap-us $g 1048576 1060000 || exit 1; done; done
echo "== gap 500, copy-first (FEED=0)"; CHUNKFS_AMD_SMALL_FEED=0 timeout -k 10 120 python -u tools/host_probe.py --gap-us 500 1048576 || exit 1
