export TMPDIR=/tmp
timeout -k 10 120 python -u tools/small_stamps.py 1048576 1060000 4194304 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o run -- python3 tools/host_probe.py 1048576 1060000 4194304 > gpurun_out/prof_small.log 2>&1
rc=$?; tail -5 gpurun_out/prof_small.log; exit $rc
