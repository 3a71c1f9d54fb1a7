#!/bin/bash
# Kernel trace (timestamps of every dispatch) of a short headline bench run:
# tools/trace_run.sh TAG [bench args] -> gpurun_out/trace_TAG/ (diagnostics).
T=$1; shift
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$T -o run -- \
    python3 bench.py --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 --no-config5 "$@" \
    > gpurun_out/trace_$T.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/trace_$T.log; exit $rc
