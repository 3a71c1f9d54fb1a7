#!/bin/bash
# Final evidence of a round (one gpurun call): every -m gpu test, smoke(), the
# default bench line, one rocprofv3 kernel-trace pass over a full bench run
# (every timed leg: FastCDC scan/resolve, the walk kernels, SHA-256 and the
# index of config 3, the host path), then the PMC passes: the scan's
# (tools/pmc.sh: traffic JSON for this digest) and SHA-256's VALU counters.
# Stops at the first failing step.  Usage: tools/evidence.sh TAG
T=${1:-r06}
mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu.sh tests $T || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash tools/gpu.sh bench $T || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_${T}.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "rocprof ok"
# the roofline kernel alone: one stream, so every scan dispatch has the chip to
# itself and rocprofv3's scan_kernel average is the bench's roofline.kernel_ms
CHUNKFS_AMD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_alone \
    -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 \
    --no-config5 > gpurun_out/prof_${T}_alone.log 2>&1 || { echo "rocprof alone rc=$?"; exit 1; }
echo "rocprof alone ok"
[ -n "$NO_PMC" ] && exit 0
bash tools/pmc.sh $T > gpurun_out/pmc_${T}.txt 2>&1 || { echo "pmc rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --kernel-include-regex sha256_kernel --output-format csv -d gpurun_out/pmc_${T}_sha -o p -- python3 tools/leg.py config3 \
    > gpurun_out/pmc_${T}_sha.log 2>&1 || { echo "pmc sha rc=$?"; exit 1; }
echo "evidence done"
