# Round-5 evidence run (one gpurun call): every -m gpu test, the bench line, a
# rocprofv3 kernel-stats pass of the bench's timed config, then the scan's PMC
# passes (tools/pmc.sh).  Stops at the first failure.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r05}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/${T}_bench.json').read().splitlines()[-1]); print(json.dumps(d['summary'])[:1500]); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-host-path --no-sweep --no-algos --no-config4 --no-config5 \
    > gpurun_out/prof_${T}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "$PMC" ] && bash tools/pmc.sh $T
exit 0
