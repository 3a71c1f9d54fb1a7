#!/bin/bash
# One parameterised driver for GPU-box runs (via gpurun), replacing the
# one-off per-round probe scripts.  Every step has its own time limit, and the
# script stops at the first failing step.
#   tools/gpu.sh tests TAG [pytest args]      -m gpu tests -> gpurun_out/TAG_pytest.log
#   tools/gpu.sh bench TAG [bench args]       bench line   -> gpurun_out/TAG_bench.json
#   tools/gpu.sh ab TAG REPS "ENV1" "ENV2"... headline-only bench per env setting, interleaved
#   tools/gpu.sh prof TAG [bench args]        rocprofv3 --kernel-trace --stats of a bench run
#   tools/gpu.sh pmc TAG                      scan PMC passes (tools/pmc.sh)
mkdir -p gpurun_out && export TMPDIR=/tmp
cmd=$1; T=$2; shift 2
HEAD="--cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 --no-config5"
case $cmd in
tests)
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${T}_pytest.log; exit $rc ;;
bench)
  timeout -k 10 900 python3 -u bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${T}_bench.err
  [ $rc -eq 0 ] && python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().splitlines()[-1]); print(json.dumps(d['summary']))"
  exit $rc ;;
ab)
  REPS=$1; shift
  for rep in $(seq 1 $REPS); do
    i=0
    for e in "$@"; do
      i=$((i+1))
      env $e timeout -k 10 300 python3 -u bench.py $HEAD > gpurun_out/${T}_v${i}_$rep.json 2> gpurun_out/${T}_v${i}_$rep.err
      rc=$?; [ $rc -eq 0 ] || { echo "variant $i ($e) rc=$rc"; tail -5 gpurun_out/${T}_v${i}_$rep.err; exit $rc; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${T}_v${i}_$rep.json').read().splitlines()[-1]); s=d['summary']; print('$i [$e] rep $rep:', round(d['value'],1), 'GiB/s', round(d['ms_per_step'],4), 'ms/step scan', round(d['phase_ms']['scan'],4), 'alone', round(d['phase_ms'].get('scan_alone') or 0,4), 'res', round(d['phase_ms']['resolve'],4), 'sus', round(s['sustained_ms_per_step'] or 0,4), 'lat', round(s['sync_latency_ms'] or 0,4), 'par', d.get('parity_vs_oracle'))"
    done
  done ;;
prof)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- \
      python3 bench.py "$@" > gpurun_out/prof_${T}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_${T}.log; exit $rc ;;
pmc)
  bash tools/pmc.sh $T ;;
*) echo "usage: tools/gpu.sh tests|bench|ab|prof|pmc TAG ..."; exit 2 ;;
esac
