#!/bin/bash
# Headline ms/step of the driver's command shape (--steps 20 --warmup 5) and
# a longer run, two-stream default vs one stream (diagnostics).
mkdir -p gpurun_out
H="--cpu-seconds 0 --no-host-path --no-sweep --no-algos --no-config4 --no-config5 --no-parity"
T=${1:-r06s}
for rep in 1 2; do
for v in "CHUNKFS_AMD_X=1" "CHUNKFS_AMD_OVERLAP=0"; do
for sw in "20 5" "100 10"; do
  set -- $sw
  f=gpurun_out/${T}_${v##*=}_$1_$rep.json
  env $v timeout -k 10 300 python3 -u bench.py $H --steps $1 --warmup $2 > $f 2> ${f%.json}.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), 'sus', round(d['sustained']['ms_per_step'],4), 'scan', round(d['phase_ms']['scan'],4), 'alone', round(d['phase_ms']['scan_alone'],4))" $f "$v" "$sw"
done; done; done
