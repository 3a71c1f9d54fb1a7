# Round-5 probe: Rabin bitmap pass variants (persistent blocks, host-built out table):
# Rabin GPU tests through each variant, then rbits kernel time by rocprofv3, interleaved.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05aa}
for v in ${VARIANTS}; do
  CHUNKFS_AMD_LIB=_exp/$v/lib.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py -k rabin > gpurun_out/${T}_pytest_$v.log 2>&1
  rc=$?; echo "pytest $v: $(tail -1 gpurun_out/${T}_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
for v in base ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L WB_ALGOS=rabin timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$rep -o run -- python3 -u tools/walk_bench.py > gpurun_out/${T}_walk_${v}_$rep.log 2>&1; rc=$?
  echo "== $v ($rep) $(grep '^rabin' gpurun_out/${T}_walk_${v}_$rep.log)"; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${T}_prof_${v}_$rep/run_kernel_stats.csv')):
    if 'rbits' in r['Name']: print('rbits', r['Calls'], float(r['AverageNs'])/1000)"
done
done
exit 0
