# Round-5 probe: Rabin bitmap pass with non-temporal second-half loads -- Rabin
# GPU tests through the variant, rbits kernel time (rocprofv3) and FETCH_SIZE.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05y}
CHUNKFS_AMD_LIB=_exp/rnt/lib.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py -k rabin > gpurun_out/${T}_pytest_rnt.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_pytest_rnt.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base rnt; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L WB_ALGOS=rabin timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$rep -o run -- python3 -u tools/walk_bench.py > gpurun_out/${T}_walk_${v}_$rep.log 2>&1; rc=$?
  echo "== $v ($rep)"; grep "^rabin" gpurun_out/${T}_walk_${v}_$rep.log; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${T}_prof_${v}_$rep/run_kernel_stats.csv')):
    if 'rbits' in r['Name']: print('rbits', r['Calls'], float(r['AverageNs'])/1000)"
done
done
for v in base rnt; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L WB_ALGOS=rabin timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rbits_kernel" --output-format csv -d gpurun_out/${T}_pmc_${v} -o p -- python3 tools/walk_bench.py > gpurun_out/${T}_pmc_${v}.log 2>&1; rc=$?
  f=$(find gpurun_out/${T}_pmc_${v} -name "*counter_collection.csv" | head -1)
  echo "== FETCH $v rc=$rc"; [ -n "$f" ] && python3 -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if r['Counter_Name']=='FETCH_SIZE']
print(len(v), 'raw x1024', sum(v)/len(v)*1024/2**30, 'x2', sum(v)/len(v)*2048/2**30)"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
