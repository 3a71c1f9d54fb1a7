# Round-5 probe: scan variant with non-temporal second-half loads -- parity via
# the pipe probe, scan kernel time by rocprofv3 stats, FETCH_SIZE per variant.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05x}
for rep in 1 2; do
for v in base ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$rep -o run -- python3 -u tools/pipe_probe.py 20 > gpurun_out/${T}_${v}_pipe_$rep.log 2>&1; rc=$?
  echo "== $v ($rep)"; grep -v amdgpu gpurun_out/${T}_${v}_pipe_$rep.log | tail -2; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/${T}_prof_${v}_$rep -name "*kernel_stats.csv" | head -1); grep -h "scan_kernel\|resolve_kernel" $f | cut -d, -f1-4 | sed 's/(cdc::StreamTable.*",/",/'
done
done
for v in base ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "p3::.*scan_kernel" --output-format csv -d gpurun_out/${T}_pmc_${v} -o p -- python3 tools/pipe_probe.py 4 > gpurun_out/${T}_pmc_${v}.log 2>&1; rc=$?
  f=$(find gpurun_out/${T}_pmc_${v} -name "*counter_collection.csv" | head -1)
  echo "== FETCH $v rc=$rc"; [ -n "$f" ] && python3 -c "
import csv,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if r['Counter_Name']=='FETCH_SIZE']
print(len(v), sum(v)/len(v)*2048/2**30)"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
