# Round-5 probe: rbits_kernel variants timed by rocprofv3 kernel stats (walk_bench,
# Rabin only), interleaved; then the resolve's block-span stamps (CHUNKFS_AMD_DIAG=64).
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05q}
for rep in 1 2; do
for v in base ${WVARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L WB_ALGOS=rabin timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$rep -o run -- python3 -u tools/walk_bench.py > gpurun_out/${T}_walk_${v}_$rep.log 2>&1; rc=$?
  echo "== walk $v ($rep)"; grep -v amdgpu gpurun_out/${T}_walk_${v}_$rep.log | grep rabin | tail -1; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/${T}_prof_${v}_$rep -name "*kernel_stats.csv" | head -1); grep -h "rbits\|wwalk" $f | cut -d, -f1-4
done
done
CHUNKFS_AMD_DIAG=64 timeout -k 10 120 python3 -u tools/diag_resolve.py 64 > gpurun_out/${T}_d64.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/${T}_d64.log | tail -6
exit $rc
