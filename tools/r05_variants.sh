# Round-5 probe: experiment builds (_exp/<name>/lib.so): resolve timings (sync and
# diag 128) and pipelined steps per variant.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05v}
for v in ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/diag_resolve.py 0 > gpurun_out/${T}_${v}_d0.log 2>&1; rc=$?
  echo "== $v"; tail -1 gpurun_out/${T}_${v}_d0.log; [ $rc -eq 0 ] || exit $rc
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/diag_resolve.py 128 > gpurun_out/${T}_${v}_d128.log 2>&1; rc=$?
  grep phases gpurun_out/${T}_${v}_d128.log | tail -1; [ $rc -eq 0 ] || exit $rc
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/pipe_probe.py 20 > gpurun_out/${T}_${v}_pipe.log 2>&1; rc=$?
  grep -v amdgpu gpurun_out/${T}_${v}_pipe.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
