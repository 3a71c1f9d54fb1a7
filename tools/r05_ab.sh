# A/B on one box: the shipped build vs experiment builds, interleaved, pipelined steps.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05ab}
for rep in 1 2; do
for v in base ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/pipe_probe.py 20 > gpurun_out/${T}_${v}_$rep.log 2>&1; rc=$?
  echo "== $v ($rep)"; grep -v amdgpu gpurun_out/${T}_${v}_$rep.log | tail -2; [ $rc -eq 0 ] || exit $rc
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/diag_resolve.py 0 2>&1 | tail -1 | cut -c1-90
done
done
