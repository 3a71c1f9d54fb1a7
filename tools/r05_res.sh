# Round-5 probe: resolve variants -- FastCDC parity subset on the shipped build,
# then per variant the block-span stamps (CHUNKFS_AMD_DIAG=64) and pipelined steps.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05r}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base ${VARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/diag_resolve.py 64 > gpurun_out/${T}_${v}_d64_$rep.log 2>&1; rc=$?
  echo "== $v ($rep)"; grep "resolve blocks" gpurun_out/${T}_${v}_d64_$rep.log | tail -2; [ $rc -eq 0 ] || exit $rc
  CHUNKFS_AMD_LIB=$L timeout -k 10 120 python3 -u tools/pipe_probe.py 20 > gpurun_out/${T}_${v}_pipe_$rep.log 2>&1; rc=$?
  grep -v amdgpu gpurun_out/${T}_${v}_pipe_$rep.log | head -1; [ $rc -eq 0 ] || exit $rc
done
done
exit 0
