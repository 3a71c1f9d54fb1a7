# Round-5 probe: experiment builds (_exp/<name>/lib.so): FastCDC parity subset, then timings.
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARIANTS}; do
  if [ -n "$PARITY" ]; then
    CHUNKFS_AMD_LIB=_exp/$v/lib.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_resolve_paths.py > gpurun_out/r05v_${v}_pytest.log 2>&1
    rc=$?; echo "== $v parity"; tail -2 gpurun_out/r05v_${v}_pytest.log; [ $rc -eq 0 ] || exit $rc
  fi
  CHUNKFS_AMD_LIB=_exp/$v/lib.so timeout -k 10 120 python3 -u tools/diag_resolve.py ${DIAG:-2048} > gpurun_out/r05v_$v.log 2>&1; rc=$?; echo "== $v"; tail -2 gpurun_out/r05v_$v.log; [ $rc -eq 0 ] || exit $rc
done
