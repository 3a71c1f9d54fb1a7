# Round-5 probe: Rabin bitmap pass variants (parity, then interleaved timing) and
# scan wave-count variants of the wave-major scan.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05p}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py -k "rabin" > gpurun_out/${T}_pytest_walk.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest_walk.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base ${WVARIANTS}; do
  L=_exp/$v/lib.so; [ "$v" = base ] && L=chunkfs_amd/libchunkfs_amd.so
  CHUNKFS_AMD_LIB=$L WB_ALGOS=rabin timeout -k 10 120 python3 -u tools/walk_bench.py > gpurun_out/${T}_walk_${v}_$rep.log 2>&1; rc=$?
  echo "== walk $v ($rep)"; grep -v amdgpu gpurun_out/${T}_walk_${v}_$rep.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
done
[ -n "$VARIANTS" ] && TAG=$T bash tools/r05_ab.sh
exit 0
