# Rabin bitmap pass with two chains per lane (variant build _exp/rabin2):
# its Rabin parity tests through that library, then timing against the shipped build.
export TMPDIR=/tmp
CHUNKFS_AMD_LIB=_exp/rabin2/lib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk.py tests/test_gpu_configs.py -k "rabin" > gpurun_out/t_z.log 2>&1
rc=$?; tail -2 gpurun_out/t_z.log; [ $rc -eq 0 ] || exit $rc
TESTK=rabin WB_ALGOS=rabin bash tools/r04_probe_y.sh rabin2
