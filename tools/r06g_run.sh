mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu.sh tests r06g || exit 1
for v in c2 c4; do timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_r06g_$v -o run -- python3 tools/c4_probe.py $v 6 > gpurun_out/pmc_r06g_$v.log 2>&1 || exit 1; done
echo done
