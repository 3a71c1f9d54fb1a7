#!/bin/bash
# Runs on the GPU box: scan / resolve timing experiments over one 1 GiB stream
# (CHUNKFS_AMD_DIAG modes, see fastcdc.hip).  Diagnostics only.
TAG=${1:-exp}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for D in ${DIAGS:-0 256 512 128 0}; do
    echo "== DIAG=$D" >> $OUT/exp_$TAG.log
    timeout -k 10 120 python -u tools/diag_resolve.py $D >> $OUT/exp_$TAG.log 2>&1
    rc=$?; echo "DIAG=$D rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
cat $OUT/exp_$TAG.log
