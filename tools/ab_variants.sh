#!/bin/bash
# tools/scan_variants.sh for every _exp build, with the default (DMA) scan and
# with the register-staged scan.  Usage: tools/ab_variants.sh TAG
TAG=${1:-abv}
bash tools/scan_variants.sh ${TAG}_dma || exit $?
CHUNKFS_AMD_DIAG=1024 bash tools/scan_variants.sh ${TAG}_reg || exit $?
bash tools/scan_variants.sh ${TAG}_dma2 || exit $?
CHUNKFS_AMD_DIAG=1024 bash tools/scan_variants.sh ${TAG}_reg2 || exit $?
