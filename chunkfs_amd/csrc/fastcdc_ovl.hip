// fastcdc_ovl.hip -- the FastCDC kernels of fastcdc.hip built a second time,
// at the sizes that let a batch's resolve run beside the next batch's scan on
// every CU (namespace p3::ovl, fastcdc.hpp; Engine::fast_submit).
//
//   scan:    8 waves per CU (2 per SIMD), VGPRs capped at 128 (512 / 4; the
//            cap needs the LDS tile to be dynamic, otherwise the compiler sizes
//            registers for the occupancy its static LDS allows), 112 KiB LDS.
//   resolve: 4 waves per block (1 per SIMD, <= 256 VGPRs), 384 window records
//            per wave: 46 KiB of LDS, 32 spans per block.
// Per CU: 2 x 128 + 1 x 240 VGPRs per SIMD lane <= 512, 112 + 46 KiB <= 160 KiB.
#define CDC_OVL 1
#define CDC_SCAN_WAVES 8
#define CDC_SCAN_DYN 1
#define CDC_SCAN_MAXW 4
#define CDC_RES_WAVES 4
#define CDC_WIN_RECS 384
#include "fastcdc.hip"
