// cdc_kernels.hpp -- types shared by the gfx950 chunking kernels, and the
// fixed-size / input-generator launchers (util_kernels.hip).  The FastCDC
// pipeline's launchers are in fastcdc.hpp.
//
// Data layout in HBM (DESIGN.md "Data layout"):
//   * streams: caller-owned device buffers, 16-byte aligned, read once by the
//     scan (the only HBM-bound kernel).
//   * spans: every stream is cut into SPAN = 2^span_log2 byte spans; span g of
//     the batch belongs to stream i with span_base[i] <= g < span_base[i+1].
//   * candidates: per span, count[g] and up to `cap` u32 records
//     pos[g*cap+k] (offset in span | exact hit flags), in position order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdc {

// Same layout as cdc_chunk_t (include/chunkfs_amd.h).
struct cdc_chunk_pod {
    uint64_t offset;
    uint64_t length;
};

struct StreamTable {
    const uint8_t *const *ptrs;  // device array [n] of device pointers
    const uint64_t *lens;        // device [n]
    const uint64_t *span_base;   // device [n+1]
    uint32_t n;
    uint32_t span_log2;
    uint64_t total_spans;
};

struct FastParams {
    uint32_t min, avg, max;
    uint32_t trunc;          // positions after chunk_start+min whose in-chunk hash differs from the windowed hash
    uint64_t mask_s, mask_l; // Level1 masks
    uint64_t cmask;          // mask_s & mask_l: candidate predicate (superset of both)
    // Candidate test forms.  Aligned (cm_align): mask_s|mask_l fits in the
    // 32-bit window [w, w+32), w = ctz(mask_s|mask_l).  The scan then tracks
    // every hash pre-shifted, h' = h << tshift with tshift = 32 - w (GEAR
    // pre-shifted the same way), so the window is exactly the high dword of
    // h' and the test is one v_and_b32 -- no v_alignbit (half rate on gfx950).
    // General form: unshifted, (lo & cm_lo) | (hi & cm_hi).
    uint32_t cm_align;       // 1 = aligned form usable
    uint32_t tshift;         // scan pre-shift of every hash (0 in the general form)
    uint32_t cm32;           // aligned: (cmask << tshift) >> 32
    uint32_t cm_lo, cm_hi;   // general form
    uint64_t mask_s_sh, mask_l_sh;  // mask_s / mask_l << tshift (exact flush tests)
    uint32_t diag;           // test hooks / timing experiments (CHUNKFS_AMD_DIAG); 0 in every real run
};

struct Candidates {
    uint32_t cap;
    uint32_t *count;  // [spans]: candidates found (> cap = overflowed)
    uint32_t *pos;    // [spans*cap]: offset in span (bits 0-23) | bit30 mask_l hit | bit31 mask_s hit
};

hipError_t launch_fixed(const StreamTable &st, uint64_t chunk_size, const uint64_t *d_first, void *d_out,
                        uint64_t total, hipStream_t s);
hipError_t launch_fill_splitmix64(uint8_t *d_buf, uint64_t len, uint64_t seed, hipStream_t s);
// Read-only XOR reduction of len bytes (16-byte multiple used): one word per
// block into d_out[num_cus * 8] (zeroed by the caller).
hipError_t launch_read_reduce(const uint8_t *d_buf, uint64_t len, uint64_t *d_out, int num_cus, hipStream_t s);

}  // namespace cdc
