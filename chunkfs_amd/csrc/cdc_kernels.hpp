// cdc_kernels.hpp -- launch interface of the gfx950 chunking kernels.
//
// Data layout in HBM (DESIGN.md "Layout"):
//   * streams: caller-owned device buffers, 16-byte aligned, read exactly once
//     by the scan kernel (the only HBM-bound kernel).
//   * spans: every stream is cut into SPAN = 2^span_log2 byte spans; span g of
//     the batch belongs to stream i with span_base[i] <= g < span_base[i+1].
//     A span is both the scan unit (one wavefront) and the resolve segment
//     (one thread).
//   * candidates: per span, cand_count[g] and up to `cap` records
//     (cand_pos[g*cap+k] = offset in span, u32; cand_hash[g*cap+k] = windowed
//     gear hash, bits 0..47 exact), in increasing position order.
//   * chains: per span two ping-pong lists of chunk starts (starts[b][g*smax+k],
//     u64 stream offsets), nstarts[b][g], which[g] selects the live one,
//     entry[g], exit[2][g].
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
};

struct Candidates {
    uint32_t cap;
    uint32_t *count;  // [spans]: candidates found (> cap = overflowed)
    uint32_t *pos;    // [spans*cap]: offset in span (bits 0-23) | truncated result (24-29) | bit30 mask_l hit | bit31 mask_s hit
};

struct Chains {
    uint32_t smax;
    uint64_t *starts[2];   // [spans*smax]
    uint32_t *nstarts[2];  // [spans]
    uint8_t *which;        // [spans]
    uint64_t *entry;       // [spans]
    uint64_t *exit[2];     // [spans]
    uint32_t *changed;     // [3]: rotating "some exit changed" flags of the Jacobi passes
};

struct Compact {
    uint64_t *chunk_index;   // [spans+1]
    uint64_t *block_sums;    // [ceil(spans/1024)+1]
    uint64_t *stats;         // [4]: candidates, overflow spans, Jacobi passes run, serial used
    uint64_t *first;         // [n+1]
};

hipError_t launch_scan(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       int num_cus, hipStream_t s);
hipError_t launch_trunc(const StreamTable &st, const FastParams &fp,
                        const uint64_t *d_gear, const Candidates &cand, hipStream_t s);
hipError_t launch_spec(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       const Chains &ch, uint64_t *stats, hipStream_t s);
hipError_t launch_fixup(const StreamTable &st, const FastParams &fp,
                        const uint64_t *d_gear, const Candidates &cand,
                        const Chains &ch, int iter, uint64_t *stats, hipStream_t s);
hipError_t launch_serial(const StreamTable &st, const FastParams &fp,
                         const uint64_t *d_gear, const Candidates &cand,
                         const Chains &ch, int buf, int slot, uint64_t *stats,
                         hipStream_t s);
hipError_t launch_compact(const StreamTable &st, const Chains &ch,
                          int exit_buf, const Candidates &cand,
                          const Compact &cp, void *d_out, hipStream_t s);
hipError_t launch_fixed(const StreamTable &st, uint64_t chunk_size,
                        const uint64_t *d_first, void *d_out, uint64_t total,
                        hipStream_t s);
hipError_t launch_fill_splitmix64(uint8_t *d_buf, uint64_t len, uint64_t seed,
                                  hipStream_t s);

}  // namespace cdc
