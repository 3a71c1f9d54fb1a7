// fastcdc.hpp -- launch interface of the FastCDC pipeline (fastcdc.hip).
//
// Per batch (DESIGN.md "Pipeline and kernels"):
//   scan    -- the HBM pass: candidate records per span (coalesced loads,
//              LDS transpose to per-lane contiguous 1 KiB segments).
//   resolve -- one launch: record links, chain walks from warm-up starts,
//              block settle, a decoupled look-back over blocks for the chunk
//              prefix and the block-boundary check, the Chunk{offset,length}
//              output, first[n+1] and the statistics in host-coherent memory.
#pragma once
#include "cdc_kernels.hpp"

namespace cdc {
namespace p3 {

struct Chains {
    uint32_t smax;        // start capacity per span
    uint64_t *starts;     // [spans*smax]: chunk starts (stream offsets) inside each span
};

struct Compact {
    uint64_t *stats;      // [kStatWords] device accumulators (see kStat*)
    uint64_t *h_stats;    // host-coherent [kStatWords]
    uint64_t *h_first;    // host-coherent [n+1]
};

// Look-back descriptors, one per resolve block.  A status word is
// gen << 2 | 1 (aggregate) or 2 (inclusive, final); it is valid only for the
// batch of generation gen, so the arrays are never re-zeroed.
struct Resolve {
    uint64_t *dstat;      // status word
    uint64_t *dagg;       // chunk count of the block (aggregate)
    uint64_t *dinc;       // chunk count up to and including the block (inclusive)
    uint64_t *dE;         // entry of the block's first span (~0: it starts a stream)
    uint64_t *dXa;        // exit of the block's last span, as aggregated
    uint64_t *dXi;        // the same, final
    uint64_t gen;
};

// stats words (reset by the scan kernel of the batch)
constexpr int kStatCand = 0;      // candidate records
constexpr int kStatOvf = 1;       // spans whose record list overflowed
constexpr int kStatRewalk = 2;    // spans re-walked after the speculative walk
constexpr int kStatError = 3;     // internal error (chain overflow / output bound / look-back timeout)
constexpr int kStatOrder = 4;     // resolve blocks started (dispatch-order index)
constexpr int kStatOnDemand = 5;  // exact walk steps without a precomputed link
constexpr int kStatTicket = 6;    // resolve blocks done
constexpr int kStatDone = 7;      // host copy only: 1 once written
constexpr int kStatDiag0 = 8;     // [8, 16): resolve phase timings (CHUNKFS_AMD_DIAG & 128 only)
constexpr int kStatDiagN = 8;
constexpr int kStatWords = kStatDiag0 + kStatDiagN;

uint64_t resolve_blocks(uint64_t spans);

// d_tails[n_tails]: span ids of the ragged last spans (scanned by their own kernel).
hipError_t launch_scan(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                       const Candidates &cand, const Compact &cp, const uint64_t *d_tails, uint32_t n_tails,
                       int num_cus, hipStream_t s);
hipError_t launch_resolve(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                          const Candidates &cand, const Chains &ch, const Compact &cp, const Resolve &rs,
                          void *d_out, uint64_t out_cap, hipStream_t s);

// The overlap set (fastcdc_ovl.hip: the same kernels at other sizes) for
// back-to-back batches whose resolve runs on a second stream beside the next
// batch's scan: the scan at 8 waves per CU, <= 128 VGPRs and 112 KiB of LDS
// leaves each CU room for one 4-wave resolve block (<= 256 VGPRs per lane,
// 46 KiB of LDS, 32 spans per block).
namespace ovl {
uint64_t resolve_blocks(uint64_t spans);
hipError_t launch_scan(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                       const Candidates &cand, const Compact &cp, const uint64_t *d_tails, uint32_t n_tails,
                       int num_cus, hipStream_t s);
hipError_t launch_resolve(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                          const Candidates &cand, const Chains &ch, const Compact &cp, const Resolve &rs,
                          void *d_out, uint64_t out_cap, hipStream_t s);
}  // namespace ovl

}  // namespace p3
}  // namespace cdc
