// fastcdc.hpp -- launch interface of the FastCDC pipeline (fastcdc.hip).
//
// Per batch (DESIGN.md "Pipeline and kernels"):
//   scan    -- the HBM pass: candidate records per span (coalesced loads,
//              LDS transpose to per-lane contiguous 1 KiB segments).
//   chain   -- one wave per span: exact links for the span's records, then a
//              speculative chain walk from a warm-up start before the span.
//   fix     -- Jacobi passes over 64-span blocks: spans whose speculative
//              entry differs from their predecessor's exit are re-walked
//              (device-side early exit once converged), then one serial
//              pass that runs only if the Jacobi passes did not converge.
//   compact -- chunk-count prefix and the Chunk{offset,length} output, with
//              first[n+1] and the statistics written to host-coherent memory.
#pragma once
#include "cdc_kernels.hpp"

namespace cdc {
namespace p3 {

struct Chains {
    uint32_t smax;        // start capacity per span
    uint64_t *starts;     // [spans*smax]: chunk starts (stream offsets) inside each span
    uint32_t *nst;        // [spans]: starts in the span
    uint64_t *ent;        // [spans]: first start >= span start (stream length if none)
    uint64_t *ex;         // [spans]: first start >= span end (stream length if none)
    uint64_t *bx[2];      // [blocks of 64 spans]: exit of each block's last span, per pass parity
};

struct Compact {
    uint64_t *bsum;       // [ceil(spans/1024)]: chunk count per 1024-span block
    uint64_t *stats;      // [kStatWords] device accumulators (see kStat*)
    uint64_t *h_stats;    // host-coherent [kStatWords]
    uint64_t *h_first;    // host-coherent [n+1]
};

constexpr int kPasses = 2;        // Jacobi fix passes per batch

// stats words (reset by the scan kernel of the batch)
constexpr int kStatCand = 0;      // candidate records
constexpr int kStatOvf = 1;       // spans whose record list overflowed
constexpr int kStatRewalk = 2;    // spans re-walked by the fix passes
constexpr int kStatError = 3;     // internal error (chain overflow / output bound)
constexpr int kStatSerial = 4;    // 1 if the serial pass had to run
constexpr int kStatFlag0 = 5;     // [5, 5+kPasses): "a block exit changed" in pass p
constexpr int kStatTicket = kStatFlag0 + kPasses;  // write_kernel blocks done
constexpr int kStatDone = kStatTicket + 1;         // host copy only: 1 once written
constexpr int kStatWords = kStatDone + 1;

// d_tails[n_tails]: span ids of the ragged last spans (scanned by their own kernel).
hipError_t launch_scan(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                       const Candidates &cand, const Compact &cp, const uint64_t *d_tails, uint32_t n_tails,
                       int num_cus, hipStream_t s);
hipError_t launch_chain(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                        const Candidates &cand, const Chains &ch, const Compact &cp, hipStream_t s);
hipError_t launch_fix(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                      const Candidates &cand, const Chains &ch, const Compact &cp, hipStream_t s);
hipError_t launch_compact(const StreamTable &st, const Chains &ch, const Compact &cp,
                          void *d_out, uint64_t out_cap, hipStream_t s);

}  // namespace p3
}  // namespace cdc
