// fastcdc.hpp -- launch interface of the FastCDC pipeline (fastcdc.hip).
//
// Per batch (DESIGN.md "Pipeline and kernels"):
//   scan    -- the HBM pass: candidate records per span (coalesced loads,
//              LDS transpose to per-lane contiguous 1 KiB segments).
//   resolve -- units of 16 spans (a team of 4 waves): record links, chain walks from
//              warm-up starts, unit settle, a decoupled look-back over units
//              for the chunk prefix and the unit-boundary check, the
//              Chunk{offset,length} output, first[n+1] and the statistics in
//              host-coherent memory.  Run by the resolve waves of the NEXT
//              batch's scan launch (pipelined batches), or by its own launch.
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

// Look-back descriptors, one per resolve unit.  A status word is
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
constexpr int kStatOrder = 4;     // resolve units claimed (dispatch-order index)
constexpr int kStatOnDemand = 5;  // exact walk steps without a precomputed link
constexpr int kStatTicket = 6;    // resolve blocks done (their statistics stored)
constexpr int kStatDone = 7;      // host copy only: 1 once written
constexpr int kStatDiag0 = 8;     // [8, 16): resolve phase timings (CHUNKFS_AMD_DIAG & 128 only)
constexpr int kStatDiagN = 8;
constexpr int kStatWords = kStatDiag0 + kStatDiagN;

// Everything a resolve worker needs about one batch (fastcdc.hip "resolve").
struct ResArgs {
    StreamTable st;
    Candidates cand;
    Chains ch;
    Compact cp;
    Resolve rs;
    cdc_chunk_pod *out;
    uint64_t out_cap;
    uint64_t units;    // resolve units of the batch (0: nothing to resolve)
    uint64_t *part;    // [resolve_part_words]: per-block statistics, summed by the last block
};

// Resolve units (16 spans each: a team of 4 waves) of a batch of `spans` spans.
uint64_t resolve_units(uint64_t spans);
uint32_t resolve_part_words(int num_cus);

// The scan of a batch (d_tails[n_tails]: span ids of the ragged last spans,
// scanned by their own kernel), fused with the resolve of `prev` (the
// handle's previous batch; prev.units == 0: none).
hipError_t launch_scan(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                       const Candidates &cand, const Compact &cp, const uint64_t *d_tails, uint32_t n_tails,
                       int num_cus, const ResArgs &prev, hipStream_t s);
// The resolve of a batch on its own (the last batch of a burst).
hipError_t launch_resolve(const ResArgs &a, const FastParams &fp, const uint64_t *d_gear, int num_cus,
                          hipStream_t s);

}  // namespace p3
}  // namespace cdc
