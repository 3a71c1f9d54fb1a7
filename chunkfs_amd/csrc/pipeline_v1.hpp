// pipeline_v1.hpp -- launch interface of the round-1 validated pipeline
// (pipeline_v1.hip).  Shares StreamTable / FastParams / Candidates with the
// newer pipeline (cdc_kernels.hpp); its own chain and compaction state.
#pragma once
#include "cdc_kernels.hpp"

namespace cdc {
namespace v1 {

struct Chains {
    uint32_t smax;
    uint64_t *starts[2];   // [spans*smax] ping-pong lists of chunk starts
    uint32_t *nstarts[2];  // [spans]
    uint8_t *which;        // [spans] live list
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

constexpr int kJacobi = 3;  // device-side Jacobi passes per batch

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

}  // namespace v1
}  // namespace cdc
