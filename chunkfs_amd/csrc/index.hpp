// index.hpp -- device dedup index (index.hip) and its host object.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cdc_kernels.hpp"

namespace cdc {

constexpr uint64_t kIndexPendingCap = 4096;  // 64-bit key collisions handled per batch

struct IndexTable {
    uint64_t slots;    // power of two
    uint64_t *tag;     // [slots] 0 = empty, else the digest's first 8 bytes | 1
    uint8_t *digest;   // [slots * 32]
    uint64_t *owner;   // [slots] global index of the first chunk with this key (~0 = none)
    uint64_t *length;  // [slots] that chunk's length
};

// Database::insert for chunks [0, n) of a batch whose first chunk has global
// index `base`.  d_acc[0..4] += new digests, their bytes, bytes written,
// chunks that did not fit, 64-bit key collisions seen.  d_new (nullable)
// receives 1 for first occurrences.  Scratch: d_slot_of (n u32), d_pending
// (kIndexPendingCap u32).
hipError_t launch_index_insert(const IndexTable &t, const uint8_t *d_digests, const void *d_chunks,
                               uint64_t n, uint64_t base, uint32_t *d_slot_of, uint32_t *d_pending,
                               uint8_t *d_new, unsigned long long *d_acc, hipStream_t s);

}  // namespace cdc
