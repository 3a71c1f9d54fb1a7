// sha256.hpp -- launch interface of the per-chunk SHA-256 kernel (sha256.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cdc_kernels.hpp"

namespace cdc {

// A batch: the chunks of n_streams streams, stream i's chunks at
// chunks[first[i] .. first[i+1]) with offsets relative to base[i] (DEVICE
// arrays).  digests[8*k .. 8*k+8) (u32, big-endian bytes) = SHA-256 of chunk
// k.  counter / order: device scratch (work distribution, claim order).
struct ShaBatch {
    const cdc_chunk_pod *chunks;
    uint64_t n_chunks;
    const uint64_t *first;  // [n_streams + 1]
    const uint64_t *base;   // [n_streams]: stream base addresses (4-byte aligned)
    uint32_t n_streams;
    uint32_t *digests;
    unsigned long long *counter;  // [1 + kShaBuckets] device scratch: work counter, length histogram
    uint32_t *order;              // [n_chunks] device scratch: chunk indices, longest first
};

constexpr uint32_t kShaBuckets = 256;  // length classes of the longest-first claim order

hipError_t launch_sha256(const ShaBatch &b, int num_cus, hipStream_t s);

}  // namespace cdc
