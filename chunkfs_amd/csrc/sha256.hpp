// sha256.hpp -- launch interface of the per-chunk SHA-256 kernel (sha256.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cdc_kernels.hpp"

namespace cdc {

// digests[32*i .. 32*i+32) = SHA-256(d_data[chunks[i].offset .. +length)).
// d_counter: one device u64 of scratch (work distribution).
hipError_t launch_sha256(const uint8_t *d_data, const void *d_chunks, uint64_t n_chunks,
                         uint8_t *d_digests, unsigned long long *d_counter, int num_cus,
                         hipStream_t s);

}  // namespace cdc
