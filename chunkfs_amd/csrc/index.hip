// index.hip -- device dedup index over SHA-256 chunk fingerprints.
//
// Mirrors the reference's chunk Database (src/system/database.rs:74-87,
// HashMap with `entry(key).or_insert(value)`: the FIRST insert of a key wins)
// and the storage statistics built on it (src/system/storage.rs:193-231:
// size_written, total_cdc_size, cdc_dedup_ratio, average_chunk_size).
// SURVEY.md §8f row 3.
//
// Layout in HBM: open addressing with linear probing over C = 2^k slots
// (capacity rounded up to twice the requested unique count, so the load
// factor stays <= 1/2).  Per slot: a 64-bit key (the digest's first 8 bytes,
// bit 0 forced to 1 so a key is never 0), the full 32-byte digest, the chunk
// length, and the global index of the first chunk that carried the digest
// (atomicMin: the reference's sequential first insert).  Thread per chunk:
// claim/find by key, confirm the full digest after a kernel boundary (no
// thread ever spins on another), a serial pass for 64-bit key collisions,
// then per-chunk first-occurrence flags and totals.
#include "index.hpp"

namespace cdc {
namespace {

constexpr int kIxThreads = 256;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

__device__ __forceinline__ bool same_digest(const uint8_t *a, const uint8_t *b) {
    const uint4 *x = reinterpret_cast<const uint4 *>(a), *y = reinterpret_cast<const uint4 *>(b);
    const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
    return x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w &&
           x1.x == y1.x && x1.y == y1.y && x1.z == y1.z && x1.w == y1.w;
}

__device__ __forceinline__ uint64_t key_of(const uint8_t *d) {
    const uint2 w = *reinterpret_cast<const uint2 *>(d);
    return (((uint64_t)w.y << 32) | w.x) | 1ull;  // never 0 (0 = empty slot)
}

// Pass 1: claim or find the slot of each chunk's 64-bit key.  The claimer
// stores the full digest; no thread ever waits on another (no spin inside a
// wavefront), the full comparison happens in pass 2 after the kernel boundary.
__global__ __launch_bounds__(kIxThreads) void claim_kernel(IndexTable t, const uint8_t *__restrict__ digests,
                                                           uint64_t n, uint32_t *slot_of) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *d = digests + 32 * i;
    const uint64_t key = key_of(d);
    const uint64_t mask = t.slots - 1;
    uint64_t s = (key >> 1) & mask;
    for (uint64_t probe = 0; probe < t.slots; ++probe, s = (s + 1) & mask) {
        uint64_t cur = t.tag[s];
        if (cur == 0) {
            cur = atomicCAS((unsigned long long *)&t.tag[s], 0ull, (unsigned long long)key);
            if (cur == 0) {
                uint4 *dst = reinterpret_cast<uint4 *>(t.digest + 32 * s);
                const uint4 *src = reinterpret_cast<const uint4 *>(d);
                dst[0] = src[0];
                dst[1] = src[1];
                slot_of[i] = (uint32_t)s;
                return;
            }
        }
        if (cur == key) {
            slot_of[i] = (uint32_t)s;
            return;
        }
    }
    slot_of[i] = kNoSlot;
}

// Pass 2: confirm the full digest; record the first chunk of each key
// (atomicMin of the global chunk index); queue the rare 64-bit key collisions
// with a different digest for the serial pass.
__global__ __launch_bounds__(kIxThreads) void verify_kernel(IndexTable t, const uint8_t *__restrict__ digests,
                                                            uint64_t n, uint64_t base, uint32_t *slot_of,
                                                            uint32_t *pending, unsigned long long *acc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    if (s == kNoSlot) return;
    if (same_digest(t.digest + 32ull * s, digests + 32 * i)) {
        atomicMin((unsigned long long *)&t.owner[s], (unsigned long long)(base + i));
    } else {
        const unsigned long long k = atomicAdd(&acc[4], 1ull);
        if (k < kIndexPendingCap) pending[k] = (uint32_t)i;
        slot_of[i] = kNoSlot;
    }
}

// Pass 3 (one thread, normally no work): exact probing with full digest
// comparison for the queued chunks, in chunk order.
__global__ void serial_kernel(IndexTable t, const uint8_t *__restrict__ digests, uint64_t base,
                              uint32_t *slot_of, uint32_t *pending, const unsigned long long *acc) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const uint64_t np = acc[4] < kIndexPendingCap ? acc[4] : kIndexPendingCap;
    for (uint64_t k = 0; k < np; ++k) {  // pending order is arbitrary: take them by index
        uint64_t best = ~0ull, bk = 0;
        for (uint64_t j = 0; j < np; ++j)
            if (pending[j] != kNoSlot && pending[j] < best) {
                best = pending[j];
                bk = j;
            }
        const uint64_t i = best;
        pending[bk] = kNoSlot;
        const uint8_t *d = digests + 32 * i;
        const uint64_t key = key_of(d);
        const uint64_t mask = t.slots - 1;
        uint64_t s = (key >> 1) & mask;
        for (uint64_t probe = 0; probe < t.slots; ++probe, s = (s + 1) & mask) {
            if (t.tag[s] == 0) {
                t.tag[s] = key;
                uint4 *dst = reinterpret_cast<uint4 *>(t.digest + 32 * s);
                const uint4 *src = reinterpret_cast<const uint4 *>(d);
                dst[0] = src[0];
                dst[1] = src[1];
                t.owner[s] = base + i;
                slot_of[i] = (uint32_t)s;
                break;
            }
            if (t.tag[s] == key && same_digest(t.digest + 32 * s, d)) {
                if (base + i < t.owner[s]) t.owner[s] = base + i;
                slot_of[i] = (uint32_t)s;
                break;
            }
        }
    }
}

// Pass 4: first occurrences (the reference's first insert wins) and totals.
__global__ __launch_bounds__(kIxThreads) void mark_kernel(IndexTable t, const cdc_chunk_pod *__restrict__ chunks,
                                                          uint64_t n, uint64_t base, const uint32_t *slot_of,
                                                          uint8_t *is_new, unsigned long long *acc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t nb = 0, nc = 0, wb = 0, full = 0;
    if (i < n) {
        const uint32_t s = slot_of[i];
        const uint64_t len = chunks[i].length;
        wb = len;
        bool fresh = false;
        if (s == kNoSlot) {
            full = 1;
        } else {
            fresh = t.owner[s] == base + i;
            if (fresh) t.length[s] = len;
        }
        if (is_new) is_new[i] = fresh ? 1 : 0;
        nc = fresh;
        nb = fresh ? len : 0;
    }
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {  // one atomic per wave per counter
        nb += __shfl_xor(nb, k);
        nc += __shfl_xor(nc, k);
        wb += __shfl_xor(wb, k);
        full += __shfl_xor(full, k);
    }
    if ((threadIdx.x & 63) == 0) {
        if (nc) atomicAdd(&acc[0], (unsigned long long)nc);
        if (nb) atomicAdd(&acc[1], (unsigned long long)nb);
        if (wb) atomicAdd(&acc[2], (unsigned long long)wb);
        if (full) atomicAdd(&acc[3], (unsigned long long)full);
    }
}

}  // namespace

hipError_t launch_index_insert(const IndexTable &t, const uint8_t *d_digests, const void *d_chunks,
                               uint64_t n, uint64_t base, uint32_t *d_slot_of, uint32_t *d_pending,
                               uint8_t *d_new, unsigned long long *d_acc, hipStream_t s) {
    if (!n) return hipSuccess;
    const unsigned grid = (unsigned)((n + kIxThreads - 1) / kIxThreads);
    claim_kernel<<<grid, kIxThreads, 0, s>>>(t, d_digests, n, d_slot_of);
    verify_kernel<<<grid, kIxThreads, 0, s>>>(t, d_digests, n, base, d_slot_of, d_pending, d_acc);
    serial_kernel<<<1, 64, 0, s>>>(t, d_digests, base, d_slot_of, d_pending, d_acc);
    mark_kernel<<<grid, kIxThreads, 0, s>>>(t, reinterpret_cast<const cdc_chunk_pod *>(d_chunks), n, base,
                                            d_slot_of, d_new, d_acc);
    return hipGetLastError();
}

}  // namespace cdc
