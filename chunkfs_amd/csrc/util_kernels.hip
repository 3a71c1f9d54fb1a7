// util_kernels.hip -- the fixed-size chunker and the on-device input generator.
#include "cdc_kernels.hpp"

namespace cdc {
namespace {

// FSChunker::chunk_data (fixed_size.rs:32-43): chunk t of the batch.  first[]
// (n+1 entries) is the index of each stream's first chunk.
__global__ void fixed_kernel(const StreamTable st, uint64_t cs, const uint64_t *__restrict__ first,
                             cdc_chunk_pod *out, uint64_t total) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    uint32_t lo = 0, hi = st.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] <= t) lo = mid; else hi = mid;
    }
    const uint64_t off = (t - first[lo]) * cs;
    const uint64_t len = st.lens[lo];
    out[t] = cdc_chunk_pod{off, min(cs, len - off)};
}

// splitmix64 (the bench's synthetic input; oracle.splitmix64_bytes is the CPU
// twin): little-endian u64 word i = mix(seed + (i + 1) * golden gamma).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_kernel(uint8_t *buf, uint64_t len, uint64_t seed) {
    const uint64_t nw = len / 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride)
        reinterpret_cast<uint64_t *>(buf)[i] = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
    if (blockIdx.x == 0 && threadIdx.x == 0 && (len & 7)) {
        const uint64_t w = mix64(seed + (nw + 1) * 0x9E3779B97F4A7C15ull);
        for (uint64_t b = 0; b < (len & 7); ++b) buf[nw * 8 + b] = (uint8_t)(w >> (8 * b));
    }
}

// Read-only reduction (the measured-achievable HBM read rate the FastCDC scan
// is compared with): each block reads 16 KiB contiguous per
// iteration, four 1 KiB-per-wave-instruction loads in flight per lane, XOR-
// folded -- the fastest read pattern of tools/ubench_scan.hip (coalesced, 4 in
// flight, 8 blocks per CU: 170 us per GiB, profiles/r02_ubench_scan.txt).
typedef unsigned int rd_u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) rd_u32x4 g_rd_u32x4;
__global__ __launch_bounds__(256) void read_kernel(const uint8_t *d, uint64_t n, uint64_t *out) {
    constexpr uint64_t kPer = 256ull * 16 * 4;
    rd_u32x4 acc = {0, 0, 0, 0};
    const uint64_t full = n / kPer * kPer;
    for (uint64_t b = (uint64_t)blockIdx.x * kPer; b < full; b += (uint64_t)gridDim.x * kPer) {
        rd_u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = *(g_rd_u32x4 *)(d + b + ((uint64_t)k * 256 + threadIdx.x) * 16);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k];
    }
    for (uint64_t i = full + ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; i + 16 <= n;
         i += (uint64_t)gridDim.x * 256 * 16)
        acc ^= *(g_rd_u32x4 *)(d + i);
    uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    for (int o = 32; o > 0; o >>= 1) x ^= (uint32_t)__shfl_xor((int)x, o);
    if ((threadIdx.x & 63) == 0) atomicXor(reinterpret_cast<unsigned int *>(out + blockIdx.x), x);
}

}  // namespace

hipError_t launch_read_reduce(const uint8_t *d_buf, uint64_t len, uint64_t *d_out, int num_cus, hipStream_t s) {
    if (len < 16) return hipSuccess;
    read_kernel<<<(unsigned)(num_cus * 8), 256, 0, s>>>(d_buf, len, d_out);
    return hipGetLastError();
}

hipError_t launch_fixed(const StreamTable &st, uint64_t chunk_size, const uint64_t *d_first, void *d_out,
                        uint64_t total, hipStream_t s) {
    if (!total) return hipSuccess;
    fixed_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(st, chunk_size, d_first,
                                                                  reinterpret_cast<cdc_chunk_pod *>(d_out), total);
    return hipGetLastError();
}

hipError_t launch_fill_splitmix64(uint8_t *d_buf, uint64_t len, uint64_t seed, hipStream_t s) {
    if (!len) return hipSuccess;
    const uint64_t nw = len / 8 + 1;
    const uint64_t blocks = (nw + 255) / 256;
    fill_kernel<<<(unsigned)(blocks < 65536 ? blocks : 65536), 256, 0, s>>>(d_buf, len, seed);
    return hipGetLastError();
}

}  // namespace cdc
