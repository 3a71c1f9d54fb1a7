// sha256.hip -- SHA-256 (FIPS 180-4) of every chunk of a stream, on gfx950.
//
// The reference fingerprints each chunk with `Sha256Hasher::hash`
// (src/hashers.rs:20-36, sha2 crate), called per chunk in StorageWriter::write
// (src/system/storage.rs:324-329) -- the next-largest cost of its write path
// after chunking.
//
// Layout: one LANE per chunk (a chunk's 64-byte blocks are inherently
// sequential).  Chunk lengths vary (min..max), so lanes are refilled
// dynamically: after every block, lanes whose chunk is done take the next
// chunk indices from a global counter (one atomic per wave per refill), and a
// wave leaves only when the counter is exhausted and all its lanes are idle.
// Each block's 16 big-endian words are built from 17 aligned dwords with one
// v_perm_b32 per word (funnel shift + byte swap in one instruction); the last
// one or two blocks (0x80 terminator, bit length) take a guarded byte path.
// Integer work only: Ch/Maj lower to v_bitop3_b32, rotations to v_alignbit.
#include "sha256.hpp"

namespace cdc {
namespace {

__constant__ uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

constexpr int kShaThreads = 256;

typedef const __attribute__((address_space(1))) uint32_t g_u32;
typedef const __attribute__((address_space(1))) uint8_t g_u8;

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }

__device__ __forceinline__ void compress(uint32_t H[8], uint32_t W[16]) {
    uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t w;
        if (t < 16) {
            w = W[t];
        } else {
            const uint32_t w15 = W[(t + 1) & 15], w2 = W[(t + 14) & 15];
            const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
            w = W[t & 15] + s0 + W[(t + 9) & 15] + s1;
            W[t & 15] = w;
        }
        const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + kK[t] + w;
        const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + mj;
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d;
    H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__global__ __launch_bounds__(kShaThreads) void sha256_kernel(const uint8_t *__restrict__ data,
                                                             const cdc_chunk_pod *__restrict__ chunks,
                                                             uint64_t n_chunks, uint32_t *__restrict__ digests,
                                                             unsigned long long *counter) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lanemask_lt = (1ull << lane) - 1;
    uint64_t ci = ~0ull;      // this lane's chunk (~0: idle)
    uint64_t start = 0, len = 0, blk = 0, nblk = 0;
    uint32_t H[8];
    for (;;) {
        // Refill idle lanes: one atomic per wave, indices handed out by rank.
        const uint64_t idle = __ballot(ci == ~0ull);
        if (idle) {
            const uint32_t k = (uint32_t)__popcll(idle);
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(counter, (unsigned long long)k);
            base = __shfl(base, 0);
            if (ci == ~0ull) {
                const uint64_t mine = base + (uint64_t)__popcll(idle & lanemask_lt);
                if (mine < n_chunks) {
                    ci = mine;
                    const cdc_chunk_pod c = chunks[mine];
                    start = c.offset;
                    len = c.length;
                    blk = 0;
                    nblk = (len + 9 + 63) / 64;  // message + 0x80 + 64-bit length, padded
#pragma unroll
                    for (int i = 0; i < 8; ++i) H[i] = kH0[i];
                }
            }
        }
        if (__ballot(ci != ~0ull) == 0) break;  // counter exhausted and every lane idle
        if (ci != ~0ull) {
            uint32_t W[16];
            const uint64_t p = 64 * blk;  // block start within the chunk
            if (p + 64 <= len) {
                // Full data block: 17 aligned dwords, one v_perm per big-endian word.
                const uint64_t a = start + p;
                const uint64_t al = a & ~3ull;
                const uint32_t sh = (uint32_t)(a - al);
                g_u32 *src = (g_u32 *)(data + al);
                uint32_t d[17];
#pragma unroll
                for (int i = 0; i < 16; ++i) d[i] = src[i];
                d[16] = 0;
                if (sh) {  // the block's last bytes; never read past the chunk
                    if (al + 68 <= start + len) {
                        d[16] = src[16];
                    } else {
                        g_u8 *b = (g_u8 *)(data + al + 64);
                        for (uint32_t j = 0; j < sh; ++j) d[16] |= (uint32_t)b[j] << (8 * j);
                    }
                }
                const uint32_t sel = (sh << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
#pragma unroll
                for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(d[i + 1], d[i], sel);
            } else {
                // Tail: remaining bytes, 0x80, zeros, bit length in the last 8 bytes.
                g_u8 *src = (g_u8 *)(data + start);
                const uint64_t bits = len * 8;
                const bool last = blk + 1 == nblk;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    uint32_t w = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint64_t q = p + 4 * i + j;
                        uint32_t byte = 0;
                        if (q < len) byte = src[q];
                        else if (q == len) byte = 0x80u;
                        w = (w << 8) | byte;
                    }
                    if (last && i == 14) w = (uint32_t)(bits >> 32);
                    if (last && i == 15) w = (uint32_t)bits;
                    W[i] = w;
                }
            }
            compress(H, W);
            if (++blk == nblk) {
                uint32_t *o = digests + 8 * ci;
#pragma unroll
                for (int i = 0; i < 8; ++i) o[i] = bswap(H[i]);  // big-endian digest bytes
                ci = ~0ull;
            }
        }
    }
}

}  // namespace

hipError_t launch_sha256(const uint8_t *d_data, const void *d_chunks, uint64_t n_chunks,
                         uint8_t *d_digests, unsigned long long *d_counter, int num_cus,
                         hipStream_t s) {
    if (!n_chunks) return hipSuccess;
    hipError_t e = hipMemsetAsync(d_counter, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    const uint64_t waves = (n_chunks + 63) / 64;
    const uint64_t want = (waves + 3) / 4;
    const uint64_t cap = (uint64_t)num_cus * 8;  // resident blocks: lanes refill in place
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    sha256_kernel<<<grid, kShaThreads, 0, s>>>(d_data, reinterpret_cast<const cdc_chunk_pod *>(d_chunks),
                                               n_chunks, reinterpret_cast<uint32_t *>(d_digests), d_counter);
    return hipGetLastError();
}

}  // namespace cdc
