// sha256.hip -- SHA-256 (FIPS 180-4) of every chunk of a stream, on gfx950.
//
// The reference fingerprints each chunk with `Sha256Hasher::hash`
// (src/hashers.rs:20-36, sha2 crate), called per chunk in StorageWriter::write
// (src/system/storage.rs:324-329) -- the next-largest cost of its write path
// after chunking.
//
// Layout: one LANE per chunk (a chunk's 64-byte blocks are inherently
// sequential); a launch takes the chunks of many streams at once (a batch:
// cdc_sha256_batch_device), so a 4 GiB archive is one launch of ~1M lanes.  Chunk lengths vary (min..max), so lanes are refilled
// dynamically: after every block, lanes whose chunk is done take the next
// chunk indices from a global counter (one atomic per wave per refill), and a
// wave leaves only when the counter is exhausted and all its lanes are idle.
// Each block's 16 big-endian words are built from 17 aligned dwords with one
// v_perm_b32 per word (funnel shift + byte swap in one instruction); the last
// one or two blocks (0x80 terminator, bit length) are masked in registers.
// Integer work only: Ch/Maj and the sigmas' three-way XORs lower to
// v_bitop3_b32, rotations to v_alignbit.
#include "sha256.hpp"

#include <algorithm>

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
typedef const __attribute__((address_space(1))) uint64_t g_u64c;
// 16-byte loads at a 4-byte-aligned address (a chunk starts at any byte).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const __attribute__((address_space(1))) u32x4_a4 g_u32x4_a4;

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }
// Three-input XOR in one v_bitop3_b32 (truth table 0x96); LLVM emits two
// v_xor_b32 for the plain expression.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// kS independent messages at once (a lane's chunk slots): the rounds of all
// of them in one unrolled body, so their dependency chains interleave.
template <int kS>
__device__ __forceinline__ void compress(uint32_t (&H)[kS][8], uint32_t (&W)[kS][16]) {
    uint32_t a[kS], b[kS], c[kS], d[kS], e[kS], f[kS], g[kS], h[kS];
#pragma unroll
    for (int k = 0; k < kS; ++k) {
        a[k] = H[k][0]; b[k] = H[k][1]; c[k] = H[k][2]; d[k] = H[k][3];
        e[k] = H[k][4]; f[k] = H[k][5]; g[k] = H[k][6]; h[k] = H[k][7];
    }
#pragma unroll
    for (int t = 0; t < 64; ++t) {
#pragma unroll
        for (int k = 0; k < kS; ++k) {
            uint32_t w;
            if (t < 16) {
                w = W[k][t];
            } else {
                const uint32_t w15 = W[k][(t + 1) & 15], w2 = W[k][(t + 14) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                w = W[k][t & 15] + s0 + W[k][(t + 9) & 15] + s1;
                W[k][t & 15] = w;
            }
            const uint32_t S1 = xor3(rotr(e[k], 6), rotr(e[k], 11), rotr(e[k], 25));
            const uint32_t ch = (e[k] & f[k]) ^ (~e[k] & g[k]);
            const uint32_t t1 = h[k] + S1 + ch + kK[t] + w;
            const uint32_t S0 = xor3(rotr(a[k], 2), rotr(a[k], 13), rotr(a[k], 22));
            const uint32_t mj = (a[k] & b[k]) ^ (a[k] & c[k]) ^ (b[k] & c[k]);
            const uint32_t t2 = S0 + mj;
            h[k] = g[k];
            g[k] = f[k];
            f[k] = e[k];
            e[k] = d[k] + t1;
            d[k] = c[k];
            c[k] = b[k];
            b[k] = a[k];
            a[k] = t1 + t2;
        }
    }
#pragma unroll
    for (int k = 0; k < kS; ++k) {
        H[k][0] += a[k]; H[k][1] += b[k]; H[k][2] += c[k]; H[k][3] += d[k];
        H[k][4] += e[k]; H[k][5] += f[k]; H[k][6] += g[k]; H[k][7] += h[k];
    }
}

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// Work distribution: a lane hashes one chunk at a time and keeps the NEXT
// chunk claimed and described ahead of time, in a three-stage pipeline that
// advances one stage per block step -- (1) claim an index (one atomic per wave
// for all lanes that need one), (2) find its stream (binary search of the
// batch's first[] in LDS) and issue the loads of its record and its
// successor's, (3) take it over when the current chunk ends.  Each stage's
// latency (L2 atomic, record loads) then hides behind a step of compression
// instead of stalling the wave at every refill (~2 of 3 steps see a lane
// finish: 64 lanes, ~65 blocks per 4 KiB chunk).  Waves leave when every lane
// is idle and the counter is exhausted.
//
// A block of the message is 17 dwords from the 4-byte-aligned address below
// it, realigned by one v_perm per big-endian word; the 68-byte window is read
// with four 16-byte loads and one dword load whenever it cannot run past
// readable memory: inside the chunk, or past its end into the next chunk of
// the same stream when that one is contiguous and >= 68 bytes ("over": every
// chunk but the last one or two of a stream).  Otherwise (a stream's last
// chunk tail) each dword is loaded only if it holds a chunk byte.  The words
// of the last one or two blocks (0x80 terminator, zeros, 64-bit bit length)
// are masked in registers, without byte loops.
constexpr uint32_t kShaLdsStreams = 2048;  // stream tables up to this many streams are staged in LDS

// The 16 big-endian message words of block `blk` of the chunk at src (len
// bytes, nblk blocks with the padding): see the kernel's comment for the
// load forms.  Wave-synchronous (the padding mask runs when any lane needs it).
__device__ __forceinline__ void block_words(uint32_t (&W)[16], uint64_t src, uint64_t len, uint64_t blk,
                                            uint64_t nblk, bool over) {
    const uint64_t p = 64 * blk;  // block start within the chunk
    const uint64_t a = src + p;
    const uint32_t sh = (uint32_t)(a & 3);
    const uint64_t al = a - sh;
    uint32_t d[17];
    if (p >= len) {  // a padding-only block (or an idle slot: len 0)
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = 0;
    } else if (over || p + 68 <= len) {
        g_u32x4_a4 *q = (g_u32x4_a4 *)al;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4_a4 v = q[i];
            d[4 * i] = v.x;
            d[4 * i + 1] = v.y;
            d[4 * i + 2] = v.z;
            d[4 * i + 3] = v.w;
        }
        d[16] = sh ? *(g_u32 *)(al + 64) : 0u;
    } else {
        const uint64_t end = src + len;
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = al + 4 * i < end ? *(g_u32 *)(al + 4 * i) : 0u;
    }
    const uint32_t sel = (sh << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(d[i + 1], d[i], sel);
    if (__ballot(p + 64 > len)) {
        // Word i holds message bytes p+4i .. p+4i+3: r = len - (p+4i) of them
        // are data; the first one past the data is 0x80.
        const int64_t r0 = (int64_t)len - (int64_t)p;
        const bool last = blk + 1 == nblk;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t r = r0 - 4 * i;
            const uint32_t rk = (uint32_t)(r < 0 ? 0 : r > 4 ? 4 : r);  // data bytes kept
            const uint32_t rp = (uint32_t)(r < 0 ? 5 : r > 5 ? 5 : r);  // 0x80 position (>= 4: none)
            const uint32_t keep = (uint32_t)~(0xFFFFFFFFull >> (8 * rk));
            const uint32_t pad = (uint32_t)(0x80000000ull >> (8 * rp));
            W[i] = (W[i] & keep) | pad;
        }
        if (last) {
            W[14] = (uint32_t)(len >> 29);  // bit length, big-endian 64-bit
            W[15] = (uint32_t)(len << 3);
        }
    }
}

#ifndef CDC_SHA_WPE  // min waves per SIMD (VGPR cap 512 / n); 0: the compiler's choice
#define CDC_SHA_WPE 0
#endif
#if CDC_SHA_WPE
#define CDC_SHA_ATTR __attribute__((amdgpu_waves_per_eu(CDC_SHA_WPE)))
#else
#define CDC_SHA_ATTR
#endif
#ifndef CDC_SHA_SLOTS  // chunks per lane hashed at once (interleaved compression chains)
#define CDC_SHA_SLOTS 1  // (2: measured slower, 7.4 vs 6.9 ms per 4 GiB, profiles/r06/r06d_*)
#endif
template <bool kLds, int kS>
__global__ __launch_bounds__(kShaThreads) CDC_SHA_ATTR void sha256_kernel(const ShaBatch j) {
    extern __shared__ uint64_t tab[];  // (kLds) first[n+1] ++ base[n], (2n+1) * 8 bytes of dynamic LDS
    const uint64_t *first = j.first, *sbase = j.base;
    if constexpr (kLds) {
        for (uint32_t i = threadIdx.x; i <= 2 * j.n_streams; i += kShaThreads)
            tab[i] = i <= j.n_streams ? *(g_u64c *)(j.first + i) : *(g_u64c *)(j.base + (i - j.n_streams - 1));
        __syncthreads();
        first = tab;
        sbase = tab + j.n_streams + 1;
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lanemask_lt = (1ull << lane) - 1;
    // the lane's chunk slots (ci ~0: idle, len 0)
    uint64_t ci[kS], src[kS], len[kS], blk[kS], nblk[kS];
    bool over[kS];
    uint32_t H[kS][8];
#pragma unroll
    for (int k = 0; k < kS; ++k) {
        ci[k] = ~0ull;
        src[k] = len[k] = blk[k] = nblk[k] = 0;
        over[k] = false;
    }
    // next chunk: stage 0 = none, 1 = index claimed, 2 = described, 3 = counter exhausted
    uint32_t nst = 0;
    uint64_t ni = 0, nsrc = 0;
    cdc_chunk_pod nc{}, nn{};
    bool nhas = false;
    for (;;) {
        // (3) an idle slot takes the next chunk over
        if (nst == 2) {
            bool took = false;
#pragma unroll
            for (int k = 0; k < kS; ++k) {
                if (!took && ci[k] == ~0ull) {
                    ci[k] = ni;
                    src[k] = nsrc + nc.offset;
                    len[k] = nc.length;
                    over[k] = nhas && nn.offset == nc.offset + nc.length && nn.length >= 68;
                    blk[k] = 0;
                    nblk[k] = (nc.length + 9 + 63) / 64;  // message + 0x80 + 64-bit length, padded
#pragma unroll
                    for (int i = 0; i < 8; ++i) H[k][i] = kH0[i];
                    took = true;
                }
            }
            if (took) nst = 0;
        }
        // (2) describe a claimed index: its stream, and the loads of its record
        if (nst == 1) {
            ni = j.order[ni];  // claims go longest chunk first
            uint32_t lo = 0, hi = j.n_streams;  // largest s with first[s] <= ni
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (first[mid] <= ni) lo = mid; else hi = mid;
            }
            nsrc = sbase[lo];
            nhas = ni + 1 < first[lo + 1];
            nc = j.chunks[ni];
            nn = j.chunks[nhas ? ni + 1 : ni];
            nst = 2;
        }
        // (1) claim indices for the lanes with an empty next stage
        const uint64_t want = __ballot(nst == 0);
        if (want) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(j.counter, (unsigned long long)__popcll(want));
            base = __shfl(base, 0);
            if (nst == 0) {
                ni = base + (uint64_t)__popcll(want & lanemask_lt);
                nst = ni < j.n_chunks ? 1u : 3u;
            }
        }
        bool busy = nst == 1 || nst == 2;
#pragma unroll
        for (int k = 0; k < kS; ++k) busy |= ci[k] != ~0ull;
        if (__ballot(busy) == 0) break;  // nothing left anywhere in the wave
        // one block of every slot (an idle slot hashes a dummy block: the
        // lanes run in lockstep anyway, and its state is reset at take-over)
        uint32_t W[kS][16];
#pragma unroll
        for (int k = 0; k < kS; ++k) block_words(W[k], src[k], len[k], blk[k], nblk[k], over[k]);
        compress<kS>(H, W);
#pragma unroll
        for (int k = 0; k < kS; ++k) {
            if (ci[k] != ~0ull && ++blk[k] == nblk[k]) {
                uint32_t *o = j.digests + 8 * ci[k];
#pragma unroll
                for (int i = 0; i < 8; ++i) o[i] = bswap(H[k][i]);  // big-endian digest bytes
                ci[k] = ~0ull;
                len[k] = blk[k] = nblk[k] = 0;
            }
        }
    }
}

// Longest-first claim order (a counting sort of the chunks by length class,
// descending): lanes take chunks from a global counter, and a wave runs until
// its slowest lane is done, so the last chunks a lane takes should be the
// short ones -- in index order a lane's final chunk was as likely 8 KiB as
// 2 KiB, and waves idled up to a whole chunk in their tails.
__device__ __forceinline__ uint32_t len_class(uint64_t len) {
    const uint32_t lz = (uint32_t)__builtin_clzll(len | 1);  // log-linear classes: 8 per octave
    const uint32_t oct = 63 - lz;
    const uint32_t sub = oct >= 3 ? (uint32_t)(len >> (oct - 3)) & 7u : (uint32_t)len & 7u;
    const uint32_t c = oct * 8 + sub;
    return c < kShaBuckets ? kShaBuckets - 1 - c : 0u;  // descending length
}

__global__ __launch_bounds__(256) void sha_hist_kernel(const cdc_chunk_pod *__restrict__ chunks, uint64_t n,
                                                      unsigned long long *hist) {
    __shared__ uint32_t h[kShaBuckets];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        atomicAdd(&h[len_class(chunks[i].length)], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// One block: exclusive scan of the histogram in place (then the scatter's cursors).
__global__ __launch_bounds__(256) void sha_scan_kernel(unsigned long long *hist) {
    __shared__ unsigned long long v[kShaBuckets];
    v[threadIdx.x] = hist[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        for (uint32_t k = 0; k < kShaBuckets; ++k) {
            const unsigned long long c = v[k];
            v[k] = acc;
            acc += c;
        }
    }
    __syncthreads();
    hist[threadIdx.x] = v[threadIdx.x];
}

// Block-local scatter: a block takes kShaTile consecutive chunks, counts
// them per class in LDS, reserves each class's run with ONE global atomic
// (822k chunks into ~17 classes with one atomic per chunk took 2.4 ms of
// contention), then places them with LDS atomics.
constexpr uint32_t kShaTile = 4096;

__global__ __launch_bounds__(256) void sha_scatter_kernel(const cdc_chunk_pod *__restrict__ chunks, uint64_t n,
                                                         unsigned long long *cursor, uint32_t *order) {
    __shared__ uint32_t cnt[kShaBuckets];
    __shared__ unsigned long long base[kShaBuckets];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kShaTile; t0 < n; t0 += (uint64_t)gridDim.x * kShaTile) {
        const uint64_t t1 = t0 + kShaTile < n ? t0 + kShaTile : n;
        cnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += 256) atomicAdd(&cnt[len_class(chunks[i].length)], 1u);
        __syncthreads();
        const uint32_t c = cnt[threadIdx.x];
        base[threadIdx.x] = c ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)c) : 0ull;
        cnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += 256) {
            const uint32_t k = len_class(chunks[i].length);
            order[base[k] + atomicAdd(&cnt[k], 1u)] = (uint32_t)i;
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_sha256(const ShaBatch &b, int num_cus, hipStream_t s) {
    if (!b.n_chunks) return hipSuccess;
    hipError_t e = hipMemsetAsync(b.counter, 0, (1 + kShaBuckets) * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    unsigned long long *hist = b.counter + 1;
    const unsigned sgrid = (unsigned)std::min<uint64_t>((b.n_chunks + 255) / 256, (uint64_t)num_cus * 4);
    sha_hist_kernel<<<sgrid, 256, 0, s>>>(b.chunks, b.n_chunks, hist);
    sha_scan_kernel<<<1, 256, 0, s>>>(hist);
    const unsigned tgrid = (unsigned)std::min<uint64_t>((b.n_chunks + kShaTile - 1) / kShaTile, (uint64_t)num_cus * 4);
    sha_scatter_kernel<<<tgrid, 256, 0, s>>>(b.chunks, b.n_chunks, hist, b.order);
    // Resident waves only (the counter spreads the chunks over them): one
    // block of 4 waves per SIMD-wave slot the kernel's registers allow.
    const bool lds = b.n_streams <= kShaLdsStreams;
    const size_t dyn = lds ? (2 * b.n_streams + 1) * sizeof(uint64_t) : 0;
    int per_cu = 0;
    e = lds ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sha256_kernel<true, CDC_SHA_SLOTS>, kShaThreads, dyn)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sha256_kernel<false, CDC_SHA_SLOTS>, kShaThreads, 0);
    if (e != hipSuccess) return e;
    const uint64_t waves = (b.n_chunks + 64 * CDC_SHA_SLOTS - 1) / (64 * CDC_SHA_SLOTS);
    const uint64_t want = (waves + 3) / 4;
    const uint64_t cap = (uint64_t)num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    if (lds)
        sha256_kernel<true, CDC_SHA_SLOTS><<<grid, kShaThreads, dyn, s>>>(b);
    else
        sha256_kernel<false, CDC_SHA_SLOTS><<<grid, kShaThreads, 0, s>>>(b);
    return hipGetLastError();
}

}  // namespace cdc
