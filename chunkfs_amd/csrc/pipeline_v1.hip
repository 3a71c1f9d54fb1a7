// pipeline_v1.hip -- the round-1 GPU-validated FastCDC pipeline (default).
//
// Kept beside the newer pipeline in cdc_kernels.hip (selected with
// CHUNKFS_AMD_PIPELINE=2) until that one has passed the GPU parity suite: this
// one was bit-exact on MI355X (tests/test_gpu_parity.py, 1 GiB config-2 stream).
//
//  1. scan_kernel: wave per span; 64 contiguous bytes per lane per 4 KiB
//     wave-iteration; pass 1 hashes the lane's last 48 bytes, one DPP wave_shr
//     hands the end hash to the next lane; pass 2 tests every position;
//     GEAR lookups software-pipelined in groups of 8 (4 waves/SIMD).
//  2. trunc_kernel: per candidate record, the exact truncated-region result
//     of a chunk starting there (record bits 24..29).
//  3. spec_kernel: wave-cooperative speculative chain walk per span from a
//     2*max warm-up start.
//  4. fixup_kernel x3 (Jacobi, device early exit) + serial_kernel (no-op
//     unless the passes did not converge).
//  5. count / block_sums / write kernels: chunk index prefix, output.
#include "pipeline_v1.hpp"

namespace cdc {
namespace v1 {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kCopies = 32;           // GEAR replicas, one bank pair per lane&31
constexpr uint32_t kIterBytes = 4096; // 64 lanes x 64 contiguous bytes per wave-iteration
// 2 blocks of 16 waves per CU = 8 waves/SIMD: caps the scan at 64 VGPRs.
constexpr int kScanMinWaves = 4;
constexpr uint32_t kEntCap = 64;      // per-wave LDS list of hitting 16-byte quarters per span
// Candidate record: offset in span (spans <= 16 MiB) | exact mask hit flags.
constexpr uint32_t kCandPosMask = 0x00FFFFFFu;
constexpr uint32_t kCandHitL = 1u << 30;
constexpr uint32_t kCandHitS = 1u << 31;
// Bits 24..29: truncated-region result of the chunk starting at the record
// (written by trunc_kernel): 0..46 = first hitting offset after start+a0.
constexpr uint32_t kCandTrShift = 24;
constexpr uint32_t kCandTrMask = 0x3Fu;
constexpr uint32_t kCandTrNone = 62;
constexpr uint32_t kCandTrUnk = 63;

// Global (address space 1) views of the stream bytes.  Generic pointers would
// compile to flat_load_*, which count on both vmcnt and lgkmcnt and may return
// out of order: every LDS wait would then drain the whole prefetch ring.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ g_u32x4 *as_global4(const void *p) { return (g_u32x4 *)(p); }
__device__ __forceinline__ g_u8 *as_global1(const void *p) { return (g_u8 *)(p); }
__device__ __forceinline__ uint4 ld16(g_u32x4 *p) {
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// DPP wave_shr:1 (dpp_ctrl 0x138): lane i receives lane i-1; lane 0 keeps `fill`.
__device__ __forceinline__ uint64_t wave_shr1(uint64_t v, uint64_t fill) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(
        (int)(uint32_t)fill, (int)(uint32_t)v, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(
        (int)(uint32_t)(fill >> 32), (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane63(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

// Largest stream i with span_base[i] <= g (streams with zero spans skipped).
__device__ __forceinline__ void locate(const StreamTable &st, uint64_t g,
                                       uint32_t &si, uint64_t &off) {
    uint32_t lo = 0, hi = st.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (st.span_base[mid] <= g) lo = mid; else hi = mid;
    }
    si = lo;
    off = (g - st.span_base[lo]) << st.span_log2;
}

template <bool kAlign>
__device__ __forceinline__ uint32_t cand_test(uint64_t h, const FastParams &fp) {
    if constexpr (kAlign) {
        return (uint32_t)(h >> 32) & fp.cm32;  // h pre-shifted by tshift
    } else {
        return ((uint32_t)h & fp.cm_lo) | ((uint32_t)(h >> 32) & fp.cm_hi);
    }
}

// h = (h << 1) + g as ONE opaque v_lshl_add_u64.  Plain C lets LLVM
// reassociate a 48-term chain into a tree that keeps every lookup live (2
// VGPRs each) and spills; the asm keeps the chain strictly sequential, so each
// GEAR lookup dies right after its add.
__device__ __forceinline__ uint64_t shl1_add(uint64_t h, uint64_t g) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(h), "v"(g));
    return r;
}

// GEAR[byte b of word w] from LDS: one v_perm_b32 builds the byte address
// b*256 + replica*8, one ds_read_b64 fetches the entry.
__device__ __forceinline__ uint64_t gear_of(const char *tabb, uint32_t rep_off, uint32_t w, int b) {
    const uint32_t addr = __builtin_amdgcn_perm(rep_off, w, 0x0c0c0004u | ((uint32_t)b << 8));
    return *reinterpret_cast<const uint64_t *>(tabb + addr);
}

struct Data64 {
    uint4 q[4];
};

__device__ __forceinline__ Data64 ld64(g_u32x4 *p) {
    Data64 d;
#pragma unroll
    for (int i = 0; i < 4; ++i) d.q[i] = ld16(p + i);
    return d;
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int w) {
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}

// Hash of the lane's 64 bytes from a zero state, mod 2^48: only the last 48
// bytes can reach bits 0..47, so bytes 16..63 suffice.  It equals the TRUE
// (windowed) hash at the lane's last byte.  Uses a different GEAR replica than
// pass 2 so the compiler cannot keep these 48 lookups live for reuse.
__device__ __forceinline__ uint64_t pass1(const char *tabb, uint32_t rep_off, const Data64 &d) {
    uint64_t P = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q) {
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int b = 0; b < 4; ++b) P = shl1_add(P, gear_of(tabb, rep_off, word_of(d.q[q], w), b));
        // Bound the scheduler's lookahead to one 16-byte quarter: hoisting all
        // lookups of the lane at once costs ~2 VGPRs each and spills.
        __builtin_amdgcn_sched_barrier(0);
    }
    return P;
}

#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

struct G8 {
    uint64_t v[8];
};

__device__ __forceinline__ void look8(G8 &g, const char *tabb, uint32_t rep_off, uint32_t w0,
                                      uint32_t w1) {
#pragma unroll
    for (int b = 0; b < 4; ++b) g.v[b] = gear_of(tabb, rep_off, w0, b);
#pragma unroll
    for (int b = 0; b < 4; ++b) g.v[4 + b] = gear_of(tabb, rep_off, w1, b);
}

__device__ __forceinline__ void chain8(uint64_t &h, const G8 &g) {
#pragma unroll
    for (int i = 0; i < 8; ++i) h = shl1_add(h, g.v[i]);
}

template <bool kAlign>
__device__ __forceinline__ void chain8_test(uint64_t &h, uint32_t &acc, const G8 &g,
                                            const FastParams &fp) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        h = shl1_add(h, g.v[i]);
        acc = min(acc, cand_test<kAlign>(h, fp));
    }
}

__device__ __forceinline__ uint4 ld16_guarded(const uint8_t *base, uint32_t p, uint32_t limit) {
    if (p + 16 <= limit) return ld16(as_global4(base + p));
    uint32_t w[4] = {0, 0, 0, 0};
    if (p < limit) {
        g_u8 *gb = as_global1(base);
        for (uint32_t j = 0; p + j < limit; ++j) w[j >> 2] |= (uint32_t)gb[p + j] << (8 * (j & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// One-pass gear candidate scan.  Layout: one wavefront per span; per
// wave-iteration the 64 lanes cover 4 KiB, lane l owning the contiguous bytes
// [64 l, 64 l + 64).  Per lane: pass 1 (48 lookups) gives the lane's end hash;
// one DPP wave_shr hands it to lane l+1 as its carry-in (bits 0..47 exact: no
// multi-step scan needed once a lane owns >= 48 bytes); pass 2 walks the 64
// positions with the true hash and tests (h & cmask) == 0, min-accumulated per
// 16-byte quarter.  A hitting quarter only appends (position, hash before the
// quarter) to a per-wave LDS list; exact mask_s/mask_l flags, ordering and the
// HBM write happen once per span in the flush.
template <bool kAlign>
__global__ __launch_bounds__(kScanThreads, kScanMinWaves) void scan_kernel(
    const StreamTable st, const FastParams fp,
    const uint64_t *__restrict__ gear, const Candidates cand) {
    __shared__ uint64_t tab[256 * kCopies];  // 64 KiB: entry e, replica c at e*32+c
    __shared__ uint32_t epos[kScanWaves][kEntCap];
    __shared__ uint32_t ehlo[kScanWaves][kEntCap];
    __shared__ uint32_t ehhi[kScanWaves][kEntCap];
    __shared__ uint32_t ecnt[kScanWaves][kEntCap];
    for (int i = threadIdx.x; i < 256 * kCopies; i += kScanThreads)
        tab[i] = gear[i / kCopies] << fp.tshift;  // pre-shifted GEAR (see FastParams)
    __syncthreads();

    const char *tabb = reinterpret_cast<const char *>(tab);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t rep2 = (lane & 31) * 8;         // pass-2 replica
    const uint32_t rep1 = ((lane + 16) & 31) * 8;  // pass-1 replica (still a permutation)
    const uint64_t span = 1ull << st.span_log2;
    const uint64_t lanemask_lt = (1ull << lane) - 1;

    for (uint64_t g = (uint64_t)blockIdx.x * kScanWaves + wave; g < st.total_spans;
         g += (uint64_t)gridDim.x * kScanWaves) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        const uint8_t *base = st.ptrs[si] + off;
        const uint64_t n_left = st.lens[si] - off;
        const uint32_t span_len = (uint32_t)(n_left < span ? n_left : span);

        // Carry-in: true hash of byte off-1 = pass 1 over the 64 bytes before the span.
        uint64_t carry = 0;
        if (off != 0) {
            uint64_t P = 0;
            if (lane == 63) P = pass1(tabb, rep1, ld64(as_global4(base - 64)));
            carry = readlane63(P);
        }

        uint32_t ne = 0;  // quarter entries appended this span (wave-uniform)

        // One wave-iteration over the lane's 64 bytes in d.
        auto process = [&](const Data64 &d, uint32_t pos0, uint32_t qvalid) {
            // 14 groups of 8 lookups (pass 1: bytes 16..63 = 6 groups; pass 2:
            // bytes 0..63 = 8 groups), software-pipelined: the LDS reads of
            // group i+1 are in flight while group i's chain runs.
            G8 ga, gb;
            uint64_t P = 0;
            look8(ga, tabb, rep1, d.q[1].x, d.q[1].y);
            SCHED_FENCE();
            look8(gb, tabb, rep1, d.q[1].z, d.q[1].w);
            SCHED_FENCE();
            chain8(P, ga);
            SCHED_FENCE();
            look8(ga, tabb, rep1, d.q[2].x, d.q[2].y);
            SCHED_FENCE();
            chain8(P, gb);
            SCHED_FENCE();
            look8(gb, tabb, rep1, d.q[2].z, d.q[2].w);
            SCHED_FENCE();
            chain8(P, ga);
            SCHED_FENCE();
            look8(ga, tabb, rep1, d.q[3].x, d.q[3].y);
            SCHED_FENCE();
            chain8(P, gb);
            SCHED_FENCE();
            look8(gb, tabb, rep1, d.q[3].z, d.q[3].w);
            SCHED_FENCE();
            chain8(P, ga);
            SCHED_FENCE();
            look8(ga, tabb, rep2, d.q[0].x, d.q[0].y);  // pass 2's first group
            SCHED_FENCE();
            chain8(P, gb);
            SCHED_FENCE();
            const uint64_t cin = wave_shr1(P, carry);
            carry = readlane63(P);
            uint64_t h = cin;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t h0 = h;  // hash before the quarter (for the flush)
                uint32_t acc = 0xffffffffu;
                look8(gb, tabb, rep2, d.q[q].z, d.q[q].w);
                SCHED_FENCE();
                chain8_test<kAlign>(h, acc, ga, fp);
                SCHED_FENCE();
                if (q < 3) {
                    look8(ga, tabb, rep2, d.q[q + 1].x, d.q[q + 1].y);
                    SCHED_FENCE();
                }
                chain8_test<kAlign>(h, acc, gb, fp);
                SCHED_FENCE();
                const bool hit = acc == 0 && ((qvalid >> q) & 1u);
                const uint64_t m = __ballot(hit);
                if (m) {  // ~1 hitting quarter per 4 KiB at 12-bit masks
                    if (hit) {
                        const uint32_t slot = ne + (uint32_t)__popcll(m & lanemask_lt);
                        if (slot < kEntCap) {
                            epos[wave][slot] = pos0 + 16 * q;
                            ehlo[wave][slot] = (uint32_t)h0;
                            ehhi[wave][slot] = (uint32_t)(h0 >> 32);
                        }
                    }
                    ne += (uint32_t)__popcll(m);
                }
            }
        };

        const uint32_t nfull = span_len / kIterBytes;
        g_u32x4 *vb = as_global4(base) + lane * 4;
        uint32_t it = 0;
        if (nfull >= 2) {
            Data64 A = ld64(vb);
            __builtin_amdgcn_sched_barrier(0);
            Data64 B = ld64(vb + 256);
            __builtin_amdgcn_sched_barrier(0);
            for (; it + 2 <= nfull; it += 2) {
                // Consume a buffer, then refill it two iterations ahead (same
                // registers: no loop-carried copies of in-flight loads).
                process(A, it * kIterBytes + lane * 64, 0xFu);
                A = ld64(vb + min(it + 2, nfull - 1) * 256);
                process(B, (it + 1) * kIterBytes + lane * 64, 0xFu);
                B = ld64(vb + min(it + 3, nfull - 1) * 256);
            }
        }
        for (; it < nfull; ++it)  // remainder: only in the last span of a stream
            process(ld64(vb + it * 256), it * kIterBytes + lane * 64, 0xFu);
        if (span_len % kIterBytes) {  // ragged end of a stream: guarded loads
            const uint32_t pos0 = nfull * kIterBytes + lane * 64;
            Data64 d;
            uint32_t qvalid = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t p = pos0 + 16 * q;
                if (p < span_len) qvalid |= 1u << q;
                d.q[q] = ld16_guarded(base, p, span_len);
            }
            process(d, pos0, qvalid);
        }

        // Flush: exact flags for each hitting quarter, position order, HBM write.
        uint32_t *cpos = cand.pos + g * cand.cap;
        if (ne > kEntCap) {  // too many hits for the LDS list: resolver takes the exact slow path
            if (lane == 0) cand.count[g] = cand.cap + 1;
            continue;
        }
        uint32_t hs = 0, hl = 0, my_pos = 0;
        if (lane < ne) {
            my_pos = epos[wave][lane];
            uint64_t hh = ((uint64_t)ehhi[wave][lane] << 32) | ehlo[wave][lane];
            const uint4 v = ld16_guarded(base, my_pos, span_len);
#pragma unroll
            for (int w = 0; w < 4; ++w)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int j = 4 * w + b;
                    hh = (hh << 1) + gear_of(tabb, rep2, word_of(v, w), b);
                    if (my_pos + j < span_len) {
                        hs |= (uint32_t)((hh & fp.mask_s_sh) == 0) << j;
                        hl |= (uint32_t)((hh & fp.mask_l_sh) == 0) << j;
                    }
                }
            ecnt[wave][lane] = __popc(hs | hl);
        }
        // Output slot = records of all entries at lower positions (entries are
        // few: a linear rank over the wave's LDS list).
        uint32_t slot = 0, total = 0;
        for (uint32_t k = 0; k < ne; ++k) {
            const uint32_t c = ecnt[wave][k];
            total += c;
            if (epos[wave][k] < my_pos) slot += c;
        }
        if (lane < ne) {
            for (uint32_t m = hs | hl; m; m &= m - 1) {
                const uint32_t j = __builtin_ctz(m);
                if (slot < cand.cap)
                    cpos[slot] = (my_pos + j) | (((hs >> j) & 1u) << 31) | (((hl >> j) & 1u) << 30);
                ++slot;
            }
        }
        if (lane == 0) cand.count[g] = total;
    }
}

// ---------------------------------------------------------------------------
// Resolve (wave-cooperative).  One wavefront walks one chain; every branch
// below is wave-uniform.
//
// A chunk starting at s is cut at the first position p in [s+a0, s+re) whose
// in-chunk hash (reset at s+a0) hits its mask.  Two kinds of positions:
//  * the <= 47 "truncated" positions s+a0 .. s+a0+46, where that hash still
//    differs from the windowed one: evaluated exactly, either precomputed per
//    candidate record (a lane per record, when its span is loaded) or, for
//    chunks that do not start at a record, by one coalesced byte load + a
//    6-step shuffle prefix scan;
//  * all later positions: the scan's candidate records (position-sorted, one
//    per lane), tested with a ballot.
// So a walk step that starts at a record -- about 90% of them -- touches no
// memory.

constexpr int kResolveThreads = 256;  // 4 waves: one span (or stream) each
constexpr int kResolveWaves = kResolveThreads / 64;
constexpr uint32_t kTrUnk = 0xFF;   // truncated result not precomputed
constexpr uint32_t kTrNone = 0xFE;  // precomputed: no hit in the truncated region
constexpr uint32_t kTruncMax = 47;  // mask bits <= 47 (checked on the host)

// Inclusive scan of the gear recurrence across lanes:
// lane d returns sum_{i<=d} g_i << (d - i)  (mod 2^64).
__device__ __forceinline__ uint64_t gear_prefix(uint64_t g, uint32_t lane) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint64_t t = __shfl_up(g, k);
        if (lane >= (uint32_t)k) g += t << k;
    }
    return g;
}

typedef const __attribute__((address_space(1))) uint32_t g_u32;

// Dword at byte offset `off` (4-aligned) of a stream of n bytes, zero past n.
__device__ __forceinline__ uint32_t ld4_guarded(const uint8_t *data, uint64_t off, uint64_t n) {
    if (off + 4 <= n) return *(g_u32 *)(data + off);
    uint32_t w = 0;
    g_u8 *gb = as_global1(data);
    for (uint64_t j = 0; off + j < n; ++j) w |= (uint32_t)gb[off + j] << (8 * j);
    return w;
}

struct SpanRecs {
    uint32_t cnt = 0;   // records in the span (> cap: overflowed)
    uint32_t rec = 0;   // record `lane` (records 0..63)
    uint32_t tr = kTrUnk;
};

struct WaveWalker {
    const StreamTable &st;
    const FastParams &fp;
    const Candidates &cand;
    const uint64_t *tab;  // LDS GEAR (one copy)
    const uint8_t *data;
    uint64_t n;
    uint64_t gbase;
    uint32_t lane;
    // Spans ra and ra+1 are resident (the search window of a chunk is at most
    // max <= SPAN bytes, so it touches at most two spans).  The walk only
    // moves forward: each span is fetched once.
    uint64_t ra = ~0ull;
    bool hb = false;
    SpanRecs A, B;
    uint64_t last_cut = ~0ull;  // last cut that came from a record ...
    uint32_t last_t = kTrUnk;   // ... and that record's truncated result

    __device__ SpanRecs fetch(uint64_t sp) {
        SpanRecs R;
        if ((sp << st.span_log2) >= n) return R;  // past the stream's last span
        const uint64_t g = gbase + sp;
        // Count and record slot `lane` are loaded together (cap >= 64): one
        // round trip per span.
        R.cnt = cand.count[g];
        const uint32_t raw = cand.pos[g * cand.cap + lane];
        if (R.cnt > cand.cap || R.cnt == 0) return R;
        R.rec = lane < R.cnt ? raw : 0;
        const uint32_t t = (R.rec >> kCandTrShift) & kCandTrMask;  // from trunc_kernel
        R.tr = t == kCandTrUnk ? kTrUnk : t == kCandTrNone ? kTrNone : t;
        return R;
    }
    __device__ void ensure_a(uint64_t sp) {
        if (ra == sp) return;
        if (hb && ra + 1 == sp) {
            A = B;
        } else {
            A = fetch(sp);
        }
        ra = sp;
        hb = false;
    }
    __device__ void ensure_b() {
        if (!hb) {
            B = fetch(ra + 1);
            hb = true;
        }
    }

    // Exact hashes at positions s+p, p in [p0, p1) (p1 - p0 <= 64), chained
    // from `hin` = hash at s+p0-1 (0 = reset).  Returns the first relative
    // position that hits its mask (~0 if none); hout = hash at s+p1-1.
    __device__ uint64_t block_hits(uint64_t s, uint64_t p0, uint64_t p1, uint64_t ce,
                                   uint64_t hin, uint64_t &hout) {
        const uint64_t p = p0 + lane;
        const bool in = p < p1;
        uint64_t gv = 0;
        if (in) gv = tab[as_global1(data)[s + p]];
        uint64_t x = gear_prefix(gv, lane) + ((hin << lane) << 1);
        const bool hit = in && !(x & (p < ce ? fp.mask_s : fp.mask_l));
        const uint64_t m = __ballot(hit);
        hout = __shfl(x, (int)(p1 - p0 - 1));
        return m ? p0 + (uint64_t)(__ffsll((long long)m) - 1) : ~0ull;
    }

    // Exact scan of [a0, re) in 64-position blocks (overflowed candidate list).
    __device__ uint64_t slow_cut(uint64_t s, uint64_t a0, uint64_t re, uint64_t ce, uint64_t rem) {
        uint64_t h = 0;
        for (uint64_t b = a0; b < re; b += 64) {
            const uint64_t p = block_hits(s, b, min(b + 64, re), ce, h, h);
            if (p != ~0ull) return s + p;
        }
        return s + rem;
    }

    // Search span sp's records for the first hit in [lo, hi).  Returns the cut,
    // s+rem when a record at or past hi proves there is none, or ~0 to go on
    // with the next span.
    __device__ uint64_t search(uint64_t sp, const SpanRecs &R, uint64_t s, uint64_t lo,
                               uint64_t hi, uint64_t ce, uint64_t rem, bool &ovf) {
        if (R.cnt > cand.cap) {
            ovf = true;
            return ~0ull;
        }
        const uint64_t sp0 = sp << st.span_log2;
        const uint32_t *P = cand.pos + (gbase + sp) * cand.cap;
        for (uint32_t base = 0; base < R.cnt; base += 64) {
            const bool have = base + lane < R.cnt;
            uint32_t r = R.rec;
            if (base) r = have ? P[base + lane] : 0;
            const uint64_t c = sp0 + (r & kCandPosMask);
            const bool ok = have && c >= lo && c < hi && (r & ((c - s) < ce ? kCandHitS : kCandHitL));
            const uint64_t mo = __ballot(ok);
            if (mo) {  // position-sorted: the lowest lane is the first hit
                const int k = __ffsll((long long)mo) - 1;
                last_cut = __shfl(c, k);
                last_t = base == 0 ? (uint32_t)__shfl((int)R.tr, k) : kTrUnk;
                return last_cut;
            }
            if (__ballot(have && c >= hi)) return s + rem;
        }
        return ~0ull;
    }

    // End offset of the chunk that starts at s (SURVEY.md A.2 semantics).
    __device__ uint64_t next_cut(uint64_t s) {
        uint64_t rem = n - s;
        if (rem <= fp.min) return n;  // tail chunk
        uint64_t center = fp.avg;
        if (rem > fp.max) rem = fp.max; else if (rem < center) center = rem;
        const uint64_t a0 = (fp.min / 2) * 2, ce = (center / 2) * 2, re = (rem / 2) * 2;
        const uint64_t tl = min(a0 + (uint64_t)fp.trunc, re);
        if (s == last_cut && last_t != kTrUnk) {  // precomputed with the record
            if (last_t != kTrNone) return s + a0 + last_t;
        } else if (tl > a0) {
            uint64_t h;
            const uint64_t p = block_hits(s, a0, tl, ce, 0, h);
            if (p != ~0ull) return s + p;
        }
        if (tl >= re) return s + rem;
        const uint64_t lo = s + tl, hi = s + re;
        const uint64_t sl = lo >> st.span_log2;
        bool ovf = false;
        ensure_a(sl);
        uint64_t r = search(sl, A, s, lo, hi, ce, rem, ovf);
        if (r == ~0ull && !ovf && ((sl + 1) << st.span_log2) < hi) {
            ensure_b();
            r = search(sl + 1, B, s, lo, hi, ce, rem, ovf);
        }
        if (ovf) return slow_cut(s, a0, re, ce, rem);
        return r == ~0ull ? s + rem : r;  // none: max (or end of data)
    }
};

__device__ __forceinline__ void load_tab1(uint64_t *tab, const uint64_t *gear) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = gear[i];
    __syncthreads();
}

// Walk span g's chain from `e` (first chunk start >= span start) until it
// reaches the span end or merges with the stored chain `old` (exit
// `old_exit`).  Writes the new chain to `nl`; returns the exit.
__device__ uint64_t rewalk(WaveWalker &w, uint64_t e, uint64_t seg_end, const uint64_t *old,
                           uint32_t ocnt, uint64_t old_exit, uint64_t *nl, uint32_t &cnt) {
    const uint32_t lane = w.lane;
    uint32_t j0 = 0;
    uint64_t s = e;
    cnt = 0;
    for (;;) {
        if (s >= seg_end) return s;
        for (;;) {  // is s on the old chain?  (old is sorted)
            const uint32_t k = j0 + lane;
            const uint64_t o = k < ocnt ? old[k] : ~0ull;
            const uint64_t meq = __ballot(o == s);
            if (meq) {  // merged: the rest of the old chain holds
                const uint32_t j = j0 + (uint32_t)(__ffsll((long long)meq) - 1);
                for (uint32_t t = lane; j + t < ocnt; t += 64) nl[cnt + t] = old[j + t];
                cnt += ocnt - j;
                return old_exit;
            }
            const uint32_t nlt = (uint32_t)__popcll(__ballot(k < ocnt && o < s));
            j0 += nlt;
            if (nlt < 64) break;
        }
        if (lane == 0) nl[cnt] = s;
        ++cnt;
        s = w.next_cut(s);
    }
}

// Truncated region of the chunk that would START at each candidate record:
// one wave per span, one lane per record.  The result (first hitting offset
// 0..46, "none", or "unknown" when that chunk's centre is not avg or its
// region is short -- near the end of a stream) goes into the record's spare
// bits 24..29, so the walk needs no memory access for chunks that start at a
// record.  Bytes are staged per lane in LDS (13 dwords, odd stride: no bank
// conflicts), the 47-step chain reads them back.
__global__ __launch_bounds__(kResolveThreads) void trunc_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand) {
    __shared__ uint64_t tab[256];
    __shared__ uint32_t win[kResolveThreads * 13];
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * kResolveWaves + (threadIdx.x >> 6);
    if (g >= st.total_spans) return;
    const uint32_t cnt = cand.count[g];
    if (cnt > cand.cap) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint8_t *data = st.ptrs[si];
    const uint64_t n = st.lens[si];
    const uint64_t a0 = (fp.min / 2) * 2, cavg = (fp.avg / 2) * 2;
    uint32_t *wl = win + threadIdx.x * 13;
    for (uint32_t k = lane; k < cnt; k += 64) {
        uint32_t rec = cand.pos[g * cand.cap + k];
        const uint64_t c = off + (rec & kCandPosMask);
        const uint64_t remc = n - c;
        const uint64_t rr = remc > fp.max ? fp.max : remc;
        uint32_t t = kCandTrUnk;
        if (remc > fp.min && remc >= fp.avg && (rr / 2) * 2 >= a0 + fp.trunc) {
            const uint64_t w0 = c + a0, al = w0 & ~3ull;
            uint32_t w[13];
            if (al + 52 <= n) {  // all 13 loads in flight at once
#pragma unroll
                for (int i = 0; i < 13; ++i) w[i] = *(g_u32 *)(data + al + 4 * i);
            } else {
#pragma unroll
                for (int i = 0; i < 13; ++i) w[i] = ld4_guarded(data, al + 4 * i, n);
            }
#pragma unroll
            for (int i = 0; i < 13; ++i) wl[i] = w[i];
            const uint8_t *bytes = reinterpret_cast<const uint8_t *>(wl) + (w0 - al);
            uint64_t h = 0;
            t = kCandTrNone;
#pragma unroll 8
            for (uint32_t d = 0; d < kTruncMax; ++d) {  // no early exit: LDS reads pipeline
                h = shl1_add(h, tab[bytes[d]]);
                const bool hit = d < fp.trunc && !(h & ((a0 + d) < cavg ? fp.mask_s : fp.mask_l));
                t = hit ? min(t, d) : t;
            }
        }
        rec = (rec & ~(kCandTrMask << kCandTrShift)) | (t << kCandTrShift);
        cand.pos[g * cand.cap + k] = rec;
    }
}

// Speculative chain of span g.  The walk starts 2*max bytes before the span
// (exact when that is the stream start), so by the time it reaches span g it
// has almost always merged with the true chain: the Jacobi passes then find
// entry[g] == exit[g-1] and do no work.
__global__ __launch_bounds__(kResolveThreads) void spec_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const Chains ch, uint64_t *stats) {
    __shared__ uint64_t tab[256];
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * kResolveWaves + (threadIdx.x >> 6);
    if (g == 0 && lane == 0) {
        for (int i = 0; i < 3; ++i) ch.changed[i] = 0;
        for (int i = 0; i < 4; ++i) stats[i] = 0;
    }
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    WaveWalker w{st, fp, cand, tab, st.ptrs[si], st.lens[si], st.span_base[si], lane};
    const uint64_t span = 1ull << st.span_log2;
    const uint64_t seg_end = min(off + span, w.n);
    uint64_t *list = ch.starts[0] + g * ch.smax;
    uint32_t cnt = 0;
    // Warm-up start: 2*max before the span (the stream start when closer).
    const uint64_t warm = 2ull * fp.max;
    uint64_t s = off > warm ? off - warm : 0;
    // Both spans the walk begins in, fetched together (one round trip).
    w.ensure_a(s >> st.span_log2);
    w.ensure_b();
    while (s < seg_end) {
        if (s >= off) {
            if (lane == 0) list[cnt] = s;
            ++cnt;
        }
        s = w.next_cut(s);
    }
    if (lane == 0) {
        ch.nstarts[0][g] = cnt;
        ch.which[g] = 0;
        ch.entry[g] = cnt ? list[0] : s;
        ch.exit[0][g] = s;
    }
}

// Jacobi pass `iter`: reads exits from buffer iter&1, writes the other one.
// Exits early (writing a 0 flag) once the previous pass changed nothing, so a
// fixed number of launches needs no host round trip.
__global__ __launch_bounds__(kResolveThreads) void fixup_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const Chains ch, int iter, uint64_t *stats) {
    __shared__ uint64_t tab[256];
    uint32_t *flag = ch.changed;
    const int b = iter & 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * kResolveWaves + (threadIdx.x >> 6);
    if (iter > 0 && flag[(iter - 1) % 3] == 0) {  // converged: propagate "no change"
        if (g == 0 && lane == 0) flag[iter % 3] = 0;
        return;
    }
    if (g == 0 && lane == 0) {
        flag[(iter + 1) % 3] = 0;
        atomicAdd((unsigned long long *)&stats[2], 1ull);
    }
    load_tab1(tab, gear);
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t ein = ch.exit[b][g];
    if (off == 0) {  // first span of a stream: its entry (0) is exact
        if (lane == 0) ch.exit[1 - b][g] = ein;
        return;
    }
    const uint64_t e = ch.exit[b][g - 1];
    if (e == ch.entry[g]) {
        if (lane == 0) ch.exit[1 - b][g] = ein;
        return;
    }
    WaveWalker w{st, fp, cand, tab, st.ptrs[si], st.lens[si], st.span_base[si], lane};
    const uint64_t seg_end = min(off + (1ull << st.span_log2), w.n);
    const int wb = ch.which[g];
    uint32_t cnt;
    const uint64_t ex = rewalk(w, e, seg_end, ch.starts[wb] + g * ch.smax, ch.nstarts[wb][g], ein,
                               ch.starts[1 - wb] + g * ch.smax, cnt);
    if (lane == 0) {
        ch.nstarts[1 - wb][g] = cnt;
        ch.which[g] = (uint8_t)(1 - wb);
        ch.entry[g] = e;
        ch.exit[1 - b][g] = ex;
        if (ex != ein) atomicOr(&flag[iter % 3], 1u);
    }
}

// Serial catch-up, one wave per stream, after the Jacobi passes: a no-op
// unless the last pass still changed an exit (chains that do not merge within
// a span, e.g. long runs of max-length cuts in constant data).  Then it walks
// the stream's spans in order, re-walking only spans whose entry is stale:
// exact in one pass, O(stale chunks) steps.
__global__ __launch_bounds__(kResolveThreads) void serial_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const Chains ch, int buf, int slot, uint64_t *stats) {
    __shared__ uint64_t tab[256];
    if (ch.changed[slot] == 0) return;
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * kResolveWaves + (threadIdx.x >> 6);
    if (i >= st.n) return;
    if (i == 0 && lane == 0) stats[3] = 1;
    const uint64_t g0 = st.span_base[i], g1 = st.span_base[i + 1];
    if (g1 - g0 < 2) return;
    WaveWalker w{st, fp, cand, tab, st.ptrs[i], st.lens[i], g0, lane};
    uint64_t prev = ch.exit[buf][g0];
    for (uint64_t g = g0 + 1; g < g1; ++g) {
        if (prev == ch.entry[g]) {
            prev = ch.exit[buf][g];
            continue;
        }
        const uint64_t off = (g - g0) << st.span_log2;
        const uint64_t seg_end = min(off + (1ull << st.span_log2), w.n);
        const int wb = ch.which[g];
        uint32_t cnt;
        const uint64_t ex = rewalk(w, prev, seg_end, ch.starts[wb] + g * ch.smax, ch.nstarts[wb][g],
                                   ch.exit[buf][g], ch.starts[1 - wb] + g * ch.smax, cnt);
        if (lane == 0) {
            ch.nstarts[1 - wb][g] = cnt;
            ch.which[g] = (uint8_t)(1 - wb);
            ch.entry[g] = prev;
            ch.exit[buf][g] = ex;
        }
        prev = ex;
    }
}

// ---------------------------------------------------------------------------
// Compaction: exclusive scan of per-span chunk counts (1024 per block).

constexpr int kScanBlock = 1024;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *sm,
                                                    uint64_t &total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl += t;
    }
    if (lane == 63) sm[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        const uint32_t nw = blockDim.x >> 6;
        const uint64_t x = lane < nw ? sm[lane] : 0;
        uint64_t xi = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t t = __shfl_up(xi, d);
            if (lane >= (uint32_t)d) xi += t;
        }
        if (lane < nw) sm[lane] = xi - x;
        if (lane == 63) sm[16] = xi;
    }
    __syncthreads();
    const uint64_t r = sm[wave] + incl - v;
    total = sm[16];
    __syncthreads();
    return r;
}

// Per span: chunk count -> block-local exclusive prefix (chunk_index) and
// per-block sums; also the candidate / overflow statistics.
__global__ __launch_bounds__(kScanBlock) void count_kernel(
    const StreamTable st, const Chains ch, const Candidates cand, const Compact cp) {
    __shared__ uint64_t sm[17];
    const uint64_t g = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
    uint64_t c = 0, nc = 0, ov = 0;
    if (g < st.total_spans) {
        c = ch.nstarts[ch.which[g]][g];
        const uint32_t k = cand.count[g];
        nc = k;
        ov = k > cand.cap;
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan(c, sm, tot);
    if (g < st.total_spans) cp.chunk_index[g] = ex;
    if (threadIdx.x == 0) cp.block_sums[blockIdx.x] = tot;
    uint64_t tnc, tov;
    block_excl_scan(nc, sm, tnc);
    block_excl_scan(ov, sm, tov);
    if (threadIdx.x == 0) {
        atomicAdd((unsigned long long *)&cp.stats[0], (unsigned long long)tnc);
        atomicAdd((unsigned long long *)&cp.stats[1], (unsigned long long)tov);
    }
}

__global__ __launch_bounds__(kScanBlock) void block_sums_kernel(uint64_t *bs, uint64_t nb) {
    __shared__ uint64_t sm[17];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += kScanBlock) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? bs[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan(v, sm, tot);
        if (i < nb) bs[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) bs[nb] = carry;
}

// One wave per span: lane k writes Chunk{offset,length} k of the span
// (coalesced 16-byte stores), plus first[stream] for a stream's first span and
// first[n] = total for the last span.  Zero-length streams own no span; the
// host fills their first[] entries.
__global__ __launch_bounds__(kResolveThreads) void write_kernel(
    const StreamTable st, const Chains ch, int eb, const Compact cp, cdc_chunk_pod *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * kResolveWaves + (threadIdx.x >> 6);
    if (g >= st.total_spans) return;
    const int w = ch.which[g];
    const uint32_t c = ch.nstarts[w][g];
    const uint64_t idx = cp.block_sums[g / kScanBlock] + cp.chunk_index[g];
    const uint64_t *list = ch.starts[w] + g * ch.smax;
    const uint64_t ex = ch.exit[eb][g];
    for (uint32_t k = lane; k < c; k += 64) {
        const uint64_t s = list[k];
        const uint64_t nx = k + 1 < c ? list[k + 1] : ex;
        out[idx + k] = cdc_chunk_pod{s, nx - s};
    }
    if (lane == 0) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        if (off == 0) cp.first[si] = idx;
        if (g + 1 == st.total_spans) cp.first[st.n] = idx + c;
    }
}

}  // namespace

hipError_t launch_scan(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       int num_cus, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t groups = (st.total_spans + kScanWaves - 1) / kScanWaves;
    const uint64_t cap = (uint64_t)num_cus * (kScanMinWaves * 4 / kScanWaves);
    const unsigned grid = (unsigned)(groups < cap ? groups : cap);
    if (fp.cm_align)
        scan_kernel<true><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand);
    else
        scan_kernel<false><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand);
    return hipGetLastError();
}

hipError_t launch_spec(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       const Chains &ch, uint64_t *stats, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + kResolveWaves - 1) / kResolveWaves);
    spec_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand, ch, stats);
    return hipGetLastError();
}

hipError_t launch_trunc(const StreamTable &st, const FastParams &fp,
                        const uint64_t *d_gear, const Candidates &cand, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + kResolveWaves - 1) / kResolveWaves);
    trunc_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand);
    return hipGetLastError();
}

hipError_t launch_fixup(const StreamTable &st, const FastParams &fp,
                        const uint64_t *d_gear, const Candidates &cand,
                        const Chains &ch, int iter, uint64_t *stats, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + kResolveWaves - 1) / kResolveWaves);
    fixup_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand, ch, iter, stats);
    return hipGetLastError();
}

hipError_t launch_serial(const StreamTable &st, const FastParams &fp,
                         const uint64_t *d_gear, const Candidates &cand,
                         const Chains &ch, int buf, int slot, uint64_t *stats, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (st.n + kResolveWaves - 1) / kResolveWaves;
    serial_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand, ch, buf, slot, stats);
    return hipGetLastError();
}

hipError_t launch_compact(const StreamTable &st, const Chains &ch, int exit_buf,
                          const Candidates &cand, const Compact &cp,
                          void *d_out, hipStream_t s) {
    const uint64_t nb = (st.total_spans + kScanBlock - 1) / kScanBlock;
    if (!nb) return hipSuccess;
    count_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(st, ch, cand, cp);
    block_sums_kernel<<<1, kScanBlock, 0, s>>>(cp.block_sums, nb);
    write_kernel<<<(unsigned)((st.total_spans + kResolveWaves - 1) / kResolveWaves), kResolveThreads, 0, s>>>(
        st, ch, exit_buf, cp, reinterpret_cast<cdc_chunk_pod *>(d_out));
    return hipGetLastError();
}

}  // namespace v1
}  // namespace cdc
