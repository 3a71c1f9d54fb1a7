// cdc_kernels.hip -- hand-written gfx950 (CDNA4) kernels for FastCDC v2020.
//
// The reference computes cut points one chunk at a time with a byte loop
// (fastcdc 3.1.0 `cut_gear`, called from chunkfs src/chunkers/fast.rs:37;
// restated in SURVEY.md Appendix A.2 and oracle/cdc_oracle.c).  That loop is
// sequential: each cut depends on the previous one through the min-skip and
// the hash reset.  The GPU decomposition (DESIGN.md "Pipeline and kernels"):
//
//  1. scan_kernel    (the HBM pass): for EVERY position i the windowed gear
//     hash W_i (bits 0..47 exact -- the masks never test bit 48 or above),
//     and a candidate record when (W_i & (mask_s & mask_l)) == 0.  One
//     wavefront per span, 64 contiguous bytes per lane per 4 KiB
//     wave-iteration, one DPP shift carries the hash across lanes; GEAR in
//     LDS as 32 bank-disjoint replicas.
//  2. next_kernel    (lane per candidate record): where the chunk after one
//     that starts at the record begins -- the truncated positions after
//     start+min checked exactly, then the first qualifying record.
//  3. walk_kernel    (lane per span, ticket order): the chain walk over those
//     links, in-wave consistency, decoupled look-back across waves for the
//     true entry and the output index, Chunk{offset,length} output.
#include <type_traits>

#include "cdc_kernels.hpp"

namespace cdc {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kCopies = 32;           // GEAR replicas, one bank pair per lane&31
// One block of 16 waves per CU = 4 waves/SIMD: up to 128 VGPRs, room for two
// groups of 8 GEAR lookups in flight per wave (latency hidden inside the wave).
constexpr int kScanMinWaves = 4;
constexpr uint32_t kEntCap = 64;      // per-wave LDS list of hitting 16-byte quarters per span
// Candidate record: offset in span (spans <= 16 MiB) | exact mask hit flags.
constexpr uint32_t kCandPosMask = 0x00FFFFFFu;
constexpr uint32_t kCandHitL = 1u << 30;
constexpr uint32_t kCandHitS = 1u << 31;

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

constexpr uint32_t kLineBytes = 128;  // one cache line per lane-iteration
constexpr uint32_t kFastIters = 8;    // 64 KiB spans: 1 KiB per lane = 8 lines

struct Line128 {
    uint4 q[8];
};

__device__ __forceinline__ Line128 ld128(g_u32x4 *p) {
    Line128 d;
#pragma unroll
    for (int i = 0; i < 8; ++i) d.q[i] = ld16(p + i);
    return d;
}

__device__ __forceinline__ Data64 ld64(g_u32x4 *p) {
    Data64 d;
#pragma unroll
    for (int i = 0; i < 4; ++i) d.q[i] = ld16(p + i);
    return d;
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int w) {
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}

#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// Eight GEAR lookups (bytes 0..3 of w0, then of w1) kept in registers so the
// next group's LDS reads overlap this group's chain.
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

// One-pass gear candidate scan.  Layout: one wavefront per span; lane l owns
// the contiguous sub-span [l*sub, (l+1)*sub) (sub = span/64 >= 1 KiB) and
// walks it 128 bytes (one full cache line, eight 16-byte loads) per
// iteration, so the hash simply carries along the lane: 1 hash step per byte
// plus a 48-byte warm-up per sub-span (the windowed hash depends only on the
// last 48 bytes).  Every position is tested against (h & cmask) == 0, the
// result min-accumulated per 16-byte quarter.  A hitting quarter only appends
// (position, hash before the quarter) to a per-wave LDS list; exact
// mask_s/mask_l flags, position order and the HBM write happen once per span
// in the flush.
template <bool kAlign>
__global__ __launch_bounds__(kScanThreads, kScanMinWaves) void scan_kernel(
    const StreamTable st, const FastParams fp,
    const uint64_t *__restrict__ gear, const Candidates cand, const Lookback lb) {
    __shared__ uint64_t tab[256 * kCopies];  // 64 KiB: entry e, replica c at e*32+c
    __shared__ uint32_t epos[kScanWaves][kEntCap];
    __shared__ uint32_t ehlo[kScanWaves][kEntCap];
    __shared__ uint32_t ehhi[kScanWaves][kEntCap];
    __shared__ uint32_t ecnt[kScanWaves][kEntCap];
    for (int i = threadIdx.x; i < 256 * kCopies; i += kScanThreads)
        tab[i] = gear[i / kCopies] << fp.tshift;  // pre-shifted GEAR (see FastParams)
    if (blockIdx.x == 0 && threadIdx.x < 4) {  // reset the resolve's look-back state
        lb.stats[threadIdx.x] = 0;
        if (threadIdx.x < 2) lb.ticket[threadIdx.x] = 0;
    }
    __syncthreads();

    const char *tabb = reinterpret_cast<const char *>(tab);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t rep2 = (lane & 31) * 8;  // this lane's GEAR replica
    const uint64_t span = 1ull << st.span_log2;
    const uint64_t lanemask_lt = (1ull << lane) - 1;
    const uint32_t sub_log2 = st.span_log2 - 6;
    const uint32_t sub = 1u << sub_log2;      // bytes per lane per span
    const uint32_t iters = sub / kLineBytes;  // >= 8, a power of two
    const uint32_t lo = lane << sub_log2;     // lane's first byte in the span

    for (uint64_t g = (uint64_t)blockIdx.x * kScanWaves + wave; g < st.total_spans;
         g += (uint64_t)gridDim.x * kScanWaves) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        const uint8_t *base = st.ptrs[si] + off;
        const uint64_t n_left = st.lens[si] - off;
        const uint32_t span_len = (uint32_t)(n_left < span ? n_left : span);
        if (lane == 0) {
            lb.desc[g] = 0;
            lb.ent[g] = 0;
        }

        // Warm-up: the true hash just before the lane's first byte is the
        // hash of the 48 bytes before it (zero at the stream start).
        uint64_t h = 0;
        const bool warm = off + lo != 0 && lo < span_len;
        auto warm_up = [&](const Data64 &w) {  // w = the 64 bytes before lo; 16..63 used
            G8 ga, gb;
            look8(ga, tabb, rep2, w.q[1].x, w.q[1].y);
            SCHED_FENCE();
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint4 &v = w.q[1 + ((k + 1) >> 1)];
                if (k & 1) look8(ga, tabb, rep2, v.x, v.y); else look8(gb, tabb, rep2, v.z, v.w);
                SCHED_FENCE();
                chain8(h, (k & 1) ? gb : ga);
                SCHED_FENCE();
            }
            chain8(h, gb);
            SCHED_FENCE();
        };

        uint32_t ne = 0;  // quarter entries appended this span (wave-uniform)

        // One 128-byte line of the lane: 16 groups of 8 lookups, software-
        // pipelined so the LDS reads of group i+1 overlap group i's chain.
        auto process = [&](const Line128 &d, uint32_t pos0, uint32_t qvalid) {
            G8 ga, gb;
            look8(ga, tabb, rep2, d.q[0].x, d.q[0].y);
            SCHED_FENCE();
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint64_t h0 = h;  // hash before the quarter (for the flush)
                uint32_t acc = 0xffffffffu;
                look8(gb, tabb, rep2, d.q[q].z, d.q[q].w);
                SCHED_FENCE();
                chain8_test<kAlign>(h, acc, ga, fp);
                SCHED_FENCE();
                if (q < 7) {
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

        g_u32x4 *vb = as_global4(base + lo);
        if (span_len == span && iters == kFastIters) {
            // Full 64 KiB span (sub = 1 KiB): fully unrolled, so every load
            // and wait is static.  Warm-up bytes first, then two lines in
            // flight; each line buffer is refilled right after use (the same
            // registers: no loop-carried copies of in-flight loads).
            Data64 w{};
            if (warm) w = ld64(as_global4(base + lo - 64));
            __builtin_amdgcn_sched_barrier(0);
            Line128 A = ld128(vb);
            __builtin_amdgcn_sched_barrier(0);
            Line128 B = ld128(vb + 8);
            __builtin_amdgcn_sched_barrier(0);
            if (warm) warm_up(w);
#pragma unroll
            for (uint32_t it = 0; it < kFastIters; it += 2) {
                process(A, lo + it * kLineBytes, 0xFFu);
                if (it + 2 < kFastIters) A = ld128(vb + (it + 2) * 8);
                process(B, lo + (it + 1) * kLineBytes, 0xFFu);
                if (it + 3 < kFastIters) B = ld128(vb + (it + 3) * 8);
            }
        } else if (span_len == span) {
            if (warm) warm_up(ld64(as_global4(base + lo - 64)));
            for (uint32_t it = 0; it < iters; ++it) process(ld128(vb + it * 8), lo + it * kLineBytes, 0xFFu);
        } else {
            // Ragged last span of a stream: guarded loads, per-quarter validity.
            if (warm) warm_up(ld64(as_global4(base + lo - 64)));
            for (uint32_t it = 0; it < iters; ++it) {
                const uint32_t pos0 = lo + it * kLineBytes;
                Line128 d;
                uint32_t qvalid = 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t p = pos0 + 16 * q;
                    if (p < span_len) qvalid |= 1u << q;
                    d.q[q] = ld16_guarded(base, p, span_len);
                }
                process(d, pos0, qvalid);
            }
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
// Resolve: from candidate records to the exact FastCDC chunk chain.
//
// A chunk starting at s is cut at the first p in [s+a0, s+re) whose in-chunk
// hash (reset at s+a0) hits mask_s below the centre or mask_l above it, else
// at s+rem (max, or the end of the data).  The in-chunk hash equals the
// windowed one except at the <= 47 "truncated" positions s+a0 .. s+a0+46, so
// a cut is either found among those (evaluated exactly from the bytes) or is
// the first candidate record in [s+a0+47, s+re) with the right hit flag.
//
//  * next_kernel: for a chunk starting at EACH candidate record, the start of
//    the following chunk (and its record index when it is a record), one
//    lane per record, records of 4 spans packed per wave.  About 90% of
//    chunks start at a record, so the chain walk below mostly follows links.
//  * walk_kernel: one LANE per span, 64 spans per wave.  Each lane walks its
//    span's chain from a warm-up start 2*max before the span (exact when that
//    is the stream start) -- following links, computing the rare non-record
//    steps itself (lane_next), or, where a record list overflowed, with the
//    whole wave's help (coop_next).  Lanes whose entry disagrees with the
//    previous lane's exit re-walk from it until the wave is self-consistent;
//    across waves a decoupled look-back (desc/ent words, ticket order) finds
//    the true entry of lane 0 and the chunk index, then each lane writes its
//    Chunk{offset,length} records.

constexpr int kResolveThreads = 256;  // 4 waves
constexpr int kResolveWaves = kResolveThreads / 64;
constexpr uint32_t kTruncMax = 47;    // mask bits <= 47 (checked on the host)
constexpr int kNextSpans = 4;         // spans whose records one next_kernel wave packs
constexpr uint32_t kMaxCap = 256;     // Engine clamps the record capacity to <= 256
constexpr uint64_t kNoRec = ~0ull;

// nxt[g*cap+k], chunk starting at record k of span g:
//   bit 63 valid | bits 25..62 record index + 1 of the next start (0: not a
//   record) | bits 0..24 next start - record position (<= max <= 16 MiB).
constexpr uint64_t kNxtValid = 1ull << 63;
constexpr uint32_t kNxtDeltaBits = 25;
constexpr uint64_t kNxtDeltaMask = (1ull << kNxtDeltaBits) - 1;
constexpr uint64_t kNxtRecMask = (1ull << 38) - 1;

typedef const __attribute__((address_space(1))) uint32_t g_u32;

// Dword at byte offset `off` (4-aligned) of a stream of n bytes, zero past n.
__device__ __forceinline__ uint32_t ld4_guarded(const uint8_t *data, uint64_t off, uint64_t n) {
    if (off + 4 <= n) return *(g_u32 *)(data + off);
    uint32_t w = 0;
    g_u8 *gb = as_global1(data);
    for (uint64_t j = 0; off + j < n; ++j) w |= (uint32_t)gb[off + j] << (8 * j);
    return w;
}

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

__device__ __forceinline__ void load_tab1(uint64_t *tab, const uint64_t *gear) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = gear[i];
    __syncthreads();
}

struct Regime {
    uint64_t rem, a0, ce, re, tl;
};

// Chunk regime at start s: rem clipped to max, centre, and
// the even-rounded scan bounds; tl = end of the truncated positions.
__device__ __forceinline__ Regime regime(const FastParams &fp, uint64_t s, uint64_t n) {
    Regime R;
    uint64_t rem = n - s, center = fp.avg;
    if (rem > fp.max) rem = fp.max; else if (rem < center) center = rem;
    R.rem = rem;
    R.a0 = (fp.min / 2) * 2;
    R.ce = (center / 2) * 2;
    R.re = (rem / 2) * 2;
    R.tl = min(R.a0 + (uint64_t)fp.trunc, R.re);
    return R;
}

// First hitting offset p in [a0, tl) of the chunk starting at s (hash reset
// at s+a0), or ~0u.  Lane-level: the <= 52 bytes are staged in this thread's
// 13-dword LDS slot `wl`, then a predicated 47-step chain.
__device__ __forceinline__ uint32_t trunc_first(const uint8_t *data, uint64_t n, uint64_t s,
                                                const Regime &R, const FastParams &fp,
                                                const uint64_t *tab, uint32_t *wl) {
    const uint64_t w0 = s + R.a0, al = w0 & ~3ull;
    const uint32_t len = (uint32_t)(R.tl - R.a0);
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
    uint32_t t = ~0u;
#pragma unroll 8
    for (uint32_t d = 0; d < kTruncMax; ++d) {  // no early exit: the LDS reads pipeline
        h = shl1_add(h, tab[bytes[d]]);
        const bool hit = d < len && !(h & ((R.a0 + d) < R.ce ? fp.mask_s : fp.mask_l));
        t = hit ? min(t, d) : t;
    }
    return t;
}

// Start of the chunk after the one starting at s, lane-level and exact.
// *rec = global record index of that start (kNoRec: not a record).  Returns
// ~0ull when a record list it needs overflowed (caller: coop_next).
__device__ __noinline__ uint64_t lane_next(const StreamTable st, const FastParams fp,
                                           const Candidates cand, const uint64_t *tab, uint32_t *wl,
                                           const uint8_t *data, uint64_t n, uint64_t gbase,
                                           uint64_t s, uint64_t *rec) {
    *rec = kNoRec;
    if (n - s <= fp.min) return n;  // tail chunk
    const Regime R = regime(fp, s, n);
    if (R.tl > R.a0) {
        const uint32_t t = trunc_first(data, n, s, R, fp, tab, wl);
        if (t != ~0u) return s + R.a0 + t;
    }
    if (R.tl >= R.re) return s + R.rem;
    const uint64_t lo = s + R.tl, hi = s + R.re;
    for (uint64_t sp = lo >> st.span_log2; (sp << st.span_log2) < hi; ++sp) {
        const uint64_t g = gbase + sp;
        const uint32_t cnt = cand.count[g];
        if (cnt > cand.cap) return ~0ull;
        const uint32_t *P = cand.pos + g * cand.cap;
        const uint64_t sp0 = sp << st.span_log2;
        const uint32_t lo_rel = lo > sp0 ? (uint32_t)(lo - sp0) : 0u;
        uint32_t a = 0, b = cnt;  // first record at or after lo
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            if ((P[m] & kCandPosMask) < lo_rel) a = m + 1; else b = m;
        }
        for (uint32_t j = a; j < cnt; ++j) {
            const uint32_t r = P[j];
            const uint64_t c = sp0 + (r & kCandPosMask);
            if (c >= hi) return s + R.rem;
            if (r & ((c - s) < R.ce ? kCandHitS : kCandHitL)) {
                *rec = g * cand.cap + j;
                return c;
            }
        }
    }
    return s + R.rem;
}

// The same, wave-cooperative, from the bytes alone (64 positions per step:
// one coalesced byte load + a 6-step shuffle prefix scan).  For chains that
// cross an overflowed record list.  Wave-uniform arguments.
__device__ __noinline__ uint64_t coop_next(const FastParams fp, const uint64_t *tab,
                                           const uint8_t *data, uint64_t n, uint64_t s,
                                           uint32_t lane) {
    if (n - s <= fp.min) return n;
    const Regime R = regime(fp, s, n);
    uint64_t h = 0;
    for (uint64_t b = R.a0; b < R.re; b += 64) {
        const uint64_t p1 = min(b + 64, R.re);
        const uint64_t p = b + lane;
        const bool in = p < p1;
        const uint64_t gv = in ? tab[as_global1(data)[s + p]] : 0;
        const uint64_t x = gear_prefix(gv, lane) + ((h << lane) << 1);
        const bool hit = in && !(x & (p < R.ce ? fp.mask_s : fp.mask_l));
        const uint64_t m = __ballot(hit);
        if (m) return s + b + (uint64_t)(__ffsll((long long)m) - 1);
        h = __shfl(x, (int)(p1 - b - 1));
    }
    return s + R.rem;
}

// Links for chunks that start at candidate records: lane per record, the
// records of kNextSpans consecutive spans packed into each wave; searches use
// the records of those spans and the one after, staged in LDS.
__global__ __launch_bounds__(kResolveThreads) void next_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, uint64_t *__restrict__ nxt) {
    __shared__ uint64_t tab[256];
    __shared__ uint32_t srec[kResolveWaves][kNextSpans + 1][kMaxCap];
    __shared__ uint32_t win[kResolveThreads * 13];
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t G0 = ((uint64_t)blockIdx.x * kResolveWaves + wave) * kNextSpans;
    if (G0 >= st.total_spans) return;  // no block-level barrier below
    const uint64_t span = 1ull << st.span_log2;
    uint32_t cnt[kNextSpans + 1], ssi[kNextSpans + 1];
    uint64_t soff[kNextSpans + 1];
#pragma unroll
    for (int i = 0; i <= kNextSpans; ++i) {
        const uint64_t g = G0 + i;
        cnt[i] = 0;
        ssi[i] = ~0u;
        soff[i] = 0;
        if (g < st.total_spans) {
            locate(st, g, ssi[i], soff[i]);
            cnt[i] = cand.count[g];
            const uint32_t c = min(cnt[i], cand.cap);
            for (uint32_t k = lane; k < c; k += 64) srec[wave][i][k] = cand.pos[g * cand.cap + k];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t pre[kNextSpans + 1];
    pre[0] = 0;
#pragma unroll
    for (int i = 0; i < kNextSpans; ++i) pre[i + 1] = pre[i] + (cnt[i] <= cand.cap ? cnt[i] : 0u);
    uint32_t *wl = win + threadIdx.x * 13;
    for (uint32_t r0 = 0; r0 < pre[kNextSpans]; r0 += 64) {
        const uint32_t r = r0 + lane;
        const bool act = r < pre[kNextSpans];
        int i = 0;
#pragma unroll
        for (int j = 1; j < kNextSpans; ++j) i += r >= pre[j];
        const uint32_t k = r - pre[i];
        uint64_t val = 0;  // invalid: the walk computes this step itself
        uint64_t c = 0, lo = 0, hi = 0, ce = 0;
        bool search = false;
        const uint32_t si = ssi[i];
        if (act) {
            const uint64_t n = st.lens[si];
            c = soff[i] + (srec[wave][i][k] & kCandPosMask);
            if (n - c > fp.min) {
                const Regime R = regime(fp, c, n);
                const uint8_t *data = st.ptrs[si];
                const uint32_t t = R.tl > R.a0 ? trunc_first(data, n, c, R, fp, tab, wl) : ~0u;
                if (t != ~0u) {
                    val = kNxtValid | (R.a0 + t);
                } else if (R.tl >= R.re) {
                    val = kNxtValid | R.rem;
                } else {
                    search = true;
                    lo = c + R.tl;
                    hi = c + R.re;
                    ce = R.ce;
                    val = kNxtValid | R.rem;  // no qualifying record: cut at max / end
                }
            } else {
                val = kNxtValid | (n - c);  // tail chunk: next start is the end of the data
            }
        }
        // First qualifying record at or after lo: one uniform pass over the
        // staged records (LDS broadcast reads), each lane testing its window.
        bool done = !search;
#pragma unroll
        for (int j2 = 0; j2 <= kNextSpans; ++j2) {
            if (__ballot(!done) == 0) break;
            const bool mine = !done && ssi[j2] == si && soff[j2] < hi && soff[j2] + span > lo;
            if (cnt[j2] > cand.cap) {  // overflowed list in the window: leave it to the walk
                if (mine) {
                    val = 0;
                    done = true;
                }
                continue;
            }
            const uint32_t cj = cnt[j2];
            for (uint32_t j = 0; j < cj; ++j) {
                const uint32_t rr = srec[wave][j2][j];
                const uint64_t cc = soff[j2] + (rr & kCandPosMask);
                if (mine && !done && cc >= lo) {
                    if (cc >= hi) {
                        done = true;
                    } else if (rr & ((cc - c) < ce ? kCandHitS : kCandHitL)) {
                        val = kNxtValid | ((G0 + j2) * cand.cap + j + 1) << kNxtDeltaBits | (cc - c);
                        done = true;
                    }
                }
            }
        }
        if (act) nxt[(G0 + i) * cand.cap + k] = val;
    }
}

// ---- walk_kernel ----------------------------------------------------------
// Look-back words (one per WAVE of 64 spans, in lb.desc / lb.ent):
//   desc = status(62-63: 1 SPEC, 2 FINAL) | chunk count (25-61; FINAL:
//          inclusive) | exit - end of the wave's last span (0-24)
//   ent  = valid(63) | wave starts a stream(62) | lane 0's entry - its span start
// Each word carries its own status: single 64-bit relaxed agent-scope
// atomics, no fences between words.
constexpr uint64_t kDescSpec = 1ull << 62, kDescFinal = 2ull << 62;
constexpr uint32_t kDescExitBits = 25;  // exit - span end < max <= 16 MiB
constexpr uint64_t kDescExitMask = (1ull << kDescExitBits) - 1;
constexpr uint64_t kDescCntMask = (1ull << 37) - 1;
constexpr uint64_t kEntValid = 1ull << 63, kEntFirst = 1ull << 62;
constexpr uint64_t kEntRelMask = kEntFirst - 1;
// A look-back wait longer than this (100 MHz s_memrealtime ticks = 2 s) can
// only be a bug: the wave records it and leaves, so the grid always drains.
constexpr uint64_t kSpinTicks = 200000000ull;

__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) v += __shfl_xor(v, k);
    return v;
}

__device__ __forceinline__ uint64_t wave_excl_scan(uint64_t v, uint32_t lane) {
    uint64_t x = v;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint64_t t = __shfl_up(x, k);
        if (lane >= (uint32_t)k) x += t;
    }
    return x - v;
}

struct LaneSpan {
    bool act;            // lane holds a span
    bool first;          // span starts its stream
    uint32_t si;
    uint64_t off, seg_end, n, gbase;
    const uint8_t *data;
};

// Walk every lane with go=true from (s, r) to its span end, recording the
// chunk starts >= off in the span's list.  Wave-synchronous: steps a lane
// cannot take alone (overflowed record lists) are done by the whole wave.
__device__ void walk_lanes(const StreamTable &st, const FastParams &fp, const Candidates &cand,
                           const uint64_t *nxt, const uint64_t *tab, uint32_t *wl,
                           const LaneSpan &L, uint64_t *list, uint32_t smax, uint32_t lane,
                           bool go, uint64_t &s, uint64_t &r, uint32_t &cnt, uint64_t &entry) {
    cnt = 0;
    entry = s;
    go = go && s < L.seg_end;
    for (;;) {
        bool need = false;
        if (go) {
            if (s >= L.off) {
                if (cnt == 0) entry = s;
                if (cnt < smax) list[cnt] = s;
                ++cnt;
            }
            uint64_t v = 0;
            if (r != kNoRec) v = nxt[r];
            uint64_t ns, nr = kNoRec;
            if (v & kNxtValid) {
                ns = s + (v & kNxtDeltaMask);
                const uint64_t rr = (v >> kNxtDeltaBits) & kNxtRecMask;
                nr = rr ? rr - 1 : kNoRec;
            } else {
                ns = lane_next(st, fp, cand, tab, wl, L.data, L.n, L.gbase, s, &nr);
                need = ns == ~0ull;
            }
            if (!need) {
                s = ns;
                r = nr;
                go = s < L.seg_end;
            }
        }
        for (uint64_t m = __ballot(need); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const uint64_t sl = __shfl(s, l), nl = __shfl(L.n, l);
            const uint8_t *dl = reinterpret_cast<const uint8_t *>(
                __shfl(reinterpret_cast<uint64_t>(L.data), l));
            const uint64_t ns = coop_next(fp, tab, dl, nl, sl, lane);
            if ((int)lane == l) {
                s = ns;
                r = kNoRec;
                go = s < L.seg_end;
            }
        }
        if (__ballot(go) == 0) break;
    }
    if (cnt == 0) entry = s;
}

__global__ __launch_bounds__(kResolveThreads) void walk_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const uint64_t *__restrict__ nxt, const Chains ch,
    const Lookback lb, cdc_chunk_pod *out, uint64_t out_cap) {
    __shared__ uint64_t tab[256];
    __shared__ uint32_t win[kResolveThreads * 13];
    __shared__ uint32_t grp;
    __shared__ uint64_t sacc[kResolveWaves][4];
    if (threadIdx.x == 0) grp = atomicAdd(&lb.ticket[0], 1u);
    load_tab1(tab, gear);  // (its barrier also publishes grp)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)grp * kResolveWaves + wave;  // wave of spans 64w .. 64w+63
    const uint64_t nwaves = (st.total_spans + 63) / 64;
    uint32_t *wl = win + threadIdx.x * 13;
    uint64_t n_cand = 0, n_ovf = 0, n_re = 0, n_to = 0;
    if (w < nwaves) {
        const uint64_t g = w * 64 + lane;
        LaneSpan L{};
        L.act = g < st.total_spans;
        if (L.act) {
            locate(st, g, L.si, L.off);
            L.n = st.lens[L.si];
            L.data = st.ptrs[L.si];
            L.gbase = st.span_base[L.si];
            L.seg_end = min(L.off + (1ull << st.span_log2), L.n);
            L.first = L.off == 0;
            const uint32_t kc = cand.count[g];
            n_cand = kc <= cand.cap ? kc : 0;
            n_ovf = kc > cand.cap;
        }
        uint64_t *list = ch.starts[0] + g * ch.smax;

        // 1. Speculative walk from the warm-up start.
        const uint64_t warm = 2ull * fp.max;
        uint64_t s = L.off > warm ? L.off - warm : 0, r = kNoRec;
        uint32_t cnt;
        uint64_t entry;
        walk_lanes(st, fp, cand, nxt, tab, wl, L, list, ch.smax, lane, L.act, s, r, cnt, entry);
        uint64_t exit = s, xr = r;

        // 2. In-wave consistency: lane l's entry must be lane l-1's exit.
        //    Lane 0's predecessor is the previous wave's last lane; `pe0`
        //    is it once known (step 3), else lane 0 stands as walked.
        auto settle = [&](bool have0, uint64_t pe0) {
            for (;;) {
                uint64_t pe = __shfl_up(exit, 1), pr = __shfl_up(xr, 1);
                if (lane == 0) {
                    pe = pe0;
                    pr = kNoRec;
                }
                const bool stale = L.act && !L.first && (lane > 0 || have0) && entry != pe;
                if (__ballot(stale) == 0) break;
                uint64_t s2 = pe, r2 = pr;
                uint32_t c2;
                uint64_t e2;
                walk_lanes(st, fp, cand, nxt, tab, wl, L, list, ch.smax, lane, stale, s2, r2, c2, e2);
                if (stale) {
                    cnt = c2;
                    entry = e2;
                    exit = s2;
                    xr = r2;
                    n_re += 1;
                }
            }
        };
        settle(false, 0);

        // 3. Publish the wave's speculative summary, then look back.
        const uint32_t last = (uint32_t)min((uint64_t)63, st.total_spans - 1 - w * 64);
        auto publish = [&](uint64_t status, uint64_t count) {
            const uint64_t ex = __shfl(exit, (int)last), se = __shfl(L.seg_end, (int)last);
            if (lane == 0) st_agent(&lb.desc[w], status | (count << kDescExitBits) | (ex - se));
        };
        const bool first0 = __shfl((int)L.first, 0) != 0;
        const uint64_t my_ent = kEntValid | (first0 ? kEntFirst : 0) | (__shfl(entry, 0) - __shfl(L.off, 0));
        if (lane == 0) st_agent(&lb.ent[w], my_ent);
        publish(kDescSpec, wave_sum(L.act ? cnt : 0));

        uint64_t before = 0;
        bool own_stale = false;
        uint64_t pe0 = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        if (w > 0) {
            uint64_t acc = 0;
            int64_t base = (int64_t)w;
            for (;;) {
                // Lane k: predecessor wave p = base-1-k, its successor q = p+1.
                const int64_t p = base - 1 - (int64_t)lane;
                uint64_t d = kDescFinal, e = kEntValid | kEntFirst;  // before wave 0
                if (p >= 0) {
                    d = ld_agent(&lb.desc[p]);
                    e = p + 1 == (int64_t)w ? my_ent : ld_agent(&lb.ent[p + 1]);
                }
                const uint64_t stat = d & (3ull << 62);
                const bool avail = stat != 0 && (e & kEntValid);
                const bool cons = (e & kEntFirst) || (e & kEntRelMask) == (d & kDescExitMask);
                const uint64_t mfin = __ballot(stat == kDescFinal);
                const int kf = mfin ? __ffsll((long long)mfin) - 1 : 64;
                const uint64_t upto = kf >= 63 ? ~0ull : ((2ull << kf) - 1);  // lanes 0..kf
                const bool first_win = base == (int64_t)w;
                const uint64_t bad = __ballot(!cons) & upto;
                if ((__ballot(!avail) & upto) || (bad & (first_win ? ~1ull : ~0ull))) {
                    // a predecessor is unpublished or re-walking: wait for it
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
                        n_to = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                    acc = 0;
                    base = (int64_t)w;
                    own_stale = false;
                    continue;
                }
                if (first_win && (bad & 1)) {
                    own_stale = true;  // waves (j, w) are exact, so exit(w-1) is
                    pe0 = __shfl(L.off, 0) + (__shfl(d, 0) & kDescExitMask);
                }
                acc += wave_sum(lane < (uint32_t)kf ? (d >> kDescExitBits) & kDescCntMask : 0);
                if (kf < 64) {
                    before = acc + ((__shfl(d, kf) >> kDescExitBits) & kDescCntMask);
                    break;
                }
                base -= 64;
            }
        }
        if (!n_to) {
            if (own_stale) settle(true, pe0);
            const uint64_t c64 = L.act ? cnt : 0;
            const uint64_t excl = wave_excl_scan(c64, lane);
            const uint64_t total = wave_sum(c64);
            publish(kDescFinal, before + total);
            // 4. Output: this lane's chunks at their final index.
            const uint64_t base = before + excl;
            if (L.act) {
                const uint32_t c = cnt;
                if (base + c > out_cap || c > ch.smax) {
                    n_to = 1;  // impossible for a correct chain: report, never write out of bounds
                } else {
                    for (uint32_t k = 0; k < c; ++k) {
                        const uint64_t c0 = list[k];
                        const uint64_t nx = k + 1 < c ? list[k + 1] : exit;
                        out[base + k] = cdc_chunk_pod{c0, nx - c0};
                    }
                }
                if (L.first) lb.h_first[L.si] = base;
                if (g + 1 == st.total_spans) lb.h_first[st.n] = base + c;
            }
        }
    }
    // Statistics: one atomic per workgroup; the last group copies them to the host.
    n_cand = wave_sum(n_cand);
    n_ovf = wave_sum(n_ovf);
    n_re = wave_sum(n_re);
    if (lane == 0) {
        sacc[wave][0] = n_cand;
        sacc[wave][1] = n_ovf;
        sacc[wave][2] = n_re;
        sacc[wave][3] = n_to;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < 4; ++k) {
            uint64_t a = 0;
            for (int i = 0; i < kResolveWaves; ++i) a += sacc[i][k];
            if (a) atomicAdd((unsigned long long *)&lb.stats[k], (unsigned long long)a);
        }
        __threadfence();
        if (atomicAdd(&lb.ticket[1], 1u) + 1 == gridDim.x) {
            __threadfence();
            for (int i = 0; i < 4; ++i) lb.h_stats[i] = ld_agent(&lb.stats[i]);
        }
    }
}

// FSChunker::chunk_data (fixed_size.rs:32-43): chunk t of the batch.
__global__ void fixed_kernel(const StreamTable st, uint64_t cs,
                             const uint64_t *__restrict__ first,
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

}  // namespace

hipError_t launch_scan(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       const Lookback &lb, int num_cus, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t groups = (st.total_spans + kScanWaves - 1) / kScanWaves;
    // One resident wave of blocks (kScanMinWaves waves per SIMD, 4 SIMDs per
    // CU); the span loop inside the kernel is grid-strided.
    const uint64_t cap = (uint64_t)num_cus * (kScanMinWaves * 4 / kScanWaves);
    const unsigned grid = (unsigned)(groups < cap ? groups : cap);
    if (fp.cm_align)
        scan_kernel<true><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand, lb);
    else
        scan_kernel<false><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand, lb);
    return hipGetLastError();
}

hipError_t launch_next(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand, uint64_t *nxt,
                       hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t per_block = (uint64_t)kResolveWaves * kNextSpans;
    const unsigned grid = (unsigned)((st.total_spans + per_block - 1) / per_block);
    next_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand, nxt);
    return hipGetLastError();
}

hipError_t launch_resolve(const StreamTable &st, const FastParams &fp,
                          const uint64_t *d_gear, const Candidates &cand,
                          const uint64_t *nxt, const Chains &ch, const Lookback &lb,
                          void *d_out, uint64_t out_cap, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t nwaves = (st.total_spans + 63) / 64;
    const unsigned grid = (unsigned)((nwaves + kResolveWaves - 1) / kResolveWaves);
    walk_kernel<<<grid, kResolveThreads, 0, s>>>(st, fp, d_gear, cand, nxt, ch, lb,
                                                 reinterpret_cast<cdc_chunk_pod *>(d_out), out_cap);
    return hipGetLastError();
}

hipError_t launch_fixed(const StreamTable &st, uint64_t chunk_size,
                        const uint64_t *d_first, void *d_out, uint64_t total,
                        hipStream_t s) {
    if (!total) return hipSuccess;
    fixed_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
        st, chunk_size, d_first, reinterpret_cast<cdc_chunk_pod *>(d_out), total);
    return hipGetLastError();
}

hipError_t launch_fill_splitmix64(uint8_t *d_buf, uint64_t len, uint64_t seed,
                                  hipStream_t s) {
    if (!len) return hipSuccess;
    const uint64_t nw = len / 8 + 1;
    const uint64_t blocks = (nw + 255) / 256;
    fill_kernel<<<(unsigned)(blocks < 65536 ? blocks : 65536), 256, 0, s>>>(d_buf, len, seed);
    return hipGetLastError();
}

}  // namespace cdc
