// fastcdc.hip -- hand-written gfx950 (CDNA4) kernels for FastCDC v2020.
//
// The reference computes cut points one chunk at a time with a byte loop
// (fastcdc 3.1.0 `cut_gear`, called from chunkfs src/chunkers/fast.rs:37;
// restated in SURVEY.md Appendix A.2 and oracle/cdc_oracle.c).  Each cut
// depends on the previous one through the min-skip and the hash reset; the GPU
// splits the work into a data-parallel HBM pass and a small resolve:
//
//  scan_kernel    for EVERY position i the windowed gear hash W_i (bits
//                 0..47 exact: the masks never test bit 48 or above) and a
//                 candidate record where (W_i & (mask_s & mask_l)) == 0.
//                 Wave per span; lane l owns the contiguous 1 KiB segment
//                 [l*sub, (l+1)*sub) and hashes it serially (one v_lshl_add_u64
//                 per byte).  The bytes arrive with fully coalesced loads --
//                 each wave-instruction reads 16 complete 64-byte pieces --
//                 and are transposed to their owning lanes through a 4 KiB
//                 per-wave LDS tile (tools/ubench_scan.hip: lane-strided loads
//                 cap the read rate at 4.1 TB/s, grouped ones reach 6.0).
//                 A lane starts from hash 0 and re-tests its first 48
//                 positions at the end, with the true carry-in taken from
//                 lane l-1 by one DPP shift: no warm-up bytes are re-read.
//  chain_kernel   wave per span: the exact successor ("link") of every
//                 candidate record in reach, lane per record, then a chain
//                 walk over those links from a warm-up start before the span.
//  fix_kernel     Jacobi passes over 64-span blocks: spans whose speculative
//                 entry differs from their predecessor's exit are re-walked.
//  serial_kernel  the same, one wave over all blocks in order, only when the
//                 passes did not converge (degenerate data).
//  count/write    chunk-count prefix and the Chunk{offset,length} output.
#include "fastcdc.hpp"

#include <type_traits>

namespace cdc {
namespace p3 {
namespace {

// ---- common helpers --------------------------------------------------------

constexpr uint32_t kCandPosMask = 0x00FFFFFFu;
constexpr uint32_t kCandHitL = 1u << 30;
constexpr uint32_t kCandHitS = 1u << 31;

// Global (address space 1) views: generic pointers compile to flat_load_*,
// which count on both vmcnt and lgkmcnt and would drain the LDS pipeline.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ g_u32x4 *as_global4(const void *p) { return (g_u32x4 *)(p); }
__device__ __forceinline__ g_u8 *as_global1(const void *p) { return (g_u8 *)(p); }
__device__ __forceinline__ uint4 ld16(g_u32x4 *p) {
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Largest stream i with span_base[i] <= g (streams with zero spans skipped).
__device__ __forceinline__ void locate(const StreamTable &st, uint64_t g, uint32_t &si, uint64_t &off) {
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

// h = (h << 1) + g as ONE opaque v_lshl_add_u64: plain C lets LLVM
// reassociate the 48-term chain into a tree that keeps every lookup live.
__device__ __forceinline__ uint64_t shl1_add(uint64_t h, uint64_t g) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(h), "v"(g));
    return r;
}

// DPP wave_shr:1 (dpp_ctrl 0x138): lane i receives lane i-1; lane 0 keeps `fill`.
__device__ __forceinline__ uint64_t wave_shr1(uint64_t v, uint64_t fill) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(
        (int)(uint32_t)fill, (int)(uint32_t)v, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(
        (int)(uint32_t)(fill >> 32), (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
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

// ---- scan ------------------------------------------------------------------

constexpr int kScanThreads = 1024;    // 16 waves, one block per CU (LDS-bound)
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kCopies = 32;           // GEAR replicas: lane&31 picks a bank pair
constexpr uint32_t kEntCap = 64;      // per-wave list of hitting 16-byte quarters per span
constexpr uint32_t kStep = 64;        // bytes per lane per step (4 quarters)

// GEAR[byte b of word w] from the replicated LDS table: one v_perm_b32
// builds the byte address b*256 + replica*8, one ds_read_b64 fetches it.
// All helpers are force-inlined on the kernel's own __shared__ table (which
// sits at LDS address 0), so the address space and the zero base fold away.
__device__ __forceinline__ uint64_t gear_of(const uint64_t *tab, uint32_t rep_off, uint32_t w, int b) {
    const uint32_t addr = __builtin_amdgcn_perm(rep_off, w, 0x0c0c0004u | ((uint32_t)b << 8));
    return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + addr);
}

struct G4 {
    uint64_t v[4];
};

__device__ __forceinline__ void look4(G4 &g, const uint64_t *tab, uint32_t rep, uint32_t w) {
#pragma unroll
    for (int b = 0; b < 4; ++b) g.v[b] = gear_of(tab, rep, w, b);
}

template <bool kAlign>
__device__ __forceinline__ void chain4_test(uint64_t &h, uint32_t &acc, const G4 &g, const FastParams &fp) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h = shl1_add(h, g.v[i]);
        acc = min(acc, cand_test<kAlign>(h, fp));
    }
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int w) {
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}

__device__ __forceinline__ uint4 ld16_guarded(const uint8_t *base, uint32_t p, uint32_t limit) {
    if (p + 16 <= limit) return ld16(as_global4(base + p));
    uint32_t w[4] = {0, 0, 0, 0};
    if (p < limit) {
        g_u8 *gb = as_global1(base);
        for (uint32_t j = 0; p + j < limit; ++j) w[j >> 2] |= (uint32_t)gb[p + j] << (8 * j);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

struct EntryList {
    uint32_t *pos, *hlo, *hhi, *cnt;
};

// Append (quarter position, hash before the quarter) for every lane whose
// quarter hit; ne is wave-uniform.
__device__ __forceinline__ void append_hits(bool hit, uint32_t pos, uint64_t h0, uint32_t &ne,
                                            const EntryList &E) {
    const uint64_t m = __ballot(hit);
    if (m) {  // ~1 hitting quarter per 4 KiB at 12-bit masks
        if (hit) {
            // hitting lanes below this one (v_mbcnt: no lane-mask register)
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t slot = ne + below;
            if (slot < kEntCap) {
                E.pos[slot] = pos;
                E.hlo[slot] = (uint32_t)h0;
                E.hhi[slot] = (uint32_t)(h0 >> 32);
            }
        }
        ne += (uint32_t)__popcll(m);
    }
}

// 16 positions of one quarter, the lookups of each dword one dword ahead.
template <bool kAlign>
__device__ __forceinline__ uint32_t quarter(uint64_t &h, const uint4 &v, const uint64_t *tab, uint32_t rep,
                                            const FastParams &fp) {
    G4 ga, gb;
    uint32_t acc = 0xffffffffu;
    look4(ga, tab, rep, v.x);
    SCHED_FENCE();
    look4(gb, tab, rep, v.y);
    SCHED_FENCE();
    chain4_test<kAlign>(h, acc, ga, fp);
    SCHED_FENCE();
    look4(ga, tab, rep, v.z);
    SCHED_FENCE();
    chain4_test<kAlign>(h, acc, gb, fp);
    SCHED_FENCE();
    look4(gb, tab, rep, v.w);
    SCHED_FENCE();
    chain4_test<kAlign>(h, acc, ga, fp);
    SCHED_FENCE();
    chain4_test<kAlign>(h, acc, gb, fp);
    SCHED_FENCE();
    return acc;
}

// One 64-byte step of a lane (4 quarters in C), lookups one dword ahead of
// the chain across the whole step (8 VGPRs per group keeps the kernel
// within 128 VGPRs = 16 waves per CU; the other waves cover LDS latency).
// Quarters 0..skip-1 are left to the fix-up.
struct Q4 {
    uint4 q[4];
};

template <bool kAlign>
__device__ __forceinline__ void process_step(const Q4 &C, uint64_t &h, uint32_t pos0, uint32_t skip, uint32_t &ne,
                                             const EntryList &E, const uint64_t *tab, uint32_t rep,
                                             const FastParams &fp) {
    G4 ga, gb;
    look4(ga, tab, rep, C.q[0].x);
    SCHED_FENCE();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t h0 = h;
        uint32_t acc = 0xffffffffu;
#pragma unroll
        for (int w = 0; w < 4; w += 2) {
            look4(gb, tab, rep, word_of(C.q[q], w + 1));
            SCHED_FENCE();
            chain4_test<kAlign>(h, acc, ga, fp);
            SCHED_FENCE();
            if (q < 3 || w < 2) {
                look4(ga, tab, rep, w < 2 ? word_of(C.q[q], w + 2) : word_of(C.q[q + 1], 0));
                SCHED_FENCE();
            }
            chain4_test<kAlign>(h, acc, gb, fp);
            SCHED_FENCE();
        }
        append_hits(acc == 0 && (uint32_t)q >= skip, pos0 + 16 * q, h0, ne, E);
    }
}

// The 4 coalesced loads of step t: instruction i reads piece (lane%4) of the
// step of segment 16 i + lane/4 (16 complete 64-byte pieces per instruction).
__device__ __forceinline__ void gload_step(Q4 &X, const uint8_t *gp, uint64_t istride, uint32_t t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) X.q[i] = ld16(as_global4(gp + i * istride + t * kStep));
}

// Transpose through the wave's LDS tile: row o (80 bytes: 64 data + 16 pad)
// holds segment o's step.  Rows are 20 dwords apart, so both directions are
// bank-conflict free (ds_write_b128: 8 contiguous lanes = 2 rows x 64 B on
// 32 distinct banks; ds_read_b128: 16 lanes of distinct l mod 16 start 20 l
// mod 64 apart = 16 distinct 4-bank groups), and every address is a per-lane
// base plus an immediate.  LDS is in order per wave, so the reads see the
// writes and the next step's writes land after these reads; the barriers
// only keep the compiler from moving LDS traffic across them.
__device__ __forceinline__ void stage_step(Q4 &C, const Q4 &X, uint4 *wrow, const uint4 *rrow) {
#pragma unroll
    for (int i = 0; i < 4; ++i) wrow[i * 16 * 5] = X.q[i];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) C.q[k] = rrow[k];
    __builtin_amdgcn_wave_barrier();
}

// Flush of one span: exact mask_s / mask_l flags for each hitting quarter
// (re-hashed from the hash before it), position order, HBM write.
__device__ __forceinline__ void flush_span(uint64_t g, const uint8_t *base, uint32_t span_len, uint32_t ne,
                                           const EntryList &E, const uint64_t *tab, uint32_t rep,
                                           const FastParams &fp, const Candidates &cand, uint32_t lane) {
    wave_sync_lds();
    uint32_t *cpos = cand.pos + g * cand.cap;
    if (ne > kEntCap) {  // too many hits for the LDS list: resolve takes the exact slow path
        if (lane == 0) cand.count[g] = cand.cap + 1;
        wave_sync_lds();
        return;
    }
    uint32_t hs = 0, hl = 0, my_pos = 0;
    if (lane < ne) {
        my_pos = E.pos[lane];
        uint64_t hh = ((uint64_t)E.hhi[lane] << 32) | E.hlo[lane];
        const uint4 v = ld16_guarded(base, my_pos, span_len);
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * w + b;
                hh = (hh << 1) + gear_of(tab, rep, word_of(v, w), b);
                if (my_pos + j < span_len) {
                    hs |= (uint32_t)((hh & fp.mask_s_sh) == 0) << j;
                    hl |= (uint32_t)((hh & fp.mask_l_sh) == 0) << j;
                }
            }
        E.cnt[lane] = __popc(hs | hl);
    }
    wave_sync_lds();
    // Output slot = records of all entries at lower positions (entries are
    // few: a linear rank over the wave's LDS list).
    uint32_t slot = 0, total = 0;
    for (uint32_t k = 0; k < ne; ++k) {
        const uint32_t c = E.cnt[k];
        total += c;
        if (E.pos[k] < my_pos) slot += c;
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
    wave_sync_lds();
}

struct ScanLds {
    uint64_t tab[256 * kCopies];           // 64 KiB: entry e, replica c at e*32+c (LDS address 0)
    uint4 stage[kScanWaves][64 * 5];       // 80 KiB: per-wave transpose tile, 80-byte rows
    uint32_t epos[kScanWaves][kEntCap];    // 16 KiB: hitting quarters of the current span
    uint32_t ehlo[kScanWaves][kEntCap];
    uint32_t ehhi[kScanWaves][kEntCap];
    uint32_t ecnt[kScanWaves][kEntCap];
};

// Full spans.  Lane l owns the contiguous segment [l*sub, (l+1)*sub) and
// hashes it serially from hash 0; its first 48 positions are re-tested at the
// end with the true carry-in (lane l-1's final hash, one DPP shift; lane 0's
// from the 48 bytes before the span).  Ragged last spans: scan_tail_kernel.
template <bool kAlign>
__global__ __launch_bounds__(kScanThreads, 1) void scan_kernel(const StreamTable st, const FastParams fp,
                                                                const uint64_t *__restrict__ gear,
                                                                const Candidates cand, const Compact cp) {
    __shared__ ScanLds L;
    const uint64_t *tab = L.tab;
    for (int i = threadIdx.x; i < 256 * kCopies; i += kScanThreads)
        L.tab[i] = gear[i / kCopies] << fp.tshift;  // pre-shifted GEAR (see FastParams)
    if (blockIdx.x == 0 && threadIdx.x < kStatWords) cp.stats[threadIdx.x] = 0;  // later kernels accumulate
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t rep = (lane & 31) * 8;  // this lane's GEAR replica
    const uint64_t span = 1ull << st.span_log2;
    const uint32_t sub_log2 = st.span_log2 - 6;
    const uint32_t sub = 1u << sub_log2;   // bytes per lane per span (>= 1 KiB)
    const uint32_t steps = sub / kStep;    // >= 16, a power of two
    const uint32_t lo = lane << sub_log2;  // lane's first byte in the span
    const uint64_t istride = 16ull * sub;
    const EntryList E{L.epos[wave], L.ehlo[wave], L.ehhi[wave], L.ecnt[wave]};
    uint4 *wrow = &L.stage[wave][(lane >> 2) * 5 + (lane & 3)];
    const uint4 *rrow = &L.stage[wave][lane * 5];

    for (uint64_t g = (uint64_t)blockIdx.x * kScanWaves + wave; g < st.total_spans;
         g += (uint64_t)gridDim.x * kScanWaves) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        const uint8_t *base = st.ptrs[si] + off;
        if (st.lens[si] - off < span) continue;  // ragged last span: scan_tail_kernel
        uint32_t ne = 0;  // quarter entries appended this span (wave-uniform)
        uint64_t h = 0;
        // Lane 0's carry-in: the true hash of the 48 bytes before the span
        // (zero at a stream start), one byte per lane + a shuffle scan.
        uint32_t wb = 0;
        if (off != 0 && lane < 48) wb = as_global1(base)[(int)lane - 48];
        const uint8_t *gp = base + (uint64_t)(lane >> 2) * sub + (lane & 3) * 16;
        Q4 A, B, C;
        uint4 F0, F1, F2;
        // Two steps in flight while one is hashed (A/B ring).  The loop body
        // issues its loads unconditionally -- a conditional load leaves the
        // compiler unsure how many are outstanding at the back edge, and it
        // then waits for all of them -- so the last two steps are peeled.
        gload_step(A, gp, istride, 0);
        SCHED_FENCE();
        gload_step(B, gp, istride, 1);
        SCHED_FENCE();
        stage_step(C, A, wrow, rrow);
        F0 = C.q[0];
        F1 = C.q[1];
        F2 = C.q[2];
        gload_step(A, gp, istride, 2);
        SCHED_FENCE();
#define CDC_SCAN_PAIR(T, LOAD_B, STAGE_A, LOAD_A)                                   \
    do {                                                                            \
        process_step<kAlign>(C, h, lo + (T) * kStep, (T) == 0 ? 3u : 0u, ne, E, tab, rep, fp); \
        SCHED_FENCE();                                                              \
        stage_step(C, B, wrow, rrow);                                               \
        if (LOAD_B) gload_step(B, gp, istride, (T) + 3);                            \
        SCHED_FENCE();                                                              \
        process_step<kAlign>(C, h, lo + ((T) + 1) * kStep, 0u, ne, E, tab, rep, fp); \
        SCHED_FENCE();                                                              \
        if (STAGE_A) stage_step(C, A, wrow, rrow);                                  \
        if (LOAD_A) gload_step(A, gp, istride, (T) + 4);                            \
        SCHED_FENCE();                                                              \
    } while (0)
        uint32_t t = 0;
        for (; t + 4 < steps; t += 2) CDC_SCAN_PAIR(t, true, true, true);
        CDC_SCAN_PAIR(t, true, true, false);        // steps-4, steps-3
        CDC_SCAN_PAIR(t + 2, false, false, false);  // steps-2, steps-1
#undef CDC_SCAN_PAIR
        // Fix-up: re-test the first 48 positions with the true carry-in.
        const uint64_t gw = lane < 48 ? L.tab[wb * kCopies + (lane & 31)] : 0;
        const uint64_t hw = readlane_u64(gear_prefix(gw, lane), 47);  // hash of the 48 bytes before
        h = wave_shr1(h, off != 0 ? hw : 0);
        {
            uint64_t h0 = h;
            append_hits(quarter<kAlign>(h, F0, tab, rep, fp) == 0, lo, h0, ne, E);
            h0 = h;
            append_hits(quarter<kAlign>(h, F1, tab, rep, fp) == 0, lo + 16, h0, ne, E);
            h0 = h;
            append_hits(quarter<kAlign>(h, F2, tab, rep, fp) == 0, lo + 32, h0, ne, E);
        }
        flush_span(g, base, (uint32_t)span, ne, E, tab, rep, fp, cand, lane);
    }
}

// Ragged last spans of streams (length not a multiple of the span): one wave
// each, lane-contiguous guarded loads and a 48-byte warm-up from the bytes
// before the lane's segment.  tails[] lists their span ids.
template <bool kAlign>
__global__ __launch_bounds__(64) void scan_tail_kernel(const StreamTable st, const FastParams fp,
                                                       const uint64_t *__restrict__ gear, const Candidates cand,
                                                       const uint64_t *__restrict__ tails) {
    __shared__ uint64_t tab[256 * kCopies];
    __shared__ uint32_t e_pos[kEntCap], e_hlo[kEntCap], e_hhi[kEntCap], e_cnt[kEntCap];
    for (int i = threadIdx.x; i < 256 * kCopies; i += 64) tab[i] = gear[i / kCopies] << fp.tshift;
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    const uint32_t rep = (lane & 31) * 8;
    const uint64_t g = tails[blockIdx.x];
    const EntryList E{e_pos, e_hlo, e_hhi, e_cnt};
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint8_t *base = st.ptrs[si] + off;
    const uint32_t span_len = (uint32_t)(st.lens[si] - off);
    const uint32_t sub_log2 = st.span_log2 - 6;
    const uint32_t sub = 1u << sub_log2;
    const uint32_t lo = lane << sub_log2;
    uint32_t ne = 0;
    uint64_t h = 0;
    const bool active = lo < span_len;
    if (active && off + lo != 0) {
        (void)quarter<kAlign>(h, ld16(as_global4(base + lo - 48)), tab, rep, fp);
        (void)quarter<kAlign>(h, ld16(as_global4(base + lo - 32)), tab, rep, fp);
        (void)quarter<kAlign>(h, ld16(as_global4(base + lo - 16)), tab, rep, fp);
    }
    for (uint32_t it = 0; it < sub / 16; ++it) {
        const uint32_t p = lo + 16 * it;
        bool hit = false;
        const uint64_t h0 = h;
        if (active && p < span_len) hit = quarter<kAlign>(h, ld16_guarded(base, p, span_len), tab, rep, fp) == 0;
        append_hits(hit, p, h0, ne, E);
    }
    flush_span(g, base, span_len, ne, E, tab, rep, fp, cand, lane);
}


// ---- resolve ---------------------------------------------------------------
//
// A chunk starting at s is cut at the first p in [s+a0, s+re) whose in-chunk
// hash (reset at s+a0) hits mask_s below the centre or mask_l above it, else
// at s+rem (max, or the end of the data); p itself starts the next chunk
// (SURVEY.md A.2).  The in-chunk hash equals the windowed one except at the
// <= 47 "truncated" positions s+a0 .. s+a0+46, which are tested exactly from
// the bytes; every later position comes from the scan's records.

constexpr int kResThreads = 256;      // 4 waves, one span (or one 64-span block) each
constexpr int kResWaves = kResThreads / 64;
constexpr uint32_t kMaxCap = 256;     // Engine clamps the record capacity to <= 256
constexpr uint32_t kTruncMax = 47;    // mask bits <= 47 (checked on the host)
constexpr uint32_t kNoRec = 0;        // window record index + 1; 0 = not a record

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

// Dword at byte offset `off` (4-aligned) of a stream of n bytes, zero past n.
__device__ __forceinline__ uint32_t ld4_guarded(const uint8_t *data, uint64_t off, uint64_t n) {
    if (off + 4 <= n) return *(g_u32 *)(data + off);
    uint32_t w = 0;
    g_u8 *gb = as_global1(data);
    for (uint64_t j = 0; off + j < n; ++j) w |= (uint32_t)gb[off + j] << (8 * j);
    return w;
}

// First hitting offset d in [0, tl-a0) of the truncated positions of the
// chunk starting at s, or ~0u.  Lane-level: the <= 52 bytes are staged in
// this thread's 13-dword LDS slot `wl`, then a predicated 47-step chain.
__device__ __forceinline__ uint32_t trunc_first(const uint8_t *data, uint64_t n, uint64_t s, const Regime &R,
                                                const FastParams &fp, const uint64_t *tab, uint32_t *wl) {
    const uint64_t w0 = s + R.a0, al = w0 & ~3ull;
    const uint32_t len = (uint32_t)(R.tl - R.a0);
    uint32_t w[13];
    if (al + 52 <= n) {
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

// Exact next start from the bytes alone, wave-cooperative (64 positions per
// step: one coalesced byte load + a 6-step shuffle prefix scan).  For chains
// that cross an overflowed record list.  Wave-uniform arguments.
__device__ __noinline__ uint64_t coop_next_bytes(const FastParams fp, const uint64_t *tab, const uint8_t *data,
                                                 uint64_t n, uint64_t s, uint32_t lane) {
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

// Per-wave LDS of the chain walk: the records of spans g-1, g, g+1 (window
// slots 0, 1, 2; in position order slot by slot) and the links of the
// records of slots 0 and 1.
struct WaveWin {
    uint32_t rec[3 * kMaxCap];
    uint32_t link[2 * kMaxCap];   // next start - record position (<= max <= 16 MiB)
    uint16_t lrec[2 * kMaxCap];   // window record index + 1 of the next start, 0: none
    uint16_t lok[2 * kMaxCap];    // 1: link computed
};

struct SpanCtx {
    uint64_t g, off, n, span, span_end;
    uint32_t si, cap;
    const uint8_t *data;
    uint32_t cnt[3];    // records per slot (0 when the slot is outside the stream)
    uint64_t soff[3];   // stream offset of each slot's span
    bool ovf;           // a needed record list overflowed
};

__device__ __forceinline__ uint64_t win_pos(const SpanCtx &C, const WaveWin &W, uint32_t w) {
    const uint32_t slot = w / C.cap;
    return C.soff[slot] + (W.rec[w] & kCandPosMask);
}

// Window index + 1 of the record at stream offset p, 0 if none (binary
// search per slot; records are position-sorted).
__device__ __forceinline__ uint32_t win_lookup(const SpanCtx &C, const WaveWin &W, uint64_t p) {
#pragma unroll
    for (uint32_t slot = 0; slot < 3; ++slot) {
        if (p < C.soff[slot] || p >= C.soff[slot] + C.span || C.cnt[slot] == 0) continue;
        const uint32_t rel = (uint32_t)(p - C.soff[slot]);
        const uint32_t *P = W.rec + slot * C.cap;
        uint32_t a = 0, b = C.cnt[slot];
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            if ((P[m] & kCandPosMask) < rel) a = m + 1; else b = m;
        }
        if (a < C.cnt[slot] && (P[a] & kCandPosMask) == rel) return slot * C.cap + a + 1;
        return kNoRec;
    }
    return kNoRec;
}

// First window index whose record position is >= p (3*cap if none).
__device__ __forceinline__ uint32_t win_first_from(const SpanCtx &C, const WaveWin &W, uint64_t p) {
    for (uint32_t slot = 0; slot < 3; ++slot) {
        if (p >= C.soff[slot] + C.span) continue;  // (slot 0 at off 0 wraps to 0: skipped)
        const uint32_t rel = p > C.soff[slot] ? (uint32_t)(p - C.soff[slot]) : 0u;
        const uint32_t *P = W.rec + slot * C.cap;
        uint32_t a = 0, b = C.cnt[slot];
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            if ((P[m] & kCandPosMask) < rel) a = m + 1; else b = m;
        }
        if (a < C.cnt[slot]) return slot * C.cap + a;
    }
    return 3 * C.cap;
}

// Next start after a chunk starting at s, lane-level, from the truncated
// bytes and the window records.  *wr = window index + 1 of the result when it
// is a record.  `first_w` = the first window index whose record position is
// >= s (search starts there).
__device__ uint64_t lane_next(const SpanCtx &C, const WaveWin &W, const FastParams &fp, const uint64_t *tab,
                              uint32_t *wl, uint64_t s, uint32_t first_w, uint32_t *wr) {
    *wr = kNoRec;
    if (C.n - s <= fp.min) return C.n;  // tail chunk
    const Regime R = regime(fp, s, C.n);
    uint64_t nx = s + R.rem;
    bool found = false;
    if (R.tl > R.a0) {
        const uint32_t t = trunc_first(C.data, C.n, s, R, fp, tab, wl);
        if (t != ~0u) {
            nx = s + R.a0 + t;
            found = true;
        }
    }
    if (!found && R.tl < R.re) {
        const uint64_t lo = s + R.tl, hi = s + R.re;
        for (uint32_t slot = first_w / C.cap; slot < 3 && !found; ++slot) {
            const uint32_t k0 = slot == first_w / C.cap ? first_w % C.cap : 0;
            for (uint32_t k = k0; k < C.cnt[slot]; ++k) {
                const uint32_t r = W.rec[slot * C.cap + k];
                const uint64_t c = C.soff[slot] + (r & kCandPosMask);
                if (c >= hi) {
                    found = true;  // no qualifying record: cut at max / end
                    break;
                }
                if (c < lo) continue;
                if (r & ((c - s) < R.ce ? kCandHitS : kCandHitL)) {
                    nx = c;
                    *wr = slot * C.cap + k + 1;
                    found = true;
                    break;
                }
            }
        }
    }
    if (*wr == kNoRec && nx < C.span_end) *wr = win_lookup(C, W, nx);
    return nx;
}

// Load the window (slots of spans g-1 .. g+1 that lie in g's stream).
__device__ void load_window(SpanCtx &C, WaveWin &W, const StreamTable &st, const Candidates &cand,
                            bool need_prev, uint32_t lane) {
    C.ovf = false;
#pragma unroll
    for (int slot = 0; slot < 3; ++slot) {
        C.cnt[slot] = 0;
        C.soff[slot] = C.off + (uint64_t)slot * C.span - C.span;  // wraps for slot 0 at off 0: unused then
        const bool in = slot == 1 || (slot == 0 && need_prev && C.off != 0) ||
                        (slot == 2 && C.off + C.span < C.n);
        if (!in) continue;
        const uint64_t gs = C.g + slot - 1;
        const uint32_t c = cand.count[gs];
        if (c > cand.cap) {
            C.ovf = true;
            continue;
        }
        C.cnt[slot] = c;
        for (uint32_t k = lane; k < c; k += 64) W.rec[slot * C.cap + k] = cand.pos[gs * cand.cap + k];
    }
    wave_sync_lds();
}

// Walk span g's chain from start w0 (a true start when `exact`, else a
// warm-up guess): links of every record in [w0, span_end) lane-parallel,
// then the walk.  Writes the span's starts; returns (cnt, entry, exit).
__device__ void walk_span(SpanCtx &C, WaveWin &W, const FastParams &fp, const uint64_t *tab, uint32_t *wl,
                          const Chains &ch, uint64_t w0, uint32_t lane, uint32_t &cnt_out, uint64_t &entry,
                          uint64_t &exit) {
    uint64_t *list = ch.starts + C.g * ch.smax;
    uint32_t cnt = 0;
    uint64_t s = w0;
    entry = ~0ull;
    if (C.ovf) {
        // Exact byte-level walk (degenerate data: a record list overflowed).
        while (s < C.span_end) {
            if (s >= C.off) {
                if (cnt < ch.smax && lane == 0) list[cnt] = s;
                if (cnt == 0) entry = s;
                ++cnt;
            }
            s = coop_next_bytes(fp, tab, C.data, C.n, s, lane);
        }
    } else {
        // 1. Links for every record in [w0, span_end): lane per record.
        const uint32_t nw = C.cap + C.cnt[1];  // slots 0 and 1 (slot 0 padded to cap)
        for (uint32_t w = lane; w < 2 * C.cap; w += 64) W.lok[w] = 0;
        wave_sync_lds();
        for (uint32_t w = lane; w < nw; w += 64) {
            bool act = w < nw && (w >= C.cap || w < C.cnt[0]);
            uint64_t c = 0;
            if (act) {
                c = win_pos(C, W, w);
                act = c >= w0 && c < C.span_end;
            }
            if (act) {
                uint32_t wr;
                const uint64_t nx = lane_next(C, W, fp, tab, wl, c, w + 1, &wr);
                W.link[w] = (uint32_t)(nx - c);
                W.lrec[w] = (uint16_t)wr;
                W.lok[w] = 1;
            }
        }
        wave_sync_lds();
        // 2. The walk (wave-uniform): links where the start is a record,
        //    lane 0 computes the rare other steps (after a max cut or a
        //    truncated hit) and broadcasts them.
        uint32_t wr = win_lookup(C, W, s);
        while (s < C.span_end) {
            if (s >= C.off) {
                if (cnt < ch.smax && lane == 0) list[cnt] = s;
                if (cnt == 0) entry = s;
                ++cnt;
            }
            if (wr != kNoRec && wr - 1 < 2 * C.cap && W.lok[wr - 1]) {
                const uint32_t k = wr - 1;
                s += W.link[k];
                wr = W.lrec[k];
            } else {
                uint64_t nx = 0;
                uint32_t nwr = 0;
                if (lane == 0) {
                    const uint32_t fw = win_first_from(C, W, s);
                    nx = lane_next(C, W, fp, tab, wl, s, fw, &nwr);
                }
                s = readlane_u64(nx, 0);
                wr = (uint32_t)__builtin_amdgcn_readlane((int)nwr, 0);
            }
        }
    }
    if (cnt == 0) entry = s;
    cnt_out = cnt;
    exit = s;
}

__device__ __forceinline__ void load_tab1(uint64_t *tab, const uint64_t *gear) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = gear[i];
    __syncthreads();
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) v += __shfl_xor(v, k);
    return v;
}

__device__ __forceinline__ void span_ctx(SpanCtx &C, const StreamTable &st, const Candidates &cand, uint64_t g) {
    C.g = g;
    locate(st, g, C.si, C.off);
    C.n = st.lens[C.si];
    C.data = st.ptrs[C.si];
    C.span = 1ull << st.span_log2;
    C.span_end = min(C.off + C.span, C.n);
    C.cap = cand.cap;
}

// Speculative chain of every span from a warm-up start before it (exact when
// that start is the stream start).
__global__ __launch_bounds__(kResThreads) void chain_kernel(const StreamTable st, const FastParams fp,
                                                            const uint64_t *__restrict__ gear,
                                                            const Candidates cand, const Chains ch,
                                                            const Compact cp) {
    __shared__ uint64_t tab[256];
    __shared__ WaveWin win[kResWaves];
    __shared__ uint32_t tw[kResThreads * 13];
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t g = (uint64_t)blockIdx.x * kResWaves + wave;
    if (g >= st.total_spans) return;  // no block-level barrier below
    SpanCtx C;
    span_ctx(C, st, cand, g);
    const uint64_t warm = min(2ull * fp.max, C.span);
    const uint64_t w0 = C.off > warm ? C.off - warm : 0;
    load_window(C, win[wave], st, cand, w0 < C.off, lane);
    uint32_t cnt;
    uint64_t entry, exit;
    walk_span(C, win[wave], fp, tab, tw + threadIdx.x * 13, ch, w0, lane, cnt, entry, exit);
    if (lane == 0) {
        ch.nst[g] = cnt;
        ch.ent[g] = entry;
        ch.ex[g] = exit;
        if ((g & 63) == 63 || g + 1 == st.total_spans) ch.bx[0][g >> 6] = exit;
        const uint32_t kc = cand.count[g];
        if (kc <= cand.cap) atomicAdd((unsigned long long *)&cp.stats[kStatCand], (unsigned long long)kc);
        else atomicAdd((unsigned long long *)&cp.stats[kStatOvf], 1ull);
        if (cnt > ch.smax) atomicAdd((unsigned long long *)&cp.stats[kStatError], 1ull);
    }
}

// Sequentially settle one 64-span block b: re-walk, in span order, every span
// whose entry differs from its predecessor's exit.  Lane 0's predecessor exit
// is `pred0` (valid when has_pred0).  Returns the block's last exit.
__device__ uint64_t settle_block(const StreamTable &st, const FastParams &fp, const uint64_t *tab, uint32_t *wl,
                                 const Candidates &cand, const Chains &ch, WaveWin &W, uint64_t b, bool has_pred0,
                                 uint64_t pred0, uint32_t lane, uint64_t &rewalks, uint64_t &errs) {
    const uint64_t g = b * 64 + lane;
    const bool valid = g < st.total_spans;
    uint64_t off = 0, E = 0, X = 0;
    uint32_t si = 0;
    if (valid) {
        locate(st, g, si, off);
        E = ch.ent[g];
        X = ch.ex[g];
    }
    const bool first = off == 0;
    uint64_t pred = __shfl_up(X, 1);
    if (lane == 0) pred = pred0;
    bool mism = valid && !first && (lane > 0 || has_pred0) && E != pred;
    for (uint64_t m = __ballot(mism); m; m = __ballot(mism)) {
        const int l0 = __ffsll((long long)m) - 1;
        const uint64_t e = readlane_u64(pred, l0);
        SpanCtx C;
        span_ctx(C, st, cand, b * 64 + l0);
        load_window(C, W, st, cand, false, lane);
        uint32_t cnt;
        uint64_t entry, exit;
        walk_span(C, W, fp, tab, wl, ch, e, lane, cnt, entry, exit);
        if (lane == 0) {
            ch.nst[C.g] = cnt;
            ch.ent[C.g] = entry;
            ch.ex[C.g] = exit;
            if (cnt > ch.smax) ++errs;
        }
        ++rewalks;
        if ((int)lane == l0) {
            mism = false;
            X = exit;
        }
        if ((int)lane == l0 + 1 && valid && !first) {
            pred = exit;
            mism = E != exit;
        }
    }
    const int last = (int)min((uint64_t)63, st.total_spans - 1 - b * 64);
    return readlane_u64(X, last);
}

// One Jacobi pass: wave per 64-span block; lane 0's predecessor is the
// previous block's last exit as of the previous pass (bx[pass&1]); this
// pass's block exits go to bx[(pass+1)&1].  A pass after a pass that changed
// no block exit has nothing to do and returns at once.
__global__ __launch_bounds__(kResThreads) void fix_kernel(const StreamTable st, const FastParams fp,
                                                          const uint64_t *__restrict__ gear,
                                                          const Candidates cand, const Chains ch,
                                                          const Compact cp, int pass) {
    __shared__ uint64_t tab[256];
    __shared__ WaveWin win[kResWaves];
    __shared__ uint32_t tw[kResThreads * 13];
    if (pass > 0 && __hip_atomic_load(&cp.stats[kStatFlag0 + pass - 1], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == 0)
        return;  // converged (uniform across the grid)
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t b = (uint64_t)blockIdx.x * kResWaves + wave;
    const uint64_t nblocks = (st.total_spans + 63) / 64;
    if (b >= nblocks) return;
    uint64_t rewalks = 0, errs = 0;
    const uint64_t pred0 = b > 0 ? ch.bx[pass & 1][b - 1] : 0;
    const uint64_t last = settle_block(st, fp, tab, tw + threadIdx.x * 13, cand, ch, win[wave], b, b > 0, pred0,
                                       lane, rewalks, errs);
    if (lane == 0) {
        ch.bx[(pass + 1) & 1][b] = last;
        if (last != ch.bx[pass & 1][b])
            __hip_atomic_store(&cp.stats[kStatFlag0 + pass], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (rewalks) atomicAdd((unsigned long long *)&cp.stats[kStatRewalk], (unsigned long long)rewalks);
        if (errs) atomicAdd((unsigned long long *)&cp.stats[kStatError], (unsigned long long)errs);
    }
}

// Runs only when the last Jacobi pass still changed a block exit (degenerate
// data whose chains never merge): one wave settles every block in order.
__global__ __launch_bounds__(64) void serial_kernel(const StreamTable st, const FastParams fp,
                                                    const uint64_t *__restrict__ gear, const Candidates cand,
                                                    const Chains ch, const Compact cp) {
    __shared__ uint64_t tab[256];
    __shared__ WaveWin win;
    __shared__ uint32_t tw[64 * 13];
    if (__hip_atomic_load(&cp.stats[kStatFlag0 + kPasses - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        return;
    load_tab1(tab, gear);
    const uint32_t lane = threadIdx.x;
    const uint64_t nblocks = (st.total_spans + 63) / 64;
    uint64_t rewalks = 0, errs = 0, pred0 = 0;
    for (uint64_t b = 0; b < nblocks; ++b)
        pred0 = settle_block(st, fp, tab, tw + lane * 13, cand, ch, win, b, b > 0, pred0, lane, rewalks, errs);
    if (lane == 0) {
        cp.stats[kStatSerial] = 1;
        cp.stats[kStatRewalk] += rewalks;
        cp.stats[kStatError] += errs;
    }
}

constexpr int kCompThreads = 1024;

__device__ __forceinline__ uint64_t block_sum_1024(uint64_t v, uint64_t *red) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    uint64_t t = lane < kCompThreads / 64 ? red[lane] : 0;
    t = wave_sum(t);
    __syncthreads();
    return t;
}

// Chunk count per 1024-span block.
__global__ __launch_bounds__(kCompThreads) void count_kernel(const StreamTable st, const Chains ch,
                                                             const Compact cp) {
    __shared__ uint64_t red[kCompThreads / 64];
    const uint64_t g = (uint64_t)blockIdx.x * kCompThreads + threadIdx.x;
    const uint64_t v = g < st.total_spans ? min(ch.nst[g], ch.smax) : 0;
    const uint64_t t = block_sum_1024(v, red);
    if (threadIdx.x == 0) cp.bsum[blockIdx.x] = t;
}

// Output: span g's chunks at their final index; first[] and the statistics
// straight into host-coherent memory (the last block copies the stats).
__global__ __launch_bounds__(kCompThreads) void write_kernel(const StreamTable st, const Chains ch,
                                                             const Compact cp, cdc_chunk_pod *out,
                                                             uint64_t out_cap) {
    __shared__ uint64_t red[kCompThreads / 64];
    __shared__ uint64_t wex[kCompThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t pre = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kCompThreads) pre += cp.bsum[b];
    const uint64_t base = block_sum_1024(pre, red);
    const uint64_t g = (uint64_t)blockIdx.x * kCompThreads + threadIdx.x;
    const bool valid = g < st.total_spans;
    const uint32_t cnt = valid ? ch.nst[g] : 0;
    const uint32_t c = min(cnt, ch.smax);
    // exclusive scan of c over the block
    uint64_t x = c;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint64_t t = __shfl_up(x, k);
        if (lane >= (uint32_t)k) x += t;
    }
    if (lane == 63) wex[wave] = x;
    __syncthreads();
    uint64_t wbase = 0;
    for (uint32_t w = 0; w < wave; ++w) wbase += wex[w];
    const uint64_t idx = base + wbase + x - c;
    uint64_t err = 0;
    if (valid) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        if (cnt > ch.smax || idx + c > out_cap) {
            err = 1;  // impossible for a consistent chain: report, never write out of bounds
        } else {
            const uint64_t *list = ch.starts + g * ch.smax;
            const uint64_t exit = ch.ex[g];
            for (uint32_t k = 0; k < c; ++k) {
                const uint64_t s0 = list[k];
                const uint64_t nx = k + 1 < c ? list[k + 1] : exit;
                out[idx + k] = cdc_chunk_pod{s0, nx - s0};
            }
        }
        if (off == 0) cp.h_first[si] = idx;
        if (g + 1 == st.total_spans) cp.h_first[st.n] = idx + c;
    }
    err = block_sum_1024(err, red);
    if (threadIdx.x == 0) {
        if (err) atomicAdd((unsigned long long *)&cp.stats[kStatError], (unsigned long long)err);
        __threadfence();
        if (atomicAdd((unsigned long long *)&cp.stats[kStatTicket], 1ull) + 1 == gridDim.x) {
            __threadfence();
            for (int i = 0; i < kStatTicket; ++i)
                cp.h_stats[i] = __hip_atomic_load(&cp.stats[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            cp.h_stats[kStatDone] = 1;
        }
    }
}

}  // namespace

hipError_t launch_scan(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                       const Candidates &cand, const Compact &cp, const uint64_t *d_tails, uint32_t n_tails,
                       int num_cus, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    if (n_tails) {
        if (fp.cm_align)
            scan_tail_kernel<true><<<n_tails, 64, 0, s>>>(st, fp, d_gear, cand, d_tails);
        else
            scan_tail_kernel<false><<<n_tails, 64, 0, s>>>(st, fp, d_gear, cand, d_tails);
    }
    const uint64_t groups = (st.total_spans + kScanWaves - 1) / kScanWaves;
    const unsigned grid = (unsigned)(groups < (uint64_t)num_cus ? groups : (uint64_t)num_cus);
    if (fp.cm_align)
        scan_kernel<true><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand, cp);
    else
        scan_kernel<false><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand, cp);
    return hipGetLastError();
}

hipError_t launch_chain(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                        const Candidates &cand, const Chains &ch, const Compact &cp, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + kResWaves - 1) / kResWaves);
    chain_kernel<<<grid, kResThreads, 0, s>>>(st, fp, d_gear, cand, ch, cp);
    return hipGetLastError();
}

hipError_t launch_fix(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                      const Candidates &cand, const Chains &ch, const Compact &cp, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t nblocks = (st.total_spans + 63) / 64;
    const unsigned grid = (unsigned)((nblocks + kResWaves - 1) / kResWaves);
    for (int p = 0; p < kPasses; ++p) fix_kernel<<<grid, kResThreads, 0, s>>>(st, fp, d_gear, cand, ch, cp, p);
    serial_kernel<<<1, 64, 0, s>>>(st, fp, d_gear, cand, ch, cp);
    return hipGetLastError();
}

hipError_t launch_compact(const StreamTable &st, const Chains &ch, const Compact &cp, void *d_out,
                          uint64_t out_cap, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + kCompThreads - 1) / kCompThreads);
    count_kernel<<<grid, kCompThreads, 0, s>>>(st, ch, cp);
    write_kernel<<<grid, kCompThreads, 0, s>>>(st, ch, cp, reinterpret_cast<cdc_chunk_pod *>(d_out), out_cap);
    return hipGetLastError();
}

}  // namespace p3
}  // namespace cdc
