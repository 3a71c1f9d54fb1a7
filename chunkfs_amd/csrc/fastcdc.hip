// fastcdc.hip -- hand-written gfx950 (CDNA4) kernels for FastCDC v2020.
//
// The reference computes cut points one chunk at a time with a byte loop
// (fastcdc 3.1.0 `cut_gear`, called from chunkfs src/chunkers/fast.rs:37;
// restated in SURVEY.md Appendix A.2 and oracle/cdc_oracle.c).  Each cut
// depends on the previous one through the min-skip and the hash reset; the GPU
// splits the work into a data-parallel HBM pass and a small resolve:
//
//  scan_kernel     for EVERY position i the windowed gear hash W_i (bits
//                  0..47 exact: the masks never test bit 48 or above) and a
//                  candidate record where (W_i & (mask_s & mask_l)) == 0.
//                  Wave per span; lane l owns the contiguous 1 KiB segment
//                  [l*sub, (l+1)*sub) and hashes it serially (one v_lshl_add_u64
//                  per byte).  The bytes arrive with fully coalesced loads --
//                  each wave-instruction reads 16 complete 64-byte pieces --
//                  and are transposed to their owning lanes through a 4 KiB
//                  per-wave LDS tile (tools/ubench_scan.hip: lane-strided loads
//                  cap the read rate at 4.1 TB/s, grouped ones reach 6.0).
//                  A lane starts from hash 0 and re-tests its first 48
//                  positions at the end, with the true carry-in taken from
//                  lane l-1 by one DPP shift: no warm-up bytes are re-read.
//  resolve_kernel  everything after the scan in one launch, block per 32
//                  spans: the exact successor ("link") of every candidate
//                  record in reach, chain walks over those links from a
//                  warm-up start before each span, a decoupled look-back over
//                  blocks for the chunk-count prefix and the block-boundary
//                  check, and the Chunk{offset,length} output.
#include "fastcdc.hpp"

#include <cstdlib>
#include <type_traits>

namespace cdc {
namespace p3 {
namespace {

// ---- common helpers --------------------------------------------------------

// Candidate record (u32): span offset (bits 0-23) | truncated-region result of
// a chunk starting there (bits 24-29, written by the scan's flush; 62 =
// unknown) | mask_l hit (30) | mask_s hit (31).
constexpr uint32_t kCandPosMask = 0x00FFFFFFu;
constexpr uint32_t kCandHitL = 1u << 30;
constexpr uint32_t kCandHitS = 1u << 31;

// Global (address space 1) views: generic pointers compile to flat_load_*,
// which count on both vmcnt and lgkmcnt and would drain the LDS pipeline.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint64_t g_u64;
__device__ __forceinline__ g_u32x4 *as_global4(const void *p) { return (g_u32x4 *)(p); }
__device__ __forceinline__ g_u8 *as_global1(const void *p) { return (g_u8 *)(p); }
__device__ __forceinline__ uint4 ld16(g_u32x4 *p) {
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld16_nt(g_u32x4 *p) {  // streaming hint: the line is done with
    const u32x4 v = __builtin_nontemporal_load(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Experiment builds (tools/scan_variants.sh) may override the scheduling
// fences, the lookahead and the waves per CU; defaults are the measured best.
#ifndef CDC_SCAN_NOFENCE
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define SCHED_FENCE() do {} while (0)
#endif
#ifndef CDC_SCAN_WAVES
#define CDC_SCAN_WAVES 12  // as fast as 16 (profiles/r05/r05v_scan_12_waves.log), 136 KiB of LDS
#endif
// Span g goes to wave g / gridDim of block g % gridDim (wave-major): the
// last, partial round of spans (16384 spans = 5.33 rounds of 3072 waves at
// 1 GiB) then lands on a few waves of EVERY CU instead of on all the waves
// of a third of the CUs while the other CUs idle.
#ifndef CDC_SCAN_NT_ODD
#define CDC_SCAN_NT_ODD 1  // FETCH_SIZE 1.038x vs 1.072x of the input, scan 222 us either way (profiles/r05/r05x_*)
#endif
#ifndef CDC_SCAN_WAVE_MAJOR
#define CDC_SCAN_WAVE_MAJOR 1
#endif
#ifndef CDC_SCAN_LOOK
#define CDC_SCAN_LOOK 1
#endif
#ifndef CDC_SCAN_TRUNC
#define CDC_SCAN_TRUNC 0
#endif

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
    return (h << 1) + g;
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

constexpr uint32_t kTruncMax = 47;    // mask bits <= 47 (checked on the host)
constexpr uint32_t kTruncNone = 63;   // truncated-region result: no hit
constexpr uint32_t kTruncUnknown = 62;  // record field: not precomputed (near the stream end)
constexpr int kRecTShift = 24;        // record bits 24..29: the record's truncated-region result

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

// ---- scan ------------------------------------------------------------------

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

// Entry word: quarter position in the span | kEntFix for the carry-in
// fix-up's quarters (exact hash).  Main-loop entries in a lane's first 48
// positions were hashed without the carry-in and are dropped by the flush.
constexpr uint32_t kEntFix = 1u << 31;
constexpr uint32_t kEntPos = kEntFix - 1;

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

// append_hits that also keeps the quarter's 16 bytes (the DMA scan's flush
// re-hashes from them instead of re-reading HBM).
__device__ __forceinline__ void append_hits_d(bool hit, uint32_t pos, uint64_t h0, const uint4 &q, uint32_t &ne,
                                              const EntryList &E, uint4 *edat) {
    const uint64_t m = __ballot(hit);
    if (m) {
        if (hit) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t slot = ne + below;
            if (slot < kEntCap) {
                E.pos[slot] = pos;
                E.hlo[slot] = (uint32_t)h0;
                E.hhi[slot] = (uint32_t)(h0 >> 32);
                edat[slot] = q;
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
// Step 0's quarters 0..2 (the lane's first 48 positions, hashed without the
// carry-in) may append spurious entries: the flush drops them, and the
// carry-in fix-up appends the exact ones (kEntFix).
struct Q4 {
    uint4 q[4];
};

template <bool kAlign, int kLook>
__device__ __forceinline__ void process_step(const Q4 &C, uint64_t &h, uint32_t pos0, uint32_t &ne,
                                             const EntryList &E, const uint64_t *tab, uint32_t rep,
                                             const FastParams &fp) {
    if constexpr (kLook == 1) {
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
            append_hits(acc == 0, pos0 + 16 * q, h0, ne, E);
        }
    } else {
        // two dwords (8 lookups) ahead of the chain
        G4 ga0, ga1, gb0, gb1;
        look4(ga0, tab, rep, C.q[0].x);
        look4(ga1, tab, rep, C.q[0].y);
        SCHED_FENCE();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t h0 = h;
            uint32_t acc = 0xffffffffu;
            look4(gb0, tab, rep, C.q[q].z);
            look4(gb1, tab, rep, C.q[q].w);
            SCHED_FENCE();
            chain4_test<kAlign>(h, acc, ga0, fp);
            chain4_test<kAlign>(h, acc, ga1, fp);
            SCHED_FENCE();
            if (q < 3) {
                look4(ga0, tab, rep, C.q[q + 1].x);
                look4(ga1, tab, rep, C.q[q + 1].y);
                SCHED_FENCE();
            }
            chain4_test<kAlign>(h, acc, gb0, fp);
            chain4_test<kAlign>(h, acc, gb1, fp);
            SCHED_FENCE();
            append_hits(acc == 0, pos0 + 16 * q, h0, ne, E);
        }
    }
}

// One 64-byte step of a lane for the DMA scan: process_step<kAlign, 1> whose
// entries keep their quarter's bytes.
template <bool kAlign>
__device__ __forceinline__ void process_step_d(const Q4 &C, uint64_t &h, uint32_t pos0, uint32_t &ne,
                                               const EntryList &E, uint4 *edat, const uint64_t *tab, uint32_t rep,
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
        append_hits_d(acc == 0, pos0 + 16 * q, h0, C.q[q], ne, E, edat);
    }
}

// The 4 coalesced loads of step t: instruction i reads piece (lane%4) of the
// step of segment 16 i + rsel(lane/4) (16 complete 64-byte pieces per
// instruction; rsel: see the kernel).
// Step t reads bytes [64 t, 64 t + 64) of every 1 KiB row: the first half of
// a 128-byte line at even t, its second half at odd t (ring B).  kNt marks the
// second-half loads non-temporal (CDC_SCAN_NT_ODD) so that lines whose second
// half is still to come keep their place in L2: the scan's over-fetch went
// from 7.2 % to 3.8 % (the bare read kernel: 0.0 %).
template <bool kNt = false>
__device__ __forceinline__ void gload_step(Q4 &X, const uint8_t *gp, uint64_t istride, uint32_t t) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
        X.q[i] = kNt ? ld16_nt(as_global4(gp + i * istride + t * kStep)) : ld16(as_global4(gp + i * istride + t * kStep));
}

// Transpose through the wave's LDS tile: row o (80 bytes: 64 data + 16 pad)
// holds segment o's step.  Rows are 20 dwords apart, so both directions are
// bank-conflict free (ds_write_b128, banks (a/4) mod 32: an 8-lane group
// writes rows x and x+4, 80 dwords = 16 banks apart, 32 distinct banks;
// ds_read_b128: 16 lanes of distinct l mod 16 start 20 l mod 64 apart = 16
// distinct 4-bank groups), and every address is a per-lane
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

// The resolve's per-record work, done here while the bytes stream by: the
// truncated-region result of a chunk starting at span offset c (first d in
// [0, trunc) whose in-chunk hash, reset at c + a0, hits mask_s below the
// centre / mask_l above it; kTruncNone if none) -- for chunks whose regime is
// the steady one (>= max bytes to the stream end), else kTruncUnknown.  The
// 52 bytes come as 13 dword loads realigned with v_alignbyte_b32; the table is
// the scan's pre-shifted one, so the masks are the shifted ones.
typedef const __attribute__((address_space(3))) uint64_t lds_u64;
typedef const __attribute__((address_space(3))) char lds_char;

#if CDC_SCAN_TRUNC
// Out of line (keeps the scan loop's registers free); the table pointer is
// an explicit LDS one so that the lookups stay ds_read_b64.
__device__ __noinline__ uint32_t scan_trunc(const uint8_t *base, uint32_t c, uint64_t avail, lds_u64 *ltab,
                                            uint32_t rep, uint32_t mn, uint32_t avg, uint32_t mx, uint32_t trunc,
                                            uint64_t mask_s, uint64_t mask_l) {
    const uint32_t a0 = (mn / 2) * 2, ce = (avg / 2) * 2, re = (mx / 2) * 2;
    if (avail - c < (uint64_t)mx || (uint64_t)a0 + 52 > avail - c) return kTruncUnknown;
    const uint32_t tl = min(a0 + trunc, re);
    if (tl <= a0) return kTruncNone;
    const uint32_t len = tl - a0;
    const uint64_t w0 = (uint64_t)c + a0;
    const uint64_t al = w0 & ~3ull;
    const uint32_t sh = (uint32_t)(w0 - al);
    uint32_t w[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) w[i] = *(g_u32 *)(base + al + 4 * i);
    uint64_t h = 0;
    uint32_t t = kTruncNone;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const uint32_t a = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t d = 4 * k + j;
            if (d >= kTruncMax) break;
            const uint32_t addr = __builtin_amdgcn_perm(rep, a, 0x0c0c0004u | ((uint32_t)j << 8));
            h = shl1_add(h, *reinterpret_cast<lds_u64 *>(reinterpret_cast<lds_char *>(ltab) + addr));
            const bool hit = d < len && !(h & ((a0 + d) < ce ? mask_s : mask_l));
            t = (hit && t == kTruncNone) ? d : t;
        }
    }
    return t;
}

#endif

// Flush of one span: exact mask_s / mask_l flags for each hitting quarter
// (re-hashed from the hash before it), each record's truncated-region result
// (scan_trunc), position order, HBM write.  avail = stream bytes from the span
// start.  edat: the entries' bytes in LDS (DMA scan), else re-read from base.
__device__ __forceinline__ void flush_span(uint64_t g, const uint8_t *base, uint32_t span_len, uint64_t avail,
                                           uint32_t sub_mask, uint32_t ne, const EntryList &E, const uint64_t *tab,
                                           uint32_t rep, const FastParams &fp, const Candidates &cand,
                                           uint32_t lane, const uint4 *edat = nullptr) {
    wave_sync_lds();
    uint32_t *cpos = cand.pos + g * cand.cap;
    if (ne > kEntCap) {  // too many hits for the LDS list: resolve takes the exact slow path
        if (lane == 0) cand.count[g] = cand.cap + 1;
        wave_sync_lds();
        return;
    }
    uint32_t hs = 0, hl = 0, my_pos = 0;
    const uint32_t wd = lane < ne ? E.pos[lane] : 0u;
    // (sub_mask = lane sub-span - 1; entries of the main loop at a lane's
    // first 48 positions lack the carry-in: dropped, count 0)
    const bool keep = lane < ne && ((wd & kEntFix) || (wd & sub_mask) >= 48);
    if (lane < ne) E.cnt[lane] = 0;
    if (keep) {
        my_pos = wd & kEntPos;
        uint64_t hh = ((uint64_t)E.hhi[lane] << 32) | E.hlo[lane];
        const uint4 v = edat ? edat[lane] : ld16_guarded(base, my_pos, span_len);
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
        if ((E.pos[k] & kEntPos) < my_pos) slot += c;
    }
    if (keep) {
        for (uint32_t m = hs | hl; m; m &= m - 1) {
            const uint32_t j = __builtin_ctz(m);
            // (bits 24-29: kTruncUnknown.  Precomputing the record's truncated
            // result here -- scan_trunc -- took 10 us off the resolve's link
            // pass but added 17 us of VALU to the scan: off by default,
            // CDC_SCAN_TRUNC=1 in an experiment build.)
            uint32_t t = kTruncUnknown;
#if CDC_SCAN_TRUNC
            t = scan_trunc(base, my_pos + j, avail, (lds_u64 *)tab, rep, fp.min, fp.avg, fp.max, fp.trunc,
                           fp.mask_s_sh, fp.mask_l_sh);
#endif
            if (slot < cand.cap)
                cpos[slot] = (my_pos + j) | (t << kRecTShift) | (((hs >> j) & 1u) << 31) | (((hl >> j) & 1u) << 30);
            ++slot;
        }
    }
    if (lane == 0) cand.count[g] = total;
    wave_sync_lds();
}

template <int kW>
struct ScanLds {
    uint64_t tab[256 * kCopies];     // 64 KiB: entry e, replica c at e*32+c (LDS address 0)
    uint4 stage[kW][64 * 5];         // 5 KiB per wave: transpose tile, 80-byte rows
    uint32_t epos[kW][kEntCap];      // 1 KiB per wave: hitting quarters of the current span
    uint32_t ehlo[kW][kEntCap];
    uint32_t ehhi[kW][kEntCap];
    uint32_t ecnt[kW][kEntCap];
};

// Full spans.  Lane l owns the contiguous segment [l*sub, (l+1)*sub) and
// hashes it serially from hash 0; its first 48 positions are re-tested at the
// end with the true carry-in (lane l-1's final hash, one DPP shift; lane 0's
// from the 48 bytes before the span).  Ragged last spans: scan_tail_kernel.
#ifndef CDC_SCAN_DYN
#define CDC_SCAN_DYN 0
#endif
#ifdef CDC_SCAN_MAXW  // min waves per SIMD -> VGPR cap 512 / CDC_SCAN_MAXW (needs CDC_SCAN_DYN)
#define CDC_SCAN_VGPR_ATTR __attribute__((amdgpu_flat_work_group_size(1, kW * 64), amdgpu_waves_per_eu(CDC_SCAN_MAXW)))
#else
#define CDC_SCAN_VGPR_ATTR __launch_bounds__(kW * 64, 1)
#endif
template <bool kAlign, int kW, int kLook, int kMode>
__global__ CDC_SCAN_VGPR_ATTR void scan_kernel(const StreamTable st, const FastParams fp,
                                                           const uint64_t *__restrict__ gear,
                                                           const Candidates cand, const Compact cp) {
#if CDC_SCAN_DYN
    extern __shared__ uint4 scan_dyn[];  // (dynamic: the compiler then honours the VGPR cap)
    ScanLds<kW> &L = *reinterpret_cast<ScanLds<kW> *>(scan_dyn);
#else
    __shared__ ScanLds<kW> L;
#endif
    const uint64_t *tab = L.tab;
    for (int i = threadIdx.x; i < 256 * kCopies; i += kW * 64)
        L.tab[i] = gear[i / kCopies] << fp.tshift;  // pre-shifted GEAR (see FastParams)
    if (blockIdx.x == 0 && threadIdx.x < kStatWords) cp.stats[threadIdx.x] = 0;  // the resolve accumulates
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
    // Instruction i's lane quad u = lane/4 loads row 16 i + rsel(u); the two
    // quads of one ds_write_b128 lane group (8 lanes) get rows 4 apart, so
    // their 80-byte rows sit 16 banks apart and the write is conflict-free
    // (rows u, u+1 collided on one 4-bank group: 8 extra LDS cycles per
    // store, r02av PMC); the reads (lane = row) are unchanged.
    const uint32_t rsel = ((lane >> 3) & 3) + 8 * (lane >> 5) + 4 * ((lane >> 2) & 1);
    uint4 *wrow = &L.stage[wave][rsel * 5 + (lane & 3)];
    const uint4 *rrow = &L.stage[wave][lane * 5];

    // Spans are software-pipelined: the first two steps of the next span are
    // in flight while this span's fix-up and flush run.  Ragged last spans:
    // scan_tail_kernel.
    const uint64_t gstride = (uint64_t)gridDim.x * kW;
    auto next_full = [&](uint64_t g, uint32_t &si, uint64_t &off) {
        for (; g < st.total_spans; g += gstride) {
            locate(st, g, si, off);
            if (st.lens[si] - off >= span) break;
        }
        return g;
    };
    Q4 A, B, C;
    uint32_t si, wb = 0;
    uint64_t off;
    uint64_t g = next_full(CDC_SCAN_WAVE_MAJOR ? (uint64_t)wave * gridDim.x + blockIdx.x
                                               : (uint64_t)blockIdx.x * kW + wave, si, off);
    const uint8_t *base = nullptr, *gp = nullptr;
    auto prefetch = [&]() {  // first two steps and the carry bytes of span g
        base = st.ptrs[si] + off;
        gp = base + (uint64_t)rsel * sub + (lane & 3) * 16;
        wb = 0;
        if (off != 0 && lane < 48) wb = as_global1(base)[(int)lane - 48];
        gload_step(A, gp, istride, 0);
        SCHED_FENCE();
        gload_step<(bool)CDC_SCAN_NT_ODD>(B, gp, istride, 1);
        SCHED_FENCE();
    };
    if (g < st.total_spans) prefetch();
    while (g < st.total_spans) {
        uint32_t ne = 0;  // quarter entries appended this span (wave-uniform)
        uint64_t h = 0;
        uint4 F0, F1, F2;
        // Two steps in flight while one is hashed (A/B ring).  The loop body
        // issues its loads unconditionally -- a conditional load leaves the
        // compiler unsure how many are outstanding at the back edge, and it
        // then waits for all of them -- so the last two steps are peeled.
        stage_step(C, A, wrow, rrow);
        F0 = C.q[0];
        F1 = C.q[1];
        F2 = C.q[2];
        gload_step(A, gp, istride, 2);
        SCHED_FENCE();
// kMode: 0 = the scan; 1 = loads and transposes only, 2 = hashing only (timing
// experiments: CHUNKFS_AMD_DIAG bits 8-9, results meaningless).
#define CDC_PROC(POS)                                                                          \
    do {                                                                                       \
        if constexpr (kMode == 1) h ^= (uint64_t)(C.q[0].x ^ C.q[1].y ^ C.q[2].z ^ C.q[3].w);   \
        else process_step<kAlign, kLook>(C, h, POS, ne, E, tab, rep, fp);                      \
    } while (0)
#define CDC_SCAN_PAIR(T, LOAD_B, STAGE_A, LOAD_A)                                              \
    do {                                                                                       \
        CDC_PROC(lo + (T) * kStep);                                                            \
        SCHED_FENCE();                                                                         \
        stage_step(C, B, wrow, rrow);                                                          \
        if (LOAD_B && kMode != 2) gload_step<(bool)CDC_SCAN_NT_ODD>(B, gp, istride, (T) + 3);  \
        SCHED_FENCE();                                                                         \
        CDC_PROC(lo + ((T) + 1) * kStep);                                                      \
        SCHED_FENCE();                                                                         \
        if (STAGE_A) stage_step(C, A, wrow, rrow);                                             \
        if (LOAD_A && kMode != 2) gload_step(A, gp, istride, (T) + 4);                         \
        SCHED_FENCE();                                                                         \
    } while (0)
        uint32_t t = 0;
        for (; t + 4 < steps; t += 2) CDC_SCAN_PAIR(t, true, true, true);
        CDC_SCAN_PAIR(t, true, true, false);        // steps-4, steps-3
        CDC_SCAN_PAIR(t + 2, false, false, false);  // steps-2, steps-1
#undef CDC_SCAN_PAIR
#undef CDC_PROC
        // This span's carry-in bytes and identity, then the next span's prefetch.
        const uint64_t g_cur = g, off_cur = off;
        const uint64_t avail_cur = st.lens[si] - off;
        const uint32_t wb_cur = wb;
        const uint8_t *base_cur = base;
        g = next_full(g + gstride, si, off);
        if (g < st.total_spans) prefetch();
        // Fix-up: re-test the first 48 positions with the true carry-in.
        const uint64_t gw = lane < 48 ? L.tab[wb_cur * kCopies + (lane & 31)] : 0;
        const uint64_t hw = readlane_u64(gear_prefix(gw, lane), 47);  // hash of the 48 bytes before
        h = wave_shr1(h, off_cur != 0 ? hw : 0);
        {
            uint64_t h0 = h;
            append_hits(quarter<kAlign>(h, F0, tab, rep, fp) == 0, lo | kEntFix, h0, ne, E);
            h0 = h;
            append_hits(quarter<kAlign>(h, F1, tab, rep, fp) == 0, (lo + 16) | kEntFix, h0, ne, E);
            h0 = h;
            append_hits(quarter<kAlign>(h, F2, tab, rep, fp) == 0, (lo + 32) | kEntFix, h0, ne, E);
        }
        flush_span(g_cur, base_cur, (uint32_t)span, avail_cur, sub - 1, ne, E, tab, rep, fp, cand, lane);
    }
    if (fp.diag & 64) {  // the last block's end (100 MHz stamp) for the resolve's block-span report
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax((unsigned long long *)&cp.stats[kStatDiag0 + 6],
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// ---- scan, LDS-DMA input landing (A/B path: CHUNKFS_AMD_DIAG bit 10) ---------
//
// The same scan with the bytes landed by global_load_lds_dwordx4 straight into
// a per-wave LDS ring: no VGPR staging ring and no ds_write half of the
// transpose.  DMA instruction i of a step has lane l fetch piece l >> 4 (16
// bytes) of row 16 i + (l & 15) -- 16 complete 64-byte pieces per instruction,
// the register path's coalescing -- and lands it lane-linearly, i.e.
// piece-major inside the instruction's 1 KiB, so lane r reads its 64-byte step
// with 4 ds_read_b128 whose 16-lane groups hit 16 distinct bank quads
// (tools/ubench_dma.hip).  Two waves per SIMD (the hashing runs as fast as at
// four, tools/ubench_hash.hip), two 4 KiB slots per wave: one step in flight
// while the other is hashed.  Entries keep their quarter's 16 bytes, so the
// flush re-reads nothing; the 48 carry-in bytes come by one more DMA.  The
// stream table is read through the constant address space (scalar loads):
// a vector load would make the compiler drain the untracked DMA with
// vmcnt(0).  Measured on MI355X (profiles/r03_scan/): bit-exact, but 2-4 %
// slower than scan_kernel (0.259 vs 0.251 ms per GiB, r03n): with two waves
// per SIMD the per-span fix-up and flush are not hidden (17 % more VALU than
// the loop alone, PMC pmc_r03m), so scan_kernel stays the default.

constexpr int kDmaW = 8;
constexpr uint32_t kDiagDmaScan = 1024;  // CHUNKFS_AMD_DIAG bit 10: this scan instead of scan_kernel (A/B)

struct ScanDmaLds {
    uint64_t tab[256 * kCopies];   // 64 KiB (LDS address 0)
    uint4 ring[kDmaW][2][256];     // two 4 KiB step slots per wave
    uint32_t epos[kDmaW][kEntCap];
    uint32_t ehlo[kDmaW][kEntCap];
    uint32_t ehhi[kDmaW][kEntCap];
    uint32_t ecnt[kDmaW][kEntCap];
    uint4 edat[kDmaW][kEntCap];    // each entry's 16 bytes
    uint32_t carry[kDmaW][64];     // the 48 bytes before the next span (DMA, dwords 0..11)
    uint4 recs[kDmaW][64];         // the span's candidate records, staged for one store
};

typedef const __attribute__((address_space(4))) uint64_t c_u64;
typedef const __attribute__((address_space(4))) uint32_t c_u32;

__device__ __forceinline__ uint64_t cld(const uint64_t *p) { return *(c_u64 *)p; }

// One 16-byte piece per lane into LDS at lds_dst + 16 * lane (M0 written in
// the same statement that reads it; hipcc does not count this load).
__device__ __forceinline__ void glds16(const uint8_t *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// One dword per lane into LDS at lds_dst + 4 * lane.
__device__ __forceinline__ void glds4(const uint8_t *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, kCtrl, kRowMask, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), kCtrl, kRowMask, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

// Sum of v over the wave (mod 2^64), uniform: DPP row_shr 1/2/4/8 leaves each
// row's total in its lane 15, row_bcast 15/31 carries them into lane 63.
__device__ __forceinline__ uint64_t wave_total_dpp(uint64_t v) {
    v += dpp64<0x111, 0xF>(v);
    v += dpp64<0x112, 0xF>(v);
    v += dpp64<0x114, 0xF>(v);
    v += dpp64<0x118, 0xF>(v);
    v += dpp64<0x142, 0xA>(v);
    v += dpp64<0x143, 0xC>(v);
    return readlane_u64(v, 63);
}

// flush_span for the DMA scan (full spans): the entries' bytes come from LDS,
// each lane's output slot from a readlane loop over the entries held in
// registers, and the records are staged in LDS and written with exactly two
// store instructions (the records, dwordx4 by lanes < cap/4, and the count),
// so the kernel's DMA waits can count them statically.
__device__ __forceinline__ void flush_span_d(uint64_t g, uint32_t sub_mask, uint32_t ne, const EntryList &E,
                                             const uint4 *edat, uint4 *recs, const uint64_t *tab, uint32_t rep,
                                             const FastParams &fp, const Candidates &cand, uint32_t lane) {
    wave_sync_lds();
    uint32_t hs = 0, hl = 0, my_pos = 0xFFFFFFFFu, cnt = 0;
    const bool ovf = ne > kEntCap;  // too many hits for the LDS list: resolve takes the exact slow path
    const uint32_t wd = lane < ne && !ovf ? E.pos[lane] : 0u;
    // (entries of the main loop at a lane's first 48 positions lack the carry-in)
    const bool keep = lane < ne && !ovf && ((wd & kEntFix) || (wd & sub_mask) >= 48);
    if (keep) {
        my_pos = wd & kEntPos;
        uint64_t hh = ((uint64_t)E.hhi[lane] << 32) | E.hlo[lane];
        const uint4 v = edat[lane];
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * w + b;
                hh = (hh << 1) + gear_of(tab, rep, word_of(v, w), b);
                hs |= (uint32_t)((hh & fp.mask_s_sh) == 0) << j;
                hl |= (uint32_t)((hh & fp.mask_l_sh) == 0) << j;
            }
        cnt = __popc(hs | hl);
    }
    uint32_t slot = 0, total = 0;
    const uint32_t nk = ovf ? 0u : ne;
    for (uint32_t k = 0; k < nk; ++k) {
        const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)my_pos, (int)k);
        const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)k);
        total += ck;
        slot += pk < my_pos ? ck : 0u;
    }
    uint32_t *const rec = reinterpret_cast<uint32_t *>(recs);
    if (keep) {
        for (uint32_t m = hs | hl; m; m &= m - 1) {
            const uint32_t j = __builtin_ctz(m);
            if (slot < cand.cap)
                rec[slot] = (my_pos + j) | (kTruncUnknown << kRecTShift) | (((hs >> j) & 1u) << 31) |
                            (((hl >> j) & 1u) << 30);
            ++slot;
        }
    }
    wave_sync_lds();
    // (slots at or past the count hold stale records: the resolve never reads them)
    if (lane < cand.cap / 4)
        *reinterpret_cast<uint4 *>(cand.pos + g * cand.cap + 4 * lane) = recs[lane];
    if (lane == 0) cand.count[g] = ovf ? cand.cap + 1 : total;
    wave_sync_lds();
}

__device__ __forceinline__ void locate_c(const StreamTable &st, uint64_t g, uint32_t &si, uint64_t &off) {
    uint32_t lo = 0, hi = st.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cld(st.span_base + mid) <= g) lo = mid; else hi = mid;
    }
    si = lo;
    off = (g - cld(st.span_base + lo)) << st.span_log2;
}

template <bool kAlign>
__global__ __launch_bounds__(kDmaW * 64, 1) void scan_dma_kernel(const StreamTable st, const FastParams fp,
                                                                 const uint64_t *__restrict__ gear,
                                                                 const Candidates cand, const Compact cp) {
    __shared__ ScanDmaLds L;
    const uint64_t *tab = L.tab;
    for (int i = threadIdx.x; i < 256 * kCopies; i += kDmaW * 64)
        L.tab[i] = gear[i / kCopies] << fp.tshift;  // pre-shifted GEAR (see FastParams)
    if (blockIdx.x == 0 && threadIdx.x < kStatWords) cp.stats[threadIdx.x] = 0;  // the resolve accumulates
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t rep = (lane & 31) * 8;
    const uint64_t span = 1ull << st.span_log2;
    const uint32_t sub_log2 = st.span_log2 - 6;
    const uint32_t sub = 1u << sub_log2;   // bytes per lane per span (>= 1 KiB)
    const uint32_t steps = sub / kStep;    // >= 16
    const uint32_t lo = lane << sub_log2;
    const EntryList E{L.epos[wave], L.ehlo[wave], L.ehhi[wave], L.ecnt[wave]};
    uint4 *const edat = L.edat[wave];
    const uint64_t src_lane = (uint64_t)(lane & 15) * sub + (lane >> 4) * 16;
    const uint64_t istride = 16ull * sub;
    const uint32_t ring0 = (uint32_t)(uintptr_t)&L.ring[wave][0][0];
    const uint4 *rd0 = &L.ring[wave][0][(lane >> 4) * 64 + (lane & 15)];
    const uint64_t gstride = (uint64_t)gridDim.x * kDmaW;
    auto next_full = [&](uint64_t g, uint32_t &si, uint64_t &off) {
        for (; g < st.total_spans; g += gstride) {
            locate_c(st, g, si, off);
            if (cld(st.lens + si) - off >= span) break;
        }
        return g;
    };
    auto stream_ptr = [&](uint32_t si) {
        return reinterpret_cast<const uint8_t *>(cld(reinterpret_cast<const uint64_t *>(st.ptrs) + si));
    };
    auto issue = [&](const uint8_t *src, uint32_t slot) {
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16(src + i * istride, ring0 + slot * 4096 + i * 1024);
    };
    // The 48 bytes before a span (its carry-in) by one more DMA; when the span
    // starts its stream the source is the span itself (in bounds; unused).
    const uint32_t carry0 = (uint32_t)(uintptr_t)&L.carry[wave][0];
    auto issue_carry = [&](const uint8_t *b, uint64_t o) {
        glds4(o != 0 ? b - 48 + 4 * (lane % 12) : b, carry0);
    };
    // Two steps in flight while one is hashed: a slot is refilled (step t+2)
    // as soon as its step has been read into registers.  vmcnt counts the DMAs
    // and the flush's two stores, in issue order:
    //   t = 0 (after a flush): step 1 (4) + 2 stores younger  -> vmcnt(6)
    //   t = 0 (first span):    step 1 (4)                     -> vmcnt(4)
    //   t = steps-1:           next carry (1) + next step 0 (4) -> vmcnt(5)
    //   otherwise:             step t+1 (4)                   -> vmcnt(4)
    uint32_t si;
    uint64_t off;
    uint64_t g = next_full(CDC_SCAN_WAVE_MAJOR ? (uint64_t)wave * gridDim.x + blockIdx.x
                                               : (uint64_t)blockIdx.x * kDmaW + wave, si, off);
    const uint8_t *base = nullptr;
    if (g < st.total_spans) {
        base = stream_ptr(si) + off;
        issue_carry(base, off);
        issue(base + src_lane, 0);
        issue(base + src_lane + kStep, 1);
    }
    uint32_t slot = 0;  // the slot of the step being hashed (wave-uniform)
    bool first = true;
    while (g < st.total_spans) {
        const uint64_t g_cur = g, off_cur = off;
        const uint8_t *const base_cur = base;
        g = next_full(g + gstride, si, off);
        // The next span's carry bytes and first two steps are issued during
        // this span's last two steps (when there is none, harmless re-reads
        // keep the vmcnt counts static).
        const bool more = g < st.total_spans;
        const uint8_t *const base_next = more ? stream_ptr(si) + off : base_cur;
        const uint64_t off_next = more ? off : 0;
        uint32_t ne = 0;  // quarter entries appended this span (wave-uniform)
        uint64_t h = 0;
        uint32_t wb = 0;
        uint4 F0, F1, F2;
        for (uint32_t t = 0; t < steps; ++t) {
            if (t == 0) {
                if (first) wait_vm<4>(); else wait_vm<6>();
            } else if (t + 1 == steps) {
                wait_vm<5>();
            } else {
                wait_vm<4>();
            }
            Q4 C;
            const uint4 *rd = rd0 + slot * 256;
#pragma unroll
            for (int k = 0; k < 4; ++k) C.q[k] = rd[k * 16];
            if (t == 0 && lane < 48) wb = L.carry[wave][lane >> 2];  // this span's carry bytes
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // the slot (and carry area) is read
            if (t + 2 < steps) {
                issue(base_cur + src_lane + (t + 2) * kStep, slot);
            } else if (t + 2 == steps) {
                issue_carry(base_next, off_next);
                issue(base_next + src_lane, slot);
            } else {
                issue(base_next + src_lane + kStep, slot);
            }
            if (t == 0) {
                F0 = C.q[0];
                F1 = C.q[1];
                F2 = C.q[2];
            }
            process_step_d<kAlign>(C, h, lo + t * kStep, ne, E, edat, tab, rep, fp);
            slot ^= 1;
        }
        first = false;
        base = base_next;
        // Fix-up: re-test the first 48 positions with the true carry-in (the
        // gear hash of the 48 bytes before the span: sum of G[b_i] << (47-i)).
        wb = (wb >> (8 * (lane & 3))) & 0xFFu;
        const uint64_t gw = lane < 48 ? L.tab[wb * kCopies + (lane & 31)] << (47 - lane) : 0;
        const uint64_t hw = wave_total_dpp(gw);
        h = wave_shr1(h, off_cur != 0 ? hw : 0);
        {
            uint64_t h0 = h;
            append_hits_d(quarter<kAlign>(h, F0, tab, rep, fp) == 0, lo | kEntFix, h0, F0, ne, E, edat);
            h0 = h;
            append_hits_d(quarter<kAlign>(h, F1, tab, rep, fp) == 0, (lo + 16) | kEntFix, h0, F1, ne, E, edat);
            h0 = h;
            append_hits_d(quarter<kAlign>(h, F2, tab, rep, fp) == 0, (lo + 32) | kEntFix, h0, F2, ne, E, edat);
        }
        flush_span_d(g_cur, sub - 1, ne, E, edat, L.recs[wave], tab, rep, fp, cand, lane);
    }
    wait_vm<0>();  // no DMA may land after the block's LDS is released
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
        append_hits(hit, p | kEntFix, h0, ne, E);
    }
    flush_span(g, base, span_len, span_len, 0, ne, E, tab, rep, fp, cand, lane);
}


// ---- resolve: exact steps --------------------------------------------------
//
// A chunk starting at s is cut at the first p in [s+a0, s+re) whose in-chunk
// hash (reset at s+a0) hits mask_s below the centre or mask_l above it, else
// at s+rem (max, or the end of the data); p itself starts the next chunk
// (SURVEY.md A.2).  The in-chunk hash equals the windowed one except at the
// <= 47 "truncated" positions s+a0 .. s+a0+46, which are tested exactly from
// the bytes; every later position comes from the scan's records.

#ifndef CDC_RES_WAVES
#define CDC_RES_WAVES 8  // 64 spans per block: one block per CU, all resident (r03q/r03r: 4 -> 8 waves, -7 us)
#endif
#ifndef CDC_WALK_SPANS
#define CDC_WALK_SPANS 8
#endif
#ifndef CDC_WIN_RECS
#define CDC_WIN_RECS 768
#endif
constexpr int kResWaves = CDC_RES_WAVES;
#ifndef CDC_RES_LINK_DIAG
#define CDC_RES_LINK_DIAG 0  // per-pass link timers (experiment builds only)
#endif
#ifndef CDC_RES_HOSTREL
#define CDC_RES_HOSTREL 1  // release of the resolve's host-visible output (0 none .. 3 system fence per wave)
#endif
#ifndef CDC_WALK_COOP
#define CDC_WALK_COOP 1  // walk_window's wave-cooperative exact steps (A/B: 0)
#endif
#ifndef CDC_RES_FASTTRUNC
#define CDC_RES_FASTTRUNC 1  // item_trunc's steady-regime test (A/B: 0)
#endif
constexpr int kResThreads = kResWaves * 64;

// First hitting offset d in [0, tl-a0) of the truncated positions of the
// chunk starting at c (hash reset at c+a0), or kTruncNone; w0 = c + a0.
// Lane-level: the <= 52 bytes arrive as 13 dword loads, are realigned in
// registers with v_alignbyte_b32, and all 47 GEAR lookups are independent of
// the chain, so the LDS latency is paid about once.  Needs al + 52 <= n.
__device__ __forceinline__ uint32_t trunc_words(const uint8_t *data, uint64_t w0, uint32_t len, uint64_t a0,
                                                uint64_t ce, uint64_t mask_s, uint64_t mask_l, lds_u64 *tab) {
    const uint64_t al = w0 & ~3ull;
    const uint32_t sh = (uint32_t)(w0 - al);
    uint32_t w[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) w[i] = *(g_u32 *)(data + al + 4 * i);
    uint64_t h = 0;
    uint32_t t = kTruncNone;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const uint32_t a = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);  // bytes w0+4k .. w0+4k+3
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t d = 4 * k + j;
            if (d >= kTruncMax) break;
            h = shl1_add(h, tab[(a >> (8 * j)) & 255]);
            const bool hit = d < len && !(h & ((a0 + d) < ce ? mask_s : mask_l));
            t = (hit && t == kTruncNone) ? d : t;
        }
    }
    return t;
}

// The same for any chunk start (virtual entries, exact walk steps, the dense
// path; inlined since round 5, see CDC_RES_CALLS).  Near the
// end of the stream the bytes are read one at a time (positions >= n are
// never tested: d < len).
// Inlined (default): the resolve kernel then has no call frames and no VGPR
// spills, so no private segment -- no scratch set-up on its first launch
// (0.31 ms cold with the out-of-line copies, 0.077 ms inlined) and 73-75 vs
// 73-78 us warm (profiles/r05/r05r_*).  __noinline__ is the A/B path.
#ifndef CDC_RES_CALLS
#define CDC_RES_CALLS __forceinline__
#endif
__device__ CDC_RES_CALLS uint32_t trunc_at(const uint8_t *data, uint64_t n, uint64_t c, uint64_t mask_s,
                                          uint64_t mask_l, uint32_t mn, uint32_t avg, uint32_t mx, uint32_t trunc,
                                          lds_u64 *tab) {
    if (n - c <= mn) return kTruncNone;
    uint64_t rem = n - c, center = avg;
    if (rem > mx) rem = mx; else if (rem < center) center = rem;
    const uint64_t a0 = (mn / 2) * 2, ce = (center / 2) * 2, re = (rem / 2) * 2;
    const uint64_t tl = min(a0 + (uint64_t)trunc, re);
    if (tl <= a0) return kTruncNone;
    const uint32_t len = (uint32_t)(tl - a0);
    const uint64_t w0 = c + a0;
    if ((w0 & ~3ull) + 52 <= n) return trunc_words(data, w0, len, a0, ce, mask_s, mask_l, tab);
    uint64_t h = 0;
    for (uint32_t d = 0; d < len; ++d) {
        h = (h << 1) + tab[as_global1(data)[w0 + d]];
        if (!(h & ((a0 + d) < ce ? mask_s : mask_l))) return d;
    }
    return kTruncNone;
}

__device__ __forceinline__ uint32_t trunc_call(const uint8_t *data, uint64_t n, uint64_t c, const FastParams &fp,
                                               const uint64_t *tab) {
    return trunc_at(data, n, c, fp.mask_s, fp.mask_l, fp.min, fp.avg, fp.max, fp.trunc, (lds_u64 *)tab);
}

// Exact next start from the bytes alone, wave-cooperative (64 positions per
// step: one coalesced byte load + a 6-step shuffle prefix scan).  For chains
// that cross an overflowed record list.  Wave-uniform arguments.
// (Scalar parameters, not the FastParams aggregate, which would go through a
// stack frame if this were out of line.)
__device__ CDC_RES_CALLS uint64_t coop_next_bytes(uint32_t mn, uint32_t avg, uint32_t mx, uint64_t mask_s,
                                                 uint64_t mask_l, const uint64_t *tab, const uint8_t *data,
                                                 uint64_t n, uint64_t s, uint32_t lane) {
    if (n - s <= mn) return n;
    FastParams fp{};
    fp.min = mn;
    fp.avg = avg;
    fp.max = mx;
    const Regime R = regime(fp, s, n);
    uint64_t h = 0;
    for (uint64_t b = R.a0; b < R.re; b += 64) {
        const uint64_t p1 = min(b + 64, R.re);
        const uint64_t p = b + lane;
        const bool in = p < p1;
        const uint64_t gv = in ? tab[as_global1(data)[s + p]] : 0;
        const uint64_t x = gear_prefix(gv, lane) + ((h << lane) << 1);
        const bool hit = in && !(x & (p < R.ce ? mask_s : mask_l));
        const uint64_t m = __ballot(hit);
        if (m) return s + b + (uint64_t)(__ffsll((long long)m) - 1);
        h = __shfl(x, (int)(p1 - b - 1));
    }
    return s + R.rem;
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

// Next start after a chunk starting at s, lane-level, from the bytes of the
// truncated positions and a binary search in the global record lists
// (gbase: the stream's first span).  Returns ~0ull when a record list it
// needs overflowed (the caller then uses coop_next_bytes).
__device__ __forceinline__ uint64_t lane_next_global(const StreamTable &st, const FastParams &fp,
                                                     const Candidates &cand, const uint64_t *tab,
                                                     const uint8_t *data, uint64_t n, uint64_t gbase, uint64_t s) {
    if (n - s <= fp.min) return n;
    const Regime R = regime(fp, s, n);
    const uint32_t t = trunc_call(data, n, s, fp, tab);
    if (t != kTruncNone) return s + R.a0 + t;
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
            if (r & ((c - s) < R.ce ? kCandHitS : kCandHitL)) return c;
        }
    }
    return s + R.rem;
}

struct LaneSpan {
    bool act, first;
    uint32_t si;
    uint64_t g, off, span_end, n, gbase;
    const uint8_t *data;
};

// Walk every lane with go=true from s to its span's end, exact, from the
// bytes and the global record lists (lane_next_global; across an overflowed
// record list the whole wave steps with coop_next_bytes).  For windows too
// dense for the LDS path.  The starts go through emit_start (below).
// Wave-synchronous.
struct ChainWin;
__device__ __forceinline__ void emit_start(ChainWin &W, const Chains &ch, const LaneSpan &L, uint32_t l, uint64_t s,
                                           uint32_t &cnt, uint64_t &entry);
__device__ __forceinline__ void walk_lanes(const StreamTable &st, const FastParams &fp, const Candidates &cand,
                                           const uint64_t *tab, ChainWin &W, const Chains &ch, const LaneSpan &L,
                                           uint32_t lane, bool go, uint64_t s, uint32_t &cnt, uint64_t &entry,
                                           uint64_t &exit, uint64_t &steps) {
    cnt = 0;
    entry = ~0ull;
    go = go && s < L.span_end;
    for (;;) {
        bool need = false;
        if (go) {
            emit_start(W, ch, L, lane, s, cnt, entry);
            ++steps;
            const uint64_t nx = lane_next_global(st, fp, cand, tab, L.data, L.n, L.gbase, s);
            if (nx == ~0ull) need = true; else s = nx;
            go = !need && s < L.span_end;
        }
        for (uint64_t m = __ballot(need); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const uint64_t sl = readlane_u64(s, l), nl = readlane_u64(L.n, l);
            const uint8_t *dl = reinterpret_cast<const uint8_t *>(readlane_u64(reinterpret_cast<uint64_t>(L.data), l));
            const uint64_t nx = coop_next_bytes(fp.min, fp.avg, fp.max, fp.mask_s, fp.mask_l, tab, dl, nl, sl, lane);
            if ((int)lane == l) {
                s = nx;
                go = s < L.span_end;
            }
        }
        if (__ballot(go) == 0) break;
    }
    if (cnt == 0) entry = s;
    exit = s;
}

// ---- resolve: window, links, walks, look-back --------------------------------
//
// One block = kResWaves waves = kBlockSpans consecutive spans.  Wave w walks
// kWalkSpans of them (lane l: span G0 + l), each from a warm-up start
// kWarmSpans spans back, over links held in a compact per-wave LDS window:
//   1. window metadata and every record of the window's kWinSlots spans, one
//      batch of global loads;
//   2. the truncated-region result of every record in reach (lane per record);
//   3. the link of every record in reach -- the next chunk start after a chunk
//      starting there -- lane per record, an LDS search.  Next starts that
//      are not records (max cuts, truncated hits) become "virtual" entries,
//      whose links are computed the same way from the bytes until none is new;
//   4. the walks: LDS pointer chasing; the spans' chunk starts go to HBM;
//   5. block settle: a span whose entry differs from its predecessor's exit
//      is re-walked from that exit (rare; in order);
//   6. decoupled look-back over blocks in dispatch order: the chunk-count
//      prefix and the block-boundary check (this block's entry == the
//      predecessor's exit).  A failed check waits for the block at fault to
//      publish its final state; a block whose own entry is stale re-walks;
//   7. Chunk{offset,length} at the final index, first[] and the statistics.
constexpr int kWalkSpans = CDC_WALK_SPANS;
#ifndef CDC_WARM_SPANS
#define CDC_WARM_SPANS 2
#endif
constexpr int kWarmSpans = CDC_WARM_SPANS;
constexpr int kWinSlots = kWarmSpans + kWalkSpans + 1;  // + 1: searched, never walked
constexpr int kReach = kWarmSpans + kWalkSpans;         // slots whose records get links
constexpr uint32_t kWinRecs = CDC_WIN_RECS;  // per-wave record budget (denser windows: global path)
constexpr uint32_t kVirt = 128;     // virtual entries per wave
constexpr int kBlockSpans = kResWaves * kWalkSpans;
constexpr uint64_t kNoDep = ~0ull;  // block entry of a block that starts a stream
constexpr uint64_t kAgg = 1, kInc = 2;
constexpr uint32_t kSpinMax = 1u << 26;  // look-back poll bound: an error, never a hang

constexpr uint32_t kLdsStarts = 24;  // chunk starts per walked span kept in LDS (the rest: HBM)
constexpr int kKeyShift = 40;        // record key: stream << 40 | stream offset (sorted in a window)
constexpr uint64_t kKeyPos = (1ull << kKeyShift) - 1;

struct ChainWin {
    uint64_t key[kWinRecs];           // the window's records: stream << 40 | stream offset, sorted
    uint32_t rec[kWinRecs];           // the records themselves (hit flags)
    uint32_t link[kWinRecs + kVirt];  // next start - entry position (0: not computed)
    uint16_t lrec[kWinRecs + kVirt];  // entry index + 1 of that next start (0: not an entry)
    uint8_t rslot[kWinRecs];          // slot of each record
    uint8_t vslot[kVirt];             // virtual entries: slot, stream offset
    uint64_t vpos[kVirt];
    uint32_t st[kWalkSpans][kLdsStarts];  // first chunk starts of each walked span (offset in span)
    uint64_t soff[kWinSlots];         // stream offset of each slot's span
    uint64_t slen[kWinSlots];         // its stream's length
    const uint8_t *sptr[kWinSlots];   // its stream's bytes
    uint32_t ssi[kWinSlots];          // its stream (~0u: no span)
    uint32_t scnt[kWinSlots];         // its records (> cap: overflowed)
    uint32_t pre[kWinSlots + 1];      // compact start of each slot's records
    uint32_t wpre[kWalkSpans + 1];    // output: chunk prefix of the walked spans
    uint32_t nrec, nvirt;
};

struct BlockState {
    uint64_t E[kBlockSpans];  // entry: first start >= span start
    uint64_t X[kBlockSpans];  // exit: first start >= span end
    uint32_t N[kBlockSpans];  // starts in the span
    uint8_t F[kBlockSpans];   // 1: the span starts a stream
    uint64_t b, base, pred;
    uint64_t t0;              // entry stamp (diag & 64)
    uint32_t rewalk;
    uint64_t stat[kResWaves][3];  // per wave: candidates << 24 | overflowed, re-walks, exact steps
    uint64_t diag[kResWaves][kStatDiagN];  // per wave phase times (diag & 128)
};

__device__ __forceinline__ uint64_t skey(uint32_t si) { return (uint64_t)si << kKeyShift; }

// Index of the first window record whose key is >= k (nrec when none).
__device__ __forceinline__ uint32_t win_lower(const ChainWin &W, uint64_t k) {
    uint32_t a = 0, b = W.nrec;
    while (a < b) {
        const uint32_t m = (a + b) >> 1;
        if (W.key[m] < k) a = m + 1; else b = m;
    }
    return a;
}

// Entry index + 1 of a start exactly at p of stream si (a record or a
// virtual entry), or 0.
__device__ __forceinline__ uint32_t win_entry_at(const ChainWin &W, uint32_t si, uint64_t p) {
    const uint64_t k = skey(si) | p;
    const uint32_t f = win_lower(W, k);
    if (f < W.nrec && W.key[f] == k) return f + 1;
    for (uint32_t v = 0; v < W.nvirt; ++v)
        if (W.vpos[v] == p && W.ssi[W.vslot[v]] == si) return kWinRecs + v + 1;
    return 0;
}

// First qualifying window record for a chunk starting at c (stream si,
// regime R): a linear scan from local index i0 over the sorted keys.
// Returns the position, or c + rem when none is below c + re.  *lr = local
// index + 1.
__device__ __forceinline__ uint64_t win_search(const ChainWin &W, uint32_t si, uint64_t c, const Regime &R,
                                               uint32_t i0, uint32_t *lr) {
    *lr = 0;
    const uint64_t s = skey(si);
    const uint64_t lo = s | (c + R.tl), hi = s | (c + R.re), ce = s | (c + R.ce);
    for (uint32_t i = i0; i < W.nrec; ++i) {
        const uint64_t k = W.key[i];
        if (k >= hi) break;
        if (k >= lo && (W.rec[i] & (k < ce ? kCandHitS : kCandHitL))) {
            *lr = i + 1;
            return k & kKeyPos;
        }
    }
    return c + R.rem;
}

// Next start after a chunk starting at c (stream si, n bytes): the truncated
// result `tr` (or from the bytes when kTrKnown is false), else the first
// qualifying window record from local index i0 on, else the max / end cut.
// *lr = local index + 1 of the result when it is a window record.
template <bool kTrKnown>
__device__ __forceinline__ uint64_t win_next(const ChainWin &W, const FastParams &fp, const uint64_t *tab,
                                             const uint8_t *data, uint64_t n, uint32_t si, uint64_t c,
                                             uint32_t i0, uint32_t tr, uint32_t *lr) {
    *lr = 0;
    if (n - c <= fp.min) return n;  // tail chunk
    const Regime R = regime(fp, c, n);
    if (R.tl > R.a0) {
        const uint32_t t = kTrKnown ? tr : trunc_call(data, n, c, fp, tab);
        if (t != kTruncNone) return c + R.a0 + t;
    }
    if (R.tl >= R.re) return c + R.rem;
    if (fp.diag & 8) return c + R.rem;  // timing experiment only
    return win_search(W, si, c, R, i0, lr);
}

// Wave-uniform allocation of virtual entries: slot of this lane's new entry
// (kVirt when the window's budget is spent); nv counts every request.
__device__ __forceinline__ uint32_t virt_alloc(bool mk, uint32_t &nv) {
    const uint64_t m = __ballot(mk);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t v = nv + below;
    nv += (uint32_t)__popcll(m);
    return v < kVirt ? v : kVirt;
}

// Record the start s of the walked span in lane slot l: the first
// kLdsStarts in LDS, the rest in HBM.
__device__ __forceinline__ void emit_start(ChainWin &W, const Chains &ch, const LaneSpan &L, uint32_t l, uint64_t s,
                                           uint32_t &cnt, uint64_t &entry) {
    if (s >= L.off) {
        if (cnt < kLdsStarts) W.st[l][cnt] = (uint32_t)(s - L.off);
        else if (cnt < ch.smax) ch.starts[L.g * ch.smax + cnt] = s;
        if (cnt == 0) entry = s;
        ++cnt;
    }
}

// Walk every lane with go=true from s (entry index + 1 wr, 0: none) to its
// span's end over the window links.  A start without a link (a stream start,
// a spent virtual budget) takes one exact step from the bytes.
// Wave-synchronous.
__device__ __forceinline__ void walk_window(ChainWin &W, const FastParams &fp, const uint64_t *tab,
                                            const LaneSpan &L, const Chains &ch, uint32_t lane, bool go, uint64_t s,
                                            uint32_t wr, uint32_t &cnt, uint64_t &entry, uint64_t &exit,
                                            uint64_t &steps) {
    cnt = 0;
    entry = ~0ull;
    go = go && s < L.span_end;
    for (;;) {
        while (go) {
            emit_start(W, ch, L, lane, s, cnt, entry);
            if (wr == 0) break;
            const uint32_t d = W.link[wr - 1];
            if (d == 0) break;
            wr = W.lrec[wr - 1];
            s += d;
            go = s < L.span_end;
        }
        if (!__ballot(go)) break;
#if CDC_WALK_COOP
        // Exact steps, wave-cooperative: lane l + 8 j takes the next start
        // after c_j = s_l + j max for walker l (lanes 0..7), so a run of
        // record-free max cuts (zero-filled or constant regions) costs one
        // memory latency per 8 chunks instead of one per chunk; the walker
        // follows the run while each next start is the next c_j.
        static_assert(kWalkSpans == 8, "walkers are lanes 0..7");
        {
            const int wl = (int)(lane & 7);
            const uint32_t jj = lane >> 3;
            const uint64_t c0 = __shfl(s, wl);
            const bool g0 = __shfl(go ? 1 : 0, wl) != 0;
            const uint64_t nw = __shfl(L.n, wl);
            const uint32_t siw = (uint32_t)__shfl((int)L.si, wl);
            const uint8_t *dw = reinterpret_cast<const uint8_t *>(__shfl(reinterpret_cast<uint64_t>(L.data), wl));
            const uint64_t cj = c0 + (uint64_t)jj * fp.max;
            uint64_t nx = 0;
            uint32_t lrj = 0;
            if (g0 && cj < nw) nx = win_next<false>(W, fp, tab, dw, nw, siw, cj, win_lower(W, skey(siw) | cj), 0, &lrj);
            bool run = go;
            uint64_t cur = s;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t n_j = __shfl(nx, wl + 8 * j);
                const uint32_t l_j = (uint32_t)__shfl((int)lrj, wl + 8 * j);
                if (run) {
                    ++steps;
                    const uint64_t c_next = cur + fp.max;
                    if (j < 7 && l_j == 0 && n_j == c_next && c_next < L.span_end) {
                        emit_start(W, ch, L, lane, c_next, cnt, entry);  // (the run goes on from c_next)
                        cur = c_next;
                    } else {
                        s = n_j;
                        wr = l_j;
                        go = s < L.span_end;
                        run = false;
                    }
                }
            }
        }
#else
        if (go) {
            ++steps;
            uint32_t lr;
            s = win_next<false>(W, fp, tab, L.data, L.n, L.si, s, win_lower(W, skey(L.si) | s), 0, &lr);
            wr = lr;
            go = s < L.span_end;
        }
#endif
    }
    if (cnt == 0) entry = s;
    exit = s;
}

// Re-walk, in order, every span of this wave whose entry differs from its
// predecessor's exit (lane 0's predecessor: pred0, when has0).  Lanes
// 0..kWalkSpans-1 own the wave's spans B.*[k0 + lane].
__device__ __forceinline__ void wave_settle(const StreamTable &st, const FastParams &fp, const Candidates &cand,
                                            const uint64_t *tab, const Chains &ch, ChainWin &W, bool dense,
                                            const LaneSpan &L, uint32_t lane, uint32_t k0, bool has0,
                                            uint64_t pred0, BlockState &B, uint64_t &rewalks, uint64_t &steps) {
    const bool mine = lane < kWalkSpans && L.act;
    uint64_t E = mine ? B.E[k0 + lane] : 0, X = mine ? B.X[k0 + lane] : 0;
    for (;;) {
        uint64_t pred = __shfl_up(X, 1);
        if (lane == 0) pred = pred0;
        const bool mism = mine && !L.first && (lane > 0 || has0) && E != pred;
        const uint64_t m = __ballot(mism);
        if (m == 0) break;
        const bool ready = mism && !(lane > 0 && ((m >> (lane - 1)) & 1ull));  // predecessor settled
        uint32_t cnt = 0;
        uint64_t entry = 0, exit = 0;
        if (dense)
            walk_lanes(st, fp, cand, tab, W, ch, L, lane, ready, pred, cnt, entry, exit, steps);
        else
            walk_window(W, fp, tab, L, ch, lane, ready, pred, ready ? win_entry_at(W, L.si, pred) : 0u, cnt, entry,
                        exit, steps);
        if (ready) {
            B.E[k0 + lane] = E = entry;
            B.X[k0 + lane] = X = exit;
            B.N[k0 + lane] = cnt;
            ++rewalks;
        }
    }
}

// One entry of the link pass: a record in reach or a virtual entry, with the
// parameters of its truncated region (fast: its 52 bytes lie before n).
struct LinkItem {
    bool act, fast;
    int j;
    uint32_t e, i0, si, len;
    uint32_t known;  // the record's precomputed truncated result, or kTruncUnknown
    uint64_t c, n, a0, ce, w0;
    const uint8_t *data;
};

__device__ __forceinline__ LinkItem link_item(const ChainWin &W, const FastParams &fp, bool virt, uint32_t x,
                                              uint32_t e1) {
    LinkItem it{};
    it.known = kTruncUnknown;
    it.act = x < e1;
    if (!it.act) return it;
    if (virt) {
        it.e = kWinRecs + x;
        it.j = W.vslot[x];
        it.c = W.vpos[x];
        it.i0 = win_lower(W, skey(W.ssi[it.j]) | it.c);
    } else {
        it.e = x;
        it.j = W.rslot[x];
        it.c = W.key[x] & kKeyPos;
        it.i0 = x + 1;
        it.known = (W.rec[x] >> kRecTShift) & 63u;
    }
    it.si = W.ssi[it.j];
    it.n = W.slen[it.j];
    it.data = W.sptr[it.j];
    if (it.n - it.c > fp.min) {
        const Regime R = regime(fp, it.c, it.n);
        if (R.tl > R.a0) {
            it.len = (uint32_t)(R.tl - R.a0);
            it.a0 = R.a0;
            it.ce = R.ce;
            it.w0 = it.c + R.a0;
            it.fast = (it.w0 & ~3ull) + 52 <= it.n && it.known == kTruncUnknown;
        }
    }
    return it;
}

// The 13 dwords holding an item's truncated region (a harmless read of
// `safe` when it has none in reach).  (Four 16-byte loads plus a select
// realignment measured slower: the extra registers cost occupancy.)
__device__ __forceinline__ void item_load(const LinkItem &it, const void *safe, uint32_t (&w)[13]) {
    if (!__ballot(it.fast)) return;  // records carry the scan's result: no bytes needed (w unused)
    const uint8_t *src = it.fast ? it.data + (it.w0 & ~3ull) : static_cast<const uint8_t *>(safe);
#pragma unroll
    for (int i = 0; i < 13; ++i) w[i] = *(g_u32 *)(src + 4 * i);
}

// Branch-free: 12 GEAR lookups issued together per batch (one LDS latency per
// batch instead of one per 4 bytes), hit bits collected in a mask, the first
// one wins (the same result as trunc_words).
__device__ __forceinline__ uint32_t item_trunc(const LinkItem &it, const uint32_t (&w)[13], const FastParams &fp,
                                               const uint64_t *tab, const uint64_t *tabs) {
    if (!it.act || it.len == 0) return kTruncNone;
    if (it.known != kTruncUnknown) return it.known;  // from the scan's flush
    if (!it.fast) return trunc_call(it.data, it.n, it.c, fp, tab);
    const uint32_t r = (uint32_t)(it.w0 & 3);
    const uint32_t ns = it.ce > it.a0 ? (uint32_t)min(it.ce - it.a0, (uint64_t)64) : 0u;  // d < ns: mask_s
    if (CDC_RES_FASTTRUNC && fp.cm_align && it.len == kTruncMax && ns >= kTruncMax) {
        // Steady regime (every tested position under mask_s): with the GEAR
        // table pre-shifted by tshift the mask is the hash's high dword, so a
        // position costs the chain step, one AND and one MIN; only a region
        // that hits (~0.3 % of records) takes the exact loop below.
        const uint32_t ms = (uint32_t)(fp.mask_s_sh >> 32);
        uint64_t h = 0;
        uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
        for (int k0 = 0; k0 < 12; k0 += 3) {
            uint64_t g[12];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t a = __builtin_amdgcn_alignbyte(w[k0 + k + 1], w[k0 + k], r);
#pragma unroll
                for (int b = 0; b < 4; ++b) g[4 * k + b] = tabs[(a >> (8 * b)) & 255];
            }
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                if (4 * k0 + i >= (int)kTruncMax) break;
                h = shl1_add(h, g[i]);
                acc = min(acc, (uint32_t)(h >> 32) & ms);
            }
        }
        if (acc != 0) return kTruncNone;
    }
    uint64_t h = 0, hits = 0;
#pragma unroll
    for (int k0 = 0; k0 < 12; k0 += 3) {
        uint64_t g[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t a = __builtin_amdgcn_alignbyte(w[k0 + k + 1], w[k0 + k], r);
#pragma unroll
            for (int b = 0; b < 4; ++b) g[4 * k + b] = tab[(a >> (8 * b)) & 255];
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const uint32_t d = 4 * k0 + i;
            if (d >= kTruncMax) break;
            h = shl1_add(h, g[i]);
            hits |= (uint64_t)((h & (d < ns ? fp.mask_s : fp.mask_l)) == 0) << d;
        }
    }
    hits &= it.len >= 64 ? ~0ull : (1ull << it.len) - 1;
    return hits ? (uint32_t)__builtin_ctzll(hits) : kTruncNone;
}

// The item's link into W.link/W.lrec; a next start that is neither a record
// nor past the walked slots becomes a new virtual entry.  Wave-synchronous.
__device__ __forceinline__ void item_link(ChainWin &W, const FastParams &fp, const uint64_t *tab,
                                          const LinkItem &it, uint32_t tr, uint32_t sl2, uint32_t &nv) {
    bool mk = false;
    uint64_t nx = 0;
    uint32_t lr = 0;
    int jt = 0;
    if (it.act) {
        nx = win_next<true>(W, fp, tab, nullptr, it.n, it.si, it.c, it.i0, tr, &lr);
        W.link[it.e] = (uint32_t)(nx - it.c);
        jt = it.j + (int)((nx - W.soff[it.j]) >> sl2);  // <= j + 1: max <= span
        mk = lr == 0 && nx < it.n && jt < kReach && W.ssi[jt] == it.si;
    }
    const uint32_t v = virt_alloc(mk, nv);
    if (mk && v < kVirt) {
        W.vpos[v] = nx;
        W.vslot[v] = (uint8_t)jt;
        lr = kWinRecs + v + 1;
    }
    if (it.act) W.lrec[it.e] = (uint16_t)lr;
}

// Inter-block words (MI355X_MICROARCH.md "inter-workgroup visibility"; the
// programming guide's Guideline 16 recipe R1): every descriptor word is
// stored and loaded with agent-scope relaxed atomics (sc1: past the per-CU
// L1 and the per-XCD L2), the payload drained before its status word.
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load((g_u64 *)const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store((g_u64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void publish(const Resolve &rs, uint64_t b, uint64_t status, uint64_t cnt, uint64_t E,
                                        uint64_t X, uint32_t lane) {
    if (lane == 0) {
        if (status == kAgg) {
            st_agent(&rs.dagg[b], cnt);
            st_agent(&rs.dE[b], E);
            st_agent(&rs.dXa[b], X);
        } else {
            st_agent(&rs.dinc[b], cnt);
            st_agent(&rs.dXi[b], X);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(&rs.dstat[b], (rs.gen << 2) | status);
    }
}

// Poll block j's status word until it is final (bounded: false on timeout).
__device__ __forceinline__ bool wait_final(const Resolve &rs, uint64_t j) {
    const uint64_t inc = (rs.gen << 2) | kInc;
    for (uint32_t k = 0; k < kSpinMax; ++k) {
        if (ld_agent(&rs.dstat[j]) == inc) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: loads stay below)
            return true;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return false;
}

// Exclusive chunk-count prefix of block b >= 1 (wave 0): walks back over the
// predecessors' descriptors, kLbGroups x 64 per step (every lane polls
// kLbGroups of them, all loads of a step in flight together: one round trip
// for the statuses, one for the payloads), to the nearest final (inclusive)
// one, checking every block boundary on the way (exit of block j == entry of
// block j+1, unless j+1 starts a stream).  Item i of a step is predecessor
// j0 - i, i = lane + 64 k.  Returns 1 with acc = the prefix when this block's
// entry Eb holds; 0 with acc = the predecessor's inclusive count and pred =
// its final exit when this block must re-walk from pred; -1 on a poll
// timeout.  (64 per step made the last of 512 blocks per GiB take 8 steps.)
constexpr int kLbGroups = 4;

__device__ int lookback(const Resolve &rs, uint64_t b, uint64_t Eb, uint32_t lane, uint64_t &acc, uint64_t &pred) {
    const uint64_t agg_w = (rs.gen << 2) | kAgg, inc_w = (rs.gen << 2) | kInc;
    for (uint32_t attempt = 0; attempt < 1024; ++attempt) {  // each retry follows a stale block going final
        acc = 0;
        uint64_t expect = Eb;  // entry of the block after this step's item 0
        int64_t j0 = (int64_t)b - 1;
        int64_t stale = -1;
        for (;;) {
            int64_t j[kLbGroups];
            uint64_t w[kLbGroups];
#pragma unroll
            for (int k = 0; k < kLbGroups; ++k) {
                j[k] = j0 - (int64_t)lane - 64 * k;
                w[k] = j[k] >= 0 ? 0 : inc_w;
            }
            // lim = first item (in distance order) whose status is final; every
            // item up to it must be published (aggregate or final).
            int kl = kLbGroups - 1;
            uint32_t ll = 63;
            uint64_t mi[kLbGroups];
            for (uint32_t spins = 0;; ++spins) {
#pragma unroll
                for (int k = 0; k < kLbGroups; ++k)
                    if (w[k] != agg_w && w[k] != inc_w) w[k] = ld_agent(&rs.dstat[j[k]]);
                bool ready = true, found = false;
#pragma unroll
                for (int k = 0; k < kLbGroups; ++k) {
                    mi[k] = __ballot(w[k] == inc_w);
                    const uint64_t mp = __ballot(w[k] == agg_w || w[k] == inc_w);
                    if (found) continue;
                    if (mi[k]) {
                        found = true;
                        kl = k;
                        ll = (uint32_t)__ffsll((long long)mi[k]) - 1;
                        const uint64_t need = (2ull << ll) - 1;
                        if ((mp & need) != need) ready = false;
                    } else if (mp != ~0ull) {
                        ready = false;
                    }
                }
                if (!found) {
                    kl = kLbGroups - 1;
                    ll = 63;
                }
                if (ready) break;
                if (spins >= kSpinMax) return -1;
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: loads stay below)
            uint64_t cnt[kLbGroups], E[kLbGroups], X[kLbGroups];
#pragma unroll
            for (int k = 0; k < kLbGroups; ++k) {
                const bool in = k < kl || (k == kl && lane <= ll);
                const bool inc = w[k] == inc_w;
                cnt[k] = 0;
                E[k] = kNoDep;
                X[k] = 0;
                if (j[k] >= 0 && in) {
                    cnt[k] = ld_agent(inc ? &rs.dinc[j[k]] : &rs.dagg[j[k]]);
                    X[k] = ld_agent(inc ? &rs.dXi[j[k]] : &rs.dXa[j[k]]);
                    if (!inc) E[k] = ld_agent(&rs.dE[j[k]]);
                }
            }
            // boundary checks in distance order: item i's exit vs item i-1's entry
            int64_t bad = -1;
#pragma unroll
            for (int k = 0; k < kLbGroups; ++k) {
                if (k > kl) break;
                uint64_t En = __shfl_up(E[k], 1);
                if (lane == 0) En = k == 0 ? expect : readlane_u64(E[k - 1], 63);
                const bool in = k < kl || lane <= ll;
                const uint64_t mb = __ballot(in && En != kNoDep && X[k] != En);
                if (mb && bad < 0) bad = 64 * k + (__ffsll((long long)mb) - 1);
            }
            if (bad >= 0) {
                stale = j0 - bad + 1;  // the block whose entry is stale
                break;
            }
            uint64_t part = 0;
#pragma unroll
            for (int k = 0; k < kLbGroups; ++k)
                if (k < kl || (k == kl && lane <= ll)) part += cnt[k];
            acc += wave_sum(part);
            if (mi[kl]) return 1;  // a final descriptor was reached (item ll of group kl)
            expect = readlane_u64(E[kLbGroups - 1], 63);
            j0 -= 64 * kLbGroups;
        }
        if (stale == (int64_t)b) {  // this block's own entry: the predecessor's final exit decides
            if (!wait_final(rs, b - 1)) return -1;
            acc = ld_agent(&rs.dinc[b - 1]);
            pred = ld_agent(&rs.dXi[b - 1]);
            return pred == Eb ? 1 : 0;
        }
        if (!wait_final(rs, (uint64_t)stale)) return -1;  // then look again
    }
    return -1;
}

// Chunk starts are re-read by the wave that stored them: nt loads (past L1).
__device__ __forceinline__ uint64_t ld_nt(const uint64_t *p) {
    return __builtin_nontemporal_load((const g_u64 *)p);
}

// Phase timer (diag & 128): per-wave durations in registers, summed per block
// at the end (one atomic per phase per block, not per wave).
#define CDC_DIAG_T(k)                                                  \
    do {                                                               \
        if ((fp.diag & 128) && !(CDC_RES_LINK_DIAG && (fp.diag & 8192))) { \
            const uint64_t t_ = __builtin_amdgcn_s_memrealtime();       \
            dt[k] += t_ - t_prev;                                      \
            t_prev = t_;                                               \
        }                                                              \
    } while (0)

// FastParams.diag (CHUNKFS_AMD_DIAG, read at cdc_create) -- test hooks and
// timing experiments only, 0 in every real run: 1 = walks start at the span
// start (no warm-up: nearly every boundary re-walks), 2 = every wave takes the
// dense (global record list) path, 128 = phase timings into the stats.
#ifndef CDC_RES_ATTR
#define CDC_RES_ATTR __launch_bounds__(kResThreads, 2)
#endif
__global__ CDC_RES_ATTR void resolve_kernel(const StreamTable st, const FastParams fp,
                                                              const uint64_t *__restrict__ gear,
                                                              const Candidates cand, const Chains ch,
                                                              const Compact cp, const Resolve rs,
                                                              cdc_chunk_pod *out, uint64_t out_cap) {
    __shared__ uint64_t tab[256];
    __shared__ uint64_t tabs[256];  // the same, pre-shifted by tshift (item_trunc's steady-regime test)
    __shared__ ChainWin win[kResWaves];
    __shared__ BlockState B;
    // Blocks take their index in dispatch order, so the look-back only ever
    // waits on blocks that are already running or done.
    if (threadIdx.x == 0) {
        if (fp.diag & 64) B.t0 = __builtin_amdgcn_s_memrealtime();
        B.b = atomicAdd((unsigned long long *)&cp.stats[kStatOrder], 1ull);
        B.base = B.pred = 0;
        B.rewalk = 0;
    }
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tabs[i] = gear[i] << fp.tshift;
    load_tab1(tab, gear);
    const uint64_t b = B.b;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t sl2 = st.span_log2;
    const uint64_t span = 1ull << sl2;
    const uint64_t g0 = b * kBlockSpans;
    const uint32_t nsp = (uint32_t)min((uint64_t)kBlockSpans, st.total_spans - g0);
    const uint32_t k0 = wave * kWalkSpans;  // block index of this wave's first span
    const uint64_t G0 = g0 + k0;
    const uint32_t cap = cand.cap;
    ChainWin &W = win[wave];
    uint64_t t_prev = (fp.diag & 128) ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t dt[kStatDiagN] = {};
    uint64_t steps = 0, rewalks = 0, cstat = 0;
    LaneSpan L{};
    bool dense = false;

    if (k0 < nsp) {
        const int64_t gfirst = (int64_t)G0 - kWarmSpans;  // span of slot 0
        // 1. window metadata, then every record of the window (one batch of loads)
        if (lane < kWinSlots) {
            const int64_t g = gfirst + lane;
            uint32_t si = ~0u, c = 0;
            uint64_t off = 0, n = 0;
            const uint8_t *p = nullptr;
            if (g >= 0 && (uint64_t)g < st.total_spans) {
                locate(st, (uint64_t)g, si, off);
                c = cand.count[g];
                n = st.lens[si];
                p = st.ptrs[si];
            }
            W.ssi[lane] = si;
            W.soff[lane] = off;
            W.scnt[lane] = c;
            W.slen[lane] = n;
            W.sptr[lane] = p;
        }
        wave_sync_lds();
        if (lane == 0) {
            uint32_t acc = 0;
            bool dn = (fp.diag & 2) != 0;
#pragma unroll 1
            for (int j = 0; j < kWinSlots; ++j) {
                W.pre[j] = acc;
                const uint32_t c = W.scnt[j];
                if (c > cap) dn = true; else acc += c;
            }
            if (acc > kWinRecs) dn = true;
            W.pre[kWinSlots] = dn ? 0 : acc;
            W.nrec = dn ? 0 : acc;
            W.nvirt = dn ? 1u : 0u;  // (the dense flag, for the other lanes)
        }
        wave_sync_lds();
        dense = W.nvirt != 0;
        if (lane < kWalkSpans && k0 + lane < nsp) {  // the walker's span: slot kWarmSpans + lane
            const int j = kWarmSpans + (int)lane;
            L.act = true;
            L.g = G0 + lane;
            L.si = W.ssi[j];
            L.off = W.soff[j];
            L.n = W.slen[j];
            L.data = W.sptr[j];
            L.gbase = L.g - (L.off >> sl2);
            L.span_end = min(L.off + span, L.n);
            L.first = L.off == 0;
            const uint32_t c = W.scnt[j];
            cstat = c > cap ? 1ull : (uint64_t)c << 24;
        }
        CDC_DIAG_T(0);
        uint32_t cnt = 0;
        uint64_t entry = 0, exit = 0;
        if (dense) {
            // Degenerate data: exact walks from the bytes and the global record lists.
            uint64_t s0 = 0;
            if (L.act && !L.first) s0 = L.off > kWarmSpans * span ? L.off - kWarmSpans * span : 0;
            if (L.act && !L.first && (fp.diag & 1)) s0 = L.off;  // test hook: no warm-up
            walk_lanes(st, fp, cand, tab, W, ch, L, lane, L.act, s0, cnt, entry, exit, steps);
        } else {
            const uint32_t nrec = W.nrec;
            {
                uint32_t v[kWinSlots];
#pragma unroll
                for (int j = 0; j < kWinSlots; ++j) {
                    const uint32_t c = W.scnt[j];
                    v[j] = cand.pos[lane < c ? (uint64_t)(gfirst + j) * cap + lane : 0];
                }
#pragma unroll 1
                for (int j = 0; j < kWinSlots; ++j) {
                    const uint64_t kb = skey(W.ssi[j]) | W.soff[j];
                    const uint32_t c = W.scnt[j], p0 = W.pre[j];
                    for (uint32_t k = lane; k < c; k += 64) {  // (k >= 64: rare dense-ish slots)
                        const uint32_t r = k < 64 ? v[0] : cand.pos[(uint64_t)(gfirst + j) * cap + k];
                        W.rec[p0 + k] = r;
                        W.key[p0 + k] = kb + (r & kCandPosMask);
                        W.rslot[p0 + k] = (uint8_t)j;
                    }
#pragma unroll
                    for (int q = 0; q + 1 < kWinSlots; ++q) v[q] = v[q + 1];  // next slot's batch into v[0]
                }
            }
            wave_sync_lds();
            CDC_DIAG_T(1);
            // 2-3. per entry (records in reach, then virtual entries until none
            // is new): its truncated-region result, then its link -- the next
            // chunk start after a chunk starting there -- by an LDS search.
            // Next starts that are neither records nor past the walked slots
            // become new virtual entries.
            const uint32_t nlink = W.pre[kReach];
            for (uint32_t i = nlink + lane; i < nrec; i += 64) W.link[i] = 0;  // searched only
            uint32_t nv = 0, e0 = 0, e1 = nlink;
            bool virt = false;
            for (;;) {
                // (the next pass's bytes are loaded while this pass evaluates:
                // one memory latency per round instead of one per pass)
                LinkItem A = link_item(W, fp, virt, e0 + lane, e1);
                uint32_t wa[13];
                item_load(A, gear, wa);
                for (uint32_t base = e0; base < e1; base += 64) {
                    // (CDC_RES_LINK_DIAG builds, diag & 8192: the pass split into
                    // issue / truncated test / link, slots 0-2 for records, 3-5 for
                    // virtual entries; profiles/r06/r06k_*)
                    constexpr bool kLinkDiag = CDC_RES_LINK_DIAG;
                    uint64_t f0 = (kLinkDiag && (fp.diag & 8192)) ? __builtin_amdgcn_s_memrealtime() : 0;
                    const LinkItem B2 = link_item(W, fp, virt, base + 64 + lane, e1);
                    uint32_t wb[13];
                    item_load(B2, gear, wb);
                    uint64_t f1 = (kLinkDiag && (fp.diag & 8192)) ? __builtin_amdgcn_s_memrealtime() : 0;
                    const uint32_t tr = (fp.diag & 4) ? kTruncNone : item_trunc(A, wa, fp, tab, tabs);
                    if (kLinkDiag && (fp.diag & 8192)) __builtin_amdgcn_s_waitcnt(0);
                    uint64_t f2 = (kLinkDiag && (fp.diag & 8192)) ? __builtin_amdgcn_s_memrealtime() : 0;
                    item_link(W, fp, tab, A, tr, sl2, nv);
                    if (kLinkDiag && (fp.diag & 8192)) {
                        const uint64_t f3 = __builtin_amdgcn_s_memrealtime();
                        const int o = virt ? 3 : 0;
                        dt[o] += f1 - f0;
                        dt[o + 1] += f2 - f1;
                        dt[o + 2] += f3 - f2;
                    }
                    A = B2;
#pragma unroll
                    for (int i = 0; i < 13; ++i) wa[i] = wb[i];
                }
                wave_sync_lds();
                if (!virt) CDC_DIAG_T(4);
                const uint32_t vend = min(nv, kVirt);
                if (virt ? e1 >= vend : vend == 0) break;
                e0 = virt ? e1 : 0;
                e1 = vend;
                virt = true;
            }
            if (lane == 0) W.nvirt = min(nv, kVirt);
            wave_sync_lds();
            CDC_DIAG_T(3);
            // 4. the walks, from the first record kWarmSpans spans back (exact
            // from a stream start)
            uint64_t s = 0;
            uint32_t wr = 0;
            if (L.act && !L.first && L.off >= kWarmSpans * span) {
                const int jw = (int)lane;  // slot of span g - kWarmSpans
                if (W.pre[jw + 1] > W.pre[jw]) {
                    wr = W.pre[jw] + 1;
                    s = W.key[W.pre[jw]] & kKeyPos;
                } else {
                    s = W.soff[jw];
                }
            }
            if (L.act && !L.first && (fp.diag & 1)) {  // test hook: no warm-up
                s = L.off;
                wr = 0;
            }
            walk_window(W, fp, tab, L, ch, lane, L.act, s, wr, cnt, entry, exit, steps);
        }
        if (L.act) {
            B.E[k0 + lane] = entry;
            B.X[k0 + lane] = exit;
            B.N[k0 + lane] = cnt;
            B.F[k0 + lane] = L.first ? 1 : 0;
        }
        CDC_DIAG_T(5);
    }
    __syncthreads();

    // 5-6. block settle (round 0), then the look-back; a block whose entry
    // turns out stale settles again from the predecessor's final exit (round 1).
#pragma unroll 1
    for (int round = 0; round < 2; ++round) {
        bool need;
        if (round == 0) {
            const uint32_t k = threadIdx.x;
            need = __syncthreads_or(k > 0 && k < nsp && !B.F[k] && B.E[k] != B.X[k - 1]) != 0;
        } else {
            if (wave == 0) {
                uint64_t C = 0;
                for (uint32_t k = lane; k < nsp; k += 64) C += B.N[k];
                C = wave_sum(C);
                const uint64_t Eb = B.F[0] ? kNoDep : B.E[0];
                const uint64_t Xb = B.X[nsp - 1];
                uint64_t acc = 0, pred = 0;
                int ok = 1;
                if (b > 0) {
                    publish(rs, b, kAgg, C, Eb, Xb, lane);
                    ok = lookback(rs, b, Eb, lane, acc, pred);
                }
                if (ok != 0) publish(rs, b, kInc, acc + C, 0, Xb, lane);  // (a timeout too: never strand waiters)
                if (lane == 0) {
                    B.base = acc;
                    B.pred = pred;
                    B.rewalk = ok == 0 ? 1u : 0u;
                    if (ok < 0) atomicAdd((unsigned long long *)&cp.stats[kStatError], 1ull);
                }
                CDC_DIAG_T(6);
            }
            __syncthreads();
            need = B.rewalk != 0;
        }
        if (need) {
            for (uint32_t w2 = 0; w2 < (uint32_t)kResWaves; ++w2) {
                if (wave == w2 && k0 < nsp)
                    wave_settle(st, fp, cand, tab, ch, W, dense, L, lane, k0, w2 > 0 || round > 0,
                                w2 > 0 ? B.X[k0 - 1] : B.pred, B, rewalks, steps);
                __syncthreads();
            }
        }
    }
    CDC_DIAG_T(2);
    if (B.rewalk && wave == 0) {
        uint64_t C = 0;
        for (uint32_t k = lane; k < nsp; k += 64) C += B.N[k];
        C = wave_sum(C);
        publish(rs, b, kInc, B.base + C, 0, B.X[nsp - 1], lane);
    }

    // 7. output: this wave's spans' chunks at their final index
    if (k0 < nsp) {
        uint32_t wpre0 = 0;
        for (uint32_t k = 0; k < k0; ++k) wpre0 += B.N[k];
        const uint32_t myN = L.act ? B.N[k0 + lane] : 0;
        uint32_t x = myN;
#pragma unroll
        for (int o = 1; o < kWalkSpans; o <<= 1) {
            const uint32_t t = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += t;
        }
        if (lane < kWalkSpans) W.wpre[lane + 1] = x;
        if (lane == 0) W.wpre[0] = 0;
        const uint32_t wtot = (uint32_t)__shfl(x, kWalkSpans - 1);
        const uint64_t obase = B.base + wpre0;
        const bool bad = __ballot(L.act && myN > ch.smax) != 0 || obase + wtot > out_cap;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's chunk-start stores, before its loads
        wave_sync_lds();
        if (!bad) {
            for (uint32_t i = lane; i < wtot; i += 64) {
                int k = 0;
                while (k + 1 < kWalkSpans && W.wpre[k + 1] <= i) ++k;
                const uint32_t r = i - W.wpre[k];
                const uint64_t *list = ch.starts + (G0 + k) * ch.smax;
                const uint64_t off_k = W.soff[kWarmSpans + k];
                const uint64_t s0 = r < kLdsStarts ? off_k + W.st[k][r] : ld_nt(list + r);
                const uint64_t nx = r + 1 >= B.N[k0 + k] ? B.X[k0 + k]
                                    : r + 1 < kLdsStarts ? off_k + W.st[k][r + 1] : ld_nt(list + r + 1);
                out[obase + i] = cdc_chunk_pod{s0, nx - s0};
            }
            if (L.act) {
                if (L.first) cp.h_first[L.si] = obase + x - myN;
                if (L.g + 1 == st.total_spans) cp.h_first[st.n] = obase + x;
            }
        }
        const uint64_t cs = wave_sum(cstat), rw = wave_sum(rewalks), sp = wave_sum(steps);
        if (lane == 0) {
            B.stat[wave][0] = cs;
            B.stat[wave][1] = rw;
            B.stat[wave][2] = sp + (bad ? (1ull << 40) : 0);
        }
        CDC_DIAG_T(7);
    } else if (lane == 0) {
        B.stat[wave][0] = B.stat[wave][1] = B.stat[wave][2] = 0;
    }
    if ((fp.diag & 128) && lane == 0)
        for (int k = 0; k < kStatDiagN; ++k) B.diag[wave][k] = dt[k];
    // The chunk list and first[] may be coherent host memory that the host
    // reads as soon as it sees the done word: every wave waits for its own
    // stores before the block takes its ticket, so the last block's done
    // word cannot overtake them.  (A system-scope fence per wave -- an L2
    // write-back each -- cost the two-stream step 37 us.)
#if CDC_RES_HOSTREL >= 3
    __threadfence_system();
#elif CDC_RES_HOSTREL >= 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t cs = 0, rw = 0, sp = 0;
        for (int w = 0; w < kResWaves; ++w) {
            cs += B.stat[w][0];
            rw += B.stat[w][1];
            sp += B.stat[w][2];
        }
        if (fp.diag & 64) {  // block spans (100 MHz stamps): min / max start, max / min end, max / sum duration
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime(), t0 = B.t0;
            unsigned long long *d = (unsigned long long *)&cp.stats[kStatDiag0];
            atomicMax(d + 0, (unsigned long long)~t0);
            atomicMax(d + 1, (unsigned long long)t0);
            atomicMax(d + 2, (unsigned long long)t1);
            atomicMax(d + 3, (unsigned long long)~t1);
            atomicMax(d + 4, (unsigned long long)(t1 - t0));
            atomicAdd(d + 5, (unsigned long long)(t1 - t0));
        } else if (fp.diag & 128)
            for (int k = 0; k < kStatDiagN; ++k) {
                uint64_t d = 0;
                for (int w = 0; w < kResWaves; ++w) d += B.diag[w][k];
                atomicAdd((unsigned long long *)&cp.stats[kStatDiag0 + k], (unsigned long long)d);
            }
        const uint64_t err = sp >> 40;
        sp &= (1ull << 40) - 1;
        if (cs) atomicAdd((unsigned long long *)&cp.stats[kStatCand], (unsigned long long)cs);
        if (rw) atomicAdd((unsigned long long *)&cp.stats[kStatRewalk], (unsigned long long)rw);
        if (sp) atomicAdd((unsigned long long *)&cp.stats[kStatOnDemand], (unsigned long long)sp);
        if (err) atomicAdd((unsigned long long *)&cp.stats[kStatError], (unsigned long long)err);
#if CDC_RES_HOSTREL >= 2
        __threadfence_system();
#else
        __threadfence();
#endif
        if (atomicAdd((unsigned long long *)&cp.stats[kStatTicket], 1ull) + 1 == gridDim.x) {
            __threadfence_system();
            for (int i = 0; i < kStatWords; ++i)
                if (i != kStatDone) cp.h_stats[i] = ld_agent(&cp.stats[i]);
            const uint64_t c = cp.h_stats[kStatCand];
            cp.h_stats[kStatCand] = c >> 24;
            cp.h_stats[kStatOvf] = c & 0xFFFFFF;
            __threadfence_system();
            cp.h_stats[kStatDone] = 1;
        }
    }
}
#undef CDC_DIAG_T

}  // namespace

#ifdef CDC_OVL
namespace ovl {  // the overlap set (fastcdc_ovl.hip): this file built again with its sizes
#endif

// Dynamic LDS of the scan (CDC_SCAN_DYN): the size and, once per kernel, the
// attribute that admits more than 64 KiB.
template <bool kAlign, int kW, int kLook, int kMode>
static hipError_t scan_launch(unsigned grid, const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                              const Candidates &cand, const Compact &cp, hipStream_t s) {
    size_t lds = 0;
    if (CDC_SCAN_DYN) {
        lds = sizeof(ScanLds<kW>);
        static bool attr = false;
        if (!attr) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&scan_kernel<kAlign, kW, kLook, kMode>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            attr = true;
        }
    }
    scan_kernel<kAlign, kW, kLook, kMode><<<grid, kW * 64, lds, s>>>(st, fp, d_gear, cand, cp);
    return hipSuccess;
}

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
    // 12 waves per CU (3 per SIMD: as fast as 16, r05v_scan_12_waves.log, with
    // up to 168 VGPRs), GEAR lookups one dword ahead of the chain.  (Measured:
    // 12 waves with two dwords of lookahead is slower.)
    constexpr int W = CDC_SCAN_WAVES, K = CDC_SCAN_LOOK;
    const uint32_t mode = (fp.diag >> 8) & 3;
    if (mode == 0 && (fp.diag & kDiagDmaScan)) {  // LDS-DMA input landing (measured, not adopted)
        const uint64_t groups = (st.total_spans + kDmaW - 1) / kDmaW;
        const unsigned grid = (unsigned)(groups < (uint64_t)num_cus ? groups : (uint64_t)num_cus);
        if (fp.cm_align)
            scan_dma_kernel<true><<<grid, kDmaW * 64, 0, s>>>(st, fp, d_gear, cand, cp);
        else
            scan_dma_kernel<false><<<grid, kDmaW * 64, 0, s>>>(st, fp, d_gear, cand, cp);
        return hipGetLastError();
    }
    const uint64_t groups = (st.total_spans + W - 1) / W;
    const unsigned grid = (unsigned)(groups < (uint64_t)num_cus ? groups : (uint64_t)num_cus);
    hipError_t e;
    if (mode == 1 && fp.cm_align)
        e = scan_launch<true, W, K, 1>(grid, st, fp, d_gear, cand, cp, s);
    else if (mode == 2 && fp.cm_align)
        e = scan_launch<true, W, K, 2>(grid, st, fp, d_gear, cand, cp, s);
    else if (fp.cm_align)
        e = scan_launch<true, W, K, 0>(grid, st, fp, d_gear, cand, cp, s);
    else
        e = scan_launch<false, W, K, 0>(grid, st, fp, d_gear, cand, cp, s);
    return e != hipSuccess ? e : hipGetLastError();
}

uint64_t resolve_blocks(uint64_t spans) { return (spans + kBlockSpans - 1) / kBlockSpans; }

hipError_t launch_resolve(const StreamTable &st, const FastParams &fp, const uint64_t *d_gear,
                          const Candidates &cand, const Chains &ch, const Compact &cp, const Resolve &rs,
                          void *d_out, uint64_t out_cap, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    resolve_kernel<<<(unsigned)resolve_blocks(st.total_spans), kResThreads, 0, s>>>(
        st, fp, d_gear, cand, ch, cp, rs, reinterpret_cast<cdc_chunk_pod *>(d_out), out_cap);
    return hipGetLastError();
}

#ifdef CDC_OVL
}  // namespace ovl
#endif
}  // namespace p3
}  // namespace cdc
