// small.hip -- FastCDC v2020 for one small stream in ONE launch (gfx950).
//
// The reference's StorageWriter calls Chunker::chunk_data once per 1 MiB
// segment plus the carried chunk (src/system/storage.rs:302-357); through the
// C ABI every such call is a host buffer of ~1 MiB.  At that size the
// two-kernel pipeline of fastcdc.hip is all latency (scan ~26 us + resolve
// ~35 us of a ~175 us call, profiles/r03aw_bench.json).  small_kernel does the
// whole job in one launch:
//
//   every block     8 waves, a 4 KiB piece per wave staged through LDS by
//                   coalesced 16-byte loads (the input may be device memory or
//                   a pinned host slot read over PCIe); lane l hashes the 64
//                   bytes [64 l, 64 l + 64) of its piece after 48 warm-up bytes,
//                   so every tested hash is the exact windowed one (SURVEY.md
//                   A.3); positions whose windowed hash hits mask_s or mask_l
//                   become records (position | hit flags) written, in position
//                   order, to the block's own region; then an arrival ticket.
//   the last block  (the one whose ticket add returns gridDim - 1) gathers the
//                   records into LDS and computes the link -- the next chunk
//                   start of a chunk starting there -- of every record, of the
//                   stream start and of every other start the chain can reach
//                   (max cuts, truncated-region hits), in rounds until no new
//                   start appears; walks the chain from offset 0; writes
//                   Chunk{offset,length}, first[] and the done word.
//
// A link is exact: a chunk starting at c is cut at the first
// p in [c+a0, c+re) whose in-chunk hash (reset at c+a0) hits mask_s below the
// centre / mask_l above it, else at c+rem.  Positions c+a0 .. c+tl-1 (the <= 47
// "truncated" ones) are tested from the bytes; every later position from the
// records, whose windowed hash equals the in-chunk hash there.
//
// Whatever the LDS budgets cannot hold (dense records on low-entropy data, a
// chain longer than the start budget, too many rounds) raises the fallback
// word and the host runs the regular pipeline: no result is ever guessed.
#include "small.hpp"

namespace cdc {
namespace small {
namespace {

#ifndef CDC_SMALL_FEED_ACQ
#define CDC_SMALL_FEED_ACQ 1
#endif
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr uint32_t kPiece = 4096;      // bytes per wave
constexpr uint32_t kLaneHits = 4;      // records a lane keeps (more: fallback)
constexpr uint32_t kCopies = 32;       // GEAR replicas (lane & 31): conflict-free ds_read_b64
constexpr uint32_t kEntCap = kRecCap + 1024;  // + starts that are not records
constexpr uint32_t kRankIters = 12;    // list-ranking doublings: 2^12 > kEntCap + 1
constexpr uint32_t kRounds = 48;       // link rounds (typical data: 1-2)
constexpr uint32_t kNone = 0xFFFFFFFFu;  // link not computed
constexpr uint32_t kEnd = 0xFFFFFFFEu;   // the chunk ends the stream
constexpr uint32_t kHitS = 1u << 31, kHitL = 1u << 30, kPosMask = (1u << 30) - 1;
constexpr uint32_t kTruncNone = 63, kTruncUnknown = 62;
static_assert((1u << kRankIters) > kEntCap + 1, "list ranking depth");

static_assert(kBlockBytes == kWaves * kPiece, "small.hpp block geometry");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint32_t g_u32w;

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    const u32x4 v = *(g_u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 bytes at p (stream offset) of an n-byte stream, zero past the end.
__device__ __forceinline__ uint4 ld16_guarded(const uint8_t *data, uint64_t p, uint64_t n) {
    if (p + 16 <= n) return ld16(data + p);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; p + j < n && j < 16; ++j) w[j >> 2] |= (uint32_t)((g_u8 *)data)[p + j] << (8 * j);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Inter-block words, agent scope (MI355X_MICROARCH.md "Valid forms", the
// last-arriver row: every store and load of the handed-off records is sc1).
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
    __hip_atomic_store((g_u32w *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load((g_u32w *)const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
typedef __attribute__((address_space(1))) uint64_t g_u64w;
__device__ __forceinline__ void st_sc1_64(uint64_t *p, uint64_t v) {
    __hip_atomic_store((g_u64w *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1_64(const uint64_t *p) {
    return __hip_atomic_load((g_u64w *)const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The host's feed words (pinned host memory): system-scope loads, never cached.
__device__ __forceinline__ uint64_t ld_sys_64(const uint64_t *p) {
    return __hip_atomic_load((g_u64w *)const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr uint32_t kPollMax = 1u << 17;  // bounded polls (~0.1-0.3 s): a stuck wait is a fallback, never a hang

struct ScanPart {
    uint4 buf[kWaves][(64 + kPiece) / 16];  // 48 warm-up bytes (+16 pad) ++ the piece
};

// Entries: every record (index = record index), the stream start (index
// nrec), then starts that are not records, appended as rounds find them.
struct ResolvePart {
    uint32_t rec[kRecCap];    // records (position | flags), sorted by position
    uint16_t rtr[kRecCap];    // their truncated results, and those of their max-cut successors << 8
    uint16_t ehint[kEntCap];  // entry: a lower bound of the index of its first record after it
    uint32_t epos[kEntCap];   // entry position
    uint32_t enx[kEntCap];    // entry of the next start (kNone: not computed, kEnd: the chunk ends the stream)
    uint8_t etr[kEntCap];     // truncated-region result (kTruncUnknown: not computed)
    uint8_t tent[kEntCap];    // 1: link assumes no truncated-region hit (a record-free max-cut run)
    uint16_t jmp[2][kEntCap + 1];   // list ranking: 2^k-th successor (kEntCap: past the end)
    uint16_t rank[2][kEntCap + 1];  // list ranking: starts from here to the end of the stream
    uint8_t reach[kEntCap + 1];     // 1: on the chain from offset 0
    uint32_t bbase[kMaxBlocks + 1];
};

struct Lds {
    uint64_t tab[256 * kCopies];  // 64 KiB, LDS address 0: entry e, replica c at e*256 + c*8
    union {
        ScanPart s;
        ResolvePart r;
    } u;
    uint32_t wcnt[kWaves + 1];
    uint32_t nent, fail, last, nstart;
    uint32_t feed_ok;     // 0: the host's feed words never arrived (fallback)
    uint32_t brec[kBlockRecCap];  // this block's records, in position order
    uint8_t bt[kBlockRecCap], btv[kBlockRecCap];  // their truncated results (own, max-cut successor's)
    uint32_t pcnt;                // the previous block's record count (> kBlockRecCap: none)
    uint64_t prec[kBlockRecCap];  // its records (record | tinfo << 32)
    uint8_t pt[kBlockRecCap], ptv[kBlockRecCap];
    uint32_t dcyc[4];     // diag: round 0's max cycles per lane (load + trunc, link, non-record successor)
    uint64_t dround[4];   // diag: end of rounds 0..3 (s_memrealtime)
};

// DPP wave_shr:1 (dpp_ctrl 0x138): lane i receives lane i-1; lane 0 gets `fill`.
__device__ __forceinline__ uint64_t wave_shr1(uint64_t v, uint64_t fill) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)fill, (int)(uint32_t)v, 0x138, 0xF, 0xF,
                                                              false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(fill >> 32), (int)(uint32_t)(v >> 32),
                                                              0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// GEAR[byte b of w] for replica offset rep (v_perm_b32 builds b*256 + rep).
__device__ __forceinline__ uint64_t gear(const uint64_t *tab, uint32_t rep, uint32_t w, int b) {
    const uint32_t addr = __builtin_amdgcn_perm(rep, w, 0x0c0c0004u | ((uint32_t)b << 8));
    return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + addr);
}

__device__ __forceinline__ uint32_t word4(const uint4 &v, int i) {
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

struct Regime {
    uint64_t rem, a0, ce, re, tl;
};

// Chunk regime at start c (fastcdc.hip regime()).
__device__ __forceinline__ Regime regime(const FastParams &fp, uint64_t c, uint64_t n) {
    Regime R;
    uint64_t rem = n - c, center = fp.avg;
    if (rem > fp.max) rem = fp.max; else if (rem < center) center = rem;
    R.rem = rem;
    R.a0 = (fp.min / 2) * 2;
    R.ce = (center / 2) * 2;
    R.re = (rem / 2) * 2;
    R.tl = min(R.a0 + (uint64_t)fp.trunc, R.re);
    return R;
}

// The truncated region of a chunk starting at c: positions c+a0 .. c+tl-1,
// whose in-chunk hash (reset at c+a0) differs from the windowed one.  trunc
// result = the first d in [0, tl - a0) that hits mask_s below the centre /
// mask_l above it, or kTruncNone.  Its <= 47 bytes come as 13 dwords (one
// batch of loads, issued before they are needed) realigned with
// v_alignbyte_b32.
// (cap: readable bytes at data; four 16-byte loads and a 4-way select when
// the aligned 64 bytes around the region are readable, else dword loads,
// the last readable one assembled byte by byte -- all independent; bytes
// past cap read as zero, and positions >= n are never tested)
__device__ __forceinline__ void trunc_load(const uint8_t *data, uint64_t cap, uint64_t w0, uint32_t (&w)[13]) {
    const uint64_t b16 = w0 & ~15ull;
    if (b16 + 64 <= cap) {
        uint32_t W[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 x = ld16(data + b16 + 16 * i);
            W[4 * i] = x.x;
            W[4 * i + 1] = x.y;
            W[4 * i + 2] = x.z;
            W[4 * i + 3] = x.w;
        }
        const uint32_t q = (uint32_t)(w0 >> 2) & 3;
#pragma unroll
        for (int k = 0; k < 13; ++k) w[k] = q == 0 ? W[k] : q == 1 ? W[k + 1] : q == 2 ? W[k + 2] : W[k + 3];
        return;
    }
    const uint64_t a0 = w0 & ~3ull;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
        const uint64_t a = a0 + 4 * i;
        if (a + 4 <= cap) {
            w[i] = *(g_u32 *)(data + a);
        } else {
            uint32_t x = 0;
            for (uint32_t j = 0; j < 4 && a + j < cap; ++j) x |= (uint32_t)((g_u8 *)data)[a + j] << (8 * j);
            w[i] = x;
        }
    }
}

// Branch-free: 12 GEAR lookups issued together per batch (one LDS latency
// per batch, not per byte), hit bits collected in a mask, the first one wins.
// Out of line, every argument by value (an array or struct reference would go
// through scratch): its five callers share one copy of the unrolled body, so
// the last block runs code its CU has already fetched (inlined copies were
// instruction-cache misses on the last block's critical path).
typedef const __attribute__((address_space(3))) uint64_t lds_u64;
typedef const __attribute__((address_space(3))) char lds_char;
__device__ __noinline__ uint32_t trunc_eval_nl(uint32_t w0_, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                                               uint32_t w5, uint32_t w6, uint32_t w7, uint32_t w8, uint32_t w9,
                                               uint32_t w10, uint32_t w11, uint32_t w12, uint32_t sh, uint32_t len,
                                               uint32_t ns, uint64_t mask_s, uint64_t mask_l, lds_u64 *tab,
                                               uint32_t rep) {
    const uint32_t w[13] = {w0_, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12};
    uint64_t h = 0, hits = 0;
#pragma unroll
    for (int k0 = 0; k0 < 12; k0 += 3) {
        uint64_t g[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t a = __builtin_amdgcn_alignbyte(w[k0 + k + 1], w[k0 + k], sh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t addr = __builtin_amdgcn_perm(rep, a, 0x0c0c0004u | ((uint32_t)j << 8));
                g[4 * k + j] = *reinterpret_cast<lds_u64 *>(reinterpret_cast<lds_char *>(tab) + addr);
            }
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const uint32_t d = 4 * k0 + i;
            if (d >= 47) break;
            h = (h << 1) + g[i];
            const uint64_t m = d < ns ? mask_s : mask_l;
            hits |= (uint64_t)((h & m) == 0) << d;
        }
    }
    hits &= len >= 64 ? ~0ull : (1ull << len) - 1;
    return hits ? (uint32_t)__builtin_ctzll(hits) : kTruncNone;
}

__device__ __forceinline__ uint32_t trunc_eval(const uint32_t (&w)[13], uint64_t w0, const Regime &R,
                                               const FastParams &fp, const uint64_t *tab, uint32_t rep) {
    const uint32_t len = (uint32_t)(R.tl - R.a0), sh = (uint32_t)(w0 & 3);
    const uint32_t ns = R.ce > R.a0 ? (uint32_t)min(R.ce - R.a0, (uint64_t)64) : 0u;  // d < ns: mask_s
    return trunc_eval_nl(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], w[8], w[9], w[10], w[11], w[12], sh, len,
                         ns, fp.mask_s, fp.mask_l, (lds_u64 *)tab, rep);
}

// Next start after a chunk starting at c whose truncated result is t: the
// truncated hit, else the first qualifying record (*ri = its index), else the
// max / end cut.
// `hint` is a lower bound of the index of the first record after c (records
// are sorted): the search walks forward from it (~max / 4 KiB records).
__device__ __forceinline__ uint64_t link_from(const uint32_t *rec, uint32_t nrec, uint32_t hint, uint64_t c,
                                              const Regime &R, uint32_t t, uint32_t *ri) {
    *ri = kNone;
    if (t != kTruncNone) return c + R.a0 + t;
    if (R.tl < R.re) {
        for (uint32_t i = hint; i < nrec; ++i) {
            const uint32_t r = rec[i];
            const uint64_t p = r & kPosMask;
            if (p < c + R.tl) continue;
            if (p >= c + R.re) break;
            if (r & (p - c < R.ce ? kHitS : kHitL)) {
                *ri = i;
                return p;
            }
        }
    }
    return c + R.rem;
}

// Max cuts from p on, while the chunk there has no record in its search
// window (so that, barring a truncated hit, it ends at the next max cut):
// the length of that run, p included.
__device__ __forceinline__ uint32_t run_len(const uint32_t *rec, uint32_t nrec, uint32_t hint, const FastParams &fp,
                                           uint64_t n, uint64_t p) {
    uint32_t k = 1, i = hint;
    for (uint64_t v = p; k < 64 && n - v > fp.max; v += fp.max, ++k) {
        const Regime R = regime(fp, v, n);
        while (i < nrec && (uint64_t)(rec[i] & kPosMask) < v + R.tl) ++i;
        if (i < nrec && (uint64_t)(rec[i] & kPosMask) < v + R.re) break;
    }
    return k;
}

// The truncated regions a chunk starting at c needs (its own and, when its
// link may be the max cut v = c + max, v's): their word-aligned first bytes,
// and whether each lies wholly before `reach`.
struct TNeed {
    Regime R, Rv;
    uint64_t v, ac, av;  // ac / av: (w0 & ~3) of c's / v's region
    bool live, hasc, spec, hasv;
};

__device__ __forceinline__ TNeed tneed(uint64_t c, uint64_t n, const FastParams &fp) {
    TNeed T{};
    T.live = n - c > fp.min;  // (else the chunk ends the stream: no result is used)
    if (!T.live) return T;
    T.R = regime(fp, c, n);
    T.v = c + T.R.rem;
    T.spec = T.R.rem == fp.max && n - T.v > fp.min;
    T.Rv = regime(fp, T.spec ? T.v : c, n);
    T.hasc = T.R.tl > T.R.a0;
    T.hasv = T.spec && T.Rv.tl > T.Rv.a0;
    T.ac = (c + T.R.a0) & ~3ull;
    T.av = (T.v + T.Rv.a0) & ~3ull;
    return T;
}

__global__ __launch_bounds__(kThreads, 1) void small_kernel(const uint8_t *__restrict__ data, uint64_t n,
                                                            const FastParams fp, const uint64_t *__restrict__ gtab,
                                                            Scratch ws, cdc_chunk_pod *out, uint64_t out_cap,
                                                            uint64_t *h_stats, uint64_t *h_first, bool stage,
                                                            const Feed feed) {
    __shared__ Lds L;
    // The last block's truncated-region bytes: when the input is host memory
    // (a pinned ring slot read over PCIe), from a device copy the scanning
    // blocks write as they go (HBM latency, not a PCIe round trip per load).
    const uint8_t *const tdata = stage ? ws.copy : data;
    const uint64_t tcap = stage ? kMaxBytes + 64 : n;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t rep = (lane & 31) * 8;
    const bool diag = (fp.diag & kDiagStamps) != 0;
    uint64_t st[6] = {0, 0, 0, 0, 0, 0};
    if (diag && blockIdx.x == 0 && tid == 0) ws.stamp[0] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = tid; i < 256 * kCopies; i += kThreads) L.tab[i] = gtab[i / kCopies];
    const uint64_t P0 = (uint64_t)blockIdx.x * kBlockBytes;  // this block's first byte
    if (tid == 0) {
        L.nent = 0;
        L.fail = 0;
        L.feed_ok = 1;
        for (int k = 0; k < 4; ++k) {
            L.dcyc[k] = 0;
            L.dround[k] = 0;
        }
        // streamed input: every piece holding this block's bytes (and the 64
        // before them) must be in the ring slot (the host stores seq after each)
        if (feed.ready) {
            const uint64_t lo = (P0 >= 64 ? P0 - 64 : 0) >> kFeedLog2, hi = (min(P0 + kBlockBytes, n) - 1) >> kFeedLog2;
            for (uint64_t k = lo; k <= hi && L.feed_ok; ++k) {
                uint32_t i = 0;
                while (ld_sys_64(feed.ready + k) != feed.seq && ++i < kPollMax) __builtin_amdgcn_s_sleep(2);
                if (i >= kPollMax) L.feed_ok = 0;
            }
#if CDC_SMALL_FEED_ACQ
            // system-scope acquire: the slot's bytes are read after their
            // feed words, never from cache lines of the slot's earlier use
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
        }
        if (diag && blockIdx.x == 0) ws.stamp[1] = __builtin_amdgcn_s_memrealtime();
        if (diag) ws.bstamp[blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const bool fed = L.feed_ok != 0;

    // ---- scan: this wave's piece, staged through LDS --------------------------
    const uint64_t P = P0 + (uint64_t)wave * kPiece;
    uint4 *B = L.u.s.buf[wave];
    if (P < n && fed) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 x = ld16_guarded(data, P + i * 1024 + lane * 16, n);
            B[4 + i * 64 + lane] = x;
            if (stage) {  // write-through: the next block reads it with sc1 loads
                uint64_t *d = reinterpret_cast<uint64_t *>(ws.copy + P + i * 1024 + lane * 16);
                st_sc1_64(d, ((uint64_t)x.y << 32) | x.x);
                st_sc1_64(d + 1, ((uint64_t)x.w << 32) | x.z);
            }
        }
        // bytes P-64 .. P-1 (the first lane's 48 warm-up bytes); zeros at the
        // stream start, where no record can be used (positions < a0 + 47)
        if (lane < 4) B[lane] = P ? ld16(data + P - 64 + lane * 16) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();  // (also the GEAR table)
    if (diag && tid == 0) ws.bstamp[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    // Hashing, in two passes of four independent 16-byte chains per lane (the
    // lane's 64 bytes [64 l + 16 k, 64 l + 16 k + 16), k = 0..3) -- 32 chain
    // steps of depth instead of a 112-step warm-up-and-scan chain:
    //   pass 1  each chain's end value e_k from hash 0, plus (lanes 0..2) the
    //           chains over the 48 bytes before the wave's piece;
    //   carry   the windowed hash (bits 0..47) just before chain k is
    //           e_{k-1} + e_{k-2} << 16 + e_{k-3} << 32, the e_{<0} being lane
    //           l-1's e_3, e_2, e_1 (one DPP wave_shr:1 each; lane 0 takes the
    //           header chains);
    //   pass 2  each chain re-run from its carry: every hash is the exact
    //           windowed one, tested against mask_s / mask_l.
    uint64_t HS = 0, HL = 0;  // bit j: position p0 + j hits mask_s / mask_l
    const uint64_t p0 = P + 64 * lane;
    if (P < n && fed) {  // (wave-uniform: the DPP below needs every lane)
        const uint4 *q = B + 4 + 4 * lane;
        const uint4 hx = B[1 + (lane < 3 ? lane : 0)];
        uint64_t e[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
#pragma unroll
                for (int k = 0; k < 4; ++k) e[k] = (e[k] << 1) + gear(L.tab, rep, word4(q[k], w), b);
                e[4] = (e[4] << 1) + gear(L.tab, rep, word4(hx, w), b);
            }
        const uint64_t p1 = wave_shr1(e[1], readlane_u64(e[4], 0));  // lane l-1's chains (lane 0: the header's)
        const uint64_t p2 = wave_shr1(e[2], readlane_u64(e[4], 1));
        const uint64_t p3 = wave_shr1(e[3], readlane_u64(e[4], 2));
        uint64_t hc[4];
        hc[0] = p3 + (p2 << 16) + (p1 << 32);
        hc[1] = e[0] + (p3 << 16) + (p2 << 32);
        hc[2] = e[1] + (e[0] << 16) + (p3 << 32);
        hc[3] = e[2] + (e[1] << 16) + (e[0] << 32);
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    hc[k] = (hc[k] << 1) + gear(L.tab, rep, word4(q[k], w), b);
                    const int j = 16 * k + 4 * w + b;
                    HS |= (uint64_t)((hc[k] & fp.mask_s) == 0) << j;
                    HL |= (uint64_t)((hc[k] & fp.mask_l) == 0) << j;
                }
        // positions past the stream end; the stream's first 48 (no full window:
        // never a usable cut, min >= 64)
        const uint64_t keep = p0 >= n ? 0ull : n - p0 >= 64 ? ~0ull : (1ull << (n - p0)) - 1;
        HS &= keep & (p0 == 0 ? ~0xFFFFFFFFFFFFull : ~0ull);
        HL &= keep & (p0 == 0 ? ~0xFFFFFFFFFFFFull : ~0ull);
    }
    if (diag && tid == 0) ws.bstamp[blockIdx.x * 8 + 2] = __builtin_amdgcn_s_memrealtime();  // (wave 0 hashed)
    // The lane's records in position order (the stream start first: a
    // flagless record at offset 0, the entry of the chain).
    uint32_t hits[kLaneHits] = {0, 0, 0, 0};
    uint32_t nh = p0 == 0 ? 1u : 0u;
    for (uint64_t M = HS | HL; M; M &= M - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(M);
        const uint32_t r = (uint32_t)(p0 + j) | ((HS >> j) & 1 ? kHitS : 0u) | ((HL >> j) & 1 ? kHitL : 0u);
#pragma unroll
        for (uint32_t s2 = 0; s2 < kLaneHits; ++s2)
            if (nh == s2) hits[s2] = r;
        ++nh;
    }
    // Records in position order (lanes of a wave, then the block's waves)
    // into LDS, then their truncated results (tinfo) block-wide, one lane per
    // region (a record's own and its max-cut successor's): from LDS when the
    // region lies in this block's bytes (the buffer of the wave holding the
    // region's last byte starts 64 bytes before that wave's piece, so it holds
    // the whole <= 52-byte region).  The others stay unknown and the last
    // block computes them from the device copy: reading them here over PCIe
    // queues behind the bulk transfer (~10 us), and waiting for a neighbour
    // block's copy puts a hand-off on every block's path (measured slower).
    const bool lane_ovf = nh > kLaneHits || !fed;
    const uint32_t c = lane_ovf ? 0u : nh;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += t;
    }
    const bool wave_ovf = __ballot(lane_ovf) != 0;
    if (lane == 63) L.wcnt[wave] = wave_ovf ? kBlockRecCap + 1 : x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    bool ovf = false;
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t cw = L.wcnt[w];
        ovf |= cw > kBlockRecCap;
        if (w < (int)wave) wbase += cw;
        total += cw;
    }
    ovf |= total > kBlockRecCap;
    if (!ovf) {
        const uint32_t b0 = wbase + x - c;
#pragma unroll
        for (uint32_t s = 0; s < kLaneHits; ++s)
            if (s < c) L.brec[b0 + s] = hits[s];
    }
    __syncthreads();
    // (regions past the stream end read its zero padding in LDS: positions
    // >= n are never tested)
    const uint64_t lds_end = P0 + kBlockBytes;
    if (!ovf && tid < 2 * total) {
        const uint32_t i = tid >> 1;
        const bool vside = tid & 1;
        const uint64_t cp = L.brec[i] & kPosMask;
        const TNeed T = tneed(cp, n, fp);
        uint32_t t = kTruncUnknown;
        if (T.live && (vside ? T.spec : true)) {
            const bool has = vside ? T.hasv : T.hasc;
            const uint64_t a = vside ? T.av : T.ac;
            if (!has) {
                t = kTruncNone;
            } else if (a + 52 <= lds_end) {
                const uint64_t wo = (a + 51 - P0) >> 12;  // wave piece holding the region's last byte
                const uint32_t *src = reinterpret_cast<const uint32_t *>(
                    reinterpret_cast<const uint8_t *>(L.u.s.buf[wo]) + (a - (P0 + (wo << 12) - 64)));
                uint32_t w[13];
#pragma unroll
                for (int k = 0; k < 13; ++k) w[k] = src[k];
                t = vside ? trunc_eval(w, T.v + T.Rv.a0, T.Rv, fp, L.tab, rep) : trunc_eval(w, cp + T.R.a0, T.R, fp, L.tab, rep);
            }
        }
        (vside ? L.btv : L.bt)[i] = (uint8_t)t;
    }
    __syncthreads();
    if (diag && tid == 0) ws.bstamp[blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memrealtime();  // (tinfo)
    uint64_t *region = ws.brec + (uint64_t)blockIdx.x * kBlockRecCap;
    if (!ovf && tid < total)
        st_sc1_64(region + tid, ((uint64_t)(L.bt[tid] | ((uint32_t)L.btv[tid] << 8)) << 32) | L.brec[tid]);
    const uint32_t bcount = ovf ? kBlockRecCap + 1 : total;
    if (tid == 0) st_sc1(ws.bcnt + blockIdx.x, bcount);
    // Publish the records (sc1 stores, drained, then an sc1 flag:
    // MI355X_MICROARCH.md, Valid forms) for the next block.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_sc1_64(ws.bpub + blockIdx.x, (feed.seq << 32) | bcount);

    // ---- the previous block's records: the regions in this block's bytes ---
    // A record c of block b-1 whose region (own, or its max-cut successor's)
    // runs past b-1's bytes has it in this block's first a0 + max + 52 bytes
    // (4/8/16 KiB: 20.5 KiB), i.e. in this block's LDS: evaluate it here.  The
    // wait is on a LOWER block (dispatched first, done loading first under the
    // in-order feed), bounded; results out of reach stay unknown (the last
    // block computes them).
    if (blockIdx.x > 0) {
        if (tid == 0) {
            uint32_t i = 0;
            uint64_t v;
            while (((v = ld_sc1_64(ws.bpub + blockIdx.x - 1)) >> 32) != feed.seq && ++i < kPollMax)
                __builtin_amdgcn_s_sleep(1);
            L.pcnt = i >= kPollMax ? kBlockRecCap + 1 : (uint32_t)v;
        }
        __syncthreads();
        const uint32_t pc = L.pcnt;
        uint64_t *preg = region - kBlockRecCap;
        if (pc <= kBlockRecCap) {
            if (tid < pc) L.prec[tid] = ld_sc1_64(preg + tid);
            __syncthreads();
            if (tid < 2 * pc) {
                const uint32_t i = tid >> 1;
                const bool vside = tid & 1;
                const uint64_t r = L.prec[i];
                uint32_t t = (uint32_t)(r >> (vside ? 40 : 32)) & 0xFF;
                const uint64_t cp = (uint32_t)r & kPosMask;
                if (t == kTruncUnknown) {
                    const TNeed T = tneed(cp, n, fp);
                    const bool has = vside ? T.hasv : T.hasc;
                    const uint64_t a = vside ? T.av : T.ac;
                    if (T.live && has && (vside ? T.spec : true) && a + 51 >= P0 && a + 52 <= lds_end) {
                        const uint64_t wo = (a + 51 - P0) >> 12;
                        const uint32_t *src = reinterpret_cast<const uint32_t *>(
                            reinterpret_cast<const uint8_t *>(L.u.s.buf[wo]) + (a - (P0 + (wo << 12) - 64)));
                        uint32_t w[13];
#pragma unroll
                        for (int k = 0; k < 13; ++k) w[k] = src[k];
                        t = vside ? trunc_eval(w, T.v + T.Rv.a0, T.Rv, fp, L.tab, rep)
                                  : trunc_eval(w, cp + T.R.a0, T.R, fp, L.tab, rep);
                    }
                }
                (vside ? L.ptv : L.pt)[i] = (uint8_t)t;
            }
            __syncthreads();
            if (tid < pc) {
                const uint64_t r = L.prec[tid];
                const uint64_t nr = ((uint64_t)(L.pt[tid] | ((uint32_t)L.ptv[tid] << 8)) << 32) | (uint32_t)r;
                if (nr != r) st_sc1_64(preg + tid, nr);
            }
        }
    }
    // Hand-off (MI355X_MICROARCH.md, Valid forms): every storing wave drains
    // its stores, a barrier, one lane releases and takes the ticket; the block
    // whose add returns gridDim - 1 is the last and reads everyone's records.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (diag && tid == 0) ws.bstamp[blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (diag) ws.bstamp[blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memrealtime();
        const uint32_t t = __hip_atomic_fetch_add(ws.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.last = t == gridDim.x - 1 ? 1u : 0u;
        if (L.last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(ws.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        }
    }
    __syncthreads();
    if (!L.last) return;
    if (diag) st[1] = __builtin_amdgcn_s_memrealtime();

    // ---- the last block: gather the records ------------------------------------
    ResolvePart &Q = L.u.r;
    const uint32_t G = gridDim.x;
    if (tid < G) Q.bbase[tid + 1] = ld_sc1(ws.bcnt + tid);
    __syncthreads();
    if (wave == 0) {  // inclusive prefix of the block counts (G <= kMaxBlocks = 2 per lane)
        const uint32_t i0 = 2 * lane + 1, i1 = 2 * lane + 2;
        const uint32_t a = i0 <= G ? Q.bbase[i0] : 0u, b = i1 <= G ? Q.bbase[i1] : 0u;
        const bool bad = __ballot(a > kBlockRecCap || b > kBlockRecCap) != 0;
        uint32_t s = a + b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(s, o);
            if (lane >= (uint32_t)o) s += t;
        }
        if (i0 <= G) Q.bbase[i0] = s - b;
        if (i1 <= G) Q.bbase[i1] = s;
        if (lane == 0) {
            Q.bbase[0] = 0;
            if (bad) L.fail = 1;
        }
    }
    __syncthreads();
    const uint32_t nrec = Q.bbase[G];
    if (L.fail || nrec > kRecCap) {
        if (tid == 0) L.fail = 1;
    } else {
        for (uint32_t i = tid; i < nrec; i += kThreads) {
            uint32_t a = 0, b = G;  // block of record i: last k with bbase[k] <= i
            while (b - a > 1) {
                const uint32_t m = (a + b) >> 1;
                if (Q.bbase[m] <= i) a = m; else b = m;
            }
            const uint64_t r = ld_sc1_64(ws.brec + (uint64_t)a * kBlockRecCap + (i - Q.bbase[a]));
            Q.rec[i] = (uint32_t)r;
            Q.rtr[i] = (uint16_t)(r >> 32);
        }
    }
    __syncthreads();
    if (diag) st[2] = __builtin_amdgcn_s_memrealtime();
    if (L.fail) goto finish;
    {
        // Entries: every record (record 0 is the flagless one at offset 0,
        // the stream start), with the truncated results the scan computed.
        for (uint32_t i = tid; i < nrec; i += kThreads) {
            Q.epos[i] = Q.rec[i] & kPosMask;
            Q.enx[i] = kNone;
            Q.etr[i] = (uint8_t)(Q.rtr[i] & 0xFF);
            Q.tent[i] = 0;
            Q.ehint[i] = (uint16_t)(i + 1);
        }
        if (tid == 0) L.nent = nrec;
        __syncthreads();
        // ---- links, in rounds -------------------------------------------------
        // An entry's truncated bytes and those of its max-cut successor v =
        // c + max are loaded together (one round trip), unless the scanning
        // block already computed them.  A link that is not a record (the max
        // cut, a truncated hit) becomes a head entry whose own link is
        // computed at once (its bytes: those loaded with v, else one more
        // round trip in this lane), so typical data needs one round.  Starts
        // that are still not records (a max cut after a max cut, a truncated
        // hit after a head) become entries for the next round; record-free
        // runs of max cuts are added whole (run_len), linked tentatively until
        // their truncated results are known.
        uint32_t e0 = 0, e1 = nrec, round = 0;
        for (; e0 < e1 && round < kRounds; ++round) {
            for (uint32_t e = e0 + tid; e < e1; e += kThreads) {
                if (Q.enx[e] != kNone && !Q.tent[e]) continue;  // linked when it was added (a head)
                if (diag && round == 1) atomicAdd(&L.dcyc[3], 1u << 16);
                const uint64_t c = Q.epos[e];
                if (n - c <= fp.min) {  // the tail chunk: it ends the stream
                    Q.enx[e] = kEnd;
                    continue;
                }
                const Regime R = regime(fp, c, n);
                const uint64_t v = c + R.rem;
                const bool spec = R.rem == fp.max && n - v > fp.min;
                const Regime Rv = regime(fp, spec ? v : c, n);
                const uint64_t ts0 = diag ? __builtin_amdgcn_s_memtime() : 0;
                uint32_t t = Q.etr[e];
                const uint32_t tvk = e < nrec ? (uint32_t)(Q.rtr[e] >> 8) : kTruncUnknown;
                const uint32_t hint = Q.ehint[e];
                uint32_t wc[13], wv[13];
                const bool ldc = t == kTruncUnknown && R.tl > R.a0;
                const bool ldv = spec && tvk == kTruncUnknown && Rv.tl > Rv.a0;
                if (ldc) trunc_load(tdata, tcap, c + R.a0, wc);
                if (ldv) trunc_load(tdata, tcap, v + Rv.a0, wv);
                if (t == kTruncUnknown) t = R.tl <= R.a0 ? kTruncNone : trunc_eval(wc, c + R.a0, R, fp, L.tab, rep);
                const uint64_t ts1 = diag ? __builtin_amdgcn_s_memtime() : 0;
                if (Q.tent[e] && t == kTruncNone) continue;  // the run's link stands
                uint32_t ri;
                const uint64_t nx = link_from(Q.rec, nrec, hint, c, R, t, &ri);
                const uint64_t ts2 = diag ? __builtin_amdgcn_s_memtime() : 0;
                uint32_t link;
                if (nx >= n) {
                    link = kEnd;
                } else if (ri != kNone) {
                    link = ri;
                } else {
                    // nx is not a record: a head entry with its link computed
                    // now, then (rarely) a run of entries for the next round.
                    const Regime Rn = regime(fp, nx, n);
                    uint32_t tn = kTruncNone;
                    if (n - nx > fp.min && Rn.tl > Rn.a0) {
                        if (spec && nx == v) {
                            tn = tvk != kTruncUnknown ? tvk : trunc_eval(wv, v + Rv.a0, Rv, fp, L.tab, rep);
                        } else {  // a truncated hit (or an end-regime cut): its bytes now
                            uint32_t wn[13];
                            trunc_load(tdata, tcap, nx + Rn.a0, wn);
                            tn = trunc_eval(wn, nx + Rn.a0, Rn, fp, L.tab, rep);
                        }
                    }
                    uint32_t hl = kNone, rk = 0;
                    uint64_t rp = 0;
                    if (n - nx <= fp.min) {
                        hl = kEnd;
                    } else {
                        uint32_t r2;
                        const uint64_t nx2 = link_from(Q.rec, nrec, hint, nx, Rn, tn, &r2);
                        if (nx2 >= n) {
                            hl = kEnd;
                        } else if (r2 != kNone) {
                            hl = r2;
                        } else {
                            rp = nx2;
                            rk = nx2 == nx + Rn.rem && Rn.rem == fp.max ? run_len(Q.rec, nrec, hint, fp, n, nx2) : 1;
                        }
                    }
                    // A single start after the head (a max cut after a max
                    // cut, or a truncated hit): its link too, now -- one more
                    // round trip in this lane instead of a whole round.
                    uint32_t rl = kNone, rt = kTruncUnknown;
                    if (rk == 1) {
                        if (n - rp <= fp.min) {
                            rl = kEnd;
                        } else {
                            const Regime Rp = regime(fp, rp, n);
                            rt = kTruncNone;
                            if (Rp.tl > Rp.a0) {
                                uint32_t wp2[13];
                                trunc_load(tdata, tcap, rp + Rp.a0, wp2);
                                rt = trunc_eval(wp2, rp + Rp.a0, Rp, fp, L.tab, rep);
                            }
                            uint32_t r3;
                            const uint64_t nx3 = link_from(Q.rec, nrec, hint, rp, Rp, rt, &r3);
                            rl = nx3 >= n ? kEnd : r3 != kNone ? r3 : kNone;
                        }
                    }
                    const uint32_t tot = 1u + rk;
                    const uint32_t b = atomicAdd(&L.nent, tot);
                    if (b + tot > kEntCap) {
                        L.fail = 1;
                        link = kNone;
                    } else {
                        Q.epos[b] = (uint32_t)nx;
                        Q.etr[b] = (uint8_t)tn;
                        Q.enx[b] = hl != kNone ? hl : b + 1;
                        Q.tent[b] = 0;
                        Q.ehint[b] = (uint16_t)hint;
                        for (uint32_t j = 0; j < rk; ++j) {
                            Q.epos[b + 1 + j] = (uint32_t)(rp + (uint64_t)j * fp.max);
                            Q.etr[b + 1 + j] = rk == 1 && rl != kNone ? (uint8_t)rt : (uint8_t)kTruncUnknown;
                            Q.enx[b + 1 + j] = j + 1 < rk ? b + 2 + j : rk == 1 ? rl : kNone;
                            Q.tent[b + 1 + j] = j + 1 < rk ? 1 : 0;
                            Q.ehint[b + 1 + j] = (uint16_t)hint;
                        }
                        link = b;
                    }
                }
                Q.enx[e] = link;
                Q.etr[e] = (uint8_t)t;
                Q.tent[e] = 0;
                if (diag && round == 0) {
                    const uint64_t ts3 = __builtin_amdgcn_s_memtime();
                    atomicMax(&L.dcyc[0], (uint32_t)(ts1 - ts0));
                    atomicMax(&L.dcyc[1], (uint32_t)(ts2 - ts1));
                    atomicMax(&L.dcyc[2], (uint32_t)(ts3 - ts2));
                }
            }
            if (diag && tid == 0 && round < 4) L.dround[round] = __builtin_amdgcn_s_memrealtime();
            if (diag && tid == 0 && round == 0) atomicAdd(&L.dcyc[3], min(L.nent - nrec, 0xFFFFu));
            __syncthreads();
            e0 = e1;
            e1 = min(L.nent, kEntCap);
            if (L.fail) break;
            __syncthreads();
        }
        if (tid == 0 && (e0 < e1 || round >= kRounds)) L.fail = 1;
        if (diag) {
            st[3] = __builtin_amdgcn_s_memrealtime();
            st[0] = round;
        }
        __syncthreads();
        if (L.fail) goto finish;
        // ---- the chain from offset 0: list ranking ------------------------------
        // rank[e] = chunks from entry e to the end of the stream, jmp = the
        // 2^k-th successor (Wyllie doubling, ne = past the end); reach marks
        // the entries within 2^(k+1) steps of the start (entry 0) after round k, so
        // after the last round exactly the chain.  Chunk i of the stream
        // starts at the reached entry of rank rank[start] - i.
        const uint32_t ne = L.nent;
        for (uint32_t e = tid; e <= ne; e += kThreads) {
            const uint32_t x = e < ne ? Q.enx[e] : kEnd;
            Q.jmp[0][e] = (uint16_t)(x >= ne ? ne : x);  // (kNone on the chain: caught below)
            Q.rank[0][e] = e < ne ? 1 : 0;
            Q.reach[e] = e == 0 ? 1 : 0;
        }
        __syncthreads();
        uint32_t b = 0;
        for (uint32_t it = 0; it < kRankIters; ++it, b ^= 1) {
            for (uint32_t e = tid; e <= ne; e += kThreads) {
                const uint32_t j = Q.jmp[b][e];
                if (Q.reach[e]) Q.reach[j] = 1;
                Q.rank[b ^ 1][e] = (uint16_t)(Q.rank[b][e] + Q.rank[b][j]);
                Q.jmp[b ^ 1][e] = Q.jmp[b][j];
            }
            __syncthreads();
        }
        const uint32_t K = Q.rank[b][0];
        if (diag) st[4] = __builtin_amdgcn_s_memrealtime();
        if (K > out_cap) {
            if (tid == 0) L.fail = 1;
        } else {
            for (uint32_t e = tid; e < ne; e += kThreads) {
                if (!Q.reach[e]) continue;
                const uint32_t x = Q.enx[e];
                if (x == kNone) {
                    L.fail = 1;
                    continue;
                }
                const uint64_t s = Q.epos[e];
                const uint64_t nx = x == kEnd ? n : (uint64_t)Q.epos[x];
                out[K - Q.rank[b][e]] = cdc_chunk_pod{s, nx - s};
            }
        }
        if (tid == 0) L.nstart = K;
    }
finish:
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const bool fail = L.fail != 0;
        if (diag) {
            h_stats[kWordStamp0] = __hip_atomic_load(ws.stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int k = 1; k < 5; ++k) h_stats[kWordStamp0 + k] = st[k];
            h_stats[kWordStamp0 + 5] = __builtin_amdgcn_s_memrealtime();
            h_stats[kWordStamp0 + 7] = st[0];
            h_stats[kWordStamp0 + 6] = (uint64_t)L.dcyc[0] | ((uint64_t)L.dcyc[1] << 21) | ((uint64_t)L.dcyc[2] << 42);
            for (int k = 0; k < 4; ++k) h_first[2 + k] = L.dround[k];  // (the staging block has room past first[1])
            h_first[6] = __hip_atomic_load(ws.stamp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // block 0 fed
            h_first[7] = L.dcyc[3];  // entries added by round 0 | entries round 1 worked on << 16
        }
        h_stats[kWordRecords] = nrec;
        h_stats[kWordFallback] = fail ? 1 : 0;
        h_first[0] = 0;
        h_first[1] = fail ? 0 : L.nstart;
        __threadfence_system();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(h_stats + kWordDone, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

hipError_t launch_small(const uint8_t *data, uint64_t n, const FastParams &fp, const uint64_t *d_gear,
                        const Scratch &ws, void *out, uint64_t out_cap, uint64_t *h_stats, uint64_t *h_first,
                        bool stage, const Feed &feed, hipStream_t s) {
    const uint64_t blocks = (n + kBlockBytes - 1) / kBlockBytes;
    if (n == 0 || blocks > kMaxBlocks || feed.seq == 0 || feed.seq >= (1ull << 32)) return hipErrorInvalidValue;
    small_kernel<<<(unsigned)blocks, kThreads, 0, s>>>(data, n, fp, d_gear, ws,
                                                       reinterpret_cast<cdc_chunk_pod *>(out), out_cap, h_stats,
                                                       h_first, stage, feed);
    return hipGetLastError();
}

}  // namespace small
}  // namespace cdc
