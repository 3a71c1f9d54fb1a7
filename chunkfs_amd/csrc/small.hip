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
    uint32_t dcyc[4];     // diag: round 0's max cycles per lane (load + trunc, link, non-record successor)
    uint64_t dround[4];   // diag: end of rounds 0..3 (s_memrealtime)
};

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
// v_alignbyte_b32; near the stream end byte by byte.
__device__ __forceinline__ bool trunc_words_ok(const Regime &R, uint64_t c, uint64_t n) {
    return R.tl > R.a0 && ((c + R.a0) & ~3ull) + 52 <= n;
}

// (cap: readable bytes at data; four 16-byte loads and a 4-way select when
// the aligned 64 bytes around the region are readable, else 13 dword loads)
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
    const uint8_t *p = data + (w0 & ~3ull);
#pragma unroll
    for (int i = 0; i < 13; ++i) w[i] = *(g_u32 *)(p + 4 * i);
}

// Branch-free: 12 GEAR lookups issued together per batch (one LDS latency
// per batch, not per byte), hit bits collected in a mask, the first one wins.
__device__ __forceinline__ uint32_t trunc_eval(const uint32_t (&w)[13], uint64_t w0, const Regime &R,
                                               const FastParams &fp, const uint64_t *tab, uint32_t rep) {
    const uint32_t len = (uint32_t)(R.tl - R.a0), sh = (uint32_t)(w0 & 3);
    const uint32_t ns = R.ce > R.a0 ? (uint32_t)min(R.ce - R.a0, (uint64_t)64) : 0u;  // d < ns: mask_s
    uint64_t h = 0, hits = 0;
#pragma unroll
    for (int k0 = 0; k0 < 12; k0 += 3) {
        uint64_t g[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t a = __builtin_amdgcn_alignbyte(w[k0 + k + 1], w[k0 + k], sh);
#pragma unroll
            for (int j = 0; j < 4; ++j) g[4 * k + j] = gear(tab, rep, a, j);
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const uint32_t d = 4 * k0 + i;
            if (d >= 47) break;
            h = (h << 1) + g[i];
            const uint64_t m = d < ns ? fp.mask_s : fp.mask_l;
            hits |= (uint64_t)((h & m) == 0) << d;
        }
    }
    hits &= len >= 64 ? ~0ull : (1ull << len) - 1;
    return hits ? (uint32_t)__builtin_ctzll(hits) : kTruncNone;
}

// (Out of line, arguments by value: a reference would force the caller's
// Regime / FastParams into scratch memory.)
__device__ __noinline__ uint32_t trunc_bytes_at(const uint8_t *data, uint64_t w0, uint32_t len, uint32_t ns,
                                                uint64_t mask_s, uint64_t mask_l, const uint64_t *tab) {
    uint64_t h = 0;
    for (uint32_t d = 0; d < len; ++d) {
        h = (h << 1) + tab[(uint32_t)((g_u8 *)data)[w0 + d] * kCopies];
        if (!(h & (d < ns ? mask_s : mask_l))) return d;
    }
    return kTruncNone;
}

__device__ __forceinline__ uint32_t trunc_bytes(const uint8_t *data, uint64_t c, const Regime &R, const FastParams &fp,
                                                const uint64_t *tab) {
    const uint32_t ns = R.ce > R.a0 ? (uint32_t)min(R.ce - R.a0, (uint64_t)64) : 0u;
    return trunc_bytes_at(data, c + R.a0, (uint32_t)(R.tl - R.a0), ns, fp.mask_s, fp.mask_l, tab);
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

__global__ __launch_bounds__(kThreads, 1) void small_kernel(const uint8_t *__restrict__ data, uint64_t n,
                                                            const FastParams fp, const uint64_t *__restrict__ gtab,
                                                            Scratch ws, cdc_chunk_pod *out, uint64_t out_cap,
                                                            uint64_t *h_stats, uint64_t *h_first, bool stage) {
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
    if (tid == 0) {
        L.nent = 0;
        L.fail = 0;
        for (int k = 0; k < 4; ++k) {
            L.dcyc[k] = 0;
            L.dround[k] = 0;
        }
    }

    // ---- scan: this wave's piece, staged through LDS --------------------------
    const uint64_t P = ((uint64_t)blockIdx.x * kWaves + wave) * kPiece;
    uint4 *B = L.u.s.buf[wave];
    if (P < n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 x = ld16_guarded(data, P + i * 1024 + lane * 16, n);
            B[4 + i * 64 + lane] = x;
            if (stage) *reinterpret_cast<uint4 *>(ws.copy + P + i * 1024 + lane * 16) = x;
        }
        // bytes P-64 .. P-1 (the first lane's 48 warm-up bytes); zeros at the
        // stream start, where no record can be used (positions < a0 + 47)
        if (lane < 4) B[lane] = P ? ld16(data + P - 64 + lane * 16) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();  // (also the GEAR table)
    uint32_t hits[kLaneHits] = {0, 0, 0, 0};
    uint32_t nh = 0;
    const uint64_t p0 = P + 64 * lane;
    if (p0 == 0) nh = 1;  // a flagless record at offset 0: the entry of the stream start (hits[0] = 0)
    if (p0 < n) {
        // 112 bytes from LDS: 48 warm-up + the lane's 64 (16-byte aligned)
        const uint4 *q = B + 1 + 4 * lane;
        uint64_t h = 0;
#pragma unroll
        for (int v = 0; v < 7; ++v) {
            const uint4 x = q[v];
#pragma unroll
            for (int w = 0; w < 4; ++w)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    h = (h << 1) + gear(L.tab, rep, word4(x, w), b);
                    const int k = 16 * v + 4 * w + b - 48;  // position p0 + k
                    if (k >= 0) {
                        const uint32_t f = ((h & fp.mask_s) == 0 ? kHitS : 0u) | ((h & fp.mask_l) == 0 ? kHitL : 0u);
                        if (f && p0 + k < n) {
                            const uint32_t r = (uint32_t)(p0 + k) | f;
#pragma unroll
                            for (uint32_t s = 0; s < kLaneHits; ++s)
                                if (nh == s) hits[s] = r;
                            ++nh;
                        }
                    }
                }
        }
    }
    // (The records' truncated results are computed by the last block from the
    // device copy: loads from the host slot here would put a PCIe round trip
    // per record on every block's critical path.)
    const uint32_t tinfo[kLaneHits] = {kTruncUnknown | (kTruncUnknown << 8), kTruncUnknown | (kTruncUnknown << 8),
                                       kTruncUnknown | (kTruncUnknown << 8), kTruncUnknown | (kTruncUnknown << 8)};
    // Records in position order: lanes of a wave, then the block's waves.
    const bool lane_ovf = nh > kLaneHits;
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
    uint64_t *region = ws.brec + (uint64_t)blockIdx.x * kBlockRecCap;
    if (!ovf) {
        const uint32_t b0 = wbase + x - c;
#pragma unroll
        for (uint32_t s = 0; s < kLaneHits; ++s)
            if (s < c) st_sc1_64(region + b0 + s, ((uint64_t)tinfo[s] << 32) | hits[s]);
    }
    if (tid == 0) st_sc1(ws.bcnt + blockIdx.x, ovf ? kBlockRecCap + 1 : total);
    // Hand-off (MI355X_MICROARCH.md, Valid forms): every storing wave drains
    // its stores, a barrier, one lane releases and takes the ticket; the block
    // whose add returns gridDim - 1 is the last and reads everyone's records.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
        // c + max are loaded together (one round trip): when the link is that
        // max cut -- ~10 % of chunks at 4/8/16 KiB -- v's own link follows from
        // the records at once, so typical data needs one round.  New starts
        // that are not records (truncated hits, a max cut after a max cut)
        // become entries for the next round; record-free runs of max cuts are
        // added whole (run_len), linked tentatively until their truncated
        // results are known.
        uint32_t e0 = 0, e1 = nrec, round = 0;
        for (; e0 < e1 && round < kRounds; ++round) {
            for (uint32_t e = e0 + tid; e < e1; e += kThreads) {
                if (Q.enx[e] != kNone && !Q.tent[e]) continue;  // linked when it was added (a head)
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
                const bool ldc = t == kTruncUnknown && trunc_words_ok(R, c, n);
                const bool ldv = spec && tvk == kTruncUnknown && trunc_words_ok(Rv, v, n);
                if (ldc) trunc_load(tdata, tcap, c + R.a0, wc);
                if (ldv) trunc_load(tdata, tcap, v + Rv.a0, wv);
                if (t == kTruncUnknown)
                    t = R.tl <= R.a0 ? kTruncNone : ldc ? trunc_eval(wc, c + R.a0, R, fp, L.tab, rep)
                                                        : trunc_bytes(tdata, c, R, fp, L.tab);
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
                    // nx is not a record.  Head entry (v, when nx is the max
                    // cut whose bytes came with this round) with its link
                    // computed now, then a run of entries for the next round.
                    bool head = false;
                    uint32_t hl = kNone, tv = kTruncNone;
                    uint64_t rp = nx;
                    uint32_t rk = 0;
                    if (spec && nx == v) {
                        head = true;
                        tv = tvk != kTruncUnknown ? tvk : Rv.tl <= Rv.a0 ? kTruncNone
                             : ldv ? trunc_eval(wv, v + Rv.a0, Rv, fp, L.tab, rep) : trunc_bytes(tdata, v, Rv, fp, L.tab);
                        uint32_t r2;
                        const uint64_t nx2 = link_from(Q.rec, nrec, hint, v, Rv, tv, &r2);
                        if (nx2 >= n) {
                            hl = kEnd;
                        } else if (r2 != kNone) {
                            hl = r2;
                        } else {
                            rp = nx2;
                            rk = nx2 == v + Rv.rem && Rv.rem == fp.max ? run_len(Q.rec, nrec, hint, fp, n, nx2) : 1;
                        }
                    } else {
                        rk = nx == c + R.rem && R.rem == fp.max ? run_len(Q.rec, nrec, hint, fp, n, nx) : 1;
                    }
                    const uint32_t tot = (head ? 1u : 0u) + rk;
                    const uint32_t b = atomicAdd(&L.nent, tot);
                    if (b + tot > kEntCap) {
                        L.fail = 1;
                        link = kNone;
                    } else {
                        if (head) {
                            Q.epos[b] = (uint32_t)v;
                            Q.etr[b] = (uint8_t)tv;
                            Q.enx[b] = hl != kNone ? hl : b + 1;
                            Q.tent[b] = 0;
                            Q.ehint[b] = (uint16_t)hint;
                        }
                        const uint32_t r0 = b + (head ? 1u : 0u);
                        for (uint32_t j = 0; j < rk; ++j) {
                            Q.epos[r0 + j] = (uint32_t)(rp + (uint64_t)j * fp.max);
                            Q.etr[r0 + j] = kTruncUnknown;
                            Q.enx[r0 + j] = j + 1 < rk ? r0 + j + 1 : kNone;
                            Q.tent[r0 + j] = j + 1 < rk ? 1 : 0;
                            Q.ehint[r0 + j] = (uint16_t)hint;
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
                        bool stage, hipStream_t s) {
    const uint64_t blocks = (n + kBlockBytes - 1) / kBlockBytes;
    if (n == 0 || blocks > kMaxBlocks) return hipErrorInvalidValue;
    small_kernel<<<(unsigned)blocks, kThreads, 0, s>>>(data, n, fp, d_gear, ws,
                                                       reinterpret_cast<cdc_chunk_pod *>(out), out_cap, h_stats,
                                                       h_first, stage);
    return hipGetLastError();
}

}  // namespace small
}  // namespace cdc
