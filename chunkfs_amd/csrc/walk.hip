// walk.hip -- hand-written gfx950 kernels of the segment-walk engine: Rabin,
// UltraCDC, LeapCDC and SeqCDC chunk_data (reference src/chunkers/rabin.rs:
// 34-56, ultra.rs:30-44, leap.rs:30-44, seq.rs:40-55).  See walk.hpp.
//
// The cut rules below restate the published algorithms exactly as
// oracle/cdc_oracle.c does (the oracle is the checker, never linked here);
// constants come from include/chunkfs_amd_cdc_params.h.  PARITY UNPINNED vs
// the reference's crate (cdc-chunkers 0.1.3, absent offline).
//
// Kernels, one launch each, all on the handle's stream:
//   walk_kernel    lane per segment: warm-up walk, then the segment's starts
//   fix_kernel     lane per segment: re-walk where entry != predecessor exit
//   serial_kernel  one lane: in-order re-walk from the lowest changed segment
//   sum/scan/emit  block sums of N -> block prefix -> per-segment prefix and
//                  the Chunk{offset,length} output; first[] per stream
#include "walk.hpp"

#include "../../include/chunkfs_amd_cdc_params.h"

namespace cdc {
namespace walk {
namespace {

constexpr int kWalkBlock = 64;  // one wave per block: lanes own independent segments

// Largest stream i with span_base[i] <= g.
__device__ __forceinline__ void locate(const StreamTable &st, uint64_t g, uint32_t &si, uint64_t &off) {
    uint32_t lo = 0, hi = st.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (st.span_base[mid] <= g) lo = mid; else hi = mid;
    }
    si = lo;
    off = (g - st.span_base[lo]) << st.span_log2;
}

// Byte reader over one stream: a per-lane window of kWin bytes in LDS.  A
// lane that steps outside its window makes EVERY active lane of the wave
// re-centre its own window at its current position in the same refill (one
// ballot, kWin/16 global_load_dwordx4 per lane in flight together), so a wave
// pays one memory latency per >= kWin - kBack - 16 bytes of progress instead
// of one per divergent 16-byte miss.  Bytes past the stream end read as 0 and
// are never loaded.
constexpr uint32_t kWin = 256;                // window bytes per lane
constexpr uint32_t kBack = 64;                // bytes kept behind the position at a refill
constexpr uint32_t kSlot = kWin + 16;         // LDS stride per lane (bank spread)

// Refill of one lane's window (out of line: one copy per kernel, called from
// every read site); returns the new window start.
__device__ __noinline__ uint64_t refill_window(const uint8_t *base, uint64_t len, uint8_t *slot, uint64_t p) {
    const uint64_t w0 = (p > kBack ? p - kBack : 0) & ~15ull;
    uint4 v[kWin / 16];
#pragma unroll
    for (uint32_t k = 0; k < kWin / 16; ++k) {
        const uint64_t a = w0 + 16 * k;
        if (a + 16 <= len) {
            v[k] = *reinterpret_cast<const uint4 *>(base + a);
        } else {
            uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
            for (uint32_t j = 0; a + j < len && j < 16; ++j) {
                const uint32_t x = (uint32_t)base[a + j] << (8 * (j & 3));
                if (j < 4) t0 |= x;
                else if (j < 8) t1 |= x;
                else if (j < 12) t2 |= x;
                else t3 |= x;
            }
            v[k] = make_uint4(t0, t1, t2, t3);
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < kWin / 16; ++k) reinterpret_cast<uint4 *>(slot)[k] = v[k];
    return w0;
}

struct Reader {
    const uint8_t *base;
    uint64_t len;
    uint64_t w0;     // window start (stream offset, 16-aligned)
    uint8_t *slot;   // this lane's LDS window

    __device__ void init(const uint8_t *b, uint64_t l, uint8_t *lds_slot) {
        base = b;
        len = l;
        w0 = ~0ull >> 1;  // empty: the first at() refills
        slot = lds_slot;
    }
    // Make [lo, hi] (hi - lo < kWin - kBack - 16) resident; then raw() reads it.
    __device__ __forceinline__ void ensure(uint64_t lo, uint64_t hi) {
        const bool miss = lo - w0 >= kWin || hi - w0 >= kWin;  // (below w0 wraps to a miss)
        if (__ballot(miss)) w0 = refill_window(base, len, slot, lo);  // every active lane, at its own position
    }
    __device__ __forceinline__ uint32_t raw(uint64_t p) const { return slot[p - w0]; }
    __device__ __forceinline__ uint32_t at(uint64_t p) {
        ensure(p, p);
        return raw(p);
    }
    __device__ __forceinline__ uint64_t at8(uint64_t p) {
        ensure(p, p + 7);
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v |= (uint64_t)raw(p + j) << (8 * j);
        return v;
    }
};

struct Tabs {
    const uint64_t *mod, *out, *leap;
};

// ---- cut rules: length of the chunk starting at s, n = bytes left ----------

// Rabin fingerprint over the last CDC_RABIN_WINDOW bytes (window reset at the
// chunk start, fed from s + min - W so every tested digest is a full window).
__device__ uint64_t cut_rabin(Reader &in, uint64_t s, uint64_t n, const WalkParams &wp, const Tabs &T) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    constexpr uint64_t W = CDC_RABIN_WINDOW;
    const uint64_t start = wp.min >= W ? wp.min - W : 0;
    uint64_t d = 0;
    for (uint64_t i = start; i < end; ++i) {
        in.ensure(s + i - (i >= start + W ? W : 0), s + i);
        const uint32_t o = i >= start + W ? in.raw(s + i - W) : 0u;
        d ^= T.out[o];
        const uint64_t top = d >> wp.rabin_shift;
        d = ((d << 8) | in.raw(s + i)) ^ T.mod[top];
        if (i + 1 >= wp.min && (d & wp.rabin_mask) == 0) return i + 1;
    }
    return end;
}

// UltraCDC: Hamming distance of the 8 bytes before each position to the
// 0xAA pattern (kept incrementally), MASK_S before `normal`, MASK_L after;
// LEST identical 8-byte blocks in a row cut early.
__device__ uint64_t cut_ultra(Reader &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    uint64_t normal = wp.avg, end = n;
    if (n >= wp.max) end = wp.max;
    else if (n <= normal) normal = n;
    constexpr uint64_t pat = 0x0101010101010101ull * CDC_ULTRA_PATTERN;
    uint64_t outw = r.at8(s + wp.min - 8);
    uint32_t dist = (uint32_t)__popcll(outw ^ pat);
    uint32_t lec = 0;
    for (uint64_t i = wp.min; i + 8 <= end; i += 8) {
        const uint64_t inw = r.at8(s + i);
        if (inw == outw) {
            if (++lec >= CDC_ULTRA_LEST) return i + 8;
            continue;
        }
        lec = 0;
        const uint32_t mask = i >= normal ? CDC_ULTRA_MASK_L : CDC_ULTRA_MASK_S;
        const uint64_t ib = inw ^ pat, ob = outw ^ pat;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((dist & mask) == 0) return i + j;
            dist += (uint32_t)__popc((uint32_t)(ib >> (8 * j)) & 0xFFu);
            dist -= (uint32_t)__popc((uint32_t)(ob >> (8 * j)) & 0xFFu);
        }
        outw = inw;
    }
    return end;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, uint32_t r) { return r ? (x << r) | (x >> (64 - r)) : x; }

// LeapCDC: 24 eligible windows ending at c-1, c-2, ..., c-24 (22 primary,
// 2 secondary); a failure at distance k leaps the candidate by 24 - k.
__device__ uint64_t cut_leap(Reader &r, uint64_t s, uint64_t n, const WalkParams &wp, const Tabs &T) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    uint64_t c = wp.min;
    while (c <= end) {
        uint32_t k = 0;
        for (; k < CDC_LEAP_WINDOWS; ++k) {
            const uint64_t p = s + c - 1 - k;
            r.ensure(p - (CDC_LEAP_WSIZE - 1), p);
            uint64_t h = 0;
#pragma unroll
            for (uint32_t j = 0; j < CDC_LEAP_WSIZE; ++j) h += rotl64(T.leap[r.raw(p - j)], 11 * j);
            const uint32_t v = k < CDC_LEAP_PRIMARY ? (uint32_t)(h >> 32) : (uint32_t)h;
            if (v >= wp.leap_thr) break;
        }
        if (k == CDC_LEAP_WINDOWS) return c;
        c += CDC_LEAP_WINDOWS - k;
    }
    return end;
}

// SeqCDC: seq_len consecutive pairs in the mode's direction cut after the
// last byte; seq_trig opposing pairs jump seq_jump bytes ahead.
__device__ uint64_t cut_seq(Reader &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    uint32_t cnt = 0, opp = 0;
    uint64_t i = wp.min;
    uint32_t a = r.at(s + i - 1);
    while (i < end) {
        const uint32_t b = r.at(s + i);
        if (wp.seq_mode ? b < a : b > a) {
            if (++cnt >= wp.seq_len) return i + 1;
        } else {
            cnt = 0;
            if (++opp >= wp.seq_trig) {
                opp = 0;
                i += wp.seq_jump;
                if (i < end) a = r.at(s + i - 1);
                continue;
            }
        }
        a = b;
        ++i;
    }
    return end;
}

template <int kAlgo>
__device__ __forceinline__ uint64_t cut(Reader &r, uint64_t s, uint64_t len, const WalkParams &wp, const Tabs &T) {
    if constexpr (kAlgo == 2) return cut_rabin(r, s, len - s, wp, T);
    else if constexpr (kAlgo == 4) return cut_ultra(r, s, len - s, wp);
    else if constexpr (kAlgo == 5) return cut_leap(r, s, len - s, wp, T);
    else return cut_seq(r, s, len - s, wp);
}

// Walk from chunk start c (< seg_end) to the first start >= seg_end,
// recording the starts in the segment's list.
template <int kAlgo>
__device__ void walk_from(uint64_t c, uint64_t g, uint64_t seg_end, uint64_t len, Reader &r,
                          const WalkParams &wp, const Tabs &T, const WalkState &ws) {
    ws.E[g] = c;
    uint32_t cnt = 0;
    uint64_t *list = ws.list + g * wp.cap;
    while (c < seg_end) {
        if (cnt < wp.cap) list[cnt] = c;
        ++cnt;
        c += cut<kAlgo>(r, c, len, wp, T);
    }
    ws.X[g] = c;
    ws.N[g] = cnt;
    if (cnt > wp.cap) atomicAdd(&ws.flags[1], 1ull);
}

__device__ __forceinline__ void load_tabs(uint64_t *sh, const uint64_t *g) {
    for (int i = threadIdx.x; i < 768; i += blockDim.x) sh[i] = g[i];
    __syncthreads();
}

template <int kAlgo>
__global__ __launch_bounds__(kWalkBlock) void walk_kernel(const StreamTable st, const WalkParams wp,
                                                          const WalkState ws) {
    __shared__ uint64_t tab[768];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWalkBlock * kSlot];
    load_tabs(tab, wp.tabs);
    const Tabs T{tab, tab + 256, tab + 512};
    const uint64_t g = (uint64_t)blockIdx.x * kWalkBlock + threadIdx.x;
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t len = st.lens[si];
    const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
    Reader r;
    r.init(st.ptrs[si], len, win + threadIdx.x * kSlot);
    // Warm-up start: `warm` bytes back, on the max-length grid of the stream
    // (so runs of max-length cuts from the stream start are in phase).
    uint64_t c = 0;
    if (off != 0) {
        c = off > wp.warm ? off - wp.warm : 0;
        c = c / wp.max * wp.max;
        while (c < off) c += cut<kAlgo>(r, c, len, wp, T);
    }
    walk_from<kAlgo>(c, g, seg_end, len, r, wp, T, ws);
}

template <int kAlgo>
__global__ __launch_bounds__(kWalkBlock) void fix_kernel(const StreamTable st, const WalkParams wp,
                                                         const WalkState ws) {
    __shared__ uint64_t tab[768];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWalkBlock * kSlot];
    load_tabs(tab, wp.tabs);
    const Tabs T{tab, tab + 256, tab + 512};
    const uint64_t g = (uint64_t)blockIdx.x * kWalkBlock + threadIdx.x;
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    if (off == 0) return;  // a stream's first segment starts exactly at 0
    const uint64_t x = ws.Xs[g - 1];
    if (ws.E[g] == x) return;
    const uint64_t len = st.lens[si];
    const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
    Reader r;
    r.init(st.ptrs[si], len, win + threadIdx.x * kSlot);
    walk_from<kAlgo>(x, g, seg_end, len, r, wp, T, ws);
    atomicAdd(&ws.flags[0], 1ull);
    atomicMin(&ws.flags[2], (unsigned long long)g);
}

template <int kAlgo>
__global__ __launch_bounds__(kWalkBlock) void serial_kernel(const StreamTable st, const WalkParams wp,
                                                            const WalkState ws) {
    __shared__ uint64_t tab[768];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWalkBlock * kSlot];
    load_tabs(tab, wp.tabs);
    const Tabs T{tab, tab + 256, tab + 512};
    if (threadIdx.x != 0) return;
    for (uint64_t g = ws.flags[2]; g < st.total_spans; ++g) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        if (off == 0) continue;
        const uint64_t x = ws.X[g - 1];
        if (ws.E[g] == x) continue;
        const uint64_t len = st.lens[si];
        const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
        Reader r;
        r.init(st.ptrs[si], len, win + threadIdx.x * kSlot);
        walk_from<kAlgo>(x, g, seg_end, len, r, wp, T, ws);
    }
}

// ---- prefix and output -----------------------------------------------------

__device__ __forceinline__ uint64_t block_exclusive(uint64_t v, uint64_t *sh, uint64_t &total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kScanBlock; o <<= 1) {
        const uint64_t a = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    total = sh[kScanBlock - 1];
    const uint64_t ex = sh[t] - v;
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(kScanBlock) void sum_kernel(const StreamTable st, const WalkState ws) {
    __shared__ uint64_t sh[kScanBlock];
    const uint64_t g = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
    const uint64_t v = g < st.total_spans ? ws.N[g] : 0;
    uint64_t total;
    (void)block_exclusive(v, sh, total);
    if (threadIdx.x == 0) ws.bsum[blockIdx.x] = total;
}

// One block: exclusive prefix of the nb block sums in place; bsum[nb] = total.
__global__ __launch_bounds__(kScanBlock) void scan_kernel(const WalkState ws, uint64_t nb) {
    __shared__ uint64_t sh[kScanBlock];
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += kScanBlock) {
        const uint64_t i = b0 + threadIdx.x;
        const uint64_t v = i < nb ? ws.bsum[i] : 0;
        uint64_t total;
        const uint64_t ex = block_exclusive(v, sh, total);
        if (i < nb) ws.bsum[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) ws.bsum[nb] = carry;
}

__global__ __launch_bounds__(kScanBlock) void emit_kernel(const StreamTable st, const WalkParams wp,
                                                          const WalkState ws, cdc_chunk_pod *out,
                                                          uint64_t out_cap) {
    __shared__ uint64_t sh[kScanBlock];
    const uint64_t g = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
    const uint32_t n = g < st.total_spans ? ws.N[g] : 0;
    uint64_t total;
    const uint64_t p = ws.bsum[blockIdx.x] + block_exclusive(n, sh, total);
    if (g >= st.total_spans) return;
    ws.P[g] = p;
    if (n > wp.cap || p + n > out_cap) {
        atomicAdd(&ws.flags[1], 1ull);
        return;
    }
    const uint64_t *list = ws.list + g * wp.cap;
    for (uint32_t k = 0; k < n; ++k) {
        const uint64_t s = list[k];
        const uint64_t nx = k + 1 < n ? list[k + 1] : ws.X[g];
        out[p + k] = cdc_chunk_pod{s, nx - s};
    }
}

__global__ void first_kernel(const StreamTable st, const WalkState ws, uint64_t nb) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > st.n) return;
    const uint64_t g = i < st.n ? st.span_base[i] : st.total_spans;
    ws.first[i] = g < st.total_spans ? ws.P[g] : ws.bsum[nb];
}

template <int kAlgo>
hipError_t walk_dispatch(int which, const StreamTable &st, const WalkParams &wp, const WalkState &ws,
                         hipStream_t s) {
    const unsigned blocks = (unsigned)((st.total_spans + kWalkBlock - 1) / kWalkBlock);
    if (which == 0) walk_kernel<kAlgo><<<blocks, kWalkBlock, 0, s>>>(st, wp, ws);
    else if (which == 1) fix_kernel<kAlgo><<<blocks, kWalkBlock, 0, s>>>(st, wp, ws);
    else serial_kernel<kAlgo><<<1, kWalkBlock, 0, s>>>(st, wp, ws);
    return hipGetLastError();
}

hipError_t dispatch(int which, const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    switch (wp.algo) {
        case 2: return walk_dispatch<2>(which, st, wp, ws, s);
        case 4: return walk_dispatch<4>(which, st, wp, ws, s);
        case 5: return walk_dispatch<5>(which, st, wp, ws, s);
        case 6: return walk_dispatch<6>(which, st, wp, ws, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_walk(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    return dispatch(0, st, wp, ws, s);
}

hipError_t launch_fix(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    hipError_t e = hipMemcpyAsync(ws.Xs, ws.X, st.total_spans * 8, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    return dispatch(1, st, wp, ws, s);
}

hipError_t launch_serial(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    return dispatch(2, st, wp, ws, s);
}

hipError_t launch_emit(const StreamTable &st, const WalkParams &wp, const WalkState &ws, void *d_out,
                       uint64_t out_cap, hipStream_t s) {
    const uint64_t nb = (st.total_spans + kScanBlock - 1) / kScanBlock;
    if (nb) {
        sum_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(st, ws);
        scan_kernel<<<1, kScanBlock, 0, s>>>(ws, nb);
        emit_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(st, wp, ws, reinterpret_cast<cdc_chunk_pod *>(d_out),
                                                        out_cap);
    }
    first_kernel<<<(unsigned)((st.n + 1 + 255) / 256), 256, 0, s>>>(st, ws, nb);
    return hipGetLastError();
}

}  // namespace walk
}  // namespace cdc
