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
//   *bits_kernel   per-position predicate bitmaps (data-parallel pass)
//   jtab_kernel    LeapCDC: per-word orbit tables
//   wwalk_kernel   wave per segment: warm-up walk, then the segment's starts
//                  (bitmap mode; walk_kernel = lane per segment, byte mode and
//                  the CHUNKFS_AMD_WAVE=0 A/B path)
//   wfix_kernel    re-walk where entry != predecessor exit, running ahead
//                  into unscheduled successors (fix_kernel: lane version)
//   wserial_kernel wave per stream: in-order re-walk from the lowest changed
//                  segment (serial_kernel: lane per stream)
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

// The data-parallel passes (bitmaps, Leap tables) run over pieces of
// 2^wp.piece_log2 bytes, so their parallelism does not shrink when the walk
// segments grow.  Piece q: segment g, stream si, stream offset off, and the
// index of its first 64-position word in the segment-major bitmap arrays.
struct Piece {
    uint64_t g, off, wbase;
    uint32_t si;
};

__device__ __forceinline__ bool piece_of(const StreamTable &st, const WalkParams &wp, uint64_t q, Piece &p) {
    const uint32_t k = st.span_log2 - wp.piece_log2;
    p.g = q >> k;
    if (p.g >= st.total_spans) return false;
    uint64_t off;
    locate(st, p.g, p.si, off);
    const uint64_t sub = q & ((1ull << k) - 1);
    p.off = off + (sub << wp.piece_log2);
    p.wbase = p.g * wp.seg_words + (sub << (wp.piece_log2 - 6));
    return true;
}

// Byte reader over one stream: a per-lane window of kWin bytes in LDS.  A
// lane that steps outside its window makes EVERY active lane of the wave
// re-centre its own window at its current position in the same refill (one
// ballot, kWin/16 global_load_dwordx4 per lane in flight together), so a wave
// pays one memory latency per >= kWin - kBack - 16 bytes of progress instead
// of one per divergent 16-byte miss.  Bytes past the stream end read as 0 and
// are never loaded.
constexpr uint32_t kWin = 512;                // window bytes per lane
constexpr uint32_t kBack = 64;                // bytes kept behind the position at a refill
constexpr uint32_t kSlot = kWin + 16;         // LDS stride per lane (bank spread)

// Refill of one lane's window (out of line: one copy per kernel, called from
// every read site); returns the new window start.  The window is loaded in
// batches of 16 global_load_dwordx4 with the next batch in flight while the
// previous one is written to LDS (64 + 64 VGPRs, no spills).  512 B windows
// (39 KiB per one-wave walk block) keep 4 walk waves per CU: 1 KiB windows
// held 2 and ran inputs above 1 GiB in batches (profiles/r02at, r02au).
constexpr uint32_t kBatch = 16;

__device__ __forceinline__ uint4 load_piece(const uint8_t *base, uint64_t len, uint64_t a) {
    if (a + 16 <= len) return *reinterpret_cast<const uint4 *>(base + a);
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    for (uint32_t j = 0; a + j < len && j < 16; ++j) {
        const uint32_t x = (uint32_t)base[a + j] << (8 * (j & 3));
        if (j < 4) t0 |= x;
        else if (j < 8) t1 |= x;
        else if (j < 12) t2 |= x;
        else t3 |= x;
    }
    return make_uint4(t0, t1, t2, t3);
}

__device__ __noinline__ uint64_t refill_window(const uint8_t *base, uint64_t len, uint8_t *slot, uint64_t p) {
    const uint64_t w0 = (p > kBack ? p - kBack : 0) & ~15ull;
    constexpr uint32_t nb = kWin / 16 / kBatch;
    uint4 v[2][kBatch];
#pragma unroll
    for (uint32_t k = 0; k < kBatch; ++k) v[0][k] = load_piece(base, len, w0 + 16 * k);
#pragma unroll
    for (uint32_t b = 0; b < nb; ++b) {
        if (b + 1 < nb) {
#pragma unroll
            for (uint32_t k = 0; k < kBatch; ++k)
                v[(b + 1) & 1][k] = load_piece(base, len, w0 + 16 * ((b + 1) * kBatch + k));
        }
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) reinterpret_cast<uint4 *>(slot)[b * kBatch + k] = v[b & 1][k];
    }
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
    // Bitmap mode: word widx (8-byte aligned in the stream's bitmap bytes).
    __device__ __forceinline__ uint64_t word(uint64_t widx) {
        ensure(widx * 8, widx * 8 + 7);
        return *reinterpret_cast<const uint64_t *>(slot + (widx * 8 - w0));
    }
    // n (1..64) bits of bitmap b from position p, bit j = position p + j.
    __device__ __forceinline__ uint64_t bits(uint32_t nbm, uint32_t b, uint64_t p, uint32_t n) {
        const uint64_t k = p >> 6;
        const uint32_t sh = (uint32_t)(p & 63);
        uint64_t v;
        if (sh + n <= 64) {
            v = word(k * nbm + b) >> sh;
        } else {
            ensure(k * nbm * 8, ((k + 1) * nbm + b) * 8 + 7);
            const uint64_t lo = *reinterpret_cast<const uint64_t *>(slot + ((k * nbm + b) * 8 - w0));
            const uint64_t hi = *reinterpret_cast<const uint64_t *>(slot + (((k + 1) * nbm + b) * 8 - w0));
            v = (lo >> sh) | (hi << (64 - sh));
        }
        return n == 64 ? v : v & ((1ull << n) - 1);
    }
    __device__ __forceinline__ uint64_t at8(uint64_t p) {
        ensure(p, p + 7);
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v |= (uint64_t)raw(p + j) << (8 * j);
        return v;
    }
};

// Bitmap reader straight from global memory (L1 / L2), for the link kernels'
// one-chunk walks: an aligned window of 8 words (4 x 16-byte loads issued
// together) stays in registers.  Same interface as Reader's bitmap
// accessors; words past the end read 0.
struct GReader {
    const uint64_t *w;
    uint64_t nw;              // words of the stream's bitmaps
    uint64_t ck = ~0ull;      // first word of the cached window (multiple of 8)
    uint64_t c[8];

    __device__ void init(const uint64_t *base, uint64_t nwords) {
        w = base;
        nw = nwords;
        ck = ~0ull;
    }
    __device__ __forceinline__ uint64_t word(uint64_t i) {
        const uint64_t k = i & ~7ull;
        if (k != ck) {
            ck = k;
            if (k + 8 <= nw) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(w + k + 2 * q);
                    c[2 * q] = ((uint64_t)v.y << 32) | v.x;
                    c[2 * q + 1] = ((uint64_t)v.w << 32) | v.z;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) c[q] = k + q < nw ? w[k + q] : 0;
            }
        }
        uint64_t v = c[0];
#pragma unroll
        for (int q = 1; q < 8; ++q)
            if ((i & 7) == (uint64_t)q) v = c[q];
        return v;
    }
    __device__ __forceinline__ uint64_t bits(uint32_t nbm, uint32_t b, uint64_t p, uint32_t n) {
        const uint64_t k = p >> 6;
        const uint32_t sh = (uint32_t)(p & 63);
        uint64_t v = word(k * nbm + b) >> sh;
        if (sh + n > 64) v |= word((k + 1) * nbm + b) << (64 - sh);
        return n == 64 ? v : v & ((1ull << n) - 1);
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

// ---- the same rules over the predicate bitmaps (bits_kernel) ---------------
// Rabin (min >= 48): every tested digest is a full 48-byte window, so a hit is
// the bitmap bit; the cut is the first hit in [s+min-1, s+end-1], plus one.
template <class R>
__device__ uint64_t cut_rabin_bits(R &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    const uint64_t lo = s + wp.min - 1, hi = s + end - 1;
    for (uint64_t k = lo >> 6; k <= (hi >> 6); ++k) {
        uint64_t w = r.word(k);
        if (k == (lo >> 6)) w &= ~0ull << (lo & 63);
        if (k == (hi >> 6) && (hi & 63) != 63) w &= (2ull << (hi & 63)) - 1;
        if (w) return k * 64 + (uint64_t)__builtin_ctzll(w) - s + 1;
    }
    return end;
}

// UltraCDC over bitmaps 0 (dist & MASK_S == 0), 1 (dist & MASK_L == 0) and
// 2 (the 8 bytes at q repeat the 8 before).  64 positions at a time while no
// block start repeats and no position hits, else block by block as cut_ultra.
template <class R>
__device__ uint64_t cut_ultra_bits(R &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    uint64_t normal = wp.avg, end = n;
    if (n >= wp.max) end = wp.max;
    else if (n <= normal) normal = n;
    uint32_t lec = 0;
    uint64_t i = wp.min;
    while (i + 8 <= end) {
        if (i + 64 <= end && (i >= normal || i + 56 < normal)) {
            const uint64_t e = r.bits(3, 2, s + i, 64) & 0x0101010101010101ull;
            const uint64_t m = r.bits(3, i >= normal ? 1 : 0, s + i, 64);
            if ((e | m) == 0) {
                lec = 0;
                i += 64;
                continue;
            }
            // The blocks before the first event neither repeat nor hit: skip
            // to the event's block (lec is 0 after them, as block by block).
            const uint32_t b = (uint32_t)__builtin_ctzll(e | m) >> 3;
            if (b) {
                lec = 0;
                i += 8 * b;
            }
        }
        if (r.bits(3, 2, s + i, 1)) {
            if (++lec >= CDC_ULTRA_LEST) return i + 8;
            i += 8;
            continue;
        }
        lec = 0;
        const uint64_t m = r.bits(3, i >= normal ? 1 : 0, s + i, 8);
        if (m) return i + (uint64_t)__builtin_ctzll(m);
        i += 8;
    }
    return end;
}

// LeapCDC over bitmaps 0 (primary) and 1 (secondary): the 22 primary windows
// of candidate c are bits c-22 .. c-1, the failing one nearest to c decides
// the leap; then the two secondary windows c-23, c-24.
template <class R>
__device__ uint64_t cut_leap_bits(R &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    uint64_t c = wp.min;
    // The two primary words around the candidate stay in registers while the
    // leaps (~21 positions each) move through them.
    uint64_t kc = ~0ull, wa = 0, wb = 0;
    while (c <= end) {
        const uint64_t p = s + c - CDC_LEAP_PRIMARY;
        const uint64_t k = p >> 6;
        if (k != kc) {
            wa = r.word(k * 2);
            wb = r.word(k * 2 + 2);
            kc = k;
        }
        const uint32_t sh = (uint32_t)(p & 63);
        const uint64_t v = sh ? (wa >> sh) | (wb << (64 - sh)) : wa;
        const uint64_t z = ~v & ((1ull << CDC_LEAP_PRIMARY) - 1);
        if (z) {  // window k = 21 - j failed, j = the highest zero bit
            const uint32_t j = 63u - (uint32_t)__builtin_clzll(z);
            c += CDC_LEAP_WINDOWS - (CDC_LEAP_PRIMARY - 1 - j);
            continue;
        }
        if (!r.bits(2, 1, s + c - 23, 1)) { c += CDC_LEAP_WINDOWS - 22; continue; }
        if (!r.bits(2, 1, s + c - 24, 1)) { c += CDC_LEAP_WINDOWS - 23; continue; }
        return c;
    }
    return end;
}

// Index of the n-th (1-based) set bit of z, popc(z) >= n >= 1: a halving
// search on popcounts (6 steps) instead of clearing n-1 bits one by one.
__device__ __forceinline__ uint32_t select_bit(uint64_t z, uint32_t n) {
    uint32_t pos = 0, c = (uint32_t)__popc((uint32_t)z);
    if (c < n) { n -= c; z >>= 32; pos += 32; }
    c = (uint32_t)__popc((uint32_t)z & 0xFFFFu);
    if (c < n) { n -= c; z >>= 16; pos += 16; }
    c = (uint32_t)__popc((uint32_t)z & 0xFFu);
    if (c < n) { n -= c; z >>= 8; pos += 8; }
    c = (uint32_t)__popc((uint32_t)z & 0xFu);
    if (c < n) { n -= c; z >>= 4; pos += 4; }
    c = (uint32_t)__popc((uint32_t)z & 0x3u);
    if (c < n) { n -= c; z >>= 2; pos += 2; }
    if (((uint32_t)z & 1u) < n) pos += 1;
    return pos;
}

// SeqCDC over bitmap 0 (pair p in the mode's direction), up to 64 positions
// per step: a = positions where a run of seq_len in-sequence pairs completes
// (the run carried in from the previous step included), tB = the pair at which
// the opposing count reaches jump_trigger; the earlier event decides.
template <class R>
__device__ uint64_t cut_seq_bits(R &r, uint64_t s, uint64_t n, const WalkParams &wp) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    uint32_t cnt = 0, opp = 0;
    uint64_t i = wp.min;
    while (i < end) {
        const uint32_t k = (uint32_t)min(end - i, (uint64_t)64);
        const uint64_t km = k == 64 ? ~0ull : (1ull << k) - 1;
        const uint64_t y = r.bits(1, 0, s + i, k);
        const uint64_t prev = cnt >= 64 ? ~0ull : cnt ? ~0ull << (64 - cnt) : 0ull;
        uint64_t a = y;
        for (uint32_t q = 1; q < wp.seq_len; ++q) a &= (y << q) | (prev >> (64 - q));
        a &= km;
        uint64_t z = ~y & km;
        const uint32_t need = wp.seq_trig - opp;
        const uint32_t tB = (uint32_t)__popcll(z) >= need ? select_bit(z, need) : 64u;
        const uint32_t tA = a ? (uint32_t)__builtin_ctzll(a) : 64u;
        if (tA < tB) return i + tA + 1;
        if (tB < 64) {
            opp = 0;
            cnt = 0;
            i += tB + wp.seq_jump;
            continue;
        }
        opp += (uint32_t)__popcll(~y & km);
        const uint64_t zz = ~y & km;
        cnt = zz ? k - 1 - (63u - (uint32_t)__builtin_clzll(zz)) : min(cnt + k, 1u << 30);
        i += k;
    }
    return end;
}

template <int kAlgo, bool kBits>
__device__ __forceinline__ uint64_t cut(Reader &r, uint64_t s, uint64_t len, const WalkParams &wp, const Tabs &T) {
    if constexpr (kBits) {
        if constexpr (kAlgo == 2) return cut_rabin_bits(r, s, len - s, wp);
        else if constexpr (kAlgo == 4) return cut_ultra_bits(r, s, len - s, wp);
        else if constexpr (kAlgo == 6) return cut_seq_bits(r, s, len - s, wp);
        else return cut_leap_bits(r, s, len - s, wp);
    } else {
        if constexpr (kAlgo == 2) return cut_rabin(r, s, len - s, wp, T);
        else if constexpr (kAlgo == 4) return cut_ultra(r, s, len - s, wp);
        else if constexpr (kAlgo == 5) return cut_leap(r, s, len - s, wp, T);
        else return cut_seq(r, s, len - s, wp);
    }
}

// Where a walk stands: the stream's first segment (gbase), the segment
// size, and the candidate slot of the current start (link mode; kNoCand when
// unknown or not a candidate).
struct Hop {
    uint64_t gbase;
    uint32_t sl2;
    uint32_t ci;
};

// Candidate slot of stream offset c (link mode), or kNoCand: a binary search
// in its segment's ascending list; overflowed segments have no links.
__device__ __forceinline__ uint32_t find_cand(const WalkParams &wp, const Hop &hp, uint64_t c) {
    const uint64_t h = hp.gbase + (c >> hp.sl2);
    const uint32_t n = wp.ccnt[h];
    if (n > wp.ccap) return kNoCand;
    const uint32_t *P = wp.cpos + h * wp.ccap;
    const uint32_t x = (uint32_t)(c & ((1ull << hp.sl2) - 1));
    uint32_t a = 0, b = n;
    while (a < b) {
        const uint32_t m = (a + b) >> 1;
        if (P[m] < x) a = m + 1; else b = m;
    }
    return a < n && P[a] == x ? (uint32_t)(h * wp.ccap + a) : kNoCand;
}

// The next chunk start after one starting at c: the precomputed link when c
// is a candidate (link mode), else the rule walked from c.
template <int kAlgo, bool kBits>
__device__ __forceinline__ uint64_t advance(Reader &r, uint64_t c, uint64_t len, Hop &hp, const WalkParams &wp,
                                            const Tabs &T) {
    if (wp.links && c < len) {
        if (hp.ci == kNoCand) hp.ci = find_cand(wp, hp, c);
        if (hp.ci != kNoCand) {
            uint64_t nx;
            if (hp.ci & kVirt) {
                const uint32_t v = hp.ci & ~kVirt;
                nx = wp.vnext[v];
                hp.ci = wp.vidx[v];
            } else {
                nx = wp.lnext[hp.ci];
                hp.ci = wp.lidx[hp.ci];
            }
            return nx;
        }
    }
    hp.ci = kNoCand;
    return c + cut<kAlgo, kBits>(r, c, len, wp, T);
}

// Walk from chunk start c (< seg_end) to the first start >= seg_end,
// recording the starts in the segment's list.
template <int kAlgo, bool kBits>
__device__ void walk_from(uint64_t c, uint64_t g, uint64_t seg_end, uint64_t len, Reader &r,
                          const WalkParams &wp, const Tabs &T, const WalkState &ws, Hop &hp) {
    ws.E[g] = c;
    ws.Es[g] = c;  // (round 0's snapshot: launch_fix skips its snap_kernel)
    uint32_t cnt = 0;
    uint64_t *list = ws.list + g * wp.cap;
    while (c < seg_end) {
        if (cnt < wp.cap) list[cnt] = c;
        ++cnt;
        c = advance<kAlgo, kBits>(r, c, len, hp, wp, T);
    }
    ws.X[g] = c;
    ws.Xs[g] = c;
    ws.N[g] = cnt;
    if (cnt > wp.cap) atomicAdd(&ws.flags[1], 1ull);
}

// Re-walk of segment g from x (a fix-up): the new chain usually meets the
// segment's old chain within a few chunks, and from a common start on the two
// are the same chain, so the old tail and exit stay.  Up to kNew new starts are
// held in the lane's LDS slots; then the old list is shifted behind them.
// Without a meeting point within kNew starts: a full walk_from.  Returns
// whether the exit X changed (only then can successors be affected).
constexpr uint32_t kNew = 8;

template <int kAlgo, bool kBits>
__device__ bool rewalk(uint64_t x, uint64_t g, uint64_t seg_end, uint64_t len, Reader &r, const WalkParams &wp,
                       const Tabs &T, const WalkState &ws, uint64_t *nb, Hop &hp) {
    hp.ci = kNoCand;
    uint64_t *list = ws.list + g * wp.cap;
    const uint32_t n_old = ws.N[g];
    const uint32_t lim = min(n_old, wp.cap);
    const uint64_t x_old = ws.X[g];
    uint64_t c = x;
    uint32_t m = 0, j = 0;
    while (c < seg_end && m < kNew) {
        while (j < lim && list[j] < c) ++j;
        if (j < lim && list[j] == c) {  // meets the old chain at old start j
            if (m < j) {
                for (uint32_t k = j; k < lim; ++k) list[m + k - j] = list[k];
            } else if (m > j) {
                for (uint32_t k = lim; k-- > j;)
                    if (m + k - j < wp.cap) list[m + k - j] = list[k];
            }
            for (uint32_t k = 0; k < m; ++k) list[k] = nb[k];
            ws.E[g] = x;
            ws.N[g] = m + (n_old - j);
            if (m + (n_old - j) > wp.cap) atomicAdd(&ws.flags[1], 1ull);
            return false;
        }
        nb[m++] = c;
        c = advance<kAlgo, kBits>(r, c, len, hp, wp, T);
    }
    if (c >= seg_end) {  // the whole segment in <= kNew starts, no meeting point
        for (uint32_t k = 0; k < m; ++k) list[k] = nb[k];
        ws.E[g] = x;
        ws.N[g] = m;
        ws.X[g] = c;
        return c != x_old;
    }
    hp.ci = kNoCand;
    walk_from<kAlgo, kBits>(x, g, seg_end, len, r, wp, T, ws, hp);
    return ws.X[g] != x_old;
}


// Byte mode reads the stream; bitmap mode reads the stream's bitmap words.
template <bool kBits>
__device__ __forceinline__ void init_reader(Reader &r, const StreamTable &st, const WalkParams &wp, uint32_t si,
                                            uint64_t len, uint8_t *slot) {
    if constexpr (kBits) {
        const uint64_t *b = wp.bm + st.span_base[si] * (uint64_t)wp.seg_words * wp.nbm;
        r.init(reinterpret_cast<const uint8_t *>(b), ((len + 63) >> 6) * 8ull * wp.nbm, slot);
    } else {
        r.init(st.ptrs[si], len, slot);
    }
}

__device__ __forceinline__ void load_tabs(uint64_t *sh, const uint64_t *g) {
    for (int i = threadIdx.x; i < 768; i += blockDim.x) sh[i] = g[i];
    __syncthreads();
}

template <int kAlgo, bool kBits>
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
    init_reader<kBits>(r, st, wp, si, len, win + threadIdx.x * kSlot);
    Hop hp{st.span_base[si], st.span_log2, kNoCand};
    // Warm-up start: `warm` bytes back, on the max-length grid of the stream
    // (so runs of max-length cuts from the stream start are in phase); in
    // link mode the first candidate at or after it, so that the warm-up is a
    // few hops over links instead of a walk.
    uint64_t c = 0;
    if (off != 0) {
        c = off > wp.warm ? off - wp.warm : 0;
        c = c / wp.max * wp.max;
        if (wp.links) {
            const uint64_t h = hp.gbase + (c >> hp.sl2);
            const uint32_t n = wp.ccnt[h];
            if (n >= 1 && n <= wp.ccap) {
                const uint64_t cc = (c & ~((1ull << hp.sl2) - 1)) + wp.cpos[h * wp.ccap];
                if (cc < off) {
                    c = cc;
                    hp.ci = (uint32_t)(h * wp.ccap);
                }
            }
        }
        while (c < off) c = advance<kAlgo, kBits>(r, c, len, hp, wp, T);
    }
    walk_from<kAlgo, kBits>(c, g, seg_end, len, r, wp, T, ws, hp);
}

// One Jacobi round.  Segment g is scheduled when its entry differs from its
// predecessor's exit in the round's snapshots (Es, Xs).  A lane whose re-walk
// changes the exit runs ahead into the successor when that one is NOT
// scheduled (no other lane touches it this round), and on until the chains
// meet, the stream ends, a scheduled successor, or wp.ahead segments: chains
// that take several segments to merge (SeqCDC's jumps) settle in one launch
// instead of one round per segment.  Scheduling reads only the snapshots, so a
// run-ahead write of E[g+1] never makes lane g+1 re-walk concurrently.

// A fix-up round runs only while the previous one changed exits and those
// were not mostly quiet-run re-walks (the host applies the same rule and hands
// a quiet-dominated stream to the in-order pass; WalkState::flags[3] counts,
// in its high half, the chains of flags[0] whose changed exit was a quiet run).
__device__ __forceinline__ bool round_stops(const unsigned long long *gate) {
    return gate && round_verdict(gate[0], gate[3] >> 32) != kRoundGoOn;
}

template <int kAlgo, bool kBits>
__global__ __launch_bounds__(kWalkBlock) void fix_kernel(const StreamTable st, const WalkParams wp,
                                                         const WalkState ws) {
    if (round_stops(ws.gate)) return;  // the previous round settled everything (or went quiet)
    __shared__ uint64_t tab[768];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWalkBlock * kSlot];
    __shared__ uint64_t nbuf[kWalkBlock * kNew];
    load_tabs(tab, wp.tabs);
    const Tabs T{tab, tab + 256, tab + 512};
    const uint64_t g = (uint64_t)blockIdx.x * kWalkBlock + threadIdx.x;
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    if (off == 0) return;  // a stream's first segment starts exactly at 0
    uint64_t x = ws.Xs[g - 1];
    if (ws.Es[g] == x) return;
    const uint64_t len = st.lens[si];
    const uint64_t span = 1ull << st.span_log2;
    Reader r;
    init_reader<kBits>(r, st, wp, si, len, win + threadIdx.x * kSlot);
    Hop hp{st.span_base[si], st.span_log2, kNoCand};
    uint64_t gg = g;
    for (uint32_t k = 0;; ++k) {
        const uint64_t seg_end = min(off + span, len);
        atomicAdd(&ws.flags[3], 1ull);  // segments re-walked (statistics)
        if (!rewalk<kAlgo, kBits>(x, gg, seg_end, len, r, wp, T, ws, nbuf + threadIdx.x * kNew, hp)) break;
        if (seg_end >= len) break;  // the stream's last segment: no successor
        if (k + 1 >= wp.ahead || ws.Es[gg + 1] != ws.Xs[gg]) {
            atomicAdd(&ws.flags[0], 1ull);  // a successor needs another round
            atomicMin(&ws.flags[2], (unsigned long long)gg);
            break;
        }
        x = ws.X[gg];
        ++gg;
        off += span;
    }
}

template <int kAlgo, bool kBits>
__global__ __launch_bounds__(kWalkBlock) void serial_kernel(const StreamTable st, const WalkParams wp,
                                                            const WalkState ws) {
    __shared__ uint64_t tab[768];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWalkBlock * kSlot];
    __shared__ uint64_t nbuf[kWalkBlock * kNew];
    load_tabs(tab, wp.tabs);
    const Tabs T{tab, tab + 256, tab + 512};
    // Lane per stream: streams are independent (every stream's first segment
    // starts at 0), so each lane runs its own stream's segments in order,
    // from the lowest segment the last round changed.
    const uint64_t si = (uint64_t)blockIdx.x * kWalkBlock + threadIdx.x;
    if (si >= st.n) return;
    const uint64_t g0 = st.span_base[si], g1 = st.span_base[si + 1];
    const uint64_t len = st.lens[si];
    Reader r;
    bool ready = false;
    for (uint64_t g = max(g0 + 1, ws.flags[2]); g < g1; ++g) {
        const uint64_t x = ws.X[g - 1];
        if (ws.E[g] == x) continue;
        const uint64_t off = (g - g0) << st.span_log2;
        const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
        if (!ready) {
            init_reader<kBits>(r, st, wp, (uint32_t)si, len, win + threadIdx.x * kSlot);
            ready = true;
        }
        Hop hp{g0, st.span_log2, kNoCand};
        (void)rewalk<kAlgo, kBits>(x, g, seg_end, len, r, wp, T, ws, nbuf + threadIdx.x * kNew, hp);
    }
}

// ---- wave-cooperative walks (Rabin, UltraCDC; bitmap mode) ------------------
// One wave per segment, its 64 lanes on ONE chain: a step reads 64 position-
// words of the bitmaps (4096 positions, coalesced, straight from L2 / HBM)
// and finds the first event with ballots and a lane scan, so a chain moves
// thousands of positions per step and the lanes never diverge.  (The lane-
// per-segment walks above advance 64 positions per lane step, and 64 lanes at
// unrelated points of their chains pay for each other's cut bookkeeping.)
// Every chain value (start, cut) is wave-uniform.

// One stream's bitmaps: position-word k of bitmap b at w[k * nbm + b];
// words at or past nk (the stream end) read 0.
struct WBm {
    const uint64_t *w;
    uint64_t nk;
    const uint8_t *jt = nullptr;  // LeapCDC: the stream's word tables
    uint8_t *lb = nullptr;        // LeapCDC: the wave's LDS slot (kLeapSlot bytes)
    const uint16_t *jt8 = nullptr;  // LeapCDC: the stream's block tables
    __device__ __forceinline__ uint64_t word(uint32_t nbm, uint32_t b, uint64_t k) const {
        return k < nk ? w[k * nbm + b] : 0ull;
    }
    // 64 bits from position p (bit j = position p + j); p & 63 wave-uniform.
    __device__ __forceinline__ uint64_t bits64(uint32_t nbm, uint32_t b, uint64_t p) const {
        const uint64_t k = p >> 6;
        const uint32_t sh = (uint32_t)(p & 63);
        const uint64_t lo = word(nbm, b, k);
        return sh ? (lo >> sh) | (word(nbm, b, k + 1) << (64 - sh)) : lo;
    }
};

// The wave's index in its block, as a wave-uniform (SGPR) value: segment
// indices, offsets and chain positions derived from it stay scalar, instead of
// the compiler's divergent (VGPR, exec-masked) form of threadIdx.x >> 6.
__device__ __forceinline__ uint32_t wave_id() { return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
}

// DPP lane moves (no LDS round trip, unlike __shfl_up's ds_bpermute): lanes
// the control leaves without a source (or rows the row mask disables) get old.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRowMask, 0xF, false);
}

// wave_shr:1 -- lane i receives lane i-1, lane 0 gets fill.
__device__ __forceinline__ uint32_t wave_shr1_32(uint32_t v, uint32_t fill) { return dpp32<0x138, 0xF>(v, fill); }
__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t v, uint64_t fill) {
    return ((uint64_t)wave_shr1_32((uint32_t)(v >> 32), (uint32_t)(fill >> 32)) << 32) |
           wave_shr1_32((uint32_t)v, (uint32_t)fill);
}

// Inclusive prefix sum over the wave: row_shr 1/2/4/8 within rows of 16 lanes,
// then row_bcast 15 (rows 1, 3) and 31 (rows 2, 3) carry the earlier rows.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dpp32<0x111, 0xF>(v, 0);
    v += dpp32<0x112, 0xF>(v, 0);
    v += dpp32<0x114, 0xF>(v, 0);
    v += dpp32<0x118, 0xF>(v, 0);
    v += dpp32<0x142, 0xA>(v, 0);
    v += dpp32<0x143, 0xC>(v, 0);
    return v;
}

// One step of UltraCDC's repeat-map scan: (fa, fv) after the source lane's map.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void ultra_map_step(uint32_t &fa, uint32_t &fv) {
    const uint32_t pa = dpp32<kCtrl, kRowMask>(fa, 1u), pv = dpp32<kCtrl, kRowMask>(fv, 0u);
    fv = fa ? pv + fv : fv;
    fa &= pa;
}

// Bits 0, 8, ..., 56 of x (others zero) gathered into bits 0..7.
__device__ __forceinline__ uint32_t gather8(uint64_t x) {
    return (uint32_t)((x * 0x0102040810204080ull) >> 56);
}

// Per 8-bit block of m: any bit set -> bit t of the result.
__device__ __forceinline__ uint32_t byte_any(uint64_t m) {
    m |= m >> 4;
    m |= m >> 2;
    m |= m >> 1;
    return gather8(m & 0x0101010101010101ull);
}

// Rabin: first hit in [s+min-1, s+end-1], 64 words per step.
__device__ uint64_t wcut_rabin(const WBm &B, uint64_t s, uint64_t n, const WalkParams &wp, uint32_t lane) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    const uint64_t lo = s + wp.min - 1, hi = s + end - 1;
    const uint64_t klo = lo >> 6, khi = hi >> 6;
    for (uint64_t k0 = klo; k0 <= khi; k0 += 64) {
        const uint64_t k = k0 + lane;
        uint64_t w = k <= khi ? B.word(1, 0, k) : 0ull;
        if (k == klo) w &= ~0ull << (lo & 63);
        if (k == khi && (hi & 63) != 63) w &= (2ull << (hi & 63)) - 1;
        const uint64_t m = __ballot(w != 0);
        if (m) {
            const uint32_t f = (uint32_t)__builtin_ctzll(m);
            return (k0 + f) * 64 + (uint64_t)__builtin_ctzll(rdlane64(w, f)) - s + 1;
        }
    }
    return end;
}

// UltraCDC over bitmaps 0 (mask_s hit), 1 (mask_l hit), 2 (8-byte repeat),
// 512 blocks per step, lane l on blocks 8l .. 8l+7 of the step.  Per block
// (cut_ultra): a repeat counts towards LEST (cut at its end when the run of
// repeats reaches LEST), otherwise the run resets and the block's first hit
// (mask by the block's side of the normal size) cuts.  The run entering each
// lane is a scan of per-lane maps x -> (all 8 repeat ? x + 8 : trailing
// repeats), the run carried in from the previous step included.
__device__ uint64_t wcut_ultra(const WBm &B, uint64_t s, uint64_t n, const WalkParams &wp, uint32_t lane) {
    if (n <= wp.min) return n;
    uint64_t normal = wp.avg, end = n;
    if (n >= wp.max) end = wp.max;
    else if (n <= normal) normal = n;
    if (end < (uint64_t)wp.min + 8) return end;
    const uint64_t nblk = (end - wp.min) >> 3;                                    // blocks with i + 8 <= end
    const uint64_t tnorm = normal > wp.min ? (normal - wp.min + 7) >> 3 : 0;  // first block at / after normal
    uint32_t lec = 0;
    for (uint64_t t0 = 0; t0 < nblk; t0 += 512) {
        const uint64_t tl = t0 + 8ull * lane;
        const uint64_t P = s + wp.min + 8 * tl;
        const uint64_t hs = B.bits64(3, 0, P), hl = B.bits64(3, 1, P), eq = B.bits64(3, 2, P);
        const uint32_t nv = tl < nblk ? (uint32_t)min(nblk - tl, (uint64_t)8) : 0u;
        const uint32_t vb = (1u << nv) - 1;
        const uint64_t split = tnorm > tl ? min(tnorm - tl, (uint64_t)8) : 0ull;
        const uint64_t lowm = split >= 8 ? ~0ull : (1ull << (8 * split)) - 1;
        const uint64_t m = (hs & lowm) | (hl & ~lowm);
        const uint32_t r = gather8(eq & 0x0101010101010101ull) & vb;
        const uint32_t a_hit = ~r & byte_any(m) & vb;
        const uint32_t lead = (uint32_t)__builtin_ctz(~r);                     // leading repeats (<= 8)
        const uint32_t z = ~r & 0xFFu;
        uint32_t fa = r == 0xFFu, fv = fa ? 8u : (uint32_t)__builtin_clz(z) - 24u;  // trailing repeats
        // inclusive scan of the maps (composition: later lane after earlier),
        // DPP steps as wave_incl_sum; lanes without a source get the identity
        // map (all repeats, length 0)
        ultra_map_step<0x111, 0xF>(fa, fv);
        ultra_map_step<0x112, 0xF>(fa, fv);
        ultra_map_step<0x114, 0xF>(fa, fv);
        ultra_map_step<0x118, 0xF>(fa, fv);
        ultra_map_step<0x142, 0xA>(fa, fv);
        ultra_map_step<0x143, 0xC>(fa, fv);
        const uint32_t cout = fa ? lec + fv : fv;
        const uint32_t cin = wave_shr1_32(cout, lec);
        const uint32_t tb0 = cin >= CDC_ULTRA_LEST - 1 ? 0u : CDC_ULTRA_LEST - 1 - cin;
        const uint32_t tB = tb0 < lead ? tb0 : 8u;
        const uint32_t tA = (uint32_t)__builtin_ctz(a_hit | 0x100u);
        const uint32_t te = min(tA, tB);
        const uint64_t ev = __ballot(te < 8);
        if (ev) {
            const uint32_t f = (uint32_t)__builtin_ctzll(ev);
            const uint32_t tf = (uint32_t)__builtin_amdgcn_readlane((int)te, (int)f);
            const uint32_t isb = (uint32_t)__builtin_amdgcn_readlane((int)(tB < tA), (int)f);
            const uint64_t i = wp.min + 8 * (t0 + 8ull * f + tf);
            if (isb) return i + 8;
            const uint64_t mf = rdlane64(m, f);
            return i + (uint64_t)__builtin_ctzll((mf >> (8 * tf)) & 0xFFull);
        }
        lec = (uint32_t)__builtin_amdgcn_readlane((int)cout, 63);
    }
    return end;
}

// Quiet runs.  Inside long zero-filled or constant regions every chunk of a
// rule has one fixed length L, so chains keep the phase they enter with and
// never merge; there the walks take the region's chunks many at a time.  Per
// rule (and kind), a chunk starting at s has length exactly L when every
// position of [s + lo, s + hi] is "quiet" and len - s >= L:
//   Rabin 0, Seq  L = max:          no hit / no in-direction pair in
//                                   [s+min-1, s+max-1] (no cut before max);
//   Rabin 1       L = min:          a hit at s+min-1 (zeros: the digest of a
//                                   zero window is 0, a hit everywhere);
//   UltraCDC      L = min + 8 LEST: every block from s+min an 8-byte repeat
//                                   (the run reaches LEST whatever the hashes);
//   LeapCDC       L = min:          primary and secondary windows all eligible
//                                   in [s+min-24, s+min-1] (accepted at once).
// quiet_run finds the first loud position at or after c + lo (4096 positions
// per wave step in the bitmaps, then 2 MiB per step in the per-word summary
// wp.rsum, written by the bitmap pass: kinds interleaved per summary word)
// and returns k: the chain from c takes k chunks of length L in a row, the k
// starts all < lim.
struct QuietRule {
    uint64_t L, lo, hi;
    bool ok;
};

template <int kAlgo>
constexpr int kQuietKinds = kAlgo == 2 ? 2 : 1;

template <int kAlgo, int kKind>
__device__ __forceinline__ QuietRule quiet_rule(const WalkParams &wp) {
    if constexpr (kAlgo == 4) {
        const uint64_t L = wp.min + 8ull * CDC_ULTRA_LEST;
        return {L, wp.min, L - 8, wp.max >= L};
    } else if constexpr (kAlgo == 5) {
        return {wp.min, wp.min - CDC_LEAP_WINDOWS, wp.min - 1, wp.min >= CDC_LEAP_WINDOWS};
    } else if constexpr (kKind == 1) {
        return {wp.min, wp.min - 1, wp.min - 1, wp.min >= 1 && wp.min < wp.max};
    } else {
        return {wp.max, wp.min - 1, wp.max - 1, wp.min >= 1};
    }
}

// Loud (non-quiet) positions of word k, bit j = position 64 k + j.
template <int kAlgo, int kKind>
__device__ __forceinline__ uint64_t loud_word(const WBm &B, uint64_t k) {
    if constexpr (kAlgo == 4) return ~B.word(3, 2, k);
    else if constexpr (kAlgo == 5) return ~(B.word(2, 0, k) & B.word(2, 1, k));
    else if constexpr (kKind == 1) return ~B.word(1, 0, k);
    else return B.word(1, 0, k);
}

// First loud position in [a, need), else need.  Summary bits of words at or
// past the stream end read loud (their summary words may be stale).
template <int kAlgo, int kKind>
__device__ uint64_t first_loud(const WBm &B, const uint64_t *rs, uint64_t a, uint64_t need, uint32_t lane) {
    const uint64_t ka = a >> 6;
    {
        const uint64_t k = ka + lane;
        uint64_t w = loud_word<kAlgo, kKind>(B, k);
        if (k == ka) w &= ~0ull << (a & 63);  // positions before a do not count
        const uint64_t m = __ballot(w != 0 && k * 64 < need);
        if (m) {
            const uint32_t f = (uint32_t)__builtin_ctzll(m);
            return min(need, (ka + f) * 64 + (uint64_t)__builtin_ctzll(rdlane64(w, f)));
        }
    }
    // summary words from word K on: lane l reads words k0 + 8 l .. + 7
    constexpr uint32_t kPer = 8;
    const uint64_t nsk = (B.nk + 63) >> 6;
    for (uint64_t K = ka + 64; K * 64 < need; K = ((K >> 6) + 64 * kPer) << 6) {
        const uint64_t k0 = K >> 6;
        uint32_t fi = kPer;
        uint64_t fw = ~0ull;
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint64_t sk = k0 + kPer * lane + i;
            uint64_t sw = 0;
            if (sk < nsk) {
                sw = rs[sk * kQuietKinds<kAlgo> + kKind];
                if (sk * 64 + 64 > B.nk) sw &= (1ull << (B.nk - sk * 64)) - 1;
            }
            if (sk == k0) sw |= (1ull << (K & 63)) - 1;
            if (sk * 4096 >= need) sw = ~0ull;
            const bool hit = sw != ~0ull && fi == kPer;
            fw = hit ? sw : fw;
            fi = hit ? i : fi;
        }
        const uint64_t m = __ballot(fi < kPer);
        if (m) {
            const uint32_t f = (uint32_t)__builtin_ctzll(m);
            const uint32_t i = (uint32_t)__builtin_amdgcn_readlane((int)fi, (int)f);
            const uint64_t kz = (k0 + kPer * f + i) * 64 + (uint64_t)__builtin_ctzll(~rdlane64(fw, f));
            const uint64_t z = loud_word<kAlgo, kKind>(B, kz);
            return min(need, kz * 64 + (z ? (uint64_t)__builtin_ctzll(z) : 0));
        }
    }
    return need;
}

template <int kAlgo, int kKind>
__device__ uint64_t quiet_run(const WBm &B, const uint64_t *rs, uint64_t c, uint64_t len, uint64_t lim,
                              const WalkParams &wp, uint32_t lane) {
    const QuietRule q = quiet_rule<kAlgo, kKind>(wp);
    if (!q.ok || c >= lim || len - c < q.L) return 0;
    const uint64_t kmax = min((len - c) / q.L, (lim - c + q.L - 1) / q.L);
    const uint64_t a = c + q.lo, tail = q.hi - q.lo;
    const uint64_t b = first_loud<kAlgo, kKind>(B, rs, a, a + (kmax - 1) * q.L + tail + 1, lane);
    return b > a + tail ? min(kmax, (b - a - tail + q.L - 1) / q.L) : 0;
}

// The kind a chunk of length d may start (-1: none).
template <int kAlgo>
__device__ __forceinline__ int quiet_kind(const WalkParams &wp, uint64_t d) {
    if (d == quiet_rule<kAlgo, 0>(wp).L) return 0;
    if constexpr (kQuietKinds<kAlgo> > 1)
        if (d == quiet_rule<kAlgo, 1>(wp).L) return 1;
    return -1;
}

template <int kAlgo>
__device__ __forceinline__ uint64_t quiet_run_k(int kind, const WBm &B, const uint64_t *rs, uint64_t c, uint64_t len,
                                                uint64_t lim, const WalkParams &wp, uint32_t lane, uint64_t &L) {
    if constexpr (kQuietKinds<kAlgo> > 1) {
        if (kind == 1) {
            L = quiet_rule<kAlgo, 1>(wp).L;
            return quiet_run<kAlgo, 1>(B, rs, c, len, lim, wp, lane);
        }
    }
    L = quiet_rule<kAlgo, 0>(wp).L;
    return quiet_run<kAlgo, 0>(B, rs, c, len, lim, wp, lane);
}

// In a walk, after a chunk of one kind's length L (Rabin: two in a row, pk
// = the previous chunk's kind; max-length chunks are common in its random
// data, and its quiet search is the next hit's), take the quiet run's chunks
// from c at once: the starts c + j L (j < k) go to list[cnt + j] (lanes in
// parallel).
template <int kAlgo>
constexpr bool kQuietTwice = kAlgo == 2;

template <int kAlgo>
__device__ __forceinline__ void take_run(const WBm &B, const uint64_t *rs, uint64_t d, int &pk, uint64_t &c,
                                         uint64_t len, uint64_t lim, const WalkParams &wp, uint32_t lane,
                                         uint64_t *list, uint32_t &cnt) {
    const int kind = quiet_kind<kAlgo>(wp, d);
    if (kind < 0 || (kQuietTwice<kAlgo> && kind != pk) || !rs || c >= lim) {
        pk = kind;
        return;
    }
    uint64_t L;
    const uint64_t k = quiet_run_k<kAlgo>(kind, B, rs, c, len, lim, wp, lane, L);
    if (list)
        for (uint64_t j = lane; j < k; j += 64)
            if (cnt + j < wp.cap) list[cnt + j] = c + j * L;
    cnt += (uint32_t)k;
    c += k * L;
    pk = k ? kind : -1;
}

// SeqCDC over bitmap 0 (pair p in the mode's direction), a window of 4096
// positions per load (lane l on positions 64l .. 64l+63 of it).  From a
// restart point t0 (the chunk's min, or a jump's landing) the rule is two
// events, whichever comes first: a run of seq_length in-direction pairs
// completes at t (cut after t), or the jump_trigger-th opposing pair since the
// restart is at t (jump: the next restart is t + jump_size).  Run ends come
// from shifted ANDs (the previous lane's word carried in; lane 0: the run
// carried from the previous window); the n-th opposing pair from a lane
// prefix of popcounts and a select in the one lane that holds it.  Several
// restarts per window are handled from the same registers.
//
// The walk's cost is that restart chain (~7 restarts per chunk on random
// data; a timing build without jumps walked 1 GiB in 119 us instead of 365),
// a dependent scalar sequence per restart, so each restart is kept short:
// window offsets in 32 bits (one SALU compare each, where 64-bit unsigned
// compares go through a VALU v_cmp and back), the select inside the lane by
// all lanes at once (5 VALU + 2 SALU, was a ~65-instruction scalar
// bisection), and the run event kept until the restart passes it.
__device__ uint64_t wcut_seq(const WBm &B, uint64_t s, uint64_t n, const WalkParams &wp, uint32_t lane) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    const uint32_t L = wp.seq_len, TT = wp.seq_trig, J = wp.seq_jump;
    const uint32_t Jc = min(J, 1u << 30);  // (tj + Jc fits 32 bits; a larger jump leaves the window anyway)
    uint64_t i = wp.min;        // window start (relative to s)
    uint32_t cnt = 0, opp = 0;  // run / opposing pairs carried into the window
    const uint64_t pmask = lane == 63 ? ~0ull : (2ull << lane) - 1;
    while (i < end) {
        const uint32_t lim = (uint32_t)min(end - i, (uint64_t)1 << 30);  // valid positions of the window: t < lim
        const uint32_t tl = 64u * lane;
        const uint64_t vm = tl >= lim ? 0ull : (lim - tl >= 64 ? ~0ull : (1ull << (lim - tl)) - 1);
        const uint64_t y = B.bits64(1, 0, s + i + tl) & vm;
        const uint64_t z = ~y & vm;
        const uint64_t yp = wave_shr1_64(y, cnt ? ~0ull << (64 - cnt) : 0ull);  // lane 0: the carried run
        uint64_t a = y;
        for (uint32_t q = 1; q < L; ++q) a &= (y << q) | (yp >> (64 - q));
        const uint32_t zc = (uint32_t)__popcll(z);
        const uint32_t zin = wave_incl_sum(zc);  // inclusive prefix of opposing pairs over lanes
        const uint32_t zex = zin - zc;
        // run event: the first run end at t >= thr (all its pairs at >= the
        // restart); run ends are rare, so the answer is kept while thr has not
        // passed it, and found from the lanes that hold any (mr) otherwise.
        const uint64_t mr = __ballot(a != 0);
        auto run_at = [&](uint32_t thr) -> uint32_t {
            if (thr >= 4096) return 4096;
            const uint32_t l = thr >> 6;
            uint64_t m = mr & (~0ull << l);
            while (m) {
                const uint32_t f = (uint32_t)__builtin_ctzll(m);
                uint64_t bits = rdlane64(a, f);
                if (f == l) bits &= ~0ull << (thr & 63);
                if (bits) return 64u * f + (uint32_t)__builtin_ctzll(bits);
                m &= m - 1;
            }
            return 4096;
        };
        uint32_t tr = run_at(0);  // t0 = 0 with the carried run: thr 0
        uint32_t t0 = 0;          // restart offset in the window
        uint32_t opp0 = opp;
        for (;;) {
            // jump event: the (TT - opp0)-th opposing pair at or after t0
            uint32_t before = 0;
            if (t0) {
                const uint32_t l0 = t0 >> 6, b0 = t0 & 63;
                const uint64_t zl = rdlane64(z, l0);
                before = (uint32_t)__builtin_amdgcn_readlane((int)zex, (int)l0) +
                         (b0 ? (uint32_t)__popcll(zl & ((1ull << b0) - 1)) : 0u);
            }
            const uint32_t target = before + (TT - opp0);
            const uint64_t mj = __ballot(zin >= target);
            uint32_t tj = 4096;
            if (mj) {  // select in lane f's word: lane j counts its bits 0..j (VALU, not a scalar bisection)
                const uint32_t f = (uint32_t)__builtin_ctzll(mj);
                const uint32_t need = target - (uint32_t)__builtin_amdgcn_readlane((int)zex, (int)f);
                const uint64_t ms = __ballot((uint32_t)__popcll(rdlane64(z, f) & pmask) >= need);
                tj = 64u * f + (uint32_t)__builtin_ctzll(ms);
            }
            if (tr < tj) return i + tr + 1;  // (tr < lim: bits past the end are clear)
            if (tj >= 4096) {
                if (lim <= 4096) return end;
                // no event in [t0, 4096): carry the run ending at 4095 and the count
                const uint64_t y63 = rdlane64(y, 63);
                const uint32_t r63 = ~y63 ? (uint32_t)__builtin_clzll(~y63) : 64u;
                cnt = min(r63, 4096u - t0);
                opp = opp0 + ((uint32_t)__builtin_amdgcn_readlane((int)zin, 63) - before);
                i += 4096;
                break;
            }
            // jump
            const uint32_t tn = tj + Jc;
            opp0 = 0;
            if (tn >= 4096 || tn >= lim) {
                i += (uint64_t)tj + J;
                cnt = 0;
                opp = 0;
                break;
            }
            t0 = tn;
            if (tr < t0 + L - 1) tr = run_at(t0 + L - 1);
        }
    }
    return end;
}

// ---- LeapCDC: leap rule over two words, word tables, wave walk ---------------
// Candidate C at offset x (0..63) of word w: its 24 windows end at C-1 ..
// C-24, all inside words w-1 (lo) and w (hi) of the primary (p*) and
// secondary (s*) bitmaps.  Returns the leap (1..24), or 0 when C is accepted
// (cut_leap_bits: the nearest failing primary window at field bit j leaps
// 3 + j; then the secondary windows C-23, C-24 leap 2, 1).
static_assert(CDC_LEAP_WINDOWS == CDC_LEAP_PRIMARY + 2, "two secondary windows");

__device__ __forceinline__ uint32_t leap_step(uint64_t plo, uint64_t phi, uint64_t slo, uint64_t shi, uint32_t x) {
    constexpr uint32_t kP = CDC_LEAP_PRIMARY;
    const uint32_t t = x + 64 - kP;  // bit of position C - 22 in (hi:lo)
    const uint64_t f = (t < 64 ? (plo >> t) | (phi << (64 - t)) : phi >> (t - 64)) & ((1ull << kP) - 1);
    const uint64_t z = ~f & ((1ull << kP) - 1);
    if (z) return CDC_LEAP_WINDOWS - (kP - 1 - (63u - (uint32_t)__builtin_clzll(z)));
    const uint32_t t2 = x + 63 - kP;  // C - 23
    if (!(((t2 < 64 ? slo >> t2 : shi >> (t2 - 64))) & 1)) return CDC_LEAP_WINDOWS - kP;
    const uint32_t t3 = t2 - 1;       // C - 24
    if (!(((t3 < 64 ? slo >> t3 : shi >> (t3 - 64))) & 1)) return CDC_LEAP_WINDOWS - kP - 1;
    return 0;
}

// Word tables: wave per segment (4 per block), lane per word, in two passes
// over the word's 64 candidates (unrolled, no divergence):
//  1. forward: the next candidate after each one.  With the last primary
//     failing window lz before x kept incrementally, a primary failure leaps
//     to lz + 25 (the leap 3 + j of cut_leap_bits), else the secondary windows
//     x-23, x-24 leap 2 / 1, else x is accepted.  Packed 4 per VGPR.
//  2. backward: the orbit result of each candidate, res[x] = accepted (64 + x),
//     the entry into the next word (next - 64), or res[next], kept in the
//     lane's LDS slot (68-byte stride: the 64 lanes' slots start on 64
//     different banks).
// Entries 0..23 are res[0..23].
constexpr uint32_t kJSlot = 68;

__global__ __launch_bounds__(256) void jtab_kernel(const StreamTable st, const WalkParams wp) {
    __shared__ __attribute__((aligned(16))) uint8_t res_lds[256 * kJSlot];
    const uint32_t lane = threadIdx.x & 63;
    Piece pc;
    if (!piece_of(st, wp, (uint64_t)blockIdx.x * 4 + wave_id(), pc)) return;
    uint8_t *res = res_lds + threadIdx.x * kJSlot;
    const uint32_t si = pc.si;
    const uint64_t off = pc.off;
    const uint64_t len = st.lens[si];
    const uint64_t base = st.span_base[si] * (uint64_t)wp.seg_words;
    const uint64_t *bm = wp.bm + base * 2;
    uint8_t *jt = wp.jt + base * 24;
    const uint64_t nk = (len + 63) >> 6;
    constexpr int kP = (int)CDC_LEAP_PRIMARY;
    uint16_t *jt8 = wp.jt8 + base / 8 * 24;
    for (uint32_t r = 0; r < (1u << (wp.piece_log2 - 12)); ++r) {
        const uint64_t w0 = (off >> 6) + (uint64_t)r * 64;
        if (w0 >= nk) return;  // (wave-uniform)
        const uint64_t w = w0 + lane;
        const bool in = w < nk;  // words past the stream end: tables never used
        const uint64_t phi = in ? bm[2 * w] : 0ull, shi = in ? bm[2 * w + 1] : 0ull;
        const uint64_t plo = in && w ? bm[2 * w - 2] : 0ull, slo = in && w ? bm[2 * w - 1] : 0ull;
        const uint64_t zlo = ~plo, zhi = ~phi;  // primary failing windows
        // lz: the last failing primary window before candidate 0 (offsets
        // relative to the word; -1000 = none in reach)
        int lz = zlo ? (63 - (int)__builtin_clzll(zlo)) - 64 : -1000;
        uint32_t nx[16];
#pragma unroll
        for (int x = 0; x < 64; ++x) {
            if (x > 0) {
                const bool f = x - 1 < 32 ? ((uint32_t)zhi >> (x - 1)) & 1 : ((uint32_t)(zhi >> 32) >> (x - 33)) & 1;
                lz = f ? x - 1 : lz;
            }
            // secondary windows x-23, x-24 (offsets in [-24, 40])
            const int a = x - kP - 1, b = x - kP - 2;
            const bool s23 = a >= 0 ? (shi >> a) & 1 : (slo >> (64 + a)) & 1;
            const bool s24 = b >= 0 ? (shi >> b) & 1 : (slo >> (64 + b)) & 1;
            const uint32_t nxt = lz >= x - kP ? (uint32_t)(lz + (int)CDC_LEAP_WINDOWS + 1)
                                : !s23 ? (uint32_t)(x + 2) : !s24 ? (uint32_t)(x + 1) : 255u;
            if ((x & 3) == 0) nx[x >> 2] = nxt;
            else nx[x >> 2] |= nxt << (8 * (x & 3));
        }
#pragma unroll
        for (int x = 63; x >= 0; --x) {  // branch-free: every lane reads one slot
            const uint32_t n = (nx[x >> 2] >> (8 * (x & 3))) & 0xFFu;
            const uint32_t r = res[n < 64u ? n : 0u];
            res[x] = (uint8_t)(n == 255u ? 64u + (uint32_t)x : n >= 64u ? n - 64u : r);
        }
        if (in) {
            const uint32_t *r32 = reinterpret_cast<const uint32_t *>(res);
            uint64_t *d = reinterpret_cast<uint64_t *>(jt + w * 24);
            d[0] = ((uint64_t)r32[1] << 32) | r32[0];
            d[1] = ((uint64_t)r32[3] << 32) | r32[2];
            d[2] = ((uint64_t)r32[5] << 32) | r32[4];
        }
        // Block tables: lanes 8k .. 8k+7 hold the words of block w0/8 + k
        // (w0 is a multiple of 512 words); lane 8k + j chases entries 3j ..
        // 3j+2 through the 8 words' results in the group's LDS slots.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint8_t *grp = res_lds + (threadIdx.x & ~7u) * kJSlot;
        const uint32_t j = lane & 7;
        uint16_t o8[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {  // branch-free: 8 reads, selects
            uint32_t x = 3 * j + q, v = 0xFFFF;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t u = grp[t * kJSlot + x];
                const bool hit = v == 0xFFFF && u >= 64;
                v = hit ? 512u + 64u * t + (u - 64u) : v;
                x = v == 0xFFFF ? u : x;
            }
            o8[q] = (uint16_t)(v == 0xFFFF ? x : v);
        }
        if (in) {
            uint16_t *d8 = jt8 + (w >> 3) * 24 + 3 * j;
            d8[0] = o8[0];
            d8[1] = o8[1];
            d8[2] = o8[2];
        }
        __builtin_amdgcn_wave_barrier();  // (the slots are rewritten next round)
    }
}

// cut_leap_bits for one wave: leaps within the start candidate's word (its
// four bitmap words loaded once), then the orbit through word tables up to the
// next 512-position block boundary, block tables while a whole block is at or
// before the bound E, and word tables up to E's word (an accepted position
// past E, or an exit past it, means no content-defined cut: `end`).  Tables
// are staged in the wave's LDS slot (one per lane, one load latency per
// stage) and followed there.
constexpr uint32_t kLeapSlot = 64 * 48 + 8 * 24;  // 64 block tables + 8 word tables

__device__ uint64_t wcut_leap(const WBm &B, uint64_t s, uint64_t n, const WalkParams &wp, uint32_t lane) {
    if (n <= wp.min) return n;
    const uint64_t end = n < wp.max ? n : wp.max;
    const uint64_t E = s + end;  // candidates C <= E
    uint64_t C = s + wp.min;
    uint64_t w = C >> 6;
    {
        const uint64_t phi = B.word(2, 0, w), shi = B.word(2, 1, w);
        const uint64_t plo = w ? B.word(2, 0, w - 1) : 0ull, slo = w ? B.word(2, 1, w - 1) : 0ull;
        while (C < 64 * (w + 1)) {
            if (C > E) return end;
            const uint32_t l = leap_step(plo, phi, slo, shi, (uint32_t)(C & 63));
            if (!l) return C - s;
            C += l;
        }
    }
    ++w;
    uint32_t e = (uint32_t)(C & 63);
    uint16_t *b8 = reinterpret_cast<uint16_t *>(B.lb);
    uint8_t *b1 = B.lb + 64 * 48;
    for (;;) {
        if (64 * w + e > E) return end;
        if ((w & 7) == 0 && 64 * (w + 8) - 1 <= E) {
            // whole blocks: up to 64 of them, every one at or before E
            const uint64_t nb = min((E + 1) / 512 - w / 8, (uint64_t)64);
            if (lane < nb) {
                const uint4 *src = reinterpret_cast<const uint4 *>(B.jt8 + (w / 8 + lane) * 24);
                uint4 *dst = reinterpret_cast<uint4 *>(b8 + lane * 24);
                dst[0] = src[0];
                dst[1] = src[1];
                dst[2] = src[2];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t k = 0; k < nb; ++k) {
                const uint32_t v = b8[k * 24 + e];
                if (v >= 512) return 64 * w + (v - 512) - s;
                e = v;
                w += 8;
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        // word tables up to the next block boundary or E's word
        const uint64_t wl = min(E >> 6, (w | 7));
        const uint32_t nw = (uint32_t)(wl - w + 1);  // 1 .. 8
        if (lane < nw) {
            const uint64_t *src = reinterpret_cast<const uint64_t *>(B.jt + (w + lane) * 24);
            uint64_t *dst = reinterpret_cast<uint64_t *>(b1 + lane * 24);
            dst[0] = src[0];
            dst[1] = src[1];
            dst[2] = src[2];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t k = 0; k < nw; ++k) {
            if (64 * w + e > E) return end;
            const uint32_t v = b1[k * 24 + e];
            if (v >= 64) {
                const uint64_t pos = 64 * w + (v - 64);
                return pos <= E ? pos - s : end;
            }
            e = v;
            ++w;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int kAlgo>
__device__ __forceinline__ uint64_t wcut(const WBm &B, uint64_t s, uint64_t n, const WalkParams &wp, uint32_t lane) {
    if constexpr (kAlgo == 2) return wcut_rabin(B, s, n, wp, lane);
    else if constexpr (kAlgo == 6) return wcut_seq(B, s, n, wp, lane);
    else if constexpr (kAlgo == 5) return wcut_leap(B, s, n, wp, lane);
    else return wcut_ultra(B, s, n, wp, lane);
}

// walk_kernel with a wave per segment (4 segments per 256-thread block).
template <int kAlgo>
__global__ __launch_bounds__(256) void wwalk_kernel(const StreamTable st, const WalkParams wp, const WalkState ws) {
    constexpr uint32_t nbm = kAlgo == 4 ? 3 : kAlgo == 5 ? 2 : 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + wave_id();
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t len = st.lens[si];
    const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
    __shared__ __attribute__((aligned(16))) uint8_t lslot[kAlgo == 5 ? 4 * kLeapSlot : 16];
    const WBm B{wp.bm + st.span_base[si] * (uint64_t)wp.seg_words * nbm, (len + 63) >> 6,
                kAlgo == 5 ? wp.jt + st.span_base[si] * (uint64_t)wp.seg_words * 24 : nullptr,
                lslot + (kAlgo == 5 ? wave_id() * kLeapSlot : 0),
                kAlgo == 5 ? wp.jt8 + st.span_base[si] * (uint64_t)wp.seg_words / 8 * 24 : nullptr};
    const uint64_t *rs = wp.rsum ? wp.rsum + st.span_base[si] * (uint64_t)wp.seg_words / 64 * kQuietKinds<kAlgo> : nullptr;
    uint64_t c = 0;
    int pk = -1;
    if (off != 0) {  // warm-up start as walk_kernel (max-length grid)
        c = off > wp.warm ? off - wp.warm : 0;
        c = c / wp.max * wp.max;
        uint32_t skip = 0;
        while (c < off) {
            const uint64_t d = wcut<kAlgo>(B, c, len - c, wp, lane);
            c += d;
            take_run<kAlgo>(B, rs, d, pk, c, len, off, wp, lane, nullptr, skip);
        }
    }
    if (lane == 0) {
        ws.E[g] = c;
        ws.Es[g] = c;  // (round 0's snapshot: launch_fix skips its snap_kernel)
    }
    uint32_t cnt = 0;
    uint64_t *list = ws.list + g * wp.cap;
    // Starts are held in lanes (lane j: list[cnt - nh + j]) and stored 64 at a
    // time: the wave's next window load never waits behind a start's store
    // (loads and stores share one counter on gfx9: a per-chunk store put an
    // HBM write round trip into every chunk's step).
    uint64_t held = 0;
    uint32_t nh = 0;
    auto flush = [&]() {
        const uint32_t base = cnt - nh;
        if (lane < nh && base + lane < wp.cap) list[base + lane] = held;
        nh = 0;
    };
    while (c < seg_end) {
        if (lane == nh) held = c;
        ++nh;
        ++cnt;
        if (nh == 64) flush();
        const uint64_t d = wcut<kAlgo>(B, c, len - c, wp, lane);
        c += d;
        const uint32_t c0 = cnt;
        take_run<kAlgo>(B, rs, d, pk, c, len, seg_end, wp, lane, list, cnt);
        if (cnt != c0 && nh) {  // a quiet run's starts went straight to the list
            const uint32_t k = cnt;
            cnt = c0;
            flush();
            cnt = k;
        }
    }
    flush();
    if (lane == 0) {
        ws.X[g] = c;
        ws.Xs[g] = c;
        ws.N[g] = cnt;
        if (cnt > wp.cap) atomicAdd(&ws.flags[1], 1ull);
    }
}

// rewalk() for one wave (wave-uniform chain; lane 0 writes): re-walk segment g
// from x until the new chain meets the old one (<= kNew new starts, kept in
// the wave's LDS slots), else a full walk.  xo = the segment's exit after it.
// Up to kWNew new starts are kept in registers (lane k & 63 of nb[k >> 6])
// before a meeting point; the old list is checked 64 entries at a time (lane
// l holds old start j0 + l: a meeting is one ballot), and the list is
// rewritten by all lanes.  128 covers a whole segment at the default sizes, so
// a re-walk without a meeting point does not walk the segment twice (SeqCDC's
// fix-up rounds per GiB at 4/8/16 KiB: 8 held starts 0.37 ms, 128: 0.29;
// profiles/r03_walk/r03as_rewalk_held_starts.log).
#ifndef CDC_WNEW  // (experiment builds, tools/build_variants.py)
#define CDC_WNEW 128
#endif
constexpr uint32_t kWNew = CDC_WNEW;
static_assert(kWNew <= 128, "two registers of held starts");

// Moves list[j .. lim) to list[m ..) (entries at or past cap dropped), 64 at a
// time, in the order that never overwrites an entry before it is read.
__device__ void shift_list(uint64_t *list, uint32_t j, uint32_t lim, uint32_t m, uint32_t cap, uint32_t lane) {
    const uint32_t cnt = lim - j, nch = (cnt + 63) / 64;
    for (uint32_t i = 0; i < nch; ++i) {
        const uint32_t ci = m > j ? nch - 1 - i : i;
        const uint32_t k = ci * 64 + lane;
        const uint64_t v = k < cnt ? list[j + k] : 0ull;
        if (k < cnt && m + k < cap) list[m + k] = v;
    }
}

template <int kAlgo>
__device__ bool wrewalk(uint64_t x, uint64_t g, uint64_t seg_end, uint64_t len, const WBm &B, const uint64_t *rs,
                        const WalkParams &wp, const WalkState &ws, uint32_t lane, uint64_t &xo, bool &qr) {
    qr = false;  // set: the new chain entered a quiet run (its phase will not merge)
    uint64_t *list = ws.list + g * wp.cap;
    const uint32_t n_old = ws.N[g];
    const uint32_t lim = min(n_old, wp.cap);
    const uint64_t x_old = ws.X[g];
    uint64_t c = x;
    uint32_t m = 0, j0 = 0;
    uint64_t ow = lane < lim ? list[lane] : ~0ull;  // old starts j0 + lane
    uint64_t nb0 = 0, nb1 = 0;                      // new starts lane, 64 + lane
    int pk = -1;
    while (c < seg_end && m < kWNew) {
        while (j0 + 64 < lim && rdlane64(ow, 63) < c) {
            j0 += 64;
            ow = j0 + lane < lim ? list[j0 + lane] : ~0ull;
        }
        const uint64_t hit = __ballot(ow == c);
        if (hit) {  // meets the old chain at old start j
            const uint32_t j = j0 + (uint32_t)__builtin_ctzll(hit);
            if (m != j) shift_list(list, j, lim, m, wp.cap, lane);
            if (lane < m && lane < wp.cap) list[lane] = nb0;
            if (64 + lane < m && 64 + lane < wp.cap) list[64 + lane] = nb1;
            if (lane == 0) {
                ws.E[g] = x;
                ws.N[g] = m + (n_old - j);
                if (m + (n_old - j) > wp.cap) atomicAdd(&ws.flags[1], 1ull);
            }
            xo = x_old;
            return false;
        }
        if (lane == (m & 63)) {
            if (m < 64) nb0 = c;
            else nb1 = c;
        }
        ++m;
        const uint64_t d = wcut<kAlgo>(B, c, len - c, wp, lane);
        c += d;
        const int kind = quiet_kind<kAlgo>(wp, d);  // a quiet run: chains keep their phase, walk it whole
        uint64_t L;
        if (kind >= 0 && (!kQuietTwice<kAlgo> || kind == pk) && rs && c < seg_end &&
            quiet_run_k<kAlgo>(kind, B, rs, c, len, seg_end, wp, lane, L) >= 2) {
            m = kWNew + 1;
            qr = true;
            break;
        }
        pk = kind;
    }
    if (c >= seg_end && m <= kWNew) {  // the whole segment in <= kWNew starts, no meeting point
        if (lane < m && lane < wp.cap) list[lane] = nb0;
        if (64 + lane < m && 64 + lane < wp.cap) list[64 + lane] = nb1;
        if (lane == 0) {
            ws.E[g] = x;
            ws.N[g] = m;
            ws.X[g] = c;
            if (m > wp.cap) atomicAdd(&ws.flags[1], 1ull);
        }
        xo = c;
        return c != x_old;
    }
    // full walk from x
    c = x;
    uint32_t cnt = 0;
    pk = -1;
    while (c < seg_end) {
        if (lane == 0 && cnt < wp.cap) list[cnt] = c;
        ++cnt;
        const uint64_t d = wcut<kAlgo>(B, c, len - c, wp, lane);
        c += d;
        take_run<kAlgo>(B, rs, d, pk, c, len, seg_end, wp, lane, list, cnt);
    }
    if (lane == 0) {
        ws.E[g] = x;
        ws.X[g] = c;
        ws.N[g] = cnt;
        if (cnt > wp.cap) atomicAdd(&ws.flags[1], 1ull);
    }
    xo = c;
    return c != x_old;
}

template <int kAlgo>
__device__ uint64_t serial_run(const StreamTable &st, const WalkParams &wp, const WalkState &ws, const WBm &B,
                               const uint64_t *rs, uint64_t g0, uint64_t g1, uint64_t g, uint64_t x, uint64_t len,
                               uint32_t lane, uint64_t &xe, const uint64_t *sE = nullptr,
                               const uint64_t *sX = nullptr, bool *capped = nullptr, uint64_t *xold = nullptr);

// A fix-up round's segment g (scheduled: its snapshot entry is not its
// predecessor's snapshot exit) leaves its re-walk to its predecessor's chain
// when both are wholly quiet in a common kind (qseg) and the predecessor is
// scheduled too: that chain takes the whole quiet stretch at once
// (serial_run), instead of every segment of the stretch re-walking its own
// stale phase (UltraCDC's chunk length does not divide the segment size, so
// inside a zero-filled region every segment starts out of phase).  off: g's
// offset in its stream.
__device__ __forceinline__ bool defers(const StreamTable &st, const WalkParams &wp, const WalkState &ws, uint64_t g,
                                       uint64_t off) {
    if (!wp.qseg || off < (2ull << st.span_log2)) return false;  // (g - 1 is the stream's first: never scheduled)
    return (wp.qseg[g] & wp.qseg[g - 1]) != 0 && ws.Es[g - 1] != ws.Xs[g - 2];
}

// fix_kernel with a wave per segment: same schedule (snapshots Es / Xs, run
// ahead into unscheduled successors), wave-cooperative re-walks; a chain that
// enters a quiet run crosses every segment the run covers at once.
template <int kAlgo>
__global__ __launch_bounds__(256) void wfix_kernel(const StreamTable st, const WalkParams wp, const WalkState ws) {
    if (round_stops(ws.gate)) return;  // the previous round settled everything (or went quiet)
    constexpr uint32_t nbm = kAlgo == 4 ? 3 : kAlgo == 5 ? 2 : 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + wave_id();
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    if (off == 0) return;  // a stream's first segment starts exactly at 0
    uint64_t x = ws.Xs[g - 1];
    if (ws.Es[g] == x) return;
    if (defers(st, wp, ws, g, off)) {  // the chain of an earlier segment crosses this one this round
        if (lane == 0) {
            atomicAdd(&ws.flags[0], 1ull);  // (one more round checks it)
            atomicMin(&ws.flags[2], (unsigned long long)(g - 1));
        }
        return;
    }
    const uint64_t len = st.lens[si];
    const uint64_t span = 1ull << st.span_log2;
    __shared__ __attribute__((aligned(16))) uint8_t lslot[kAlgo == 5 ? 4 * kLeapSlot : 16];
    const WBm B{wp.bm + st.span_base[si] * (uint64_t)wp.seg_words * nbm, (len + 63) >> 6,
                kAlgo == 5 ? wp.jt + st.span_base[si] * (uint64_t)wp.seg_words * 24 : nullptr,
                lslot + (kAlgo == 5 ? wave_id() * kLeapSlot : 0),
                kAlgo == 5 ? wp.jt8 + st.span_base[si] * (uint64_t)wp.seg_words / 8 * 24 : nullptr};
    const uint64_t *rs = wp.rsum ? wp.rsum + st.span_base[si] * (uint64_t)wp.seg_words / 64 * kQuietKinds<kAlgo> : nullptr;
    uint64_t gg = g;
    const uint64_t g0 = st.span_base[si], g1 = st.span_base[si + 1];
    for (uint32_t k = 0;; ++k) {
        if (lane == 0) atomicAdd(&ws.flags[3], 1ull);  // segments re-walked (statistics)
        uint64_t xo;
        bool qr = false, changed;
        uint64_t ge = gg;
        if (rs) {  // a quiet run from x through whole segments: all of them at once
            bool capped = false;
            uint64_t xold = 0;
            ge = serial_run<kAlgo>(st, wp, ws, B, rs, g0, g1, gg, x, len, lane, xo, ws.Es, ws.Xs, &capped, &xold);
            if (ge > gg) {
                gg = ge - 1;
                off = (gg - g0) << st.span_log2;
                changed = xo != xold;
                qr = capped;  // stopped inside the quiet run: phase-locked, for the hand-off count
            }
        }
        const uint64_t seg_end = min(off + span, len);
        if (ge == gg) changed = wrewalk<kAlgo>(x, gg, seg_end, len, B, rs, wp, ws, lane, xo, qr);
        if (!changed) break;
        if (seg_end >= len) break;  // the stream's last segment: no successor
        if (k + 1 >= wp.ahead || ws.Es[gg + 1] != ws.Xs[gg]) {
            if (lane == 0) {
                atomicAdd(&ws.flags[0], 1ull);  // a successor needs another round
                atomicMin(&ws.flags[2], (unsigned long long)gg);
                // Of those, the chains whose changed exit came out of a quiet
                // run (high half; the same count as flags[0], restricted): the
                // host hands rounds of mostly phase-locked quiet segments to
                // the in-order pass early.  Run-ahead steps inside one chain
                // are not counted, so scattered small quiet islands in random
                // data do not trip the hand-off.
                if (qr) atomicAdd(&ws.flags[3], 1ull << 32);
            }
            break;
        }
        x = xo;
        ++gg;
        off += span;
    }
}

// A quiet run through whole segments (the in-order pass, and the fix-up
// rounds' phase propagation): the chain from x (segment g's entry) takes k
// chunks of length L; every segment that ends at or before the run's covered
// part gets its list, entry, count and exit written directly (lanes over
// chunks, then over segments) -- a region settles as soon as its entry phase
// is known, instead of one segment per fix-up round.  In a fix-up round (sE /
// sX: the round's snapshots) the run stops before any later segment that the
// round re-walks on its own (so no two waves write one segment).  Returns the
// first segment the run does not cover whole (g: none), xe = its entry.
template <int kAlgo>
__device__ uint64_t serial_run(const StreamTable &st, const WalkParams &wp, const WalkState &ws, const WBm &B,
                               const uint64_t *rs, uint64_t g0, uint64_t g1, uint64_t g, uint64_t x, uint64_t len,
                               uint32_t lane, uint64_t &xe, const uint64_t *sE, const uint64_t *sX, bool *capped,
                               uint64_t *xold) {
    uint64_t L;
    uint64_t k = quiet_run_k<kAlgo>(0, B, rs, x, len, len, wp, lane, L);
    if constexpr (kQuietKinds<kAlgo> > 1)
        if (k < 2) k = quiet_run_k<kAlgo>(1, B, rs, x, len, len, wp, lane, L);
    const uint64_t ce = x + k * L;
    const uint32_t sl = st.span_log2;
    uint64_t ie = min(ce >> sl, g1 - g0);
    const uint64_t i0 = g - g0;
    if (k < 2 || ie <= i0) return g;
    if (sE)  // the first later segment this round re-walks by itself (scheduled, not deferring)
        for (uint64_t b = i0 + 1; b < ie; b += 64) {
            const uint64_t i = b + lane;
            const uint64_t m = __ballot(i < ie && sE[g0 + i] != sX[g0 + i - 1] &&
                                        !defers(st, wp, ws, g0 + i, i << sl));
            if (m) {
                ie = b + (uint64_t)__builtin_ctzll(m);
                if (capped) *capped = true;
                break;
            }
        }
    if (xold) *xold = ws.X[g0 + ie - 1];  // (before the writes below)
    const uint64_t send = min(ie << sl, len);  // the covered segments end here
    const uint64_t jtot = send > x ? (send - x + L - 1) / L : 0;  // run starts inside them
    for (uint64_t j = lane; j < jtot; j += 64) {
        const uint64_t p = x + j * L, i = p >> sl, o = i << sl;
        const uint64_t jl = o > x ? (o - x + L - 1) / L : 0;
        if (j - jl < wp.cap) ws.list[(g0 + i) * wp.cap + (j - jl)] = p;
    }
    for (uint64_t i = i0 + lane; i < ie; i += 64) {
        const uint64_t o = i << sl, e = min(o + (1ull << sl), len);
        const uint64_t jl = o > x ? (o - x + L - 1) / L : 0, jh = e > x ? (e - x + L - 1) / L : 0;
        ws.E[g0 + i] = x + jl * L;
        ws.X[g0 + i] = x + jh * L;
        ws.N[g0 + i] = (uint32_t)(jh - jl);
        if (jh - jl > wp.cap) atomicAdd(&ws.flags[1], 1ull);
    }
    xe = x + jtot * L;
    return g0 + ie;
}

// serial_kernel with a wave per stream (wave-cooperative re-walks).  The exit
// of a segment this pass re-walked is carried in a register (lane 0 wrote it;
// the other lanes do not read it back from memory).
template <int kAlgo>
__global__ __launch_bounds__(256) void wserial_kernel(const StreamTable st, const WalkParams wp, const WalkState ws) {
    constexpr uint32_t nbm = kAlgo == 4 ? 3 : kAlgo == 5 ? 2 : 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t si = (uint64_t)blockIdx.x * 4 + wave_id();
    if (si >= st.n) return;
    const uint64_t g0 = st.span_base[si], g1 = st.span_base[si + 1];
    const uint64_t len = st.lens[si];
    __shared__ __attribute__((aligned(16))) uint8_t lslot[kAlgo == 5 ? 4 * kLeapSlot : 16];
    const WBm B{wp.bm + g0 * (uint64_t)wp.seg_words * nbm, (len + 63) >> 6,
                kAlgo == 5 ? wp.jt + g0 * (uint64_t)wp.seg_words * 24 : nullptr,
                lslot + (kAlgo == 5 ? wave_id() * kLeapSlot : 0),
                kAlgo == 5 ? wp.jt8 + g0 * (uint64_t)wp.seg_words / 8 * 24 : nullptr};
    const uint64_t *rs = wp.rsum ? wp.rsum + g0 * (uint64_t)wp.seg_words / 64 * kQuietKinds<kAlgo> : nullptr;
    uint64_t xprev = 0;
    bool have = false;
    // entries and predecessor exits prefetched 64 segments at a time (lane l:
    // segment gb + l), so settled segments cost no dependent load each; this
    // pass rewrites only segments it has passed
    uint64_t gb = 0, eR = 0, xR = 0;
    bool pref = false;
    for (uint64_t g = max(g0 + 1, (uint64_t)ws.flags[2]); g < g1; ++g) {
        if (!pref || g - gb >= 64) {
            gb = g;
            pref = true;
            eR = g + lane < g1 ? ws.E[g + lane] : 0ull;
            xR = g + lane < g1 ? ws.X[g + lane - 1] : 0ull;
        }
        const uint32_t i = (uint32_t)(g - gb);
        const uint64_t x = have ? xprev : rdlane64(xR, i);
        have = false;
        if (rdlane64(eR, i) == x) continue;
        if (rs) {
            uint64_t xe;
            const uint64_t ge = serial_run<kAlgo>(st, wp, ws, B, rs, g0, g1, g, x, len, lane, xe);
            if (ge > g) {  // segments g .. ge-1 lie wholly inside one quiet run
                xprev = xe;
                have = true;
                g = ge - 1;
                continue;
            }
        }
        const uint64_t off = (g - g0) << st.span_log2;
        const uint64_t seg_end = min(off + (1ull << st.span_log2), len);
        uint64_t xo;
        bool qr;
        (void)wrewalk<kAlgo>(x, g, seg_end, len, B, rs, wp, ws, lane, xo, qr);
        xprev = xo;
        have = true;
    }
}

// ---- bitmap pass ------------------------------------------------------------
// Wave per segment; lane l computes the predicate bits of the positions
// [off + l*w, off + (l+1)*w), w = segment/64 (a multiple of 64), reading its
// bytes 16 at a time plus the window bytes before (and, for Ultra's repeat
// test, after) its range.  Bits of positions whose window would reach before
// the stream start are never tested by the walks (they need min >= 48 / 8 /
// 32), nor are bits at or past the stream end.

// Global (address space 1) loads: through a generic pointer these compile to
// flat_load_*, which count on lgkmcnt as well as vmcnt, so every wait for an
// LDS table lookup would also wait for the next step's prefetched bytes.
typedef unsigned int wu32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) wu32x4 gw_u32x4;
typedef const __attribute__((address_space(1))) uint8_t gw_u8;

__device__ __forceinline__ uint4 load16_guarded(const uint8_t *base, uint64_t a, uint64_t len) {
    if (a + 16 <= len) {
        const wu32x4 v = *(gw_u32x4 *)(base + a);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t t[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
        if (a + j < len) t[j >> 2] |= (uint32_t)((gw_u8 *)base)[a + j] << (8 * (j & 3));
    return make_uint4(t[0], t[1], t[2], t[3]);
}

__device__ __forceinline__ uint32_t byte_of(const uint4 &v, int j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xFFu;
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int w) {
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}

__device__ __forceinline__ uint64_t lo64(const uint4 &v) { return ((uint64_t)v.y << 32) | v.x; }
__device__ __forceinline__ uint64_t hi64(const uint4 &v) { return ((uint64_t)v.w << 32) | v.z; }

// The 8 bytes starting at byte o (0 <= o <= 40) of the 48 bytes W[0..5].
__device__ __forceinline__ uint64_t window8(const uint64_t (&W)[6], int o) {
    const int q = o >> 3, r = o & 7;
    return r == 0 ? W[q] : (W[q] >> (8 * r)) | (W[q + 1] << (64 - 8 * r));
}

// The lane's 16-byte chunks [a0, a1) in order, 64 bytes per step with the
// next 64 bytes' loads in flight while f(chunk, address) runs.
template <typename F>
__device__ __forceinline__ void for_chunks(const uint8_t *base, uint64_t len, uint64_t a0, uint64_t a1, F &&f) {
    uint4 n0 = load16_guarded(base, a0, len), n1 = load16_guarded(base, a0 + 16, len);
    uint4 n2 = load16_guarded(base, a0 + 32, len), n3 = load16_guarded(base, a0 + 48, len);
    for (uint64_t a = a0; a < a1; a += 64) {
        const uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        if (a + 64 < a1) {
            n0 = load16_guarded(base, a + 64, len);
            n1 = load16_guarded(base, a + 80, len);
            n2 = load16_guarded(base, a + 96, len);
            n3 = load16_guarded(base, a + 112, len);
        }
        f(c0, a);
        if (a + 16 < a1) f(c1, a + 16);
        if (a + 32 < a1) f(c2, a + 32);
        if (a + 48 < a1) f(c3, a + 48);
    }
}

// UltraCDC predicate bits of one 64-position word from its bytes w[4..19]
// (w[0..3] = the 16 bytes before, w[20..23] = the 16 after): bitmaps 0
// (dist & MASK_S == 0), 1 (dist & MASK_L == 0), 2 (8-byte repeat).
__device__ __forceinline__ uint64_t ultra_word(const uint32_t (&w)[24], uint64_t *out) {
    // equality bits E(i) = (b[i] == b[i-8]) for i = p0 .. p0+71 (first:
    // w is dead after the popcounts, which keeps the kernel's VGPRs low)
    uint32_t e[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 18; ++k) {
        const uint32_t x = w[k + 4] ^ w[k + 2];
        const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // bit 7 of each zero byte
        const uint32_t nib = (((z >> 7) * 0x204081u) >> 21) & 0xFu;
        e[k >> 3] |= nib << (4 * (k & 7));
    }
    constexpr uint32_t pat4 = 0x01010101u * CDC_ULTRA_PATTERN;
    uint32_t cw[18];  // per-byte popcounts of words 2..19 (positions p0-8 .. p0+63)
#pragma unroll
    for (int k = 0; k < 18; ++k) {
        uint32_t x = w[k + 2] ^ pat4;
        x = x - ((x >> 1) & 0x55555555u);
        x = (x & 0x33333333u) + ((x >> 2) & 0x33333333u);
        cw[k] = (x + (x >> 4)) & 0x0F0F0F0Fu;
    }
    // T(j) = dist(p0+j) + 128 j: one byte-select add per position (bytes
    // of 128 + c(q) - c(q-8), no borrows); the masks test bits < 7 only.
    uint32_t T = ((cw[0] * 0x01010101u) >> 24) + ((cw[1] * 0x01010101u) >> 24);  // dist(p0)
    uint32_t hs0 = 0, hs1 = 0, hl0 = 0, hl1 = 0;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const uint32_t bs = min(T & (uint32_t)CDC_ULTRA_MASK_S, 1u);  // 0 = hit
        const uint32_t bl = min(T & (uint32_t)CDC_ULTRA_MASK_L, 1u);
        if (j < 32) {
            hs0 |= bs << j;
            hl0 |= bl << j;
        } else {
            hs1 |= bs << (j - 32);
            hl1 |= bl << (j - 32);
        }
        const uint32_t dw = (cw[2 + (j >> 2)] | 0x80808080u) - cw[j >> 2];
        T += __builtin_amdgcn_ubfe(dw, 8 * (j & 3), 8);
    }
    typedef unsigned __int128 u128;
    const u128 E = ((u128)e[2] << 64) | ((u128)e[1] << 32) | e[0];
    const u128 a2 = E & (E >> 1), a4 = a2 & (a2 >> 2), a8 = a4 & (a4 >> 4);
    out[0] = ~(((uint64_t)hs1 << 32) | hs0);
    out[1] = ~(((uint64_t)hl1 << 32) | hl0);
    out[2] = (uint64_t)a8;
    return (uint64_t)a8;
}

template <int kAlgo>
__global__ __launch_bounds__(kWalkBlock) void bits_kernel(const StreamTable st, const WalkParams wp) {
    __shared__ uint64_t tab[768];
    if constexpr (kAlgo == 2 || kAlgo == 5) load_tabs(tab, wp.tabs);  // Ultra / Seq use no table
    const Tabs T{tab, tab + 256, tab + 512};
    Piece pc;
    if (!piece_of(st, wp, blockIdx.x, pc)) return;
    const uint32_t si = pc.si;
    const uint64_t off = pc.off;
    const uint64_t len = st.lens[si];
    const uint8_t *base = st.ptrs[si];
    // Fine mode (Ultra, Leap, Seq): a lane evaluates one 64-position word at a
    // time and the wave sweeps the segment 4 KiB per step, so each load
    // instruction covers 4 KiB contiguous and each bitmap store is coalesced;
    // the few window bytes before / after a word are re-read from cache.
    // Rabin keeps one 1/64 range per lane (its 48-byte warm-up per range).
    const uint64_t seg_bytes = 1ull << wp.piece_log2;  // (this piece)
    const bool fine = kAlgo != 2 && wp.bits_fine != 0;
    const uint64_t w = fine ? 64 : seg_bytes >> 6;
    const uint32_t reps = fine ? (uint32_t)(seg_bytes >> 12) : 1u;
    for (uint32_t it = 0; it < reps; ++it) {
    const uint64_t lidx = fine ? (uint64_t)it * 64 + threadIdx.x : threadIdx.x;
    const uint64_t p0 = off + lidx * w;
    if (p0 >= len) return;
    const uint64_t p1 = min(p0 + w, len);
    uint64_t *out = wp.bm + (pc.wbase + lidx * (w >> 6)) * wp.nbm;
    if constexpr (kAlgo == 2) {
        // Rolling Rabin digest from 48 bytes before p0 (out bytes 0 until
        // 48 bytes are in): the digest after byte i is the fingerprint of the
        // window [i-47, i], exactly the digest cut_rabin tests.
        const uint64_t f0 = p0 >= CDC_RABIN_WINDOW ? p0 - CDC_RABIN_WINDOW : 0;
        uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, c2 = c0;  // chunks 48, 32, 16 bytes back
        if (wp.rabin_mask <= 0xFFFFFFFFull && wp.rabin_shift >= 32 && (p0 & 63) == 0) {
            // The digest as two dwords (deg < 64): per byte one v_alignbit
            // for the 8-bit shift of the high dword, one v_lshl_or for the
            // low one, the two table XORs, and a 32-bit test; the 48-byte
            // warm-up runs without tests, then whole 64-position words.
            const uint32_t rmask = (uint32_t)wp.rabin_mask, tsh = wp.rabin_shift - 32;
            uint32_t lo = 0, hi = 0;
            auto step16 = [&](const uint4 &cur, const uint4 &old, uint32_t &bits, int sh, bool test) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint64_t o = T.out[byte_of(old, j)];
                    lo ^= (uint32_t)o;
                    hi ^= (uint32_t)(o >> 32);
                    const uint64_t m = T.mod[hi >> tsh];
                    hi = __builtin_amdgcn_alignbit(hi, lo, 24) ^ (uint32_t)(m >> 32);
                    lo = ((lo << 8) | byte_of(cur, j)) ^ (uint32_t)m;
                    if (test) bits |= min(lo & rmask, 1u) << (sh + j);
                }
            };
            uint32_t dummy = 0;
            for (uint64_t a = f0; a < p0; a += 16) {
                const uint4 cur = load16_guarded(base, a, len);
                step16(cur, c0, dummy, 0, false);
                c0 = c1;
                c1 = c2;
                c2 = cur;
            }
            uint4 n0 = load16_guarded(base, p0, len), n1 = load16_guarded(base, p0 + 16, len);
            uint4 n2 = load16_guarded(base, p0 + 32, len), n3 = load16_guarded(base, p0 + 48, len);
            for (uint64_t a = p0; a < p1; a += 64) {
                const uint4 q0 = n0, q1 = n1, q2 = n2, q3 = n3;
                if (a + 64 < p1) {
                    n0 = load16_guarded(base, a + 64, len);
                    n1 = load16_guarded(base, a + 80, len);
                    n2 = load16_guarded(base, a + 96, len);
                    n3 = load16_guarded(base, a + 112, len);
                }
                uint32_t b0 = 0, b1 = 0;
                step16(q0, c0, b0, 0, true);
                step16(q1, c1, b0, 16, true);
                step16(q2, c2, b1, 0, true);
                step16(q3, q0, b1, 16, true);
                c0 = q1;
                c1 = q2;
                c2 = q3;
                out[(a - p0) >> 6] = ~(((uint64_t)b1 << 32) | b0);  // bit set = window hit
            }
            continue;
        }
        uint64_t d = 0, acc = 0;
        for_chunks(base, len, f0, p1, [&](const uint4 &cur, uint64_t a) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t i = a + j;
                d ^= T.out[byte_of(c0, j)];
                const uint64_t top = d >> wp.rabin_shift;
                d = ((d << 8) | byte_of(cur, j)) ^ T.mod[top];
                if (i >= p0 && i < p1) {
                    acc |= (uint64_t)((d & wp.rabin_mask) == 0) << ((i - p0) & 63);
                    if (((i - p0) & 63) == 63) {
                        out[((i - p0) >> 6)] = acc;
                        acc = 0;
                    }
                }
            }
            c0 = c1;
            c1 = c2;
            c2 = cur;
        });
        if ((p1 - p0) & 63) out[(p1 - p0) >> 6] = acc;
    } else if constexpr (kAlgo == 4) {
      if (fine) {
        // One 64-position word per lane, on 32-bit words: per-byte popcounts
        // c(i) = popcount(b[i] ^ 0xAA) by SWAR, dist(q) = sum c(q-8 .. q-1)
        // kept as a running sum (+c(q) - c(q-8) per position); the repeat
        // bit of q = bytes q .. q+7 all equal the byte 8 before them, from
        // per-byte equality bits (SWAR zero-byte test of w[k] ^ w[k-2]) and
        // three shift-ANDs.  Words: w[0..3] = [p0-16, p0), w[4..19] = the
        // lane's 64 bytes, w[20..23] = [p0+64, p0+80); bytes past the stream
        // end read 0 (as load16_guarded).
        uint32_t w[24];
        {
            const uint4 a = p0 >= 16 ? load16_guarded(base, p0 - 16, len) : make_uint4(0, 0, 0, 0);
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint4 v = load16_guarded(base, p0 + 16 * k, len);
                w[4 + 4 * k] = v.x; w[5 + 4 * k] = v.y; w[6 + 4 * k] = v.z; w[7 + 4 * k] = v.w;
            }
        }
        ultra_word(w, out);
        continue;
      }
        // dist(q) = popcount of the 8 bytes before q ^ 0xAA..; repeat(q) =
        // the 8 bytes at q equal the 8 before.  A chunk's positions are
        // evaluated when the chunk after it arrives (bytes [a-16, a+32) in W).
        constexpr uint64_t pat = 0x0101010101010101ull * CDC_ULTRA_PATTERN;
        uint4 prev = p0 >= 16 ? load16_guarded(base, p0 - 16, len) : make_uint4(0, 0, 0, 0);
        uint4 cur = make_uint4(0, 0, 0, 0);
        uint64_t hs = 0, hl = 0, eq = 0;
        for_chunks(base, len, p0, p1 + 16, [&](const uint4 &nxt, uint64_t an) {
            if (an == p0) {
                cur = nxt;
                return;
            }
            const uint64_t a = an - 16;  // the chunk evaluated now
            const uint64_t W[6] = {lo64(prev), hi64(prev), lo64(cur), hi64(cur), lo64(nxt), hi64(nxt)};
            const uint32_t sh = (uint32_t)((a - p0) & 63);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t before = window8(W, 8 + j), at = window8(W, 16 + j);
                const uint32_t dist = (uint32_t)__popcll(before ^ pat);
                hs |= (uint64_t)((dist & CDC_ULTRA_MASK_S) == 0) << (sh + j);
                hl |= (uint64_t)((dist & CDC_ULTRA_MASK_L) == 0) << (sh + j);
                eq |= (uint64_t)(before == at) << (sh + j);
            }
            if (sh == 48 || a + 16 >= p1) {
                const uint64_t k = (a - p0) >> 6;
                out[k * 3 + 0] = hs;
                out[k * 3 + 1] = hl;
                out[k * 3 + 2] = eq;
                hs = hl = eq = 0;
            }
            prev = cur;
            cur = nxt;
        });
    } else if constexpr (kAlgo == 6) {
        // SeqCDC: bit p = (b[p] > b[p-1]) (increasing) or (b[p] < b[p-1]),
        // four bytes per dword (SWAR): with x, y the bytes compared, bit 7 of
        // t = (x | 0x80) - (y & 0x7F) - 1 is (x & 0x7F) > (y & 0x7F) (no
        // borrow leaves a byte), and x > y takes x's bit 7 where bits 7
        // differ, t's elsewhere; the four bit 7s gather into a nibble.
        uint32_t lastw = p0 >= 1 ? (uint32_t)base[p0 - 1] << 24 : 0u;  // b[a-1] in bits 24..31
        uint64_t acc = 0, wlast = 0;
        for_chunks(base, len, p0, p1, [&](const uint4 &cur, uint64_t a) {
            const uint32_t sh = (uint32_t)((a - p0) & 63);
            uint32_t b16 = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t W = word_of(cur, q);
                const uint32_t P = __builtin_amdgcn_alignbit(W, lastw, 24);  // byte k: b[i + k - 1]
                lastw = W;
                const uint32_t x = wp.seq_mode ? P : W, y = wp.seq_mode ? W : P;
                const uint32_t t = (x | 0x80808080u) - (y & 0x7F7F7F7Fu) - 0x01010101u;
                const uint32_t d = x ^ y;
                const uint32_t h = ((d & x) | (~d & t)) & 0x80808080u;
                b16 |= ((((h >> 7) * 0x204081u) >> 21) & 0xFu) << (4 * q);
            }
            acc |= (uint64_t)b16 << sh;
            if (sh == 48 || a + 16 >= p1) {
                out[(a - p0) >> 6] = acc;
                wlast = acc;
                acc = 0;
            }
        });
        if (fine && wp.rsum) {  // quiet-run summary: words without an in-direction pair
            const uint64_t full = __ballot(wlast == 0);
            if (threadIdx.x == 0) wp.rsum[(pc.wbase >> 6) + it] = full;
        }
    } else {
        // Leap eligibility of the 5-byte window ending at p (bytes [a-16, a+16)).
        uint4 prev = p0 >= 16 ? load16_guarded(base, p0 - 16, len) : make_uint4(0, 0, 0, 0);
        uint64_t pr = 0, se = 0;
        for_chunks(base, len, p0, p1, [&](const uint4 &cur, uint64_t a) {
            const uint32_t sh = (uint32_t)((a - p0) & 63);
            uint64_t e[21];
#pragma unroll
            for (int j = 0; j < 4; ++j) e[j] = T.leap[byte_of(prev, 12 + j)];
#pragma unroll
            for (int j = 0; j < 16; ++j) e[4 + j] = T.leap[byte_of(cur, j)];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                uint64_t h = 0;
#pragma unroll
                for (int k = 0; k < (int)CDC_LEAP_WSIZE; ++k) h += rotl64(e[4 + j - k], 11 * k);
                pr |= (uint64_t)((uint32_t)(h >> 32) < wp.leap_thr) << (sh + j);
                se |= (uint64_t)((uint32_t)h < wp.leap_thr) << (sh + j);
            }
            if (sh == 48 || a + 16 >= p1) {
                const uint64_t k = (a - p0) >> 6;
                out[k * 2 + 0] = pr;
                out[k * 2 + 1] = se;
                pr = se = 0;
            }
            prev = cur;
        });
    }
    }
}

// Rabin's bitmap pass with replicated tables: 8 pieces (waves) per block
// share 16 replicas of the mod / out tables (64 KiB of LDS; lane l reads
// replica l & 15, entry e at (16 e + r) * 8, so two lanes of a 32-lane bank
// group share a replica).  PMC of the single-copy tables showed 4x LDS cycles
// in bank conflicts (profiles/r03_walk); per GiB at 4/8/16 KiB, whole Rabin
// call: 8 replicas x 4 waves 1293 GiB/s, 8 x 8 1294, 16 x 4 1051, 16 x 8
// 1327, 32 x 16 (conflict-free, one block per CU) 1165
// (profiles/r03_walk/r03ah_rabin_bits_variants.txt).  Lane l hashes 1/64 of its wave's segment from a
// 48-byte warm-up (as bits_kernel<2>), the digest as two dwords.
#ifndef CDC_RABIN_REPS  // (experiment builds, tools/build_variants.py)
#define CDC_RABIN_REPS 16
#endif
#ifndef CDC_RABIN_WAVES
#define CDC_RABIN_WAVES 8
#endif
// Skewed replicas (CDC_RABIN_SKEW=1): entry e's 16 replicas at e * 136 bytes
// (17 slots), so the bank of a lookup depends on the entry too -- lanes l and
// l+16 share a replica and used to collide on every lookup (bank = 2r only:
// 48 % of LDS cycles were conflicts, profiles/r04_walk/r04f_pmc_walk.txt);
// with the skew they collide when their entries agree mod 16.
#ifndef CDC_RABIN_SKEW
#define CDC_RABIN_SKEW 0  // measured slower: 1262 vs 1346 GiB/s (profiles/r05/r05g_rabin_*.log)
#endif
// The leaving byte's term after the shift (CDC_RABIN_OUT2=1): d' = ((d << 8) |
// in) ^ mod[top(d)] ^ out2[leaving], out2[b] = b x^(8W) mod P (= x^8 out[b]),
// so the out lookup is off the digest's dependency chain and both table
// values fold in with one v_xor3 per half: 7 VALU per byte for the digest
// instead of 11 (the round-4 PMC had the pass VALU-issue-bound at 14.7 per byte).
#ifndef CDC_RABIN_OUT2
#define CDC_RABIN_OUT2 0  // measured slower: rbits 0.58-0.60 vs 0.55-0.57 ms (profiles/r05/r05q_*)
#endif
// A wave hashes 2^CDC_RABIN_GROUP_LOG2 consecutive pieces of one segment as
// one range (2 KiB per lane at 32 KiB pieces instead of 512 B): the 48-byte
// warm-up each lane re-hashes before its range drops from 9.4 % to 2.3 % of
// the bytes.
#ifndef CDC_RABIN_GROUP_LOG2
#define CDC_RABIN_GROUP_LOG2 0  // measured slower at 2: rbits 0.60 vs 0.55-0.57 ms (profiles/r05/r05q_*)
#endif
static_assert(CDC_RABIN_GROUP_LOG2 <= 2, "rbits_kernel: a lane's quiet bits are one 32-bit word (<= 2 KiB per lane)");
__host__ __device__ __forceinline__ uint32_t rabin_group_log2(const StreamTable &st, const WalkParams &wp) {
    const uint32_t k = st.span_log2 - wp.piece_log2;
    return k < CDC_RABIN_GROUP_LOG2 ? k : CDC_RABIN_GROUP_LOG2;
}
// (Its input loads re-fetch: FETCH_SIZE 1.76x of the input, the halves of a
// 128-byte line being asked for one iteration apart by 1024 lanes per CU.
// Non-temporal second halves made it 1.90x and the pass slower, and a whole
// line per iteration needs 169 VGPRs: profiles/r05/r05y_*.)
constexpr int kRabinReps = CDC_RABIN_REPS;
constexpr int kRabinWaves = CDC_RABIN_WAVES;  // pieces per block (64 KiB of tables shared by 8 waves)

typedef const __attribute__((address_space(3))) uint64_t lds_w64;
typedef const __attribute__((address_space(3))) char lds_wchar;

__global__ __launch_bounds__(64 * kRabinWaves) void rbits_kernel(const StreamTable st, const WalkParams wp) {
    // entry e at e * 256 bytes: 16 replicas of mod[e], then 16 of out[e]; a
    // lane's replica offset is one byte, so each lookup address is one v_perm
    // (out: the leaving byte) or one v_lshl_or (mod: the digest's top byte).
    // (Two interleaved chains per lane -- more independent lookups in flight
    // -- need ~2x the registers and spilled at the 128 VGPRs of 16 waves / CU.)
#if CDC_RABIN_SKEW
    constexpr uint32_t kStride = 136;  // bytes per entry (17 slots of 8: 16 replicas + a skew slot)
    __shared__ uint64_t rt[2 * 256 * 17];  // mod table, then out table
    static_assert(kRabinReps == 16, "rbits_kernel: 16 replicas per table");
    for (int i = threadIdx.x; i < 2 * 256 * 17; i += 64 * kRabinWaves) {
        const int t = i / (256 * 17), e = (i % (256 * 17)) / 17;
        rt[i] = wp.tabs[(t ? 256 : 0) + e];
    }
#else
    __shared__ uint64_t rt[256 * 32];
    static_assert(kRabinReps == 16, "rbits_kernel: 16 replicas per table");
    for (int i = threadIdx.x; i < 256 * 32; i += 64 * kRabinWaves) {
        const int e = i >> 5, k = i & 31;
        uint64_t v = wp.tabs[(k < 16 ? 0 : 256) + e];
        if (CDC_RABIN_OUT2 && k >= 16) v = (v << 8) ^ wp.tabs[v >> wp.rabin_shift];  // x^8 out[e] mod P
        rt[i] = v;
    }
#endif
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    Piece pc;
    const uint32_t grp = rabin_group_log2(st, wp);
    if (!piece_of(st, wp, ((uint64_t)blockIdx.x * kRabinWaves + wave_id()) << grp, pc)) return;
#if CDC_RABIN_SKEW
    const uint32_t om = (lane & 15) * 8, oo = 256 * kStride + om;  // this lane's mod / out replica
#else
    const uint32_t om = (lane & 15) * 8, oo = 128 + om;  // this lane's mod / out replica
#endif
    lds_wchar *tb = (lds_wchar *)rt;
    const uint64_t len = st.lens[pc.si];
    const uint8_t *base = st.ptrs[pc.si];
    // bytes per lane (a multiple of 64; the group's pieces are consecutive in
    // the segment, in bytes and in bitmap words)
    const uint64_t w = (1ull << (wp.piece_log2 + grp)) >> 6;
    const uint64_t p0 = pc.off + lane * w;
    uint32_t qm = 0, qa = 0;  // bit i: word i of the lane's range has no hit / only hits (quiet runs)
    if (p0 < len) {
    const uint64_t p1 = min(p0 + w, len);
        uint64_t *out = wp.bm + (pc.wbase + lane * (w >> 6));
        const uint32_t rmask = (uint32_t)wp.rabin_mask, tsh = wp.rabin_shift - 32;
        uint32_t lo = 0, hi = 0;
        auto step16 = [&](const uint4 &cur, const uint4 &old, uint32_t &bits, int sh, bool test) {
    #pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t ow = word_of(old, j >> 2), cw = word_of(cur, j >> 2);
#if CDC_RABIN_SKEW
                const uint32_t ao = __umul24((ow >> (8 * (j & 3))) & 0xFFu, kStride) + oo;
#else
                const uint32_t ao = __builtin_amdgcn_perm(oo, ow, 0x0c0c0004u | ((uint32_t)(j & 3) << 8));
#endif
                const uint64_t o = *reinterpret_cast<lds_w64 *>(tb + ao);
#if CDC_RABIN_OUT2 && !CDC_RABIN_SKEW
                // o = out2[leaving byte], folded in after the shift (off the chain)
                const uint64_t m = *reinterpret_cast<lds_w64 *>(tb + (((hi >> tsh) << 8) | om));
                hi = __builtin_amdgcn_alignbit(hi, lo, 24) ^ (uint32_t)(m >> 32) ^ (uint32_t)(o >> 32);
                // (lo << 8) | the entering byte, one v_perm
                lo = __builtin_amdgcn_perm(lo, cw, 0x06050400u | (uint32_t)(j & 3)) ^ (uint32_t)m ^ (uint32_t)o;
#else
                lo ^= (uint32_t)o;
                hi ^= (uint32_t)(o >> 32);
#if CDC_RABIN_SKEW
                const uint64_t m = *reinterpret_cast<lds_w64 *>(tb + (__umul24(hi >> tsh, kStride) + om));
#else
                const uint64_t m = *reinterpret_cast<lds_w64 *>(tb + (((hi >> tsh) << 8) | om));
#endif
                hi = __builtin_amdgcn_alignbit(hi, lo, 24) ^ (uint32_t)(m >> 32);
                lo = __builtin_amdgcn_perm(lo, cw, 0x06050400u | (uint32_t)(j & 3)) ^ (uint32_t)m;
#endif
                if (test) bits |= min(lo & rmask, 1u) << (sh + j);
            }
        };
        uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, c2 = c0;  // chunks 48, 32, 16 bytes back
        uint32_t dummy = 0;
        for (uint64_t a = p0 >= CDC_RABIN_WINDOW ? p0 - CDC_RABIN_WINDOW : p0; a < p0; a += 16) {
            const uint4 cur = load16_guarded(base, a, len);
            step16(cur, c0, dummy, 0, false);
            c0 = c1;
            c1 = c2;
            c2 = cur;
        }
        auto emit = [&](uint64_t a, uint32_t b0, uint32_t b1) {
            const uint64_t hits = ~(((uint64_t)b1 << 32) | b0);  // bit set = window hit
            const uint32_t wi = (uint32_t)((a - p0) >> 6);
            out[wi] = hits;
            qm |= (uint32_t)(hits == 0) << wi;
            qa |= (uint32_t)(hits == ~0ull) << wi;
        };
        uint4 n0 = load16_guarded(base, p0, len), n1 = load16_guarded(base, p0 + 16, len);
        uint4 n2 = load16_guarded(base, p0 + 32, len), n3 = load16_guarded(base, p0 + 48, len);
        for (uint64_t a = p0; a < p1; a += 64) {
            const uint4 q0 = n0, q1 = n1, q2 = n2, q3 = n3;
            if (a + 64 < p1) {
                n0 = load16_guarded(base, a + 64, len);
                n1 = load16_guarded(base, a + 80, len);
                n2 = load16_guarded(base, a + 96, len);
                n3 = load16_guarded(base, a + 112, len);
            }
            uint32_t b0 = 0, b1 = 0;
            step16(q0, c0, b0, 0, true);
            step16(q1, c1, b0, 16, true);
            step16(q2, c2, b1, 0, true);
            step16(q3, q0, b1, 16, true);
            c0 = q1;
            c1 = q2;
            c2 = q3;
            emit(a, b0, b1);
        }
    }
    if (wp.rsum && (w >> 6) >= 8) {  // nw >= 8 words per lane: nw / 8 whole summary bytes per kind
        const uint32_t nw = (uint32_t)(w >> 6);
        const uint64_t W = pc.wbase + lane * nw;
        uint8_t *b = reinterpret_cast<uint8_t *>(wp.rsum) + (W >> 6) * 16 + ((W >> 3) & 7);
        for (uint32_t k = 0; k < nw / 8; ++k) {
            b[k] = (uint8_t)(qm >> (8 * k));
            b[8 + k] = (uint8_t)(qa >> (8 * k));
        }
    } else if (wp.rsum) {  // the lanes' quiet bits into summary bytes (nw words per lane, 8 / nw lanes per byte)
        const uint32_t nw = (uint32_t)(w >> 6), gl = 8 / nw;
        uint32_t v = (qm | qa << 8) << (nw * (lane & (gl - 1)));
        for (uint32_t o = 1; o < gl; o <<= 1) v |= (uint32_t)__shfl_xor((int)v, (int)o);
        if ((lane & (gl - 1)) == 0) {  // kinds interleaved: summary word sk of kind q at rsum[2 sk + q]
            const uint64_t W = pc.wbase + lane * nw;
            uint8_t *b = reinterpret_cast<uint8_t *>(wp.rsum) + (W >> 6) * 16 + ((W >> 3) & 7);
            b[0] = (uint8_t)v;
            b[8] = (uint8_t)(v >> 8);
        }
    }
}

// UltraCDC's bitmap pass: 4 segments (waves) per block, lane per 64-position
// word, the wave sweeping its segment 4 KiB per step with the next step's
// six 16-byte loads in flight while ultra_word runs on the current one.
__device__ __forceinline__ void ultra_load(uint4 (&v)[6], const uint8_t *base, uint64_t len, uint64_t p0) {
    v[0] = p0 >= 16 ? load16_guarded(base, p0 - 16, len) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 5; ++k) v[1 + k] = load16_guarded(base, p0 + 16 * k, len);
}

__global__ __launch_bounds__(256) void ubits_kernel(const StreamTable st, const WalkParams wp) {
    const uint32_t lane = threadIdx.x & 63;
    Piece pc;
    if (!piece_of(st, wp, (uint64_t)blockIdx.x * 4 + wave_id(), pc)) return;
    const uint64_t off = pc.off;
    const uint64_t len = st.lens[pc.si];
    const uint8_t *base = st.ptrs[pc.si];
    const uint32_t reps = (uint32_t)((1ull << wp.piece_log2) >> 12);
    uint4 nx[6];
    ultra_load(nx, base, len, off + 64ull * lane);
    for (uint32_t it = 0; it < reps; ++it) {
        const uint64_t lidx = (uint64_t)it * 64 + lane;
        const uint64_t p0 = off + lidx * 64;
        if (p0 >= len) return;
        uint32_t w[24];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            w[4 * k] = nx[k].x; w[4 * k + 1] = nx[k].y; w[4 * k + 2] = nx[k].z; w[4 * k + 3] = nx[k].w;
        }
        if (it + 1 < reps && p0 + 4096 < len) ultra_load(nx, base, len, p0 + 4096);
        const uint64_t rep = ultra_word(w, wp.bm + (pc.wbase + lidx) * 3);
        // the 64 words' all-repeat bits (lanes past the stream end: 0)
        const uint64_t full = __ballot(rep == ~0ull);
        if (wp.rsum && lane == 0) wp.rsum[(pc.wbase >> 6) + it] = full;
    }
}

// LeapCDC's bitmap pass: 4 pieces (waves) per block sharing 8 replicas of
// the window-hash table (16 KiB; the single-copy table spent 4x its LDS
// cycles in bank conflicts, profiles/r03_walk/pmcw_r03af), lane per
// 64-position word, each byte's table value looked up once per word (the 4
// bytes before the word once), the next word's loads in flight.
constexpr int kLeapReps = 8;

__device__ __forceinline__ void leap_load(uint4 (&v)[5], const uint8_t *base, uint64_t len, uint64_t p0) {
    v[0] = p0 >= 16 ? load16_guarded(base, p0 - 16, len) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[1 + k] = load16_guarded(base, p0 + 16 * k, len);
}

__global__ __launch_bounds__(256) void lbits_kernel(const StreamTable st, const WalkParams wp) {
    __shared__ uint64_t lt[256 * kLeapReps];
    for (int i = threadIdx.x; i < 256 * kLeapReps; i += 256) lt[i] = wp.tabs[512 + i / kLeapReps];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    Piece pc;
    if (!piece_of(st, wp, (uint64_t)blockIdx.x * 4 + wave_id(), pc)) return;
    const uint64_t *tl = lt + (lane & (kLeapReps - 1));
    const uint64_t len = st.lens[pc.si];
    const uint8_t *base = st.ptrs[pc.si];
    const uint32_t reps = (uint32_t)((1ull << wp.piece_log2) >> 12);
    const uint32_t thr = wp.leap_thr;
    uint4 nx[5];
    leap_load(nx, base, len, pc.off + 64ull * lane);
    for (uint32_t it = 0; it < reps; ++it) {
        const uint64_t lidx = (uint64_t)it * 64 + lane;
        const uint64_t p0 = pc.off + lidx * 64;
        if (p0 >= len) return;
        uint4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = nx[k];
        if (it + 1 < reps && p0 + 4096 < len) leap_load(nx, base, len, p0 + 4096);
        uint64_t e[20];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[16 + j] = tl[byte_of(v[0], 12 + j) * kLeapReps];
        uint32_t pr[2] = {0, 0}, se[2] = {0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int j = 0; j < 4; ++j) e[j] = e[16 + j];  // the 4 bytes before this 16
#pragma unroll
            for (int j = 0; j < 16; ++j) e[4 + j] = tl[byte_of(v[1 + q], j) * kLeapReps];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                uint64_t h = 0;
#pragma unroll
                for (int k = 0; k < (int)CDC_LEAP_WSIZE; ++k) h += rotl64(e[4 + j - k], 11 * k);
                const int bit = 16 * (q & 1) + j;
                pr[q >> 1] |= (uint32_t)((uint32_t)(h >> 32) < thr) << bit;
                se[q >> 1] |= (uint32_t)((uint32_t)h < thr) << bit;
            }
        }
        uint64_t *out = wp.bm + (pc.wbase + lidx) * 2;
        const uint64_t prw = ((uint64_t)pr[1] << 32) | pr[0], sew = ((uint64_t)se[1] << 32) | se[0];
        out[0] = prw;
        out[1] = sew;
        // quiet-run summary: words whose windows are all eligible
        const uint64_t full = __ballot((prw & sew) == ~0ull);
        if (wp.rsum && lane == 0) wp.rsum[(pc.wbase >> 6) + it] = full;
    }
}

// ---- link mode (Rabin, UltraCDC, LeapCDC) ---------------------------------------
// Candidates: the positions where a chunk can start after a cut that is not a
// max / end / LEST cut, whatever the previous chunk's start -- so every such
// cut lands on one:
//   Rabin  q = p + 1 for a window hit at p (cut_rabin_bits returns i + 1);
//   Ultra  a mask_s or mask_l hit at q (cut_ultra_bits returns i + j there);
//   Leap   its 22 primary windows (ending at q-1 .. q-22) and 2 secondary
//          windows (q-23, q-24) eligible (cut_leap_bits returns c only
//          then): runs of 22 set bits by doubling over two words.
// Each lane produces the candidate mask of one 64-position word.
template <int kAlgo>
__device__ __forceinline__ uint64_t cand_word(const uint64_t *bm, uint64_t K) {
    if constexpr (kAlgo == 2) {  // Rabin, one bitmap
        const uint64_t h1 = bm[K], h0 = K ? bm[K - 1] : 0;
        return (h1 << 1) | (h0 >> 63);
    } else if constexpr (kAlgo == 4) {  // Ultra: mask_s | mask_l
        return bm[K * 3] | bm[K * 3 + 1];
    } else {  // Leap
        const uint64_t p1 = bm[K * 2], s1 = bm[K * 2 + 1];
        const uint64_t p0 = K ? bm[K * 2 - 2] : 0, s0 = K ? bm[K * 2 - 1] : 0;
        typedef unsigned __int128 u128;
        const u128 V = ((u128)p1 << 64) | p0, W = ((u128)s1 << 64) | s0;
        const u128 e2 = V & (V << 1), e4 = e2 & (e2 << 2), e8 = e4 & (e4 << 4), e16 = e8 & (e8 << 8);
        const u128 e22 = e16 & (e4 << 16) & (e2 << 20);  // bit b: primary bits b-21 .. b all set
        return (uint64_t)(e22 >> 63) & (uint64_t)(W >> 41) & (uint64_t)(W >> 40);
    }
}

template <int kAlgo>
__global__ __launch_bounds__(kWalkBlock) void cand_kernel(const StreamTable st, const WalkParams wp) {
    constexpr uint32_t kNbm = kAlgo == 2 ? 1 : kAlgo == 4 ? 3 : 2;
    // lowest position a cut can reach: min >= 1 (Rabin), >= 8 (Ultra), >= 32 (Leap)
    constexpr uint64_t kLow = kAlgo == 2 ? 1 : kAlgo == 4 ? 8 : 32;
    const uint64_t g = blockIdx.x;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t len = st.lens[si];
    const uint64_t gbase = st.span_base[si];
    const uint64_t *bm = wp.bm + gbase * (uint64_t)wp.seg_words * kNbm;  // the stream's bitmaps
    const uint64_t w0 = (off >> 6);                                       // stream word of the segment's start
    const uint32_t lane = threadIdx.x;
    uint32_t total = 0;
    uint32_t *out = wp.cpos + g * wp.ccap;
    for (uint32_t r = 0; r < wp.seg_words / 64; ++r) {
        const uint64_t K = w0 + (uint64_t)r * 64 + lane;  // this lane's stream word
        uint64_t m = 0;
        if (K * 64 < len) {
            m = cand_word<kAlgo>(bm, K);
            const uint64_t q0 = K * 64;  // position of bit 0
            if (q0 < kLow) m &= ~0ull << (kLow - q0);
            if (len - q0 < 64) m &= (1ull << (len - q0)) - 1;  // q < len
        }
        // ordered compaction: an exclusive prefix of the lanes' counts
        const uint32_t c = (uint32_t)__popcll(m);
        uint32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        uint32_t slot = total + x - c;
        for (uint64_t mm = m; mm; mm &= mm - 1, ++slot)
            if (slot < wp.ccap) out[slot] = (uint32_t)(((uint64_t)r * 64 + lane) * 64 + __builtin_ctzll(mm));
        total += (uint32_t)__shfl(x, 63);
    }
    if (lane == 0) wp.ccnt[g] = total;
}

// The rule's next start after a chunk starting at c, over the global bitmaps.
template <int kAlgo>
__device__ __forceinline__ uint64_t link_next(const WalkParams &wp, uint64_t gbase, uint64_t c, uint64_t len) {
    constexpr uint32_t kNbm = kAlgo == 2 ? 1 : kAlgo == 4 ? 3 : 2;
    GReader r;
    r.init(wp.bm + gbase * (uint64_t)wp.seg_words * kNbm, ((len + 63) >> 6) * kNbm);
    if constexpr (kAlgo == 2) return c + cut_rabin_bits(r, c, len - c, wp);
    else if constexpr (kAlgo == 4) return c + cut_ultra_bits(r, c, len - c, wp);
    else return c + cut_leap_bits(r, c, len - c, wp);
}

// Slot of a link's next start nx: its candidate slot, else a new virtual
// entry (to be linked by round `round`), else kNoCand (stream end, the
// budget or the rounds spent: the walk then walks the rule from there).
__device__ __forceinline__ uint32_t next_slot(const WalkParams &wp, uint32_t sl2, uint64_t gbase, uint64_t nx,
                                              uint64_t len, uint32_t round) {
    if (nx >= len) return kNoCand;
    const Hop hp{gbase, sl2, kNoCand};
    const uint32_t ci = find_cand(wp, hp, nx);
    if (ci != kNoCand || round >= kVirtRounds) return ci;
    const unsigned long long v = atomicAdd(&wp.vcnt[0], 1ull);
    if (v >= wp.vcap) return kNoCand;
    wp.vpos[v] = nx;
    wp.vseg[v] = (uint32_t)gbase;
    return kVirt | (uint32_t)v;
}

// Lane per candidate slot (k-major: the 64 lanes of a wave share k, so the
// waves of high k retire at once): the next chunk start after a chunk
// starting at the candidate, and that start's slot.
template <int kAlgo>
__global__ __launch_bounds__(256) void link_kernel(const StreamTable st, const WalkParams wp) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t S = st.total_spans;
    const uint64_t k = t / S, g = t - k * S;
    if (k >= wp.ccap) return;
    const uint32_t n = wp.ccnt[g];
    if (n > wp.ccap || k >= n) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t len = st.lens[si];
    const uint64_t gbase = st.span_base[si];
    const uint64_t slot = g * wp.ccap + k;
    const uint64_t nx = link_next<kAlgo>(wp, gbase, off + wp.cpos[slot], len);
    wp.lnext[slot] = nx;
    wp.lidx[slot] = next_slot(wp, st.span_log2, gbase, nx, len, 0);
}

// Round r of the virtual links: the entries allocated before it and after
// round r-1 started (vcnt[1 + r] .. vcnt[2 + r], snapshots by vmark_kernel).
template <int kAlgo>
__global__ __launch_bounds__(256) void vlink_kernel(const StreamTable st, const WalkParams wp, uint32_t round) {
    const uint64_t v = wp.vcnt[1 + round] + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t end = min(wp.vcnt[2 + round], (unsigned long long)wp.vcap);
    if (v >= end) return;
    const uint64_t gbase = wp.vseg[v];
    uint32_t si;
    uint64_t off;
    locate(st, gbase, si, off);
    const uint64_t len = st.lens[si];
    const uint64_t nx = link_next<kAlgo>(wp, gbase, wp.vpos[v], len);
    wp.vnext[v] = nx;
    wp.vidx[v] = next_slot(wp, st.span_log2, gbase, nx, len, round + 1);
}

// Snapshot of the allocation counter: the end of virtual round r.
__global__ void vmark_kernel(const WalkParams wp, uint32_t round) { wp.vcnt[2 + round] = wp.vcnt[0]; }

template <int kAlgo>
hipError_t links_dispatch(const StreamTable &st, const WalkParams &wp, hipStream_t s) {
    hipError_t e = hipMemsetAsync(wp.vcnt, 0, (2 * kVirtRounds + 2) * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    cand_kernel<kAlgo><<<(unsigned)st.total_spans, kWalkBlock, 0, s>>>(st, wp);
    const uint64_t threads = st.total_spans * (uint64_t)wp.ccap;
    link_kernel<kAlgo><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(st, wp);
    for (uint32_t r = 0; r < kVirtRounds; ++r) {  // round r links the entries allocated by round r - 1
        vmark_kernel<<<1, 1, 0, s>>>(wp, r);
        vlink_kernel<kAlgo><<<(unsigned)((wp.vcap + 255) / 256), 256, 0, s>>>(st, wp, r);
    }
    return hipGetLastError();
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

// The output kernels queued behind the first group of fix-up rounds (egate:
// its first flag block, egn rounds) run only when one of those rounds settled
// every segment before any round handed off to the in-order pass -- the
// host's rule in Engine::run_walk, which otherwise re-queues them.
__device__ __forceinline__ bool emit_skips(const unsigned long long *egate, uint32_t egn) {
    if (!egate) return false;
    for (uint32_t r = 0; r < egn; ++r) {
        const int v = round_verdict(egate[4 * r], egate[4 * r + 3] >> 32);
        if (v == kRoundSettled) return false;
        if (v == kRoundQuiet) return true;
    }
    return true;
}

__global__ __launch_bounds__(kScanBlock) void sum_kernel(const StreamTable st, const WalkState ws,
                                                         const unsigned long long *egate, uint32_t egn) {
    if (emit_skips(egate, egn)) return;
    __shared__ uint64_t sh[kScanBlock];
    const uint64_t g = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
    const uint64_t v = g < st.total_spans ? ws.N[g] : 0;
    uint64_t total;
    (void)block_exclusive(v, sh, total);
    if (threadIdx.x == 0) ws.bsum[blockIdx.x] = total;
}

// One block: exclusive prefix of the nb block sums in place; bsum[nb] = total.
__global__ __launch_bounds__(kScanBlock) void prefix_kernel(const WalkState ws, uint64_t nb,
                                                            const unsigned long long *egate, uint32_t egn) {
    if (emit_skips(egate, egn)) return;
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

// A wave per segment: its chunk index from the block sums (bsum, exclusive
// after prefix_kernel) plus the N of the earlier segments of its 256-segment
// block, then lanes over its chunks -- coalesced stores, 4096 waves per GiB
// (a thread per segment writing its ~40 chunks one after another took 18-25
// us per GiB on 64 waves).
// go: the fused end kernel's verdict word (finish_kernel: P[] is complete and
// the output is due); null: the gate rule itself, with the prefix from bsum.
__global__ __launch_bounds__(256) void emit_kernel(const StreamTable st, const WalkParams wp, const WalkState ws,
                                                   cdc_chunk_pod *out, uint64_t out_cap,
                                                   const unsigned long long *egate, uint32_t egn,
                                                   const uint64_t *go) {
    if (go ? *go == 0 : emit_skips(egate, egn)) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + wave_id();
    if (g >= st.total_spans) return;
    uint64_t p;
    if (go) {
        p = ws.P[g];
    } else {
        uint32_t part = 0;
        for (uint64_t j = (g & ~(uint64_t)(kScanBlock - 1)) + lane; j < g; j += 64) part += ws.N[j];
        part = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(part), 63);
        p = ws.bsum[g / kScanBlock] + part;
        if (lane == 0) ws.P[g] = p;
    }
    const uint32_t n = ws.N[g];
    if (n > wp.cap || p + n > out_cap) {
        if (lane == 0) atomicAdd(&ws.flags[1], 1ull);
        return;
    }
    const uint64_t *list = ws.list + g * wp.cap;
    const uint64_t x = ws.X[g];
    for (uint32_t k = lane; k < n; k += 64) {
        const uint64_t c = list[k];
        const uint64_t nx = k + 1 < n ? list[k + 1] : x;
        out[p + k] = cdc_chunk_pod{c, nx - c};
    }
}

__global__ void first_kernel(const StreamTable st, const WalkState ws, uint64_t nb, const unsigned long long *egate,
                             uint32_t egn) {
    if (emit_skips(egate, egn)) return;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > st.n) return;
    const uint64_t g = i < st.n ? st.span_base[i] : st.total_spans;
    ws.first[i] = g < st.total_spans ? ws.P[g] : ws.bsum[nb];
}

// The end of a call whose first group of fix-up rounds is queued (one block,
// replacing sum / prefix / first and two D2H copies): when the gate rule says
// the output is due, the exclusive prefix P[g] of every segment's count and
// first[n+1] -- into the workspace and straight into the host staging block
// -- and the go word for emit_kernel; in every case the flag blocks copied to
// the host block, and, when the output is due (the host then needs no more
// rounds), the flags reset for the next call (launch_flags_init's pattern),
// so that call launches no init kernel.  Segment counts up to kFinishMax.
constexpr uint32_t kFinishThreads = 1024;
constexpr uint64_t kFinishMax = 1u << 16;

__global__ __launch_bounds__(kFinishThreads) void finish_kernel(const StreamTable st, const WalkState ws,
                                                                const unsigned long long *egate, uint32_t egn,
                                                                uint32_t rounds, uint64_t *go, uint64_t *h_first,
                                                                uint64_t *h_flags) {
    __shared__ uint64_t part[kFinishThreads];
    const bool due = !emit_skips(egate, egn);
    const uint32_t t = threadIdx.x;
    const uint64_t S = st.total_spans;
    if (due) {
        // thread t owns segments [t*per, (t+1)*per): local sums, a block scan, then the prefixes
        const uint64_t per = (S + kFinishThreads - 1) / kFinishThreads;
        const uint64_t a = min((uint64_t)t * per, S), b = min(a + per, S);
        uint64_t sum = 0;
        for (uint64_t g = a; g < b; ++g) sum += ws.N[g];
        part[t] = sum;
        __syncthreads();
        for (uint32_t o = 1; o < kFinishThreads; o <<= 1) {
            const uint64_t v = t >= o ? part[t - o] : 0;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        uint64_t run = part[t] - sum;
        for (uint64_t g = a; g < b; ++g) {
            ws.P[g] = run;
            run += ws.N[g];
        }
        __syncthreads();  // (every P[] written before first[] reads them)
        const uint64_t total = part[kFinishThreads - 1];
        for (uint64_t i = t; i <= st.n; i += kFinishThreads) {
            const uint64_t g = i < st.n ? st.span_base[i] : S;
            const uint64_t f = g < S ? ws.P[g] : total;
            ws.first[i] = f;
            h_first[i] = f;
        }
    }
    if (t == 0) *go = due ? 1 : 0;
    const uint32_t words = 4 + 4 * rounds;
    for (uint32_t i = t; i < words; i += kFinishThreads) h_flags[i] = ws.flags[i];
    __threadfence_system();
    __syncthreads();
    if (due)
        for (uint32_t i = t; i < 4 + 4 * kMaxFixRounds; i += kFinishThreads)
            ws.flags[i] = i >= 4 && (i & 3) == 2 ? ~0ull : 0ull;
}

template <int kAlgo, bool kBits>
hipError_t walk_dispatch(int which, const StreamTable &st, const WalkParams &wp, const WalkState &ws,
                         hipStream_t s) {
    const unsigned blocks = (unsigned)((st.total_spans + kWalkBlock - 1) / kWalkBlock);
    if (which == 0) walk_kernel<kAlgo, kBits><<<blocks, kWalkBlock, 0, s>>>(st, wp, ws);
    else if (which == 1) fix_kernel<kAlgo, kBits><<<blocks, kWalkBlock, 0, s>>>(st, wp, ws);
    else serial_kernel<kAlgo, kBits><<<(st.n + kWalkBlock - 1) / kWalkBlock, kWalkBlock, 0, s>>>(st, wp, ws);
    return hipGetLastError();
}

hipError_t dispatch(int which, const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const bool bits = wp.nbm != 0;
    switch (wp.algo) {
        case 2: return bits ? walk_dispatch<2, true>(which, st, wp, ws, s) : walk_dispatch<2, false>(which, st, wp, ws, s);
        case 4: return bits ? walk_dispatch<4, true>(which, st, wp, ws, s) : walk_dispatch<4, false>(which, st, wp, ws, s);
        case 5: return bits ? walk_dispatch<5, true>(which, st, wp, ws, s) : walk_dispatch<5, false>(which, st, wp, ws, s);
        case 6: return bits ? walk_dispatch<6, true>(which, st, wp, ws, s) : walk_dispatch<6, false>(which, st, wp, ws, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool bits_write_summary(const WalkParams &wp) {
    if (!wp.wave || !wp.nbm || wp.piece_log2 < 12 || wp.piece_log2 > 15) return false;
    switch (wp.algo) {
        case 2: return wp.rabin_mask <= 0xFFFFFFFFull && wp.rabin_shift >= 32;  // rbits_kernel
        case 4: case 5: return wp.bits_fine != 0;                               // ubits / lbits_kernel
        case 6: return wp.bits_fine != 0;                                       // bits_kernel<6>, fine
        default: return false;
    }
}

// Per segment: which quiet kinds hold at every position (qseg, see WalkParams).
template <int kAlgo>
__global__ __launch_bounds__(256) void qseg_kernel(const StreamTable st, const WalkParams wp) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + wave_id();
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    uint32_t m = 0;
    if (g + 1 < st.span_base[si + 1]) {  // (a stream's last segment: 0)
        const uint64_t sw = wp.seg_words >> 6;  // summary words per segment and kind
#pragma unroll
        for (int kind = 0; kind < kQuietKinds<kAlgo>; ++kind) {
            bool all = true;
            for (uint64_t i = lane; i < sw; i += 64) all = all && wp.rsum[(g * sw + i) * kQuietKinds<kAlgo> + kind] == ~0ull;
            if (__ballot(!all) == 0) m |= 1u << kind;
        }
    }
    if (lane == 0) wp.qseg[g] = (uint8_t)m;
}

hipError_t launch_bits(const StreamTable &st, const WalkParams &wp, hipStream_t s) {
    if (!st.total_spans || !wp.nbm) return hipSuccess;
    const uint64_t pieces = st.total_spans << (st.span_log2 - wp.piece_log2);
    const unsigned blocks = (unsigned)pieces;
    if (wp.algo == 2 && wp.rabin_mask <= 0xFFFFFFFFull && wp.rabin_shift >= 32 && wp.piece_log2 >= 12)
        rbits_kernel<<<(unsigned)(((pieces >> rabin_group_log2(st, wp)) + kRabinWaves - 1) / kRabinWaves),
                       64 * kRabinWaves, 0, s>>>(st, wp);
    else if (wp.algo == 2) bits_kernel<2><<<blocks, kWalkBlock, 0, s>>>(st, wp);
    else if (wp.algo == 4 && wp.bits_fine && wp.piece_log2 >= 12)
        ubits_kernel<<<(unsigned)((pieces + 3) / 4), 256, 0, s>>>(st, wp);
    else if (wp.algo == 4) bits_kernel<4><<<blocks, kWalkBlock, 0, s>>>(st, wp);
    else if (wp.algo == 5 && wp.bits_fine && wp.piece_log2 >= 12)
        lbits_kernel<<<(unsigned)((pieces + 3) / 4), 256, 0, s>>>(st, wp);
    else if (wp.algo == 5) bits_kernel<5><<<blocks, kWalkBlock, 0, s>>>(st, wp);
    else if (wp.algo == 6) bits_kernel<6><<<blocks, kWalkBlock, 0, s>>>(st, wp);
    else return hipErrorInvalidValue;
    if (wp.algo == 5 && wp.wave && wp.jt && wp.piece_log2 >= 12)  // LeapCDC word tables
        jtab_kernel<<<(unsigned)((pieces + 3) / 4), 256, 0, s>>>(st, wp);
    if (wp.rsum && wp.qseg) {
        const unsigned qb = (unsigned)((st.total_spans + 3) / 4);
        if (wp.algo == 2) qseg_kernel<2><<<qb, 256, 0, s>>>(st, wp);
        else if (wp.algo == 4) qseg_kernel<4><<<qb, 256, 0, s>>>(st, wp);
        else if (wp.algo == 5) qseg_kernel<5><<<qb, 256, 0, s>>>(st, wp);
        else qseg_kernel<6><<<qb, 256, 0, s>>>(st, wp);
    }
    return hipGetLastError();
}

hipError_t launch_links(const StreamTable &st, const WalkParams &wp, hipStream_t s) {
    if (!st.total_spans || !wp.links) return hipSuccess;
    if (wp.algo == 2) return links_dispatch<2>(st, wp, s);
    if (wp.algo == 4) return links_dispatch<4>(st, wp, s);
    if (wp.algo == 5) return links_dispatch<5>(st, wp, s);
    return hipErrorInvalidValue;
}

hipError_t launch_walk(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    if (wp.wave && wp.nbm && st.total_spans) {
        const unsigned blocks = (unsigned)((st.total_spans + 3) / 4);
        if (wp.algo == 2) wwalk_kernel<2><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 5) wwalk_kernel<5><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 6) wwalk_kernel<6><<<blocks, 256, 0, s>>>(st, wp, ws);
        else wwalk_kernel<4><<<blocks, 256, 0, s>>>(st, wp, ws);
        return hipGetLastError();
    }
    return dispatch(0, st, wp, ws, s);
}

// A round's snapshots, both arrays in one launch (skipped with the round).
__global__ __launch_bounds__(256) void snap_kernel(const WalkState ws, uint64_t n) {
    if (round_stops(ws.gate)) return;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        ws.Xs[i] = ws.X[i];
        ws.Es[i] = ws.E[i];
    }
}

__global__ __launch_bounds__(256) void flags_init_kernel(unsigned long long *flags, uint32_t rounds) {
    for (uint32_t i = threadIdx.x; i < 4 + 4 * rounds; i += 256) flags[i] = i >= 4 && (i & 3) == 2 ? ~0ull : 0ull;
}

hipError_t launch_flags_init(unsigned long long *flags, uint32_t rounds, hipStream_t s) {
    flags_init_kernel<<<1, 256, 0, s>>>(flags, rounds);
    return hipGetLastError();
}

hipError_t launch_fix(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s,
                      bool snap) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t sb = (st.total_spans + 255) / 256;
    if (snap) snap_kernel<<<(unsigned)(sb < 1024 ? sb : 1024), 256, 0, s>>>(ws, st.total_spans);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (wp.wave && wp.nbm) {
        const unsigned blocks = (unsigned)((st.total_spans + 3) / 4);
        if (wp.algo == 2) wfix_kernel<2><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 5) wfix_kernel<5><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 6) wfix_kernel<6><<<blocks, 256, 0, s>>>(st, wp, ws);
        else wfix_kernel<4><<<blocks, 256, 0, s>>>(st, wp, ws);
        return hipGetLastError();
    }
    return dispatch(1, st, wp, ws, s);
}

hipError_t launch_serial(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s) {
    if (wp.wave && wp.nbm && st.total_spans) {
        const unsigned blocks = (unsigned)((st.n + 3) / 4);
        if (wp.algo == 2) wserial_kernel<2><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 5) wserial_kernel<5><<<blocks, 256, 0, s>>>(st, wp, ws);
        else if (wp.algo == 6) wserial_kernel<6><<<blocks, 256, 0, s>>>(st, wp, ws);
        else wserial_kernel<4><<<blocks, 256, 0, s>>>(st, wp, ws);
        return hipGetLastError();
    }
    return dispatch(2, st, wp, ws, s);
}

hipError_t launch_emit(const StreamTable &st, const WalkParams &wp, const WalkState &ws, void *d_out,
                       uint64_t out_cap, hipStream_t s, const unsigned long long *egate, uint32_t egn) {
    const uint64_t nb = (st.total_spans + kScanBlock - 1) / kScanBlock;
    if (nb) {
        sum_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(st, ws, egate, egn);
        prefix_kernel<<<1, kScanBlock, 0, s>>>(ws, nb, egate, egn);
        emit_kernel<<<(unsigned)((st.total_spans + 3) / 4), 256, 0, s>>>(
            st, wp, ws, reinterpret_cast<cdc_chunk_pod *>(d_out), out_cap, egate, egn, nullptr);
    }
    first_kernel<<<(unsigned)((st.n + 1 + 255) / 256), 256, 0, s>>>(st, ws, nb, egate, egn);
    return hipGetLastError();
}

bool finish_fits(const StreamTable &st) { return st.total_spans <= kFinishMax; }

hipError_t launch_finish_emit(const StreamTable &st, const WalkParams &wp, const WalkState &ws, void *d_out,
                              uint64_t out_cap, hipStream_t s, const unsigned long long *egate, uint32_t egn,
                              uint32_t rounds, uint64_t *go, uint64_t *h_first, uint64_t *h_flags) {
    finish_kernel<<<1, kFinishThreads, 0, s>>>(st, ws, egate, egn, rounds, go, h_first, h_flags);
    if (st.total_spans)
        emit_kernel<<<(unsigned)((st.total_spans + 3) / 4), 256, 0, s>>>(
            st, wp, ws, reinterpret_cast<cdc_chunk_pod *>(d_out), out_cap, egate, egn, go);
    return hipGetLastError();
}

}  // namespace walk
}  // namespace cdc
