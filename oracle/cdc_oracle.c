/*
 * cdc_oracle.c -- CPU ORACLE for the chunkfs chunking hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (chunkfs_amd/, include/)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and
 * bench.py's `cpu_baseline` leg may use it, and only as the checker / the
 * reported CPU baseline -- never as the thing measured or shipped.
 *
 * It is a scalar C restatement of the algorithms behind chunkfs's
 * `Chunker::chunk_data` (src/lib.rs:80):
 *
 *   - FastChunker (src/chunkers/fast.rs:29-45) -> fastcdc 3.1.0
 *     `v2020::FastCDC::new(data, min, avg, max)` (Cargo.lock:473-476), i.e.
 *     Normalization::Level1 and the crate's default (unseeded) GEAR table.  The
 *     crate is NOT present in this environment; the algorithm below follows
 *     SURVEY.md Appendix A.1-A.2 (the published fastcdc-rs v2020 `cut_gear`).
 *   - FSChunker (src/chunkers/fixed_size.rs:32-47) -- exact, in-tree.
 *   - Rabin / UltraCDC / LeapCDC / SeqCDC (src/chunkers/{rabin,ultra,leap,seq}.rs)
 *     from the published algorithm descriptions (end of file; parity unpinned).
 *   - StorageWriter 1 MiB segmentation with carry-over of the last chunk
 *     (src/system/storage.rs:78-103, 302-383).
 *
 * PARITY STATUS
 *   FastCDC : "parity unpinned" vs the Rust crate.  The GEAR table in
 *             include/chunkfs_amd_tables.h is a placeholder (see that header);
 *             the reference ships no golden vector for any CDC algorithm
 *             (SURVEY.md §4, §8c).  This oracle is self-consistent only.
 *   FSChunker / segmentation : pinned by the reference's own known answers
 *             (tests/filesystem.rs:135-166, storage.rs:471-485), checked in
 *             tests/test_oracle.py.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <time.h>

#include "../include/chunkfs_amd_tables.h"

int oracle_cdc_check(int algo, uint32_t min, uint32_t avg, uint32_t max);
int64_t oracle_cdc_chunk(int algo, const uint8_t *data, uint64_t len, uint32_t min, uint32_t avg,
                         uint32_t max, const uint32_t *seqcfg, uint64_t *offsets, uint64_t *lengths,
                         uint64_t cap);

/* fastcdc 3.1.0 v2020 size limits (assert!s in FastCDC::with_level_and_seed;
 * SURVEY.md A.1, VERIFY).  The crate panics; the oracle returns -1. */
#define ORC_MINIMUM_MIN 64u
#define ORC_MINIMUM_MAX 1048576u
#define ORC_AVERAGE_MIN 256u
#define ORC_AVERAGE_MAX 4194304u
#define ORC_MAXIMUM_MIN 1024u
#define ORC_MAXIMUM_MAX 16777216u

/* Level1 normalization: bits = round(log2(avg)); mask_s = MASKS[bits+1],
 * mask_l = MASKS[bits-1]  (SURVEY.md A.1). */
int oracle_fastcdc_masks(uint32_t min, uint32_t avg, uint32_t max,
                         uint64_t *mask_s, uint64_t *mask_l)
{
    if (min < ORC_MINIMUM_MIN || min > ORC_MINIMUM_MAX) return -1;
    if (avg < ORC_AVERAGE_MIN || avg > ORC_AVERAGE_MAX) return -1;
    if (max < ORC_MAXIMUM_MIN || max > ORC_MAXIMUM_MAX) return -1;
    unsigned bits = (unsigned)lround(log2((double)avg));
    *mask_s = CHUNKFS_AMD_MASKS[bits + 1];
    *mask_l = CHUNKFS_AMD_MASKS[bits - 1];
    return 0;
}

/* cut_gear: returns the length of the chunk that starts at
 * src[0], given n bytes available.  Two-bytes-per-iteration form with the
 * pre-shifted GEAR_LS table and mask<<1 on the even byte, exactly as the
 * crate does (odd final byte never examined; centre rounded down to even). */
static uint64_t cut_gear(const uint8_t *src, uint64_t n, uint32_t min,
                         uint32_t avg, uint32_t max, uint64_t mask_s,
                         uint64_t mask_l, const uint64_t *gear,
                         const uint64_t *gear_ls)
{
    uint64_t remaining = n;
    if (remaining <= min) return remaining;
    uint64_t center = avg;
    if (remaining > max) remaining = max;
    else if (remaining < center) center = remaining;
    const uint64_t mask_s_ls = mask_s << 1, mask_l_ls = mask_l << 1;
    uint64_t index = min / 2;
    uint64_t hash = 0;
    while (index < center / 2) {
        uint64_t a = index * 2;
        hash = (hash << 2) + gear_ls[src[a]];
        if ((hash & mask_s_ls) == 0) return a;
        hash = hash + gear[src[a + 1]];
        if ((hash & mask_s) == 0) return a + 1;
        index++;
    }
    while (index < remaining / 2) {
        uint64_t a = index * 2;
        hash = (hash << 2) + gear_ls[src[a]];
        if ((hash & mask_l_ls) == 0) return a;
        hash = hash + gear[src[a + 1]];
        if ((hash & mask_l) == 0) return a + 1;
        index++;
    }
    return remaining;
}

/* FastCDC v2020 iterator (offset = processed; length = cut; stop when
 * remaining == 0), mapped to chunkfs Chunk{offset,length} (fast.rs:40-42).
 * gear == NULL selects include/chunkfs_amd_tables.h's table.
 * Returns the chunk count (which may exceed cap: only cap are written),
 * or -1 on invalid sizes. */
int64_t oracle_fastcdc_chunk(const uint8_t *data, uint64_t len, uint32_t min,
                             uint32_t avg, uint32_t max, const uint64_t *gear,
                             uint64_t *offsets, uint64_t *lengths, uint64_t cap)
{
    uint64_t ms, ml;
    if (oracle_fastcdc_masks(min, avg, max, &ms, &ml)) return -1;
    if (!gear) gear = CHUNKFS_AMD_GEAR;
    uint64_t gear_ls[256];
    for (int i = 0; i < 256; i++) gear_ls[i] = gear[i] << 1;
    uint64_t processed = 0, count = 0;
    while (processed < len) {
        uint64_t cut = cut_gear(data + processed, len - processed, min, avg,
                                max, ms, ml, gear, gear_ls);
        if (cut == 0) break;
        if (count < cap) {
            if (offsets) offsets[count] = processed;
            if (lengths) lengths[count] = cut;
        }
        count++;
        processed += cut;
    }
    return (int64_t)count;
}

/* FSChunker::chunk_data (fixed_size.rs:32-43). */
int64_t oracle_fixed_chunk(uint64_t len, uint64_t chunk_size,
                           uint64_t *offsets, uint64_t *lengths, uint64_t cap)
{
    if (chunk_size == 0) return -1;
    uint64_t count = 0;
    for (uint64_t off = 0; off < len; off += chunk_size) {
        if (count < cap) {
            if (offsets) offsets[count] = off;
            if (lengths) lengths[count] = (len - off < chunk_size) ? len - off : chunk_size;
        }
        count++;
    }
    return (int64_t)count;
}

/* Estimate functions: FastChunker len/min (fast.rs:47-49); FSChunker
 * len/cs + 1 (fixed_size.rs:45-47). */
uint64_t oracle_estimate_fast(uint64_t len, uint32_t min) { return len / min; }
uint64_t oracle_estimate_fixed(uint64_t len, uint64_t cs) { return len / cs + 1; }

/* ChunkStorage::write + StorageWriter::{write,flush} (storage.rs:78-103,
 * 302-383) for one write call: the data is cut into seg_size slices; each
 * slice is appended to the carried-over `rest`, chunked, the last chunk is
 * carried again, the others become spans; flush emits the rest as one span.
 * algo 0 = FastCDC(min,avg,max), 1 = fixed(min), 2/4/5/6 = Rabin / Ultra /
 * Leap / Seq (default seq::Config).  Writes span lengths (up to
 * cap), returns the span count or -1.  *chunk_seconds accumulates the time
 * spent inside the chunk_data calls only (storage.rs:314-316). */
int64_t oracle_fs_write(int algo, const uint8_t *data, uint64_t len,
                        uint32_t min, uint32_t avg, uint32_t max,
                        const uint64_t *gear, uint64_t seg_size,
                        uint64_t *span_lengths, uint64_t cap,
                        double *chunk_seconds)
{
    if (seg_size == 0) return -1;
    if (algo == 0) {
        uint64_t ms, ml;
        if (oracle_fastcdc_masks(min, avg, max, &ms, &ml)) return -1;
    } else if (algo != 1 && oracle_cdc_check(algo, min, avg, max)) {
        return -1;
    }
    /* buffer = rest ++ slice; rest <= max (FastCDC) or <= min (fixed) */
    uint64_t buf_cap = seg_size + (uint64_t)(max > min ? max : min) + 1;
    uint8_t *buf = (uint8_t *)malloc(buf_cap);
    uint64_t tmp_sz = buf_cap / (min >= 2 ? 2 * (min / 2) : 1) + 2;
    uint64_t *tmp_len = (uint64_t *)malloc(tmp_sz * sizeof(uint64_t));
    if (!buf || !tmp_len) { free(buf); free(tmp_len); return -1; }
    uint64_t rest = 0, nspans = 0;
    for (uint64_t cur = 0; cur < len;) {
        uint64_t take = len - cur < seg_size ? len - cur : seg_size;
        memcpy(buf + rest, data + cur, take);
        uint64_t blen = rest + take;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        int64_t n = algo == 0 ? oracle_fastcdc_chunk(buf, blen, min, avg, max, gear, NULL, tmp_len, tmp_sz)
                  : algo == 1 ? oracle_fixed_chunk(blen, min, NULL, tmp_len, tmp_sz)
                              : oracle_cdc_chunk(algo, buf, blen, min, avg, max, NULL, NULL, tmp_len, tmp_sz);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (chunk_seconds)
            *chunk_seconds += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        if (n < 0) { free(buf); free(tmp_len); return -1; }
        cur += take;
        /* storage.rs:318-320: no chunks -> early return, rest unchanged (the
         * slice is dropped; unreachable for non-empty buffers) */
        if (n == 0) continue;
        uint64_t consumed = 0;
        for (int64_t i = 0; i < n - 1; i++) {
            if (nspans < cap && span_lengths) span_lengths[nspans] = tmp_len[i];
            nspans++;
            consumed += tmp_len[i];
        }
        rest = tmp_len[n - 1];
        memmove(buf, buf + consumed, rest);
    }
    if (rest > 0) {
        if (nspans < cap && span_lengths) span_lengths[nspans] = rest;
        nspans++;
    }
    free(buf);
    free(tmp_len);
    return (int64_t)nspans;
}

/* Synthetic input used by every config: little-endian u64
 * words, word i = mix64(seed + (i+1) * golden) (counter-based splitmix64). */
static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_fill_splitmix64(uint8_t *buf, uint64_t len, uint64_t seed)
{
    uint64_t nw = len / 8;
    for (uint64_t i = 0; i < nw; i++) {
        uint64_t w = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(buf + 8 * i, &w, 8);
    }
    if (len % 8) {
        uint64_t w = mix64(seed + (nw + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(buf + 8 * nw, &w, len % 8);
    }
}

/* CPU-baseline helper: wall seconds of one whole-buffer FastCDC pass
 * (reference "raw chunk_data" mode, single thread). */
double oracle_time_fastcdc(const uint8_t *data, uint64_t len, uint32_t min,
                           uint32_t avg, uint32_t max, int64_t *count_out)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int64_t n = oracle_fastcdc_chunk(data, len, min, avg, max, NULL, NULL, NULL, 0);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (count_out) *count_out = n;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ======================================================================
 * Rabin / UltraCDC / LeapCDC / SeqCDC (reference src/chunkers/rabin.rs:34-56,
 * ultra.rs:30-44, leap.rs:30-44, seq.rs:40-55).  PARITY UNPINNED: the
 * reference's arithmetic is in cdc-chunkers 0.1.3 (Cargo.lock:143-151), absent
 * here; these follow the published algorithm descriptions restated in
 * DESIGN.md, with the constants of include/chunkfs_amd_cdc_params.h.  Each
 * cut_* returns the length of the chunk starting at src[0] (n bytes left);
 * all of them look only forward from the chunk start and restart at every
 * boundary, like cut_gear.
 * ====================================================================== */
#include "../include/chunkfs_amd_cdc_params.h"

/* GF(2) polynomial remainder of x modulo p (deg p = 53). */
static uint64_t pol_mod(uint64_t x, uint64_t p)
{
    const int dp = 63 - __builtin_clzll(p);
    while (x && 63 - __builtin_clzll(x) >= dp) x ^= p << ((63 - __builtin_clzll(x)) - dp);
    return x;
}

/* Tables of polynomial P (RabinChunker's ChunkerParams, rabin.rs:38; the
 * built-in CDC_RABIN_POLY unless a caller passes another one). */
static void rabin_tables_p(uint64_t P, uint64_t mod_t[256], uint64_t out_t[256])
{
    const int deg = 63 - __builtin_clzll(P);
    for (uint64_t b = 0; b < 256; b++) {
        mod_t[b] = pol_mod(b << deg, P) | (b << deg);
        uint64_t h = pol_mod(b, P);
        for (uint32_t i = 1; i < CDC_RABIN_WINDOW; i++) h = pol_mod(h << 8, P);
        out_t[b] = h;
    }
}

static void rabin_tables(uint64_t mod_t[256], uint64_t out_t[256]) { rabin_tables_p(CDC_RABIN_POLY, mod_t, out_t); }

/* Degrees a Rabin polynomial may have here: the digest shifted left by 8
 * stays inside 64 bits, and the top byte index (deg - 8) is >= 1. */
int oracle_rabin_poly_ok(uint64_t P) { return P && (63 - __builtin_clzll(P)) >= 9 && (63 - __builtin_clzll(P)) <= 56; }

static uint64_t cut_rabin(const uint8_t *src, uint64_t n, uint32_t min, uint32_t max, uint64_t mask,
                          const uint64_t *mod_t, const uint64_t *out_t, int shift)
{
    if (n <= min) return n;
    const uint64_t end = n < max ? n : max;
    const uint64_t W = CDC_RABIN_WINDOW;
    const uint64_t start = min >= W ? min - W : 0;
    uint64_t d = 0;
    for (uint64_t i = start; i < end; i++) {
        d ^= out_t[i >= start + W ? src[i - W] : 0];
        const uint64_t top = d >> shift;
        d = ((d << 8) | src[i]) ^ mod_t[top];
        if (i + 1 >= min && (d & mask) == 0) return i + 1;
    }
    return end;
}

static inline uint64_t load8(const uint8_t *p)
{
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

static uint64_t cut_ultra(const uint8_t *src, uint64_t n, uint32_t min, uint32_t avg, uint32_t max)
{
    if (n <= min) return n;
    uint64_t normal = avg, end = n;
    if (n >= max) end = max;
    else if (n <= normal) normal = n;
    const uint64_t pat = 0x0101010101010101ULL * CDC_ULTRA_PATTERN;
    uint64_t out = load8(src + min - 8);
    uint32_t dist = (uint32_t)__builtin_popcountll(out ^ pat);
    uint32_t lec = 0;
    for (uint64_t i = min; i + 8 <= end; i += 8) {
        const uint64_t in = load8(src + i);
        if (in == out) {
            if (++lec >= CDC_ULTRA_LEST) return i + 8;
            continue;
        }
        lec = 0;
        const uint32_t mask = i >= normal ? CDC_ULTRA_MASK_L : CDC_ULTRA_MASK_S;
        for (int j = 0; j < 8; j++) {
            if ((dist & mask) == 0) return i + j;
            dist += (uint32_t)__builtin_popcount((unsigned)(src[i + j] ^ CDC_ULTRA_PATTERN));
            dist -= (uint32_t)__builtin_popcount((unsigned)((uint8_t)(out >> (8 * j)) ^ CDC_ULTRA_PATTERN));
        }
        out = in;
    }
    return end;
}

static void leap_table(uint64_t e[256])
{
    for (uint64_t b = 0; b < 256; b++) e[b] = mix64(CDC_LEAP_SEED + (b + 1) * 0x9E3779B97F4A7C15ULL);
}

static inline uint64_t rotl64(uint64_t x, unsigned r) { return r ? (x << r) | (x >> (64 - r)) : x; }

/* Window hash of the CDC_LEAP_WSIZE bytes ending at src[p].  STAND-IN
 * eligibility function (include/chunkfs_amd_cdc_params.h): not the published
 * Leap-based CDC one; only cut_leap's leap structure follows the paper. */
static inline uint64_t leap_hash(const uint8_t *src, uint64_t p, const uint64_t *e)
{
    uint64_t h = 0;
    for (uint32_t j = 0; j < CDC_LEAP_WSIZE; j++) h += rotl64(e[src[p - j]], 11 * j);
    return h;
}

static uint64_t cut_leap(const uint8_t *src, uint64_t n, uint32_t min, uint32_t max, uint32_t thr,
                         const uint64_t *e)
{
    if (n <= min) return n;
    const uint64_t end = n < max ? n : max;
    uint64_t c = min;
    while (c <= end) {
        uint32_t k = 0;
        for (; k < CDC_LEAP_WINDOWS; k++) {
            const uint64_t h = leap_hash(src, c - 1 - k, e);
            const uint32_t v = k < CDC_LEAP_PRIMARY ? (uint32_t)(h >> 32) : (uint32_t)h;
            if (v >= thr) break;
        }
        if (k == CDC_LEAP_WINDOWS) return c;
        c += CDC_LEAP_WINDOWS - k;
    }
    return end;
}

static uint64_t cut_seq(const uint8_t *src, uint64_t n, uint32_t min, uint32_t max, const uint32_t *cfg)
{
    if (n <= min) return n;
    const uint64_t end = n < max ? n : max;
    const int dec = cfg[0] != 0;
    uint32_t cnt = 0, opp = 0;
    for (uint64_t i = min; i < end;) {
        const uint8_t a = src[i - 1], b = src[i];
        if (dec ? b < a : b > a) {
            if (++cnt >= cfg[1]) return i + 1;
        } else {
            cnt = 0;
            if (++opp >= cfg[2]) {
                opp = 0;
                i += cfg[3];
                continue;
            }
        }
        i++;
    }
    return end;
}

uint32_t oracle_leap_threshold(uint32_t min, uint32_t avg)
{
    const uint64_t span = avg > min ? (uint64_t)(avg - min) : 1;
    uint32_t bits = cdc_log2_round(span);
    return CDC_LEAP_THRESHOLD[bits > 32 ? 32 : bits];
}

/* Size rules shared with cdc_create: 0 < min <= avg <= max,
 * Ultra min >= 8, Leap min >= 32, Rabin avg >= 2.  Returns 0 when valid. */
int oracle_cdc_check(int algo, uint32_t min, uint32_t avg, uint32_t max)
{
    if (min == 0 || min > avg || avg > max) return -1;
    if (algo == 4 && min < 8) return -1;
    if (algo == 5 && min < 32) return -1;
    if (algo == 2 && avg < 2) return -1;
    if (algo != 2 && algo != 4 && algo != 5 && algo != 6) return -1;
    return 0;
}

/* chunk_data for algo 2 (Rabin), 4 (Ultra), 5 (Leap), 6 (Seq; seqcfg =
 * {mode (0 increasing, 1 decreasing), seq_length, jump_trigger, jump_size},
 * NULL = defaults).  Same output convention as oracle_fastcdc_chunk. */
int64_t oracle_cdc_chunk_p(int algo, const uint8_t *data, uint64_t len, uint32_t min, uint32_t avg,
                           uint32_t max, const uint32_t *seqcfg, uint64_t rabin_poly, uint64_t *offsets,
                           uint64_t *lengths, uint64_t cap);

int64_t oracle_cdc_chunk(int algo, const uint8_t *data, uint64_t len, uint32_t min, uint32_t avg,
                         uint32_t max, const uint32_t *seqcfg, uint64_t *offsets, uint64_t *lengths,
                         uint64_t cap)
{
    return oracle_cdc_chunk_p(algo, data, len, min, avg, max, seqcfg, 0, offsets, lengths, cap);
}

/* oracle_cdc_chunk with a Rabin polynomial (0 = CDC_RABIN_POLY): the
 * restatement behind cdc_set_rabin_poly. */
int64_t oracle_cdc_chunk_p(int algo, const uint8_t *data, uint64_t len, uint32_t min, uint32_t avg,
                           uint32_t max, const uint32_t *seqcfg, uint64_t rabin_poly, uint64_t *offsets,
                           uint64_t *lengths, uint64_t cap)
{
    if (oracle_cdc_check(algo, min, avg, max)) return -1;
    const uint64_t P = rabin_poly ? rabin_poly : CDC_RABIN_POLY;
    if (!oracle_rabin_poly_ok(P)) return -1;
    static uint64_t mod_t[256], out_t[256], e[256], cur_p = 0;
    static int init = 0;
    if (!init) {
        leap_table(e);
        init = 1;
    }
    if (cur_p != P) {
        rabin_tables_p(P, mod_t, out_t);
        cur_p = P;
    }
    const int rshift = (63 - __builtin_clzll(P)) - 8;
    const uint32_t defcfg[4] = {0, CDC_SEQ_LENGTH, CDC_SEQ_JUMP_TRIGGER, CDC_SEQ_JUMP_SIZE};
    const uint32_t *cfg = seqcfg ? seqcfg : defcfg;
    if (algo == 6 && (cfg[0] > 1 || cfg[1] == 0 || cfg[2] == 0 || cfg[3] == 0)) return -1;
    const uint64_t rmask = (1ull << cdc_log2_round(avg)) - 1;
    const uint32_t thr = oracle_leap_threshold(min, avg);
    uint64_t processed = 0, count = 0;
    while (processed < len) {
        const uint8_t *s = data + processed;
        const uint64_t n = len - processed;
        uint64_t cut = algo == 2 ? cut_rabin(s, n, min, max, rmask, mod_t, out_t, rshift)
                     : algo == 4 ? cut_ultra(s, n, min, avg, max)
                     : algo == 5 ? cut_leap(s, n, min, max, thr, e)
                                 : cut_seq(s, n, min, max, cfg);
        if (count < cap) {
            if (offsets) offsets[count] = processed;
            if (lengths) lengths[count] = cut;
        }
        count++;
        processed += cut;
    }
    return (int64_t)count;
}

/* Tables for the Python twin (oracle.py): Rabin mod/out, Leap hash table. */
void oracle_cdc_tables(uint64_t *mod_t, uint64_t *out_t, uint64_t *leap_e)
{
    rabin_tables(mod_t, out_t);
    leap_table(leap_e);
}

/* CPU-baseline helper for algo 2/4/5/6 (single thread, whole buffer). */
double oracle_time_cdc(int algo, const uint8_t *data, uint64_t len, uint32_t min, uint32_t avg,
                       uint32_t max, int64_t *count_out)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int64_t n = oracle_cdc_chunk(algo, data, len, min, avg, max, NULL, NULL, NULL, 0);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (count_out) *count_out = n;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
