// cdc_kernels.hip -- hand-written gfx950 (CDNA4) kernels for FastCDC v2020.
//
// The reference computes cut points one chunk at a time with a byte loop
// (fastcdc 3.1.0 `cut_gear`, called from chunkfs src/chunkers/fast.rs:37;
// restated in SURVEY.md Appendix A.2 and oracle/cdc_oracle.c).  That loop is
// sequential: each cut depends on the previous one through the min-skip and
// the hash reset.  The GPU decomposition:
//
//  1. scan_kernel   (HBM-bound, one pass over the bytes): for EVERY position
//     i compute the windowed gear hash W_i = sum_k GEAR[b_{i-k}] << k (bits
//     0..47 exact -- the masks never test bit 48 or above) and emit i as a
//     candidate when (W_i & (mask_s & mask_l)) == 0.  One wavefront owns one
//     span; each lane owns 16 consecutive bytes per 1 KiB wave-iteration; the
//     hash is carried across lanes by a 3-step DPP wave_shr scan (a lane's
//     bits 0..47 depend on at most the 3 previous lanes) and across
//     iterations by lane 63's end hash.  GEAR lives in LDS as 32 replicas laid
//     out so lane l reads only banks 2(l&31), 2(l&31)+1: every ds_read_b64 is
//     bank-conflict free.
//  2. spec_kernel   (latency-bound, one thread per span): walk the cut chain
//     from the span start, speculatively treating it as a chunk start.  Each
//     cut re-tests only the <=47 positions after start+min where the in-chunk
//     hash still differs from W (A.3), then looks up the sorted candidates.
//  3. fixup_kernel  (Jacobi iterations): span k re-walks from the exit of span
//     k-1 until its chain merges with its previous chain.  A pass in which no
//     exit changes is the exact reference chain ("Resolve").
//  4. compact kernels: prefix sum of chunk counts and Chunk{offset,length}
//     output in stream order.
#include "cdc_kernels.hpp"

namespace cdc {
namespace {

constexpr int kScanThreads = 512;
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kCopies = 32;           // GEAR replicas, one bank pair per lane&31
constexpr uint32_t kIterBytes = 1024; // 64 lanes x 16 B per wave-iteration
constexpr int kPrefetch = 4;          // wave-iterations of loads kept in flight

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
        return __builtin_amdgcn_alignbit((uint32_t)(h >> 32), (uint32_t)h, fp.cm_shift) & fp.cm32;
    } else {
        return ((uint32_t)h & fp.cm_lo) | ((uint32_t)(h >> 32) & fp.cm_hi);
    }
}

// GEAR[b] for byte j (0..15) of the lane's 16 bytes: one v_perm_b32 builds the
// LDS byte address b*256 + (lane&31)*8, one ds_read_b64 fetches the entry.
__device__ __forceinline__ void gather16(const char *tabb, uint32_t lane_off,
                                         const uint4 v, uint64_t (&gj)[16]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t addr = __builtin_amdgcn_perm(
            lane_off, w[j >> 2], 0x0c0c0004u | ((uint32_t)(j & 3) << 8));
        gj[j] = *reinterpret_cast<const uint64_t *>(tabb + addr);
    }
}

template <bool kAlign>
__global__ __launch_bounds__(kScanThreads, 2) void scan_kernel(
    const StreamTable st, const FastParams fp,
    const uint64_t *__restrict__ gear, const Candidates cand) {
    __shared__ uint64_t tab[256 * kCopies];  // 64 KiB: entry e, replica c at e*32+c
    for (int i = threadIdx.x; i < 256 * kCopies; i += kScanThreads)
        tab[i] = gear[i / kCopies];
    __syncthreads();

    const char *tabb = reinterpret_cast<const char *>(tab);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t lane_off = (lane & 31) * 8;
    const uint64_t span = 1ull << st.span_log2;

    for (uint64_t g = (uint64_t)blockIdx.x * kScanWaves + wave; g < st.total_spans;
         g += (uint64_t)gridDim.x * kScanWaves) {
        uint32_t si;
        uint64_t off;
        locate(st, g, si, off);
        const uint8_t *base = st.ptrs[si] + off;
        const uint64_t n_left = st.lens[si] - off;
        const uint32_t span_len = (uint32_t)(n_left < span ? n_left : span);
        uint32_t *cpos = cand.pos + g * cand.cap;
        uint64_t *chash = cand.hash + g * cand.cap;

        // Carry-in: windowed hash of byte off-1 from the 48 bytes before the span
        // (lanes 61..63 hold them; earlier history cannot reach bits 0..47).
        uint64_t carry = 0;
        if (off != 0) {
            uint64_t P = 0;
            if (lane >= 61) {
                const uint4 v = *reinterpret_cast<const uint4 *>(base - 48 + (lane - 61) * 16);
                uint64_t gj[16];
                gather16(tabb, lane_off, v, gj);
#pragma unroll
                for (int j = 0; j < 16; ++j) P = (P << 1) + gj[j];
            }
            uint64_t E = P + (wave_shr1(P, 0) << 16);
            E = P + (wave_shr1(E, 0) << 16);
            E = P + (wave_shr1(E, 0) << 16);
            carry = readlane63(E);
        }

        uint32_t wcount = 0;  // candidates emitted so far in this span (wave-uniform)

        auto process = [&](const uint4 v, uint32_t pos0, uint32_t valid) {
            uint64_t gj[16];
            gather16(tabb, lane_off, v, gj);
            uint64_t P = 0;  // lane-local hash of its 16 bytes from a zero state
#pragma unroll
            for (int j = 0; j < 16; ++j) P = (P << 1) + gj[j];
            // End-of-lane true hash, exact mod 2^48 after 3 steps.
            uint64_t E = P + (wave_shr1(P, carry) << 16);
            E = P + (wave_shr1(E, carry) << 16);
            E = P + (wave_shr1(E, carry) << 16);
            const uint64_t cin = wave_shr1(E, carry);
            carry = readlane63(E);
            uint64_t h = cin;
            uint32_t acc = 0xffffffffu;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                h = (h << 1) + gj[j];
                acc = min(acc, cand_test<kAlign>(h, fp));
            }
            const bool maybe = acc == 0;
            if (__ballot(maybe)) {  // rare: ~1 lane in 256 per iteration at 12-bit masks
                uint32_t hm = 0;
                if (maybe) {
                    uint64_t hh = cin;
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        hh = (hh << 1) + gj[j];
                        if (cand_test<kAlign>(hh, fp) == 0 && (uint32_t)j < valid) hm |= 1u << j;
                    }
                }
                const uint32_t cnt = __popc(hm);
                uint32_t incl = cnt;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t t = __shfl_up(incl, d);
                    if (lane >= (uint32_t)d) incl += t;
                }
                const uint32_t total = __shfl(incl, 63);
                if (hm) {
                    uint32_t slot = wcount + incl - cnt;
                    uint64_t hh = cin;
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        hh = (hh << 1) + gj[j];
                        if ((hm >> j) & 1u) {
                            if (slot < cand.cap) {
                                cpos[slot] = pos0 + j;
                                chash[slot] = hh;
                            }
                            ++slot;
                        }
                    }
                }
                wcount += total;
            }
        };

        const uint32_t nfull = span_len / kIterBytes;
        const uint4 *vb = reinterpret_cast<const uint4 *>(base) + lane;
        uint4 pf[kPrefetch];
#pragma unroll
        for (int d = 0; d < kPrefetch; ++d) {
            const uint32_t it = (uint32_t)d < nfull ? d : (nfull ? nfull - 1 : 0);
            pf[d] = nfull ? vb[it * 64] : make_uint4(0, 0, 0, 0);
        }
        for (uint32_t it = 0; it < nfull; it += kPrefetch) {
#pragma unroll
            for (int d = 0; d < kPrefetch; ++d) {
                if (it + d < nfull) {
                    const uint4 v = pf[d];
                    const uint32_t nx = min(it + d + kPrefetch, nfull - 1);
                    pf[d] = vb[nx * 64];
                    process(v, (it + d) * kIterBytes + lane * 16, 16);
                }
            }
        }
        if (span_len % kIterBytes) {  // ragged end of a stream: guarded loads
            const uint32_t pos0 = nfull * kIterBytes + lane * 16;
            const uint32_t valid = pos0 < span_len ? min(span_len - pos0, 16u) : 0u;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (valid == 16) {
                v = *reinterpret_cast<const uint4 *>(base + pos0);
            } else if (valid) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (uint32_t j = 0; j < valid; ++j) w[j >> 2] |= (uint32_t)base[pos0 + j] << (8 * (j & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            process(v, pos0, valid);
        }
        if (lane == 0) cand.count[g] = wcount;
    }
}

// ---------------------------------------------------------------------------
// Resolve.  `tab` is a single LDS copy of GEAR.

// Exact sequential cut (byte-wise form of cut_gear): only used
// when a candidate list overflowed (pathological, low-entropy data).
__device__ uint64_t slow_cut(const FastParams &fp, const uint64_t *tab,
                             const uint8_t *d, uint64_t n, uint64_t s) {
    uint64_t rem = n - s;
    if (rem <= fp.min) return n;
    uint64_t center = fp.avg;
    if (rem > fp.max) rem = fp.max; else if (rem < center) center = rem;
    const uint64_t a0 = (fp.min / 2) * 2, ce = (center / 2) * 2, re = (rem / 2) * 2;
    uint64_t h = 0;
    for (uint64_t p = a0; p < re; ++p) {
        h = (h << 1) + tab[d[s + p]];
        if (!(h & (p < ce ? fp.mask_s : fp.mask_l))) return s + p;
    }
    return s + rem;
}

// Cut point (end offset) of the chunk that starts at s, from the candidates.
__device__ uint64_t next_cut(const StreamTable &st, const FastParams &fp,
                             const Candidates &cand, const uint64_t *tab,
                             const uint8_t *d, uint64_t n, uint64_t gbase,
                             uint64_t s) {
    uint64_t rem = n - s;
    if (rem <= fp.min) return n;                   // tail chunk
    uint64_t center = fp.avg;
    if (rem > fp.max) rem = fp.max; else if (rem < center) center = rem;
    const uint64_t a0 = (fp.min / 2) * 2, ce = (center / 2) * 2, re = (rem / 2) * 2;
    const uint64_t tl = min(a0 + (uint64_t)fp.trunc, re);
    // Positions where the in-chunk hash (reset at s+a0) still differs from W.
    uint64_t h = 0;
    for (uint64_t p = a0; p < tl; ++p) {
        h = (h << 1) + tab[d[s + p]];
        if (!(h & (p < ce ? fp.mask_s : fp.mask_l))) return s + p;
    }
    if (tl < re) {
        const uint64_t lo = s + tl, hi = s + re;
        for (uint64_t sp = lo >> st.span_log2; (sp << st.span_log2) < hi; ++sp) {
            const uint64_t g = gbase + sp;
            const uint32_t cnt = cand.count[g];
            if (cnt > cand.cap) return slow_cut(fp, tab, d, n, s);
            const uint32_t *P = cand.pos + g * cand.cap;
            const uint64_t *H = cand.hash + g * cand.cap;
            const uint64_t sp0 = sp << st.span_log2;
            uint32_t k = 0;
            if (lo > sp0) {
                const uint32_t target = (uint32_t)(lo - sp0);
                uint32_t l = 0, r = cnt;
                while (l < r) {
                    const uint32_t m = (l + r) >> 1;
                    if (P[m] < target) l = m + 1; else r = m;
                }
                k = l;
            }
            for (; k < cnt; ++k) {
                const uint64_t c = sp0 + P[k];
                if (c >= hi) return s + rem;
                if (!(H[k] & ((c - s) < ce ? fp.mask_s : fp.mask_l))) return c;
            }
        }
    }
    return s + rem;                                // max (or end of data)
}

__device__ __forceinline__ void load_tab1(uint64_t *tab, const uint64_t *gear) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = gear[i];
    __syncthreads();
}

__global__ __launch_bounds__(256) void spec_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const Chains ch) {
    __shared__ uint64_t tab[256];
    load_tab1(tab, gear);
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint8_t *d = st.ptrs[si];
    const uint64_t n = st.lens[si], gbase = st.span_base[si];
    const uint64_t seg_end = min(off + (1ull << st.span_log2), n);
    uint64_t *list = ch.starts[0] + g * ch.smax;
    uint32_t cnt = 0;
    uint64_t s = off;
    while (s < seg_end) {
        list[cnt++] = s;
        s = next_cut(st, fp, cand, tab, d, n, gbase, s);
    }
    ch.nstarts[0][g] = cnt;
    ch.which[g] = 0;
    ch.entry[g] = off;
    ch.exit[0][g] = s;
}

// One Jacobi pass: reads exits from buffer `b`, writes buffer 1-b.
__global__ __launch_bounds__(256) void fixup_kernel(
    const StreamTable st, const FastParams fp, const uint64_t *__restrict__ gear,
    const Candidates cand, const Chains ch, int b) {
    __shared__ uint64_t tab[256];
    load_tab1(tab, gear);
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= st.total_spans) return;
    uint32_t si;
    uint64_t off;
    locate(st, g, si, off);
    const uint64_t ein = ch.exit[b][g];
    if (off == 0) {  // first span of a stream: its entry (0) is exact
        ch.exit[1 - b][g] = ein;
        return;
    }
    const uint64_t e = ch.exit[b][g - 1];
    if (e == ch.entry[g]) {
        ch.exit[1 - b][g] = ein;
        return;
    }
    const uint8_t *d = st.ptrs[si];
    const uint64_t n = st.lens[si], gbase = st.span_base[si];
    const uint64_t seg_end = min(off + (1ull << st.span_log2), n);
    const int w = ch.which[g];
    const uint64_t *old = ch.starts[w] + g * ch.smax;
    const uint32_t ocnt = ch.nstarts[w][g];
    uint64_t *nl = ch.starts[1 - w] + g * ch.smax;
    uint32_t cnt = 0, j = 0;
    uint64_t s = e, ex;
    for (;;) {
        if (s >= seg_end) { ex = s; break; }
        while (j < ocnt && old[j] < s) ++j;
        if (j < ocnt && old[j] == s) {  // merged with the previous chain
            for (; j < ocnt; ++j) nl[cnt++] = old[j];
            ex = ein;
            break;
        }
        nl[cnt++] = s;
        s = next_cut(st, fp, cand, tab, d, n, gbase, s);
    }
    ch.nstarts[1 - w][g] = cnt;
    ch.which[g] = (uint8_t)(1 - w);
    ch.entry[g] = e;
    ch.exit[1 - b][g] = ex;
    if (ex != ein) atomicOr(ch.changed, 1u);
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
    block_excl_scan(c, sm, tot);
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

__global__ __launch_bounds__(kScanBlock) void write_kernel(
    const StreamTable st, const Chains ch, int eb, const Compact cp,
    cdc_chunk_pod *out, uint64_t nb) {
    __shared__ uint64_t sm[17];
    const uint64_t g = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
    uint32_t c = 0;
    int w = 0;
    if (g < st.total_spans) {
        w = ch.which[g];
        c = ch.nstarts[w][g];
    }
    uint64_t tot;
    const uint64_t idx = cp.block_sums[blockIdx.x] + block_excl_scan(c, sm, tot);
    if (g < st.total_spans) {
        cp.chunk_index[g] = idx;
        const uint64_t *list = ch.starts[w] + g * ch.smax;
        const uint64_t ex = ch.exit[eb][g];
        for (uint32_t k = 0; k < c; ++k) {
            const uint64_t s = list[k];
            const uint64_t nx = k + 1 < c ? list[k + 1] : ex;
            out[idx + k] = cdc_chunk_pod{s, nx - s};
        }
    }
    if (g == 0) cp.chunk_index[st.total_spans] = cp.block_sums[nb];
}

__global__ void first_kernel(const StreamTable st, const Compact cp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= st.n) cp.first[i] = cp.chunk_index[st.span_base[i]];
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
                       int num_cus, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const uint64_t groups = (st.total_spans + kScanWaves - 1) / kScanWaves;
    const uint64_t cap = (uint64_t)num_cus * 2;
    const unsigned grid = (unsigned)(groups < cap ? groups : cap);
    if (fp.cm_align)
        scan_kernel<true><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand);
    else
        scan_kernel<false><<<grid, kScanThreads, 0, s>>>(st, fp, d_gear, cand);
    return hipGetLastError();
}

hipError_t launch_spec(const StreamTable &st, const FastParams &fp,
                       const uint64_t *d_gear, const Candidates &cand,
                       const Chains &ch, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + 255) / 256);
    spec_kernel<<<grid, 256, 0, s>>>(st, fp, d_gear, cand, ch);
    return hipGetLastError();
}

hipError_t launch_fixup(const StreamTable &st, const FastParams &fp,
                        const uint64_t *d_gear, const Candidates &cand,
                        const Chains &ch, int in_buf, hipStream_t s) {
    if (!st.total_spans) return hipSuccess;
    const unsigned grid = (unsigned)((st.total_spans + 255) / 256);
    fixup_kernel<<<grid, 256, 0, s>>>(st, fp, d_gear, cand, ch, in_buf);
    return hipGetLastError();
}

hipError_t launch_compact(const StreamTable &st, const Chains &ch, int exit_buf,
                          const Candidates &cand, const Compact &cp,
                          void *d_out, hipStream_t s) {
    const uint64_t nb = (st.total_spans + kScanBlock - 1) / kScanBlock;
    if (nb) {
        count_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(st, ch, cand, cp);
        block_sums_kernel<<<1, kScanBlock, 0, s>>>(cp.block_sums, nb);
        write_kernel<<<(unsigned)nb, kScanBlock, 0, s>>>(
            st, ch, exit_buf, cp, reinterpret_cast<cdc_chunk_pod *>(d_out), nb);
    }
    first_kernel<<<(st.n + 1 + 255) / 256, 256, 0, s>>>(st, cp);
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
