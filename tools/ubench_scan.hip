// Memory-pattern and compute-only microbenchmarks for the gear scan (gfx950).
// Answers "which side bounds the scan": the HBM read pattern or the per-byte
// hash work.  Each kernel covers the same 1 GiB; the time is reported as an
// equivalent input rate in GB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_scan.hip -o chunkfs_amd/_build/ubench_scan
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
__device__ __forceinline__ g_u32x4 *G4(const void *p) { return (g_u32x4 *)(p); }
__device__ __forceinline__ u32x4 ld(const uint8_t *p) { return *G4(p); }

// 1) coalesced: each wave-instruction reads 1 KiB contiguous.  NL loads in flight per lane.
template <int NL>
__global__ __launch_bounds__(256) void rd_coalesced(const uint8_t *d, uint64_t n, uint32_t *out) {
    const uint64_t per = 256ull * 16 * NL;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t b = (uint64_t)blockIdx.x * per; b < n; b += (uint64_t)gridDim.x * per) {
        u32x4 v[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) v[k] = ld(d + b + ((uint64_t)k * 256 + threadIdx.x) * 16);
#pragma unroll
        for (int k = 0; k < NL; ++k) acc ^= v[k];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 2) lane-contiguous: wave per 64 KiB span, lane owns 1 KiB, 128 B line per
// iteration (pipeline 2's scan pattern), two lines in flight.
template <int TPB>
__global__ __launch_bounds__(TPB) void rd_lanecontig(const uint8_t *d, uint64_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int W = TPB / 64;
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t spans = n >> 16;
    for (uint64_t g = (uint64_t)blockIdx.x * W + wave; g < spans; g += (uint64_t)gridDim.x * W) {
        const uint8_t *p = d + (g << 16) + lane * 1024;
        u32x4 A[8], B[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) A[q] = ld(p + q * 16);
#pragma unroll
        for (int q = 0; q < 8; ++q) B[q] = ld(p + 128 + q * 16);
#pragma unroll
        for (int it = 0; it < 8; it += 2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) acc ^= A[q];
            if (it + 2 < 8)
#pragma unroll
                for (int q = 0; q < 8; ++q) A[q] = ld(p + (it + 2) * 128 + q * 16);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc ^= B[q];
            if (it + 3 < 8)
#pragma unroll
                for (int q = 0; q < 8; ++q) B[q] = ld(p + (it + 3) * 128 + q * 16);
        }
    }
    out[blockIdx.x * TPB + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 3) pipeline-1 pattern: 64 B per lane per 4 KiB wave-iteration.
__global__ __launch_bounds__(1024) void rd_lane64(const uint8_t *d, uint64_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t spans = n >> 16;
    for (uint64_t g = (uint64_t)blockIdx.x * 16 + wave; g < spans; g += (uint64_t)gridDim.x * 16) {
        const uint8_t *p = d + (g << 16) + lane * 64;
        u32x4 A[4], B[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) A[q] = ld(p + q * 16);
        for (int it = 0; it < 16; it += 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) B[q] = ld(p + (it + 1) * 4096 + q * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc ^= A[q];
            if (it + 2 < 16)
#pragma unroll
                for (int q = 0; q < 4; ++q) A[q] = ld(p + (it + 2) * 4096 + q * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc ^= B[q];
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 3b) grouped: each wave-instruction reads 1024/C groups of C contiguous bytes;
// group k of instruction i is the next C bytes of lane segment (i*(1024/C)+k)
// (segments 1 KiB apart, as the scan's lane sub-spans).  C = 16 is pipeline
// 2's pattern, C = 1024 a fully contiguous instruction.  With STAGE the 16-B
// pieces go through a padded LDS tile so every lane ends up with its own
// segment's C bytes (the transposition a staged scan needs).
template <int C, bool STAGE>
__global__ __launch_bounds__(512) void rd_group(const uint8_t *d, uint64_t n, uint32_t *out) {
    constexpr int PER = C / 16;         // lanes per group
    constexpr int NI = 64 / (1024 / C) ;  // instructions per wave-step: 64 segments / groups per instr
    constexpr int ROW = C + 16;         // padded LDS row per lane segment
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE ? 8 : 1][STAGE ? 64 * ROW : 16];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t spans = n >> 16;
    const uint32_t seg_in = lane / PER, piece = lane % PER;
    for (uint64_t g = (uint64_t)blockIdx.x * 8 + wave; g < spans; g += (uint64_t)gridDim.x * 8) {
        const uint8_t *p = d + (g << 16);
        for (int it = 0; it < 1024 / C; ++it) {
            u32x4 v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i)
                v[i] = ld(p + (uint64_t)(i * (1024 / C) + seg_in) * 1024 + it * C + piece * 16);
            if constexpr (STAGE) {
#pragma unroll
                for (int i = 0; i < NI; ++i)
                    *reinterpret_cast<u32x4 *>(&stage[wave][(i * (1024 / C) + seg_in) * ROW + piece * 16]) = v[i];
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int i = 0; i < NI; ++i) v[i] = *reinterpret_cast<const u32x4 *>(&stage[wave][lane * ROW + i * 16]);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int i = 0; i < NI; ++i) acc ^= v[i];
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 4) compute only: the scan's per-byte work (perm address, ds_read_b64 of a
// 32-replica GEAR table, v_lshl_add_u64 chain, and+min test) on synthetic
// bytes.  NC independent chains per lane; 1 GiB worth of byte-steps.
__device__ __forceinline__ uint64_t shl1_add(uint64_t h, uint64_t g) {
    uint64_t r;
    asm volatile("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(h), "v"(g));
    return r;
}
template <int NC, int TPB>
__global__ __launch_bounds__(TPB) void cmp_chain(uint64_t steps_per_lane, uint32_t cm, uint32_t *out) {
    __shared__ uint64_t tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += TPB) tab[i] = (uint64_t)(i / 32) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const char *tb = reinterpret_cast<const char *>(tab);
    const uint32_t rep = (threadIdx.x & 31) * 8;
    uint64_t h[NC];
    uint32_t w[NC], acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) { h[c] = c; w[c] = (threadIdx.x * 77 + c * 131 + blockIdx.x) * 2654435761u; acc[c] = ~0u; }
    for (uint64_t s = 0; s < steps_per_lane; s += 8) {
        uint64_t g[NC][8];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const uint32_t w1 = w[c] * 1664525u + 1013904223u;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t a0 = __builtin_amdgcn_perm(rep, w[c], 0x0c0c0004u | ((uint32_t)b << 8));
                const uint32_t a1 = __builtin_amdgcn_perm(rep, w1, 0x0c0c0004u | ((uint32_t)b << 8));
                g[c][b] = *reinterpret_cast<const uint64_t *>(tb + a0);
                g[c][4 + b] = *reinterpret_cast<const uint64_t *>(tb + a1);
            }
            w[c] = w1 * 1664525u + 1013904223u;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                h[c] = shl1_add(h[c], g[c][i]);
                acc[c] = min(acc[c], (uint32_t)(h[c] >> 32) & cm);
            }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) r ^= acc[c] ^ (uint32_t)h[c];
    out[blockIdx.x * TPB + threadIdx.x] = r;
}

static float timeit(void (*launch)(void *), void *arg, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch(arg);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) launch(arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

struct Args {
    const uint8_t *d;
    uint64_t n;
    uint32_t *out;
    int cus;
};
static Args g;

#define LAUNCHER(name, body) static void name(void *) { body; }
LAUNCHER(l_coal4, (rd_coalesced<4><<<g.cus * 8, 256>>>(g.d, g.n, g.out)))
LAUNCHER(l_coal8, (rd_coalesced<8><<<g.cus * 8, 256>>>(g.d, g.n, g.out)))
LAUNCHER(l_coal8x4, (rd_coalesced<8><<<g.cus * 4, 256>>>(g.d, g.n, g.out)))
LAUNCHER(l_coal16, (rd_coalesced<16><<<g.cus * 4, 256>>>(g.d, g.n, g.out)))
LAUNCHER(l_lc1024, (rd_lanecontig<1024><<<g.cus, 1024>>>(g.d, g.n, g.out)))
LAUNCHER(l_lc256, (rd_lanecontig<256><<<g.cus * 4, 256>>>(g.d, g.n, g.out)))
LAUNCHER(l_g16, (rd_group<16, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_g32, (rd_group<32, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_g64, (rd_group<64, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_g128, (rd_group<128, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_g256, (rd_group<256, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_g1024, (rd_group<1024, false><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_s64, (rd_group<64, true><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_s128, (rd_group<128, true><<<g.cus * 2, 512>>>(g.d, g.n, g.out)))
LAUNCHER(l_l64, (rd_lane64<<<g.cus, 1024>>>(g.d, g.n, g.out)))
// compute: total byte-steps = n; lanes = blocks*TPB; steps per lane = n / lanes / NC
LAUNCHER(l_c1_1024, (cmp_chain<1, 1024><<<g.cus, 1024>>>(g.n / (g.cus * 1024ull), 0x00d90103u, g.out)))
LAUNCHER(l_c2_1024, (cmp_chain<2, 1024><<<g.cus, 1024>>>(g.n / (g.cus * 1024ull) / 2, 0x00d90103u, g.out)))
LAUNCHER(l_c2_512, (cmp_chain<2, 512><<<g.cus * 2, 512>>>(g.n / (g.cus * 1024ull) / 2, 0x00d90103u, g.out)))
LAUNCHER(l_c4_512, (cmp_chain<4, 512><<<g.cus * 2, 512>>>(g.n / (g.cus * 1024ull) / 4, 0x00d90103u, g.out)))
LAUNCHER(l_c1_2048, (cmp_chain<1, 1024><<<g.cus * 2, 1024>>>(g.n / (g.cus * 2048ull), 0x00d90103u, g.out)))

int main() {
    g.n = 1ull << 30;
    hipDeviceGetAttribute(&g.cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t *d;
    hipMalloc(&d, g.n);
    hipMemset(d, 0x5a, g.n);
    hipMalloc(&g.out, 64ull << 20);
    g.d = d;
    struct {
        const char *name;
        void (*f)(void *);
    } runs[] = {
        {"read coalesced 4 in flight, 8 blk/CU", l_coal4},
        {"read coalesced 8 in flight, 8 blk/CU", l_coal8},
        {"read coalesced 8 in flight, 4 blk/CU", l_coal8x4},
        {"read coalesced 16 in flight, 4 blk/CU", l_coal16},
        {"read lane-contig 1KiB (p2), 16 waves/blk", l_lc1024},
        {"read lane-contig 1KiB (p2), 4 waves/blk", l_lc256},
        {"read 64B/lane per 4KiB (p1)", l_l64},
        {"group C=16 (64 lines/instr)", l_g16},
        {"group C=32", l_g32},
        {"group C=64", l_g64},
        {"group C=128 (8 full lines/instr)", l_g128},
        {"group C=256", l_g256},
        {"group C=1024 (contiguous)", l_g1024},
        {"group C=64 + LDS transpose", l_s64},
        {"group C=128 + LDS transpose", l_s128},
        {"compute 1 chain, 16 waves/CU", l_c1_1024},
        {"compute 1 chain, 32 waves/CU", l_c1_2048},
        {"compute 2 chains, 16 waves/CU", l_c2_1024},
        {"compute 2 chains, 8 waves/blk x2", l_c2_512},
        {"compute 4 chains, 8 waves/blk x2", l_c4_512},
    };
    for (auto &r : runs) {
        const float ms = timeit(r.f, nullptr, 10);
        const hipError_t e = hipGetLastError();
        printf("%-44s %8.1f us  %7.0f GB/s  %s\n", r.name, ms * 1e3, g.n / (ms * 1e-3) / 1e9,
               e == hipSuccess ? "" : hipGetErrorString(e));
    }
    hipFree(d);
    hipFree(g.out);
    return 0;
}
