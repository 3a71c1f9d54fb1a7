// The scan's hashing inner loop in isolation (gfx950): GEAR lookups from the
// replicated LDS table, the v_lshl_add_u64 chain and the per-quarter candidate
// test, on register-resident bytes (no global loads, no transpose).  Variants
// change the waves per CU, the independent chains per lane and how far the
// lookups run ahead of the chain, to find what the hashing half of
// scan_kernel can reach on its own.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_hash.hip -o _build/ubench_hash
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ uint64_t gear_of(const uint64_t *tab, uint32_t rep, uint32_t w, int b) {
    const uint32_t addr = __builtin_amdgcn_perm(rep, w, 0x0c0c0004u | ((uint32_t)b << 8));
    return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + addr);
}

struct G4 {
    uint64_t v[4];
};

__device__ __forceinline__ void look4(G4 &g, const uint64_t *tab, uint32_t rep, uint32_t w) {
#pragma unroll
    for (int b = 0; b < 4; ++b) g.v[b] = gear_of(tab, rep, w, b);
}

// kTest: 0 = and + min per position (the scan), 1 = no test
template <int kTest>
__device__ __forceinline__ void chain4(uint64_t &h, uint32_t &acc, const G4 &g, uint32_t cm) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h = (h << 1) + g.v[i];
        if (kTest == 0) acc = min(acc, (uint32_t)(h >> 32) & cm);
    }
}

// C chains per lane, 16 dwords (64 bytes) of data per chain per step; lookups
// LOOK dwords ahead of each chain.  Chains are interleaved dword by dword.
template <int W, int C, int LOOK, int kTest>
__global__ __launch_bounds__(W * 64, 1) void k_hash(uint64_t *out, uint32_t seed, int iters, uint32_t cm) {
    __shared__ uint64_t tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += W * 64) tab[i] = (uint64_t)(i / 32) * 0x9E3779B97F4A7C15ull ^ seed;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rep = (lane & 31) * 8;
    uint32_t d[C][16];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int k = 0; k < 16; ++k) d[c][k] = (seed + threadIdx.x * 131 + c * 977 + k * 7919) * 2654435761u;
    uint64_t h[C];
    uint32_t hits = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) h[c] = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(d[c][k]));
        G4 g[C][LOOK + 1];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int a = 0; a < LOOK; ++a) look4(g[c][a], tab, rep, d[c][a]);
        FENCE();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t acc[C];
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = 0xffffffffu;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int k = 4 * q + w;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if (k + LOOK < 16) look4(g[c][(k + LOOK) % (LOOK + 1)], tab, rep, d[c][k + LOOK]);
                }
                FENCE();
#pragma unroll
                for (int c = 0; c < C; ++c) chain4<kTest>(h[c], acc[c], g[c][k % (LOOK + 1)], cm);
                FENCE();
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint64_t m = __ballot(acc[c] == 0);
                if (m) hits += __popcll(m);
            }
        }
    }
    uint64_t s = hits;
#pragma unroll
    for (int c = 0; c < C; ++c) s += h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char *name, K kernel, int W, int C, uint64_t *d, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    kernel<<<blocks, W * 64>>>(d, 12345, iters, 0xd9030353u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(a);
        kernel<<<blocks, W * 64>>>(d, 12345, iters, 0xd9030353u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const double bytes = (double)blocks * W * 64 * iters * 64.0 * C;
    printf("%-28s %8.3f ms  %7.1f us per GiB\n", name, best, best * 1e3 / (bytes / 1073741824.0));
}

#define RUN(W, C, L, T) run(#W " waves x" #C " chains look" #L " test" #T, k_hash<W, C, L, T>, W, C, d, cus, iters)

int main() {
    uint64_t *d;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipMalloc(&d, (size_t)cus * 1024 * 8);
    const int iters = 1024;  // 64 KiB per lane-chain
    RUN(16, 1, 1, 0);
    RUN(16, 1, 2, 0);
    RUN(16, 1, 4, 0);
    RUN(8, 1, 1, 0);
    RUN(8, 1, 2, 0);
    RUN(8, 2, 1, 0);
    RUN(8, 2, 2, 0);
    RUN(12, 1, 1, 0);
    RUN(12, 1, 2, 0);
    RUN(4, 2, 2, 0);
    RUN(4, 4, 1, 0);
    RUN(4, 4, 2, 0);
    RUN(16, 2, 1, 0);
    hipFree(d);
    return 0;
}
