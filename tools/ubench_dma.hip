// LDS-DMA input landing for the scan (gfx950): global_load_lds_dwordx4 puts
// each 64-byte step of 64 lane rows straight into a per-wave LDS ring slot
// (piece-major: slot byte (r/16)*1024 + (k*16 + r%16)*16 holds piece k of
// row r, so the consumer's ds_read_b128 is conflict-free and the source of
// every DMA lane is one 16-byte piece of 16 complete 64-byte pieces per
// instruction); lane r then reads its row with 4 ds_read_b128 and hashes it
// as scan_kernel does.  No VGPR staging, no ds_write transpose.
// Measures loads alone and loads + hashing over a 1 GiB buffer.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_dma.hip -o _build/ubench_dma
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

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
__device__ __forceinline__ void chain4(uint64_t &h, uint32_t &acc, const G4 &g, uint32_t cm) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h = (h << 1) + g.v[i];
        acc = min(acc, (uint32_t)(h >> 32) & cm);
    }
}

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

// W waves per block (one block per CU, persistent), C spans hashed together
// per wave (C chains per lane), NS ring slots of C x 4 KiB per wave; kHash 0 =
// loads only (xor), 1 = the scan's hashing.
template <int W, int C, int NS, int kHash>
__global__ __launch_bounds__(W * 64, 1) void k_dma(const uint8_t *data, uint64_t nspans, uint32_t cm,
                                                    uint64_t *out) {
    __shared__ uint64_t tab[256 * 32];
    __shared__ uint4 ring[W][NS][C][256];
    for (int i = threadIdx.x; i < 256 * 32; i += W * 64) tab[i] = (uint64_t)(i / 32) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t rep = (lane & 31) * 8;
    // span groups of C consecutive spans
    const uint64_t ngroups = nspans / C;
    const uint64_t stride = (uint64_t)gridDim.x * W;
    const uint64_t g0 = (uint64_t)blockIdx.x * W + wave;
    const uint64_t nmine = g0 < ngroups ? (ngroups - g0 + stride - 1) / stride : 0;
    const uint64_t nsteps = nmine * 16;
    // DMA lane l: row 16 i + (l & 15), piece l >> 4
    const uint64_t src_off = (uint64_t)(lane & 15) * 1024 + (lane >> 4) * 16;
    const uint32_t ring_base = (uint32_t)(uintptr_t)&ring[wave][0][0][0];
    auto issue = [&](uint64_t j) {
        if (j >= nsteps) j = nsteps - 1;  // (re-reads the last step: keeps vmcnt static)
        const uint64_t g = (g0 + (j >> 4) * stride) * C;
        const uint32_t slot = ring_base + (uint32_t)(j % NS) * 4096 * C;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint8_t *p = data + ((g + c) << 16) + src_off + (j & 15) * 64;
#pragma unroll
            for (int i = 0; i < 4; ++i) glds16(p + i * 16 * 1024, slot + c * 4096 + i * 1024);
        }
    };
    uint64_t h[C], acc_all = 0;
    uint32_t hits = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) h[c] = 0;
    if (nsteps) {
#pragma unroll
        for (int j = 0; j < NS - 1; ++j) issue(j);
        for (uint64_t j = 0; j < nsteps; ++j) {
            issue(j + NS - 1);
            wait_vm<4 * C * (NS - 1)>();
            uint4 q[C][4];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint4 *rs = &ring[wave][j % NS][c][(lane >> 4) * 64 + (lane & 15)];
#pragma unroll
                for (int k = 0; k < 4; ++k) q[c][k] = rs[k * 16];
            }
            if ((j & 15) == 0)
#pragma unroll
                for (int c = 0; c < C; ++c) h[c] = 0;
            if (kHash == 0) {
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc_all ^= (uint64_t)(q[c][k].x ^ q[c][k].y) << 32 | (q[c][k].z ^ q[c][k].w);
            } else {
                G4 ga[C], gb[C];
#pragma unroll
                for (int c = 0; c < C; ++c) look4(ga[c], tab, rep, q[c][0].x);
                FENCE();
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint32_t acc[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) acc[c] = 0xffffffffu;
#pragma unroll
                    for (int c = 0; c < C; ++c) look4(gb[c], tab, rep, q[c][k].y);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) chain4(h[c], acc[c], ga[c], cm);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) look4(ga[c], tab, rep, q[c][k].z);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) chain4(h[c], acc[c], gb[c], cm);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) look4(gb[c], tab, rep, q[c][k].w);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) chain4(h[c], acc[c], ga[c], cm);
                    FENCE();
                    if (k < 3)
#pragma unroll
                        for (int c = 0; c < C; ++c) look4(ga[c], tab, rep, q[c][k + 1].x);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) chain4(h[c], acc[c], gb[c], cm);
                    FENCE();
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        const uint64_t m = __ballot(acc[c] == 0);
                        if (m) hits += __popcll(m);
                    }
                }
            }
        }
        wait_vm<0>();
    }
    uint64_t s = acc_all + hits;
#pragma unroll
    for (int c = 0; c < C; ++c) s += h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fill(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

template <typename K>
static void run(const char *name, K kernel, int W, const uint8_t *data, uint64_t nspans, uint64_t *d, int cus) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    kernel<<<cus, W * 64>>>(data, nspans, 0xd9030353u, d);
    (void)hipDeviceSynchronize();
    float best = 1e30f, sum = 0;
    const int R = 10;
    for (int r = 0; r < R; ++r) {
        (void)hipEventRecord(a);
        kernel<<<cus, W * 64>>>(data, nspans, 0xd9030353u, d);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
        sum += ms;
    }
    const double bytes = (double)nspans * 65536.0;
    printf("%-36s best %7.1f us  avg %7.1f us  %6.0f GB/s (best)\n", name, best * 1e3, sum / R * 1e3,
           bytes / (best * 1e-3) / 1e9);
}

#define RUN(W, C, NS, H)                                                                          \
    if (!sel || strcmp(sel, #W "," #C "," #NS "," #H) == 0)                                          \
        run(#W " waves x" #C " spans, " #NS " slots, hash " #H, k_dma<W, C, NS, H>, W, data, nspans, d, cus)

int main(int argc, char **argv) {
    const char *sel = argc > 1 ? argv[1] : nullptr;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint64_t bytes = 1ull << 30, nspans = bytes >> 16;
    uint8_t *data;
    uint64_t *d;
    (void)hipMalloc(&data, bytes);
    (void)hipMalloc(&d, (size_t)cus * 1024 * 8);
    fill<<<4096, 256>>>((uint64_t *)data, bytes / 8);
    (void)hipDeviceSynchronize();
    RUN(8, 1, 2, 0);
    RUN(8, 1, 3, 0);
    RUN(6, 1, 4, 0);
    RUN(4, 2, 3, 0);
    RUN(8, 1, 2, 1);
    RUN(8, 1, 3, 1);
    RUN(10, 1, 2, 1);
    RUN(6, 1, 3, 1);
    RUN(6, 1, 4, 1);
    RUN(4, 2, 2, 1);
    RUN(4, 2, 3, 1);
    RUN(6, 2, 2, 1);
    (void)hipFree(data);
    (void)hipFree(d);
    return 0;
}
