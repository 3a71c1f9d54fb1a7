// Instruction-throughput microbenchmark for the scan kernel's inner loop
// (gfx950).  Each kernel runs CH independent chains of one instruction kind
// per lane for ITERS steps; cycles per wave-instruction per SIMD are derived
// from wall time at full occupancy.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_isa.hip -o _build/ubench_isa
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH 8
#define ITERS 4096

__global__ __launch_bounds__(256) void k_lshl_add_u64(uint64_t *out, uint64_t seed) {
    uint64_t h[CH], g[CH];
    for (int c = 0; c < CH; ++c) { h[c] = seed + threadIdx.x + c; g[c] = seed * (c + 3); }
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(h[c]) : "v"(g[c]));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add_co_pair(uint64_t *out, uint64_t seed) {
    uint32_t lo[CH], hi[CH], gl[CH], gh[CH];
    for (int c = 0; c < CH; ++c) { lo[c] = seed + threadIdx.x + c; hi[c] = c; gl[c] = seed * (c + 3); gh[c] = c * 7; }
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c)
            asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                         : "+v"(lo[c]), "+v"(hi[c]) : "v"(gl[c]), "v"(gh[c]) : "vcc");
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += lo[c] + hi[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_perm(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed;
    const uint32_t sel = 0x0c0c0104u;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(y), "s"(sel));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_alignbit(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_alignbit_b32 %0, %1, %0, 16" : "+v"(x[c]) : "v"(y));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_and32(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_dsread64(uint64_t *out, uint64_t seed) {
    __shared__ uint64_t tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += 256) tab[i] = i * seed;
    __syncthreads();
    const uint32_t rep = (threadIdx.x & 31) * 8;
    uint64_t s = 0;
    uint32_t b = (seed + threadIdx.x) & 255;
    for (int i = 0; i < ITERS; ++i) {
        uint64_t v[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const uint32_t addr = (((b + c * 37) & 255) << 8) | rep;
            v[c] = *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + addr);
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) s ^= v[c];
        b = (b * 5 + 1) & 255;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


__global__ __launch_bounds__(256) void k_mov_sdwa(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed * 0x01020304u;
    for (int c = 0; c < CH; ++c) x[c] = (threadIdx.x & 31) * 8;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c)
            asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(x[c]) : "v"(y));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_min_u32(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_min_u32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_min3_u32(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed, z = seed * 3;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_min3_u32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(y), "v"(z));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_and_e32(uint64_t *out, uint64_t seed) {
    uint32_t x[CH], y = seed;
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_lshl_add_u64_dep(uint64_t *out, uint64_t seed) {
    // ONE dependent chain per lane: latency, not throughput
    uint64_t h = seed + threadIdx.x, g = seed * 3;
    for (int i = 0; i < ITERS * CH; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(h) : "v"(g));
    out[blockIdx.x * blockDim.x + threadIdx.x] = h;
}

__global__ __launch_bounds__(256) void k_lds_chain(uint64_t *out, uint64_t seed) {
    // the scan's inner step: perm address -> ds_read_b64 -> lshl_add, 8 chains
    __shared__ uint64_t tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += 256) tab[i] = i * seed;
    __syncthreads();
    const uint32_t rep = (threadIdx.x & 31) * 8;
    const uint32_t sel = 0x0c0c0104u;
    uint64_t h[CH];
    uint32_t w[CH];
    for (int c = 0; c < CH; ++c) { h[c] = c; w[c] = (seed + threadIdx.x * 77 + c * 131) * 2654435761u; }
    const char *tb = reinterpret_cast<const char *>(tab);
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            uint32_t a;
            asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a) : "v"(rep), "v"(w[c]), "s"(sel));
            const uint64_t g = *reinterpret_cast<const uint64_t *>(tb + a);
            asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(h[c]) : "v"(g));
            w[c] = w[c] * 5 + 1;
        }
    }
    uint64_t s = 0;
    for (int c = 0; c < CH; ++c) s += h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char *name, K kernel, int ops_per_step, uint64_t *d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    kernel<<<blocks, 256>>>(d, 12345);
    hipDeviceSynchronize();
    hipEventRecord(a);
    kernel<<<blocks, 256>>>(d, 12345);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double waves = blocks * 4.0;
    const double wave_instr = waves * ITERS * CH * ops_per_step;
    const double per_simd = wave_instr / (cus * 4.0);
    const double clk_ghz = 2.4;  // nominal; see the note printed below
    printf("%-16s %8.3f ms  %.2f cycles per wave-instr per SIMD @%.1f GHz nominal\n", name, ms,
           ms * 1e-3 * clk_ghz * 1e9 / per_simd, clk_ghz);
}

int main() {
    uint64_t *d;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 32 waves/CU
    hipMalloc(&d, (size_t)blocks * 256 * 8);
    run("lshl_add_u64", k_lshl_add_u64, 1, d, blocks);
    run("add_co+addc", k_add_co_pair, 2, d, blocks);
    run("perm_b32", k_perm, 1, d, blocks);
    run("alignbit_b32", k_alignbit, 1, d, blocks);
    run("xor_b32", k_and32, 1, d, blocks);
    run("ds_read_b64", k_dsread64, 1, d, blocks);
    run("mov_b32_sdwa", k_mov_sdwa, 1, d, blocks);
    run("min_u32_e32", k_min_u32, 1, d, blocks);
    run("min3_u32", k_min3_u32, 1, d, blocks);
    run("and_b32_e32", k_and_e32, 1, d, blocks);
    run("lshl_add dep1", k_lshl_add_u64_dep, 1, d, blocks);
    run("perm+ds+lshl", k_lds_chain, 1, d, blocks);
    printf("note: cycles use a nominal 2.4 GHz clock; compare ratios between rows\n");
    hipFree(d);
    return 0;
}
