// How fast can a kernel read a 1 MiB host buffer (the reference's StorageWriter
// segment) over PCIe, and what do the alternatives cost?  Diagnostics for the
// one-launch small-stream path (small.hip):
//   * kernel reads of pinned host memory, by allocation flags (default /
//     non-coherent / write-combined) and grid size, 16-byte loads, every wave
//     with its whole share in flight;
//   * one hipMemcpyAsync H2D DMA of the same bytes;
//   * CPU stores into device memory, when the allocation is host-visible.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_pcie.hip -o _build/ubench_pcie
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

// Block b reads bytes [b*per, (b+1)*per) with 16-byte loads, kLoads per thread in flight.
template <int kLoads>
__global__ __launch_bounds__(512) void k_read(const uint8_t *src, uint64_t per, uint32_t *out) {
    const uint8_t *p = src + (uint64_t)blockIdx.x * per;
    uint32_t acc = 0;
    for (uint64_t o = (uint64_t)threadIdx.x * 16; o < per; o += 512ull * 16 * kLoads) {
        u32x4 v[kLoads];
#pragma unroll
        for (int k = 0; k < kLoads; ++k)
            v[k] = o + k * 512ull * 16 < per ? *(g_u32x4 *)(p + o + k * 512ull * 16) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < kLoads; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;  // (keeps the loads)
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int run_reads(const char *name, const uint8_t *dsrc, uint64_t n, uint32_t *dout, hipStream_t s) {
    const int grids[] = {16, 32, 64, 128, 256};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int g : grids) {
        const uint64_t per = n / g;
        for (int variant = 0; variant < 2; ++variant) {
            float best = 1e9f, sum = 0;
            const int reps = 30;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(a, s));
                if (variant == 0)
                    k_read<1><<<g, 512, 0, s>>>(dsrc, per, dout);
                else
                    k_read<4><<<g, 512, 0, s>>>(dsrc, per, dout);
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
                sum += ms;
            }
            printf("%-28s n=%8llu grid %4d loads/thread-batch %d: best %7.2f us  avg %7.2f us  (%6.1f GB/s best)\n",
                   name, (unsigned long long)n, g, variant ? 4 : 1, best * 1e3, sum / reps * 1e3,
                   n / (best * 1e-3) / 1e9);
        }
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *dout;
    CK(hipMalloc(&dout, 64));
    for (uint64_t n : {(uint64_t)1 << 20, (uint64_t)4 << 20}) {
        struct Kind {
            const char *name;
            unsigned flags;
        } kinds[] = {{"hostmalloc default", hipHostMallocDefault},
                     {"hostmalloc noncoherent", hipHostMallocNonCoherent},
                     {"hostmalloc coherent", hipHostMallocCoherent},
                     {"hostmalloc writecombined", hipHostMallocWriteCombined}};
        for (auto &k : kinds) {
            uint8_t *h = nullptr, *d = nullptr;
            if (hipHostMalloc(&h, n, k.flags) != hipSuccess) {
                printf("%s: hipHostMalloc failed\n", k.name);
                continue;
            }
            memset(h, 0x5a, n);
            CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0));
            if (run_reads(k.name, d, n, dout, s)) return 1;
            CK(hipHostFree(h));
        }
        // DMA of the same bytes from default pinned memory
        uint8_t *h = nullptr, *dd = nullptr;
        CK(hipHostMalloc(&h, n, hipHostMallocDefault));
        memset(h, 0x33, n);
        CK(hipMalloc(&dd, n));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        float best = 1e9f, sum = 0;
        double wbest = 1e9, wsum = 0;
        for (int r = 0; r < 30; ++r) {
            const double t0 = now_us();
            CK(hipEventRecord(a, s));
            CK(hipMemcpyAsync(dd, h, n, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            const double t1 = now_us();
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
            wbest = t1 - t0 < wbest ? t1 - t0 : wbest;
            wsum += t1 - t0;
        }
        printf("DMA H2D n=%8llu: events best %7.2f us avg %7.2f us; wall best %7.2f avg %7.2f us\n",
               (unsigned long long)n, best * 1e3, sum / 30 * 1e3, wbest, wsum / 30);
        // device memory the host may write directly
        struct DKind {
            const char *name;
            unsigned flags;
        } dk[] = {{"device finegrained", hipDeviceMallocFinegrained}, {"device uncached", hipDeviceMallocUncached},
                  {"device default", hipDeviceMallocDefault}};
        std::vector<uint8_t> src(n, 0x44);
        for (auto &k : dk) {
            uint8_t *d = nullptr;
            if (hipExtMallocWithFlags(reinterpret_cast<void **>(&d), n, k.flags) != hipSuccess) {
                printf("%s: hipExtMallocWithFlags failed\n", k.name);
                continue;
            }
            hipPointerAttribute_t at{};
            if (hipPointerGetAttributes(&at, d) != hipSuccess) {
                printf("%s: no attributes\n", k.name);
            } else {
                printf("%s: type %d hostPointer %p devicePointer %p\n", k.name, (int)at.type, at.hostPointer,
                       at.devicePointer);
                if (at.hostPointer) {
                    uint8_t *hp = static_cast<uint8_t *>(at.hostPointer);
                    double wb = 1e9;
                    for (int r = 0; r < 10; ++r) {
                        const double t0 = now_us();
                        memcpy(hp, src.data(), n);
                        const double t1 = now_us();
                        wb = t1 - t0 < wb ? t1 - t0 : wb;
                    }
                    printf("%s: CPU memcpy into device memory best %7.2f us (%6.1f GB/s)\n", k.name, wb,
                           n / (wb * 1e-6) / 1e9);
                    if (run_reads(k.name, d, n, dout, s)) return 1;
                }
            }
            CK(hipFree(d));
        }
        CK(hipHostFree(h));
        CK(hipFree(dd));
    }
    // host memcpy rate into pinned memory (1 thread) for reference
    {
        const uint64_t n = 1 << 20;
        uint8_t *h = nullptr;
        CK(hipHostMalloc(&h, n, hipHostMallocDefault));
        std::vector<uint8_t> src(n, 7);
        double wb = 1e9;
        for (int r = 0; r < 20; ++r) {
            const double t0 = now_us();
            memcpy(h, src.data(), n);
            const double t1 = now_us();
            wb = t1 - t0 < wb ? t1 - t0 : wb;
        }
        printf("CPU memcpy 1 MiB into pinned host memory, 1 thread: best %.2f us\n", wb);
        CK(hipHostFree(h));
    }
    return 0;
}
