// index_host.cpp -- C ABI of the device dedup index (include/chunkfs_amd.h,
// "Dedup index"): the reference's chunk Database + storage statistics
// (src/system/database.rs:74-87, src/system/storage.rs:193-240).
#include <cstring>
#include <string>

#include "../../include/chunkfs_amd.h"
#include "engine.hpp"
#include "index.hpp"

struct cdc_index {
    int device = 0;
    cdc::IndexTable t{};
    uint64_t capacity = 0;        // unique digests accepted
    uint64_t *d_acc = nullptr;    // [5] per-call accumulators
    uint32_t *d_slot = nullptr;   // [slot_cap] per-chunk scratch
    uint64_t slot_cap = 0;
    uint32_t *d_pending = nullptr;
    hipStream_t stream = nullptr;
    cdc_index_stats_t st{};
};

namespace {

#define IX_TRY(expr)                                                         \
    do {                                                                     \
        hipError_t e_ = (expr);                                              \
        if (e_ != hipSuccess) {                                              \
            cdc::set_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
            return CDC_EDEVICE;                                              \
        }                                                                    \
    } while (0)

int reset(cdc_index *ix) {
    IX_TRY(hipSetDevice(ix->device));
    IX_TRY(hipMemsetAsync(ix->t.tag, 0, ix->t.slots * 8, ix->stream));
    IX_TRY(hipMemsetAsync(ix->t.owner, 0xFF, ix->t.slots * 8, ix->stream));
    IX_TRY(hipStreamSynchronize(ix->stream));
    ix->st = cdc_index_stats_t{};
    return CDC_OK;
}

void release(cdc_index *ix) {
    (void)hipSetDevice(ix->device);
    (void)hipFree(ix->t.tag);
    (void)hipFree(ix->t.digest);
    (void)hipFree(ix->t.owner);
    (void)hipFree(ix->t.length);
    (void)hipFree(ix->d_acc);
    (void)hipFree(ix->d_slot);
    (void)hipFree(ix->d_pending);
    if (ix->stream) (void)hipStreamDestroy(ix->stream);
    delete ix;
}

int create(int device, size_t capacity, cdc_index **out) {
    cdc_index *ix = new cdc_index();
    ix->device = device;
    ix->capacity = capacity ? capacity : 1;
    uint64_t slots = 1024;
    while (slots < 2 * ix->capacity) slots <<= 1;
    ix->t.slots = slots;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
        delete ix;
        cdc::set_error("no usable GPU for the dedup index");
        return CDC_EDEVICE;
    }
    auto fail = [&](hipError_t e) {
        cdc::set_error(std::string("dedup index allocation: ") + hipGetErrorString(e));
        release(ix);
        return e == hipErrorOutOfMemory ? CDC_ENOMEM : CDC_EDEVICE;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail(e);
    if ((e = hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->t.tag, slots * 8)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->t.digest, slots * 32)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->t.owner, slots * 8)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->t.length, slots * 8)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->d_acc, 5 * 8)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&ix->d_pending, cdc::kIndexPendingCap * 4)) != hipSuccess) return fail(e);
    const int rc = reset(ix);
    if (rc) {
        release(ix);
        return rc;
    }
    *out = ix;
    return CDC_OK;
}

}  // namespace

extern "C" {

int cdc_index_create(int device, size_t capacity, cdc_index_t **out) {
    if (!out) {
        cdc::set_error("cdc_index_create: out is NULL");
        return CDC_EINVAL;
    }
    *out = nullptr;
    return create(device, capacity, out);
}

void cdc_index_destroy(cdc_index_t *ix) {
    if (ix) release(ix);
}

int cdc_index_clear(cdc_index_t *ix) {
    if (!ix) {
        cdc::set_error("NULL index");
        return CDC_EINVAL;
    }
    return reset(ix);
}

int64_t cdc_index_insert_device(cdc_index_t *ix, const uint8_t *d_digests, const cdc_chunk_t *d_chunks,
                                size_t n, uint8_t *d_new, void *hip_stream) {
    if (!ix) {
        cdc::set_error("NULL index");
        return CDC_EINVAL;
    }
    if (n && (!d_digests || !d_chunks)) {
        cdc::set_error("cdc_index_insert_device: NULL argument");
        return CDC_EINVAL;
    }
    if (n == 0) return 0;
    if (ix->st.unique_chunks + n > ix->capacity) {
        // Every chunk of the batch might be new: refuse before the table can
        // pass its load limit (the reference HashMap would grow; size it).
        cdc::set_error("dedup index capacity too small for this batch");
        return CDC_ENOMEM;
    }
    IX_TRY(hipSetDevice(ix->device));
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : ix->stream;
    if (ix->slot_cap < n) {
        (void)hipFree(ix->d_slot);
        ix->d_slot = nullptr;
        ix->slot_cap = 0;
        IX_TRY(hipMalloc(&ix->d_slot, (n + n / 8 + 64) * 4));
        ix->slot_cap = n + n / 8 + 64;
    }
    IX_TRY(hipMemsetAsync(ix->d_acc, 0, 5 * 8, s));
    IX_TRY(cdc::launch_index_insert(ix->t, d_digests, d_chunks, n, ix->st.chunks_written, ix->d_slot,
                                    ix->d_pending, d_new, reinterpret_cast<unsigned long long *>(ix->d_acc), s));
    uint64_t acc[5];
    IX_TRY(hipMemcpyAsync(acc, ix->d_acc, sizeof acc, hipMemcpyDeviceToHost, s));
    IX_TRY(hipStreamSynchronize(s));
    if (acc[3] || acc[4] > cdc::kIndexPendingCap) {
        cdc::set_error("dedup index: table full or too many 64-bit key collisions");
        return CDC_ENOMEM;
    }
    ix->st.chunks_written += n;
    ix->st.bytes_written += acc[2];
    ix->st.unique_chunks += acc[0];
    ix->st.unique_bytes += acc[1];
    return (int64_t)acc[0];
}

int cdc_index_stats(const cdc_index_t *ix, cdc_index_stats_t *out) {
    if (!ix || !out) {
        cdc::set_error("NULL argument");
        return CDC_EINVAL;
    }
    *out = ix->st;
    return CDC_OK;
}

}  // extern "C"
