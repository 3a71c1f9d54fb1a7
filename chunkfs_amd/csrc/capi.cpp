// capi.cpp -- extern "C" entry points of libchunkfs_amd.so (include/chunkfs_amd.h).
#include <cstring>
#include <string>
#include <vector>

#include "../../include/chunkfs_amd.h"
#include "../../include/chunkfs_amd_debug.h"
#include "engine.hpp"

struct cdc_handle {
    cdc::Engine *engine;
};

namespace {
int64_t bad_handle() {
    cdc::set_error("NULL handle");
    return CDC_EINVAL;
}
}  // namespace

extern "C" {

int cdc_create(cdc_algo_t algo, uint32_t min, uint32_t avg, uint32_t max,
               int device, cdc_handle_t **out) {
    cdc::Engine *e = nullptr;
    const int rc = cdc::Engine::create(algo, min, avg, max, device, &e);
    if (rc != CDC_OK) return rc;
    *out = new cdc_handle{e};
    return CDC_OK;
}

int cdc_create_seq(uint32_t mode, uint32_t seq_length, uint32_t jump_trigger, uint32_t jump_size,
                   uint32_t min, uint32_t avg, uint32_t max, int device, cdc_handle_t **out) {
    const uint32_t cfg[4] = {mode, seq_length, jump_trigger, jump_size};
    cdc::Engine *e = nullptr;
    const int rc = cdc::Engine::create_seq(cfg, min, avg, max, device, &e);
    if (rc != CDC_OK) return rc;
    *out = new cdc_handle{e};
    return CDC_OK;
}

void cdc_destroy(cdc_handle_t *h) {
    if (!h) return;
    delete h->engine;
    delete h;
}

int64_t cdc_chunk_data(cdc_handle_t *h, const uint8_t *data, size_t len,
                       cdc_chunk_t *out, size_t cap) {
    if (!h) return bad_handle();
    return h->engine->chunk_host(data, len, out, cap);
}

size_t cdc_estimate_chunk_count(const cdc_handle_t *h, size_t len) {
    return h ? h->engine->estimate(len) : 0;
}

size_t cdc_max_chunk_count(const cdc_handle_t *h, size_t len) {
    return h ? h->engine->max_chunks(len) : 0;
}

const char *cdc_describe(const cdc_handle_t *h) {
    return h ? h->engine->describe() : "";
}

const char *cdc_last_error(void) { return cdc::last_error(); }

int cdc_set_gear(cdc_handle_t *h, const uint64_t gear[256]) {
    if (!h) return (int)bad_handle();
    return h->engine->set_gear(gear);
}

int cdc_set_rabin_poly(cdc_handle_t *h, uint64_t poly) {
    if (!h) return (int)bad_handle();
    return h->engine->set_rabin_poly(poly);
}

int64_t cdc_chunk_batch_device(cdc_handle_t *h, size_t n,
                               const uint8_t *const *d_streams,
                               const uint64_t *lens, cdc_chunk_t *d_out,
                               size_t out_cap, uint64_t *first,
                               void *hip_stream) {
    if (!h) return bad_handle();
    return h->engine->chunk_batch_device(n, d_streams, lens, d_out, out_cap, first,
                                         static_cast<hipStream_t>(hip_stream));
}

int64_t cdc_chunk_batch_device_async(cdc_handle_t *h, size_t n, const uint8_t *const *d_streams,
                                     const uint64_t *lens, cdc_chunk_t *d_out, size_t out_cap, uint64_t *first,
                                     void *hip_stream) {
    if (!h) return bad_handle();
    return h->engine->chunk_batch_device_async(n, d_streams, lens, d_out, out_cap, first,
                                               static_cast<hipStream_t>(hip_stream));
}

int64_t cdc_batch_sync(cdc_handle_t *h) {
    if (!h) return bad_handle();
    return h->engine->batch_sync();
}

size_t cdc_batch_max_chunks(const cdc_handle_t *h, size_t n, const uint64_t *lens) {
    return (h && lens) ? h->engine->batch_max_chunks(n, lens) : 0;
}

int cdc_debug_timing_back(cdc_handle_t *h, uint32_t back, cdc_timing_t *t, size_t t_size) {
    if (!h || !t) return (int)bad_handle();
    cdc_timing_t v{};
    const int rc = h->engine->timing_back(back, v);
    if (rc) return rc;
    std::memcpy(t, &v, t_size < sizeof v ? t_size : sizeof v);
    return CDC_OK;
}

int cdc_debug_read_bw(cdc_handle_t *h, const uint8_t *d_buf, size_t len, int reps, double *ms) {
    if (!h || !ms || (len && !d_buf) || reps < 1) return (int)bad_handle();
    return h->engine->read_bw(d_buf, len, reps, ms);
}

int64_t cdc_debug_host_placement(cdc_handle_t *h, char *buf, size_t cap) {
    if (!h || (cap && !buf)) return bad_handle();
    return h->engine->host_placement_json(buf, cap);
}

int cdc_last_timing(const cdc_handle_t *h, cdc_timing_t *t, size_t t_size) {
    if (!h || !t) return (int)bad_handle();
    const cdc_timing_t &src = h->engine->timing();
    std::memcpy(t, &src, t_size < sizeof src ? t_size : sizeof src);
    return CDC_OK;
}

int64_t cdc_fs_write(cdc_handle_t *h, const uint8_t *data, size_t len,
                     size_t seg_size, uint64_t *span_lengths, size_t cap,
                     double *chunk_seconds) {
    if (!h) return bad_handle();
    if (cap && !span_lengths) {
        cdc::set_error("cdc_fs_write: span_lengths is NULL");
        return CDC_EINVAL;
    }
    std::vector<uint64_t> spans;
    const int64_t n = h->engine->fs_write(data, len, seg_size, spans, chunk_seconds);
    if (n < 0) return n;
    for (size_t i = 0; i < spans.size() && i < cap; ++i) span_lengths[i] = spans[i];
    return n;
}

int cdc_write_begin(cdc_handle_t *h) {
    if (!h) return (int)bad_handle();
    return h->engine->write_begin();
}

int cdc_write_segment(cdc_handle_t *h, const uint8_t *data, size_t len) {
    if (!h) return (int)bad_handle();
    return h->engine->write_segment(data, len);
}

int64_t cdc_write_finish(cdc_handle_t *h, uint64_t *span_lengths, size_t cap, double *seconds) {
    if (!h) return bad_handle();
    if (cap && !span_lengths) {
        cdc::set_error("cdc_write_finish: span_lengths is NULL");
        return CDC_EINVAL;
    }
    std::vector<uint64_t> spans;
    const int64_t n = h->engine->write_finish(spans, seconds);
    if (n < 0) return n;
    for (size_t i = 0; i < spans.size() && i < cap; ++i) span_lengths[i] = spans[i];
    return n;
}

int64_t cdc_write_drain(cdc_handle_t *h, uint64_t *span_lengths, size_t cap) {
    if (!h) return bad_handle();
    return h->engine->write_drain(span_lengths, cap);
}

int cdc_debug_host_stats(const cdc_handle_t *h, double *v, size_t n) {
    if (!h || (n && !v)) return (int)bad_handle();
    return h->engine->host_stats(v, n);
}

int cdc_sha256_chunks_device(cdc_handle_t *h, const uint8_t *d_data,
                             const cdc_chunk_t *d_chunks, size_t n_chunks,
                             uint8_t *d_digests, void *hip_stream) {
    if (!h) return (int)bad_handle();
    return h->engine->sha256_device(d_data, d_chunks, n_chunks, d_digests,
                                    static_cast<hipStream_t>(hip_stream));
}

int cdc_sha256_batch_device(cdc_handle_t *h, size_t n_streams, const uint8_t *const *d_streams,
                            const uint64_t *first, const cdc_chunk_t *d_chunks, uint8_t *d_digests,
                            void *hip_stream) {
    if (!h) return (int)bad_handle();
    return h->engine->sha256_batch(n_streams, d_streams, first, d_chunks, d_digests,
                                   static_cast<hipStream_t>(hip_stream));
}

int64_t cdc_chunk_and_hash(cdc_handle_t *h, const uint8_t *data, size_t len,
                           cdc_chunk_t *out, uint8_t *digests, size_t cap) {
    if (!h) return bad_handle();
    if (cap && !digests) {
        cdc::set_error("cdc_chunk_and_hash: digests is NULL");
        return CDC_EINVAL;
    }
    return h->engine->chunk_host(data, len, out, cap, digests);
}

int cdc_fill_splitmix64_device(uint8_t *d_buf, size_t len, uint64_t seed, void *hip_stream) {
    if (len && !d_buf) {
        cdc::set_error("NULL buffer");
        return CDC_EINVAL;
    }
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    hipError_t e = cdc::launch_fill_splitmix64(d_buf, len, seed, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        cdc::set_error(std::string("fill: ") + hipGetErrorString(e));
        return CDC_EDEVICE;
    }
    return CDC_OK;
}

int cdc_debug_pipeline(const cdc_handle_t *h) { return h ? h->engine->pipeline() : (int)bad_handle(); }

uint32_t cdc_debug_record_cap(const cdc_handle_t *h) { return h ? h->engine->record_cap() : 0; }

int64_t cdc_debug_copy(cdc_handle_t *h, int what, void *out, size_t max_bytes) {
    if (!h) return bad_handle();
    if (max_bytes && !out) {
        cdc::set_error("cdc_debug_copy: out is NULL");
        return CDC_EINVAL;
    }
    return h->engine->debug_copy(what, out, max_bytes);
}

const char *cdc_version(void) { return "chunkfs_amd 0.6 gfx950 abi 4"; }

uint32_t cdc_abi_version(void) { return CHUNKFS_AMD_ABI_VERSION; }

}  // extern "C"
