// engine.hpp -- device-side orchestration behind the C ABI.
//
// One Engine = one chunker handle bound to one GPU: the FastChunker /
// FSChunker object of reference src/chunkers/{fast,fixed_size}.rs with its
// device workspace.  Not thread-safe (the reference serialises through a
// Mutex, src/lib.rs:89-90).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/chunkfs_amd.h"
#include "cdc_kernels.hpp"
#include "fastcdc.hpp"
#include "walk.hpp"

namespace cdc {

class Engine {
  public:
    // Returns CDC_OK or a negative CDC_E* code (message via set_error()).
    static int create(cdc_algo_t algo, uint32_t min, uint32_t avg, uint32_t max,
                      int device, Engine **out);
    // SeqChunker::new(mode, sizes, config) (seq.rs:16-24): seq = {mode,
    // seq_length, jump_trigger, jump_size} (mode 0 increasing, 1 decreasing).
    static int create_seq(const uint32_t seq[4], uint32_t min, uint32_t avg, uint32_t max,
                          int device, Engine **out);
    ~Engine();

    // chunk_data on a host buffer; with `digests` (32 B per chunk, cap
    // entries) also the SHA-256 of every chunk (StorageWriter's hashing).
    int64_t chunk_host(const uint8_t *data, size_t len, cdc_chunk_t *out, size_t cap,
                       uint8_t *digests = nullptr);
    // ChunkStorage::write of one whole write (storage.rs:78-103, 302-383):
    // the span lengths the StorageWriter loop produces.  Both supported
    // chunkers restart at every chunk boundary, so the carried-over `rest`
    // always begins at a boundary of the whole write and the spans do not
    // depend on the segment size: the write is chunked in
    // device windows of up to kFsWindow bytes, each window's last chunk
    // carried into the next exactly as the reference carries `rest`.
    int64_t fs_write(const uint8_t *data, size_t len, size_t seg_size, std::vector<uint64_t> &spans,
                     double *seconds);
    // SHA-256 of chunks of one device-resident stream (Sha256Hasher::hash).
    int sha256_device(const uint8_t *d_data, const cdc_chunk_t *d_chunks, size_t n,
                      uint8_t *d_digests, hipStream_t s);
    int64_t chunk_batch_device(size_t n, const uint8_t *const *d_streams,
                               const uint64_t *lens, cdc_chunk_t *d_out,
                               size_t out_cap, uint64_t *first, hipStream_t stream);
    size_t estimate(size_t len) const;
    // Strict bound: every FastCDC chunk but the last is >= 2*(min/2) bytes
    // (cut_gear starts testing at index 2*(min/2)).
    size_t min_chunk() const { return algo_ == CDC_ALGO_FASTCDC ? (min_ / 2) * 2 : min_; }
    size_t max_chunks(size_t len) const { return len / min_chunk() + 1; }
    size_t batch_max_chunks(size_t n, const uint64_t *lens) const;
    int set_gear(const uint64_t *gear);
    const char *describe() const { return describe_.c_str(); }
    const cdc_timing_t &timing() const { return timing_; }
    cdc_algo_t algo() const { return algo_; }
    int device() const { return device_; }
    int fill_splitmix64(uint8_t *d_buf, size_t len, uint64_t seed, hipStream_t s);
    // Debug (include/chunkfs_amd_debug.h): copy an intermediate array of the
    // last FastCDC batch to the host.  what: 0 = per-span candidate counts
    // (u32), 1 = candidate records (u32, cap per span).  Returns bytes copied.
    int64_t debug_copy(int what, void *out, size_t max_bytes);
    uint32_t record_cap() const { return cap_; }
    int pipeline() const { return 3; }  // (one FastCDC pipeline: scan + resolve)

  private:
    Engine() = default;
    static int create_walk(cdc_algo_t algo, const uint32_t seq[4], uint32_t min, uint32_t avg, uint32_t max,
                           int device, Engine **out);
    int init();
    int ensure_workspace(uint64_t spans, size_t n);
    int ensure_host_staging(size_t n);
    int run_fast(const StreamTable &st, cdc_chunk_t *d_out, size_t n,
                 uint64_t *first, hipStream_t s);
    int run_fixed(const StreamTable &st, size_t n, const uint64_t *lens,
                  cdc_chunk_t *d_out, uint64_t *first, hipStream_t s);
    // Rabin / Ultra / Leap / Seq: the segment-walk engine (walk.hip).
    bool is_walk() const { return algo_ != CDC_ALGO_FASTCDC && algo_ != CDC_ALGO_FIXED; }
    int init_walk(const uint32_t *seq);
    int ensure_walk_workspace(uint64_t segs, size_t n);
    int run_walk(const StreamTable &st, cdc_chunk_t *d_out, size_t n, uint64_t *first, hipStream_t s);

    cdc_algo_t algo_ = CDC_ALGO_FASTCDC;
    uint32_t min_ = 0, avg_ = 0, max_ = 0;
    int device_ = 0;
    int num_cus_ = 256;
    FastParams fp_{};
    uint32_t span_log2_ = 16;
    uint32_t cap_ = 0, smax_ = 0;
    std::string describe_;

    hipStream_t own_stream_ = nullptr;
    hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t *d_gear_ = nullptr;

    // Workspace arena (grow-only).
    void *ws_ = nullptr;
    size_t ws_bytes_ = 0;
    uint64_t ws_spans_ = 0;
    size_t ws_streams_ = 0;
    Candidates cand_{};
    p3::Chains ch3_{};             // chunk starts spilled past the resolve's LDS
    p3::Compact cp3_{};
    p3::Resolve rs3_{};            // look-back descriptors (generation-tagged, never re-zeroed)
    uint64_t res_gen_ = 0;
    uint64_t *d_tails_ = nullptr;  // [streams] ragged last span ids
    uint32_t n_tails_ = 0;
    uint64_t *d_first_ = nullptr;  // [n+1] (fixed-size path)
    const uint8_t **d_ptrs_ = nullptr;
    uint64_t *d_lens_ = nullptr;
    uint64_t *d_span_base_ = nullptr;

    // Pinned, device-visible (coherent) host staging: the small per-call
    // tables going in, stats ++ first[n+1] coming back (written by the
    // resolve kernel directly, no copy).
    void *h_stage_ = nullptr;
    size_t h_stage_streams_ = 0;

    // Host-path buffers (cdc_chunk_data).
    uint8_t *d_data_ = nullptr;
    size_t d_data_bytes_ = 0;
    cdc_chunk_t *d_out_ = nullptr;
    size_t d_out_cap_ = 0;
    uint8_t *d_dig_ = nullptr;               // [d_dig_cap_ * 32] digests (host path)
    size_t d_dig_cap_ = 0;
    unsigned long long *d_counter_ = nullptr;  // SHA-256 work counter

    cdc_timing_t timing_{};

    // Last uploaded stream tables (ptrs ++ lens) and the workspace generation
    // they were uploaded into.
    std::vector<uint64_t> tables_;
    uint64_t ws_gen_ = 0, tables_gen_ = ~0ull;
    uint64_t last_spans_ = 0;  // spans of the last FastCDC batch (debug_copy)
    uint64_t out_cap_ = 0;     // capacity of the current batch's output (resolve bound)

    // Segment-walk engine state (Rabin / Ultra / Leap / Seq).
    walk::WalkParams wp_{};
    uint32_t seg_log2_ = 14;
    uint32_t max_rounds_ = 16;     // Jacobi fix-up rounds before the serial pass
    uint32_t ahead_after_ = 8;     // rounds of plain Jacobi before run-ahead re-walks
    uint32_t ahead_max_ = 64;      // segments one lane may re-walk in a run-ahead round
    uint64_t *d_wtabs_ = nullptr;  // [768] rabin mod/out + leap hash tables
    void *wws_ = nullptr;          // walk workspace arena (grow-only)
    uint64_t wws_segs_ = 0;
    size_t wws_streams_ = 0;
    walk::WalkState wst_{};
};

void set_error(const std::string &msg);
const char *last_error();

}  // namespace cdc
