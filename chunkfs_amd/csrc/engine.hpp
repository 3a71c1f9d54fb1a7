// engine.hpp -- device-side orchestration behind the C ABI.
//
// One Engine = one chunker handle bound to one GPU: the FastChunker /
// FSChunker object of reference src/chunkers/{fast,fixed_size}.rs with its
// device workspace.  Not thread-safe (the reference serialises through a
// Mutex, src/lib.rs:89-90).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/chunkfs_amd.h"
#include "cdc_kernels.hpp"
#include "fastcdc.hpp"
#include "small.hpp"
#include "walk.hpp"

namespace cdc {

// Pageable -> pinned copies of the host path split over a few threads (one
// core copies ~20 GB/s, below what the H2D DMA takes).  One pool per process
// (CopyPool::shared), helpers spin briefly after a job (the next 1 MiB segment
// usually follows within microseconds), then sleep.  copy() returns when
// every part is done (hostpath.cpp).
// Where the host side of the boundary runs (hostpath.cpp): the device's PCIe
// address, NUMA node and link; the node's CPUs this process may use.
struct HostPlacement {
    std::string pci, link, link_max;
    int node = -1;
    int allowed = 0;          // CPUs in this process's affinity mask
    std::vector<int> cpus;    // of them, those on `node`
    bool enabled = false;     // pinned memory and copy helpers placed on `node`
    static HostPlacement probe(int device);
    hipError_t host_malloc(void **ptr, size_t bytes, unsigned flags) const;
    static int node_of(const void *addr);  // NUMA node of the page at addr (-1: unknown)
};

class CopyPool {
  public:
    CopyPool(unsigned threads, unsigned spin_us, const std::vector<int> &cpus);
    ~CopyPool();
    static CopyPool &for_node(int node, const std::vector<int> &cpus);
    void copy(void *dst, const void *src, size_t n);
    // Streamed copy for the small kernel's feed: pieces of `piece` bytes,
    // claimed by the caller and the awake helpers, each announced by
    // ready[piece index] = seq once copied (the device reads it over PCIe
    // while later pieces are still being copied).  Returns once every piece
    // is announced.
    void copy_feed(void *dst, const void *src, size_t n, size_t piece, volatile uint64_t *ready, uint64_t seq);
    unsigned threads() const { return (unsigned)th_.size() + 1; }
    unsigned pinned() const { return pinned_; }

  private:
    void run(unsigned id);
    void work();  // claim and copy pieces until none is left
    void job(void *dst, const void *src, size_t n, size_t piece, volatile uint64_t *ready, uint64_t seq);
    std::vector<std::thread> th_;
    std::mutex m_, job_m_;
    std::condition_variable cv_;
    unsigned spin_us_ = 200;
    unsigned pinned_ = 0;  // helpers bound to the node's CPUs
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false}, open_{false};
    std::atomic<unsigned> active_{0};  // helpers inside the current job
    std::atomic<size_t> next_{0}, done_{0};  // next piece to claim, pieces copied
    uint8_t *dst_ = nullptr;
    const uint8_t *src_ = nullptr;
    size_t n_ = 0, piece_ = 0, np_ = 0;
    volatile uint64_t *ready_ = nullptr;  // feed words (nullptr: a plain copy)
    uint64_t seq_ = 0;
};

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
    // the span lengths of the StorageWriter loop over seg_size segments, run
    // through the streaming write path below (hostpath.cpp).
    int64_t fs_write(const uint8_t *data, size_t len, size_t seg_size, std::vector<uint64_t> &spans,
                     double *seconds);
    // Streaming write path (hostpath.cpp): one file write as a sequence of
    // segments (write_from_stream, storage.rs:105-137); spans at finish.
    int write_begin();
    int write_segment(const uint8_t *data, size_t len);
    int64_t write_finish(std::vector<uint64_t> &spans, double *seconds);
    int64_t write_drain(uint64_t *out, size_t cap);
    // Host-path statistics: calls, upload s, total s of chunk_host; chunking s
    // and segments of the current / last streaming write.
    int host_stats(double *v, size_t n) const;
    int64_t host_placement_json(char *out, size_t cap);
    // SHA-256 of chunks of one device-resident stream (Sha256Hasher::hash).
    int sha256_device(const uint8_t *d_data, const cdc_chunk_t *d_chunks, size_t n,
                      uint8_t *d_digests, hipStream_t s);
    // The same over n streams in one launch (cdc_sha256_batch_device).
    int sha256_batch(size_t n, const uint8_t *const *d_streams, const uint64_t *first, const cdc_chunk_t *d_chunks,
                     uint8_t *d_digests, hipStream_t s);
    int64_t chunk_batch_device(size_t n, const uint8_t *const *d_streams,
                               const uint64_t *lens, cdc_chunk_t *d_out,
                               size_t out_cap, uint64_t *first, hipStream_t stream);
    // The same, enqueued (cdc_chunk_batch_device_async): FastCDC batches of
    // more than 8 MiB go back to back on the stream with no host wait, first[]
    // filled by batch_sync().  Other algorithms run synchronously.
    int64_t chunk_batch_device_async(size_t n, const uint8_t *const *d_streams, const uint64_t *lens,
                                     cdc_chunk_t *d_out, size_t out_cap, uint64_t *first, hipStream_t stream);
    // Waits for every enqueued batch (resolving the last one); the total chunk
    // count of the last batch, or a negative code.
    int64_t batch_sync();
    size_t estimate(size_t len) const;
    // Strict bound: every FastCDC chunk but the last is >= 2*(min/2) bytes
    // (cut_gear starts testing at index 2*(min/2)).
    size_t min_chunk() const { return algo_ == CDC_ALGO_FASTCDC ? (min_ / 2) * 2 : min_; }
    size_t max_chunks(size_t len) const { return len / min_chunk() + 1; }
    size_t batch_max_chunks(size_t n, const uint64_t *lens) const;
    int set_gear(const uint64_t *gear);
    int set_rabin_poly(uint64_t poly);
    const char *describe() const { return describe_.c_str(); }
    // Kernel durations of the last batch: a FastCDC batch whose done word was
    // seen returns before its kernels retire, and its events are read here,
    // on first request.
    const cdc_timing_t &timing();
    // Kernel times of the FastCDC batch `back` calls before the last one
    // (event ring, include/chunkfs_amd_debug.h).
    int timing_back(uint32_t back, cdc_timing_t &out);
    cdc_algo_t algo() const { return algo_; }
    int device() const { return device_; }
    int fill_splitmix64(uint8_t *d_buf, size_t len, uint64_t seed, hipStream_t s);
    int read_bw(const uint8_t *d_buf, size_t len, int reps, double *ms);
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
    // FastCDC regular pipeline: enqueue a batch (scan + resolve), collect a
    // batch's results, drain every batch in flight.
    int64_t batch_device(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                         size_t out_cap, uint64_t *first, hipStream_t stream, bool async);
    // ovl: the overlap kernel set (fastcdc_ovl.hip), the resolve on res_stream_.
    int64_t fast_submit(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                        size_t out_cap, uint64_t *first, uint64_t bytes, hipStream_t s, bool timed, bool ovl);
    int fast_collect(int rec);
    int64_t fast_drain();
    int64_t drain_implicit();  // fast_drain for another call: its result is kept for batch_sync
    // Async batches of the segment-walk algorithms (Rabin / Ultra / Leap /
    // Seq): two contexts -- engines with this handle's parameters, each with
    // its own stream and workspace -- run alternate batches synchronously,
    // each on its own host worker thread, so one batch's walks and fix-up
    // rounds overlap the next batch's bitmap pass on the device (a walk call
    // keeps host logic between its kernels: the round loop).
    int64_t walk_submit(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                        size_t out_cap, uint64_t *first);
    int64_t walk_drain();  // fast_drain's part for these batches
    struct WalkWorker;
    static constexpr int kWalkCtxMax = 4;
    std::unique_ptr<WalkWorker> ww_[kWalkCtxMax];
    int walk_ctx_ = 2;        // contexts in use (CHUNKFS_AMD_WALK_CTX, 2..4)
    bool wk_any_ = false;     // a walk batch is in flight
    uint64_t wk_seq_ = 0;     // walk batches submitted
    bool walk_async_ = true;  // CHUNKFS_AMD_WALK_ASYNC=0: walk batches complete inside the call
    uint32_t seq_cfg_[4] = {0, 0, 0, 0};  // create_walk's SeqCDC configuration (for the contexts)
    uint64_t rabin_poly_ = 0;             // set_rabin_poly's polynomial (0: the default), for the contexts
    // One small FastCDC stream in one launch (small.hip): CDC_OK, kSmallFallback
    // (a budget was exceeded: run the regular pipeline) or a CDC_E* code.
    static constexpr int kSmallFallback = 1;
    bool small_ok(uint64_t len) const;
    // feed_src: streamed host input -- the kernel is launched first, then the
    // bytes are copied from feed_src into feed_dst (ring slot feed_slot, which
    // `data` addresses) piece by piece, each piece announced by a feed word.
    int run_small(const uint8_t *data, uint64_t len, cdc_chunk_t *d_out, size_t out_cap, uint64_t *first,
                  hipStream_t s, bool host_input = false, const uint8_t *feed_src = nullptr,
                  uint8_t *feed_dst = nullptr, uint32_t feed_slot = 0);
    int run_fixed(const StreamTable &st, size_t n, const uint64_t *lens,
                  cdc_chunk_t *d_out, uint64_t *first, hipStream_t s);
    // Rabin / Ultra / Leap / Seq: the segment-walk engine (walk.hip).
    bool is_walk() const { return algo_ != CDC_ALGO_FASTCDC && algo_ != CDC_ALGO_FIXED; }
    int init_walk(const uint32_t *seq);
    int load_walk_tables(uint64_t rabin_poly);
    int ensure_walk_workspace(uint64_t segs, size_t n);
    int run_walk(const StreamTable &st, cdc_chunk_t *d_out, size_t n, uint64_t *first, hipStream_t s);
    // Host boundary (hostpath.cpp).
    int ensure_ring();
    int ensure_host_out(size_t chunks);
    int ensure_device_data(size_t len);
    int upload(const uint8_t *src, size_t len, uint8_t *dst, hipStream_t s, size_t piece);
    int write_window(bool final);

    cdc_algo_t algo_ = CDC_ALGO_FASTCDC;
    uint32_t min_ = 0, avg_ = 0, max_ = 0;
    int device_ = 0;
    int num_cus_ = 256;
    FastParams fp_{};
    uint32_t span_log2_ = 16;
    uint32_t small_span_log2_ = 16;                       // spans of batches <= kSmallBatch bytes
    static constexpr uint64_t kSmallBatch = uint64_t(8) << 20;
    // Batches this small with few streams read their stream tables straight
    // from the pinned staging block (no H2D copies: each small copy costs a
    // ~10 us DMA on the call's critical path).
    static constexpr size_t kZeroCopyStreams = 64;
    uint32_t cap_ = 0, smax_ = 0;
    std::string describe_;

    hipStream_t own_stream_ = nullptr;
    hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
    // FastCDC batches: events (start, scan end, resolve end) in a ring of
    // kTimeRing slots, batch k in slot k % kTimeRing.
    static constexpr uint32_t kTimeRing = 64;
    hipEvent_t tev_[kTimeRing][3] = {};
    uint64_t fast_batches_ = 0;
    uint64_t *d_gear_ = nullptr;

    // Workspace arena (grow-only).
    void *ws_ = nullptr;
    size_t ws_bytes_ = 0;
    uint64_t ws_spans_ = 0;
    size_t ws_streams_ = 0;
    Candidates cand_{};            // the last FastCDC batch's (debug_copy)
    p3::Chains ch3_{};             // chunk starts spilled past the resolve's LDS
    p3::Resolve rs3_{};            // look-back descriptors (generation-tagged, never re-zeroed)
    uint64_t res_gen_ = 0;
    uint64_t *d_tails_ = nullptr;  // [streams] ragged last span ids (walk engine: unused)
    // FastCDC batches in flight: device tables and candidates in four slots
    // (slot = sequence number % 4) whose uploaded tables are kept to skip
    // unchanged H2D copies; host staging in three slots (batch record k % 3,
    // below): batch k's block -- tables going in, stats ++ first[] coming
    // back -- is read at its collection, before submit k+3 reuses it.  A
    // device slot outlives its host block, so when batch k is submitted the
    // slot's previous user k-4 is complete (k-3 was collected): no stream
    // wait guards it, even with the resolves on a second stream.
    static constexpr int kSlots = 4, kHostSlots = 3;
    struct FastSlot {
        Candidates cand{};
        const uint8_t **d_ptrs = nullptr;
        uint64_t *d_lens = nullptr, *d_sb = nullptr, *d_tails = nullptr, *stats = nullptr;
        std::vector<uint64_t> tables;    // ptrs ++ lens as last uploaded (skip the H2D when unchanged)
        uint64_t tables_gen = ~0ull;
        uint32_t n_tails = 0;            // ragged last spans of those tables
    } fs_[kSlots];
    // Batches in flight, by sequence number % 3 (cdc_chunk_batch_device_async):
    // scan + resolve enqueued at submit, collected (done word, first[]) by the
    // submit three later or by fast_drain.
    struct FastBatch {
        bool live = false, resolved = false, timed = true, ovl = false;
        int slot = 0;                // device slot
        uint64_t *h = nullptr;       // host staging block (slot seq % kHostSlots)
        size_t n = 0;
        uint64_t *first = nullptr;  // the caller's first[n+1]
        uint64_t seq = 0, bytes = 0, spans = 0;
    } fb_[3];
    int event_every_ = 4;           // async FastCDC batches with events: 1 in event_every_ (CHUNKFS_AMD_EVENT_EVERY)
    bool tev_timed_[kTimeRing] = {};  // events recorded for ring slot
    uint64_t timing_seq_ = 0;       // the batch timing_ describes
    uint64_t fb_seq_ = 0;           // batches submitted
    hipStream_t fb_stream_ = nullptr;  // the stream of the batches in flight
    bool fb_any_ = false;           // a batch is in flight
    bool fb_ovl_ = false;           // ... with their resolves on res_stream_
    // Async batches on two streams (default, CHUNKFS_AMD_OVERLAP=2): batch k's
    // resolve on res_stream_ behind scan_ev_[slot k], batch k+1's scan on the
    // caller's stream right behind scan k.  A resolve block (148 KiB of LDS)
    // and a scan block (136 KiB) never share a CU, so nothing co-resides: the
    // next scan's blocks take each CU as its resolve block retires -- the
    // kernel-to-kernel gaps and the resolve's ragged end leave the step
    // (0.2557 vs 0.2744 ms sustained, profiles/r06/r06p_*).  res_ev_ orders the
    // caller's stream after the resolves at a drain.  CHUNKFS_AMD_OVERLAP=1:
    // the same with the overlap kernel set (fastcdc_ovl.hip, where its resolve
    // windows fit), which co-resides and measured slower (0.33 vs 0.278 ms:
    // the issue-bound scan slowed from 0.217 to 0.296 ms, profiles/r06/r06a_*);
    // 0: one stream.
    bool ovl_on_ = true;
    bool ovl_std_ = true;   // the regular kernel set on the two streams
    hipStream_t res_stream_ = nullptr;
    hipEvent_t scan_ev_[kSlots] = {};
    hipEvent_t res_ev_ = nullptr;
    hipEvent_t res_done_[3] = {};  // untimed batch k's resolve end on res_stream_ (slot k % 3)
    int64_t held_ = 0;              // result of the last implicit drain (drain_implicit)
    bool held_valid_ = false;
    const uint64_t *cur_tails_ = nullptr;  // this batch's: d_tails_ or the staging block's
    uint32_t n_tails_ = 0;
    uint64_t *d_first_ = nullptr;  // [n+1] (fixed-size path)
    const uint8_t **d_ptrs_ = nullptr;
    uint64_t *d_lens_ = nullptr;
    uint64_t *d_span_base_ = nullptr;

    // Pinned, device-visible (coherent) host staging: the small per-call
    // tables going in, stats ++ first[n+1] coming back (written by the
    // resolve kernel directly, no copy).
    void *h_stage_ = nullptr;       // slot 0 (the small and walk paths use its layout too), then slots 1-2
    size_t h_stage_streams_ = 0, h_stage_per_ = 0;

    // Host path (hostpath.cpp): pinned upload ring (slot k reused once its
    // DMA event completes), host-mapped chunk output written by the kernels,
    // a copy stream for the streaming writes and two device windows.
    static constexpr uint32_t kRingSlots = 4;
    static constexpr size_t kRingSlot = size_t(4) << 20;
    static constexpr size_t kWriteWindow = size_t(256) << 20;
    static constexpr size_t kRingDirect = size_t(16) << 20;  // chunk_data above this: pageable hipMemcpyAsync
    void *h_ring_ = nullptr;
    uint8_t *h_ring_dev_ = nullptr;  // the ring as the device addresses it (small-path kernel reads)
    CopyPool *pool_ = nullptr;  // CopyPool::for_node(the device's node)
    HostPlacement place_;
    bool place_probed_ = false;
    const HostPlacement &placement();
    hipEvent_t ring_ev_[kRingSlots] = {};
    uint32_t ring_next_ = 0;
    // Feed words of the small path's streamed input: kFeedPieces per ring
    // slot (pinned, coherent), and their device address.
    uint64_t *h_ready_ = nullptr, *h_ready_dev_ = nullptr;
    hipStream_t copy_stream_ = nullptr;
    hipEvent_t copy_done_ = nullptr, ws_ev_ = nullptr;
    cdc_chunk_t *h_out_ = nullptr, *d_hout_ = nullptr;
    size_t h_out_cap_ = 0;
    uint8_t *ws_win_[2] = {nullptr, nullptr};
    struct WriteState {
        bool active = false, failed = false;
        int cur = 0;
        size_t drained = 0;  // spans already returned by cdc_write_drain
        size_t reserve = 0, carry = 0, fill = 0;
        uint64_t bytes = 0, segments = 0;
        double t0 = 0, chunk_s = 0;
        std::vector<uint64_t> spans;
    } wr_;
    struct HostStats {
        uint64_t calls = 0;
        double upload_s = 0, total_s = 0;
    } host_;
    uint8_t *d_data_ = nullptr;
    size_t d_data_bytes_ = 0;
    cdc_chunk_t *d_out_ = nullptr;
    size_t d_out_cap_ = 0;
    uint8_t *d_dig_ = nullptr;               // [d_dig_cap_ * 32] digests (host path)
    size_t d_dig_cap_ = 0;
    unsigned long long *d_counter_ = nullptr;  // SHA-256 work counter
    uint64_t *d_sha_tab_ = nullptr, *h_sha_tab_ = nullptr;  // SHA-256 batch stream table: first[n+1] ++ bases[n]
    size_t sha_tab_cap_ = 0;
    uint32_t *d_sha_order_ = nullptr;  // SHA-256 claim order (longest chunk first)
    uint64_t sha_order_cap_ = 0;

    cdc_timing_t timing_{};
    bool timing_pending_ = false;  // FastCDC events not read yet (see timing())

    // Last uploaded stream tables (ptrs ++ lens) and the workspace generation
    // they were uploaded into.
    std::vector<uint64_t> tables_;
    uint64_t ws_gen_ = 0, tables_gen_ = ~0ull;
    // Small-stream path (small.hip): on unless CHUNKFS_AMD_SMALL=0; its input
    // straight from the pinned ring slot (no H2D copy) unless CHUNKFS_AMD_SMALL_ZC=0.
    bool small_on_ = false, small_zc_ = true;
    // Streamed input: 1 = launch first, then the copy with feed words; 0 = the
    // whole copy, then the launch; 2 = the feed copy, then the launch (A/B).
    int small_feed_ = 1;
    bool small_feed_pool_ = true;  // the feed copy on the copy pool (CHUNKFS_AMD_SMALL_FEED_POOL=0: caller only, A/B)
    uint32_t small_pmin_ = 0;  // min(popcount mask_s, popcount mask_l): records ~ 2^-pmin per byte
    bool small_skip_ = false;  // chunk_host's fallback call: the kernel already declined the bytes
    void *small_mem_ = nullptr;
    small::Scratch small_ws_{};
    uint64_t small_calls_ = 0, small_fallbacks_ = 0;
    uint64_t small_seq_ = 0;      // launch sequence number (feed words, block publication tags)
    double small_copy_s_ = 0;     // the last streamed call's host copy time
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
    uint64_t *walk_go_ = nullptr;     // finish_kernel's verdict word for the gated emit
    bool walk_flags_clean_ = false;   // the flag blocks hold the init pattern (the last call's end kernel reset them)
    bool walk_fused_ = true;          // fused end kernel (CHUNKFS_AMD_WALK_FUSED=0: sum / prefix / first + copies, A/B)
};

void set_error(const std::string &msg);
const char *last_error();

}  // namespace cdc
