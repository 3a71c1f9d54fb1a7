// engine.cpp -- host orchestration of the gfx950 chunking pipeline.
//
// Per batch (DESIGN.md "Pipeline and kernels"):
//   H2D of three tiny per-stream tables (skipped when unchanged) -> scan ->
//   next (record links) -> walk (writes the chunks to HBM and first[n+1] + stats
//   straight into coherent pinned host memory) -> one stream sync.
// Everything runs on one HIP stream; candidates, chains and the output never
// leave HBM.
#include "engine.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/chunkfs_amd_cdc_params.h"
#include "../../include/chunkfs_amd_tables.h"
#include "fastcdc.hpp"
#include "sha256.hpp"

namespace cdc {

namespace {
thread_local std::string g_last_error;

#ifndef CDC_MIN_SPAN_LOG2
#define CDC_MIN_SPAN_LOG2 16
#endif
constexpr uint32_t kMinSpanLog2 = CDC_MIN_SPAN_LOG2;  // 64 KiB spans at least (experiment builds may raise it)
constexpr uint32_t kMaxSpanLog2 = 17;  // ... and at most 128 KiB unless the max chunk needs more

// fastcdc 3.1.0 v2020 FastCDC::new asserts (VERIFY).
constexpr uint32_t kMinimumMin = 64, kMinimumMax = 1048576;
constexpr uint32_t kAverageMin = 256, kAverageMax = 4194304;
constexpr uint32_t kMaximumMin = 1024, kMaximumMax = 16777216;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint32_t ceil_log2(uint64_t x) {
    uint32_t r = 0;
    while ((1ull << r) < x) ++r;
    return r;
}
}  // namespace

void set_error(const std::string &msg) { g_last_error = msg; }
const char *last_error() { return g_last_error.c_str(); }

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));      \
            return CDC_EDEVICE;                                                \
        }                                                                      \
    } while (0)

int Engine::create(cdc_algo_t algo, uint32_t min, uint32_t avg, uint32_t max,
                   int device, Engine **out) {
    if (!out) {
        set_error("cdc_create: out is NULL");
        return CDC_EINVAL;
    }
    *out = nullptr;
    if (algo == CDC_ALGO_RABIN || algo == CDC_ALGO_ULTRA || algo == CDC_ALGO_LEAP || algo == CDC_ALGO_SEQ) {
        const uint32_t seq[4] = {0, CDC_SEQ_LENGTH, CDC_SEQ_JUMP_TRIGGER, CDC_SEQ_JUMP_SIZE};
        return create_walk(algo, seq, min, avg, max, device, out);
    }
    if (algo != CDC_ALGO_FASTCDC && algo != CDC_ALGO_FIXED) {
        set_error("SuperCDC is not implemented on MI355X: its chunk records (supercdc.rs:10, 37-50) "
                  "follow cdc-chunkers 0.1.3, absent offline (SURVEY.md §8c)");
        return CDC_ENOTSUP;
    }
    Engine *e = new Engine();
    e->algo_ = algo;
    e->min_ = min;
    e->avg_ = avg;
    e->max_ = max;
    e->device_ = device;
    if (algo == CDC_ALGO_FASTCDC) {
        if (min < kMinimumMin || min > kMinimumMax || avg < kAverageMin ||
            avg > kAverageMax || max < kMaximumMin || max > kMaximumMax) {
            set_error("FastCDC sizes out of range (fastcdc v2020 asserts: min 64..1MiB, "
                      "avg 256..4MiB, max 1KiB..16MiB)");
            delete e;
            return CDC_EINVAL;
        }
        const unsigned bits = (unsigned)std::lround(std::log2((double)avg));
        FastParams &fp = e->fp_;
        fp.min = min;
        fp.avg = avg;
        fp.max = max;
        fp.mask_s = CHUNKFS_AMD_MASKS[bits + 1];
        fp.mask_l = CHUNKFS_AMD_MASKS[bits - 1];
        fp.cmask = fp.mask_s & fp.mask_l;
        const uint64_t all = fp.mask_s | fp.mask_l;
        const uint32_t top = 63 - (uint32_t)__builtin_clzll(all);
        if (top > 47) {  // the 3-lane carry is exact mod 2^48 only
            set_error("mask tests bit >= 48: unsupported");
            delete e;
            return CDC_EINVAL;
        }
        fp.trunc = top;
        const uint32_t wlo = (uint32_t)__builtin_ctzll(all);
        fp.cm_align = (wlo <= 32 && (all >> wlo) <= 0xFFFFFFFFull) ? 1u : 0u;
        fp.tshift = fp.cm_align ? 32 - wlo : 0;
        fp.cm32 = (uint32_t)((fp.cmask << fp.tshift) >> 32);
        fp.cm_lo = (uint32_t)fp.cmask;
        fp.cm_hi = (uint32_t)(fp.cmask >> 32);
        fp.mask_s_sh = fp.mask_s << fp.tshift;
        fp.mask_l_sh = fp.mask_l << fp.tshift;
        if (const char *d = std::getenv("CHUNKFS_AMD_DIAG")) fp.diag = (uint32_t)std::atoi(d);
        if (const char *v = std::getenv("CHUNKFS_AMD_EVENT_EVERY")) e->event_every_ = std::max(1, std::atoi(v));
        if (const char *v = std::getenv("CHUNKFS_AMD_OVERLAP")) {  // (A/B; default 2)
            e->ovl_on_ = std::atoi(v) != 0;
            e->ovl_std_ = std::atoi(v) != 1;  // 1: the overlap kernel set (fastcdc_ovl.hip)
        }
        uint32_t l2 = ceil_log2(max);
        e->span_log2_ = l2 > kMinSpanLog2 ? l2 : kMinSpanLog2;
        {
            // Up to 128 KiB spans while a resolve window (11 spans) expects <=
            // 384 records, half its budget (4/8/16 KiB: 352): half the scan's
            // per-span epilogues (scan 0.222 -> 0.203 ms per GiB) and half the
            // resolve blocks, which then leave half the CUs to the next
            // batch's scan on the two streams (0.262 -> 0.237 ms per step,
            // profiles/r06/r06zc_*).  (256 KiB: windows overflow to the slow
            // global path.)
            const uint32_t pcm = (uint32_t)__builtin_popcountll(fp.cmask);
            while (e->span_log2_ < kMaxSpanLog2 && 11 * ((2ull << e->span_log2_) >> (pcm < 63 ? pcm : 63)) <= 384)
                ++e->span_log2_;
        }
        if (const char *v = std::getenv("CHUNKFS_AMD_SPAN"))  // experiments: span log2 (>= the max's, >= 14)
            e->span_log2_ = (uint32_t)std::max<int>(std::atoi(v), (int)std::max(l2, 14u));
        e->small_span_log2_ = l2 > 14 ? l2 : 14;
        if (const char *v = std::getenv("CHUNKFS_AMD_SMALL_SPAN")) {  // experiments: 0 = off
            const int x = std::atoi(v);
            e->small_span_log2_ = x == 0 ? e->span_log2_ : (uint32_t)std::max<int>(x, (int)std::max(l2, 14u));
        }
        if (e->small_span_log2_ > e->span_log2_) e->small_span_log2_ = e->span_log2_;
        const uint64_t span = 1ull << e->span_log2_;
        const uint32_t pc = (uint32_t)__builtin_popcountll(fp.cmask);
        uint64_t cap = 8 * (span >> (pc < 63 ? pc : 63));
        if (cap < 64) cap = 64;
        if (cap > 256) cap = 256;
        e->cap_ = (uint32_t)cap;
        e->smax_ = (uint32_t)(span / ((min / 2) * 2) + 2);
        // The overlap set's resolve windows hold 384 records (11 spans): keep
        // it to sizes whose windows expect <= 256 (avg >= 8 KiB at max <= 64
        // KiB); denser records would send windows to the slow global path.
        if (11 * (span >> (pc < 63 ? pc : 63)) > 256 && !e->ovl_std_) e->ovl_on_ = false;
        // Small-stream path (small.hip): its per-lane and per-block record
        // budgets assume sparse hits, ~2^-10 per position or rarer.
        const uint32_t pmin = (uint32_t)std::min(__builtin_popcountll(fp.mask_s), __builtin_popcountll(fp.mask_l));
        e->small_on_ = pmin >= 10;
        e->small_pmin_ = pmin;
        if (const char *v = std::getenv("CHUNKFS_AMD_SMALL")) e->small_on_ = e->small_on_ && std::atoi(v) != 0;
        if (const char *v = std::getenv("CHUNKFS_AMD_SMALL_ZC")) e->small_zc_ = std::atoi(v) != 0;
        if (const char *v = std::getenv("CHUNKFS_AMD_SMALL_FEED")) e->small_feed_ = std::atoi(v);
        if (const char *v = std::getenv("CHUNKFS_AMD_SMALL_FEED_POOL")) e->small_feed_pool_ = std::atoi(v) != 0;
        char buf[256];
        std::snprintf(buf, sizeof buf,
                      "FastCDC (2020), sizes: SizeParams { min: %u, avg: %u, max: %u } "
                      "[MI355X gfx950]",
                      min, avg, max);
        e->describe_ = buf;
    } else {
        if (min == 0) {
            set_error("FSChunker chunk size must be > 0");
            delete e;
            return CDC_EINVAL;
        }
        char buf[128];
        std::snprintf(buf, sizeof buf, "Fixed size chunking, chunk size: %u [MI355X gfx950]", min);
        e->describe_ = buf;
    }
    const int rc = e->init();
    if (rc != CDC_OK) {
        delete e;
        return rc;
    }
    *out = e;
    return CDC_OK;
}

int Engine::init() {
    int count = 0;
    HIP_TRY(hipGetDeviceCount(&count));
    if (device_ < 0 || device_ >= count) {
        set_error("device index out of range");
        return CDC_EDEVICE;
    }
    HIP_TRY(hipSetDevice(device_));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device_));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("chunkfs_amd kernels are built for gfx950 only; device is ") +
                  prop.gcnArchName);
        return CDC_EDEVICE;
    }
    num_cus_ = prop.multiProcessorCount;
    HIP_TRY(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking));
    for (auto &ev : ev_) HIP_TRY(hipEventCreate(&ev));
    for (auto &slot : tev_)
        for (auto &ev : slot) HIP_TRY(hipEventCreate(&ev));
    HIP_TRY(hipMalloc(&d_gear_, 256 * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&d_counter_, (1 + kShaBuckets) * sizeof(unsigned long long)));  // SHA-256 counter + histogram
    HIP_TRY(hipMemcpy(d_gear_, CHUNKFS_AMD_GEAR, 256 * sizeof(uint64_t), hipMemcpyHostToDevice));
    return CDC_OK;
}

// A walk context and the host thread that runs its batches (Engine::walk_submit).
struct Engine::WalkWorker {
    Engine *ctx = nullptr;  // owned: an engine with the handle's parameters
    int device = 0;
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    bool has_job = false, stop = false;
    bool done = true;    // no batch posted or running
    bool fresh = false;  // ran a batch since the last drain
    uint64_t seq = 0;    // that batch's number
    std::vector<const uint8_t *> ptrs;
    std::vector<uint64_t> lens;
    cdc_chunk_t *out = nullptr;
    size_t cap = 0;
    uint64_t *first = nullptr;
    int64_t rc = 0;
    std::string err;

    void loop() {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(m);
        for (;;) {
            cv.wait(lk, [&] { return stop || has_job; });
            if (has_job) {  // (a stop request waits for the batch in hand)
                has_job = false;
                lk.unlock();
                const int64_t r =
                    ctx->chunk_batch_device(ptrs.size(), ptrs.data(), lens.data(), out, cap, first, nullptr);
                std::string e = r < 0 ? std::string(last_error()) : std::string();
                lk.lock();
                rc = r;
                err = std::move(e);
                done = true;
                cv.notify_all();
                continue;
            }
            return;
        }
    }
    void wait_done(std::unique_lock<std::mutex> &lk) {
        cv.wait(lk, [&] { return done; });
    }
    ~WalkWorker() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
        delete ctx;
    }
};

Engine::~Engine() {
    if (device_ >= 0) (void)hipSetDevice(device_);
    if (fb_any_) (void)fast_drain();
    for (auto &w : ww_) w.reset();
    if (own_stream_) (void)hipStreamSynchronize(own_stream_);
    if (res_stream_) (void)hipStreamSynchronize(res_stream_);
    (void)hipFree(ws_);
    (void)hipFree(small_mem_);
    (void)hipFree(d_gear_);
    (void)hipFree(d_data_);
    (void)hipFree(d_out_);
    (void)hipFree(d_dig_);
    (void)hipFree(d_sha_tab_);
    (void)hipHostFree(h_sha_tab_);
    (void)hipFree(d_sha_order_);
    (void)hipFree(d_counter_);
    (void)hipFree(d_wtabs_);
    (void)hipFree(wws_);
    (void)hipHostFree(h_stage_);
    if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
    (void)hipHostFree(h_ring_);
    (void)hipHostFree(h_ready_);
    (void)hipHostFree(h_out_);
    for (auto &w : ws_win_) (void)hipFree(w);
    for (auto &e : ring_ev_)
        if (e) (void)hipEventDestroy(e);
    if (copy_done_) (void)hipEventDestroy(copy_done_);
    if (ws_ev_) (void)hipEventDestroy(ws_ev_);
    if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
    for (auto &ev : ev_)
        if (ev) (void)hipEventDestroy(ev);
    for (auto &slot : tev_)
        for (auto &ev : slot)
            if (ev) (void)hipEventDestroy(ev);
    if (own_stream_) (void)hipStreamDestroy(own_stream_);
    for (auto &ev : scan_ev_)
        if (ev) (void)hipEventDestroy(ev);
    if (res_ev_) (void)hipEventDestroy(res_ev_);
    for (auto &ev : res_done_)
        if (ev) (void)hipEventDestroy(ev);
    if (res_stream_) (void)hipStreamDestroy(res_stream_);
}

int Engine::set_gear(const uint64_t *gear) {
    if (!gear) {
        set_error("gear is NULL");
        return CDC_EINVAL;
    }
    if (fb_any_) {  // the batches in flight finish with the table they were submitted with
        const int64_t r = drain_implicit();
        if (r < 0) return (int)r;
    }
    if (wr_.active) {  // windows already chunked used the old table: a write never mixes two
        set_error("cdc_set_gear: a streaming write is in progress (cdc_write_finish it first)");
        return CDC_EINVAL;
    }
    HIP_TRY(hipSetDevice(device_));
    HIP_TRY(hipMemcpy(d_gear_, gear, 256 * sizeof(uint64_t), hipMemcpyHostToDevice));
    return CDC_OK;
}

size_t Engine::estimate(size_t len) const {
    if (algo_ == CDC_ALGO_FIXED) return len / min_ + 1;  // fixed_size.rs:45-47
    if (algo_ == CDC_ALGO_SEQ) return len / avg_;        // seq.rs:52-54
    return len / min_;  // fast.rs:47-49, rabin.rs:53-55, ultra.rs:41-43, leap.rs:41-43
}

size_t Engine::batch_max_chunks(size_t n, const uint64_t *lens) const {
    size_t t = 0;
    for (size_t i = 0; i < n; ++i) t += lens[i] / min_chunk() + 1;
    return t;
}

int Engine::ensure_host_staging(size_t n) {
    if (h_stage_ && h_stage_streams_ >= n) return CDC_OK;
    if (fb_any_) {  // (the batches in flight read their slots)
        set_error("internal: host staging regrown with FastCDC batches in flight");
        return CDC_EINVAL;
    }
    (void)hipHostFree(h_stage_);
    h_stage_ = nullptr;
    const size_t want = n + 64;
    // Per slot: ptrs[W] lens[W] span_base[W] tails[W] | stats ++ first[n+1]
    // (fixed: first[n+1]) -- stream tables 4 n, device-written stats / flags
    // ++ first[n+1] (n + 32), the walk's flags[4] and fix-up round flag blocks
    // (4 x walk::kMaxFixRounds).  Slots 1-2: more FastCDC batches in flight.
    h_stage_per_ = 5 * want + 36 + 4 * walk::kMaxFixRounds;
    HIP_TRY(placement().host_malloc(&h_stage_, kHostSlots * h_stage_per_ * sizeof(uint64_t), hipHostMallocCoherent));
    h_stage_streams_ = want;
    for (int k = 0; k < kSlots; ++k) fs_[k].tables.clear();
    return CDC_OK;
}

int Engine::ensure_workspace(uint64_t spans, size_t n) {
    if (ws_ && spans <= ws_spans_ && n <= ws_streams_) return CDC_OK;
    const uint64_t S = spans > ws_spans_ ? spans + spans / 4 + 16 : ws_spans_;
    const size_t N = n > ws_streams_ ? n + 64 : ws_streams_;
    const uint64_t cap = algo_ == CDC_ALGO_FASTCDC ? cap_ : 0;
    const uint64_t smax = algo_ == CDC_ALGO_FASTCDC ? smax_ : 0;
    const size_t A = 256;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align_up(off + bytes, A);
        return o;
    };
    if (fb_any_) {
        set_error("internal: workspace regrown with FastCDC batches in flight");
        return CDC_EINVAL;
    }
    size_t o_count[kSlots], o_pos[kSlots], o_ptrs[kSlots], o_lens[kSlots], o_sb[kSlots], o_stats[kSlots],
        o_tails[kSlots];
    for (int k = 0; k < kSlots; ++k) {  // per batch in flight (FastCDC); the fixed-size path uses slot 0
        o_count[k] = take(S * 4);
        o_pos[k] = take(S * cap * 4);
        o_ptrs[k] = take(N * 8);
        o_lens[k] = take(N * 8);
        o_sb[k] = take((N + 1) * 8);
        o_stats[k] = take(p3::kStatWords * 8);
        o_tails[k] = take(N * 8);
    }
    const size_t o_starts = take(S * smax * 8);  // chunk starts beyond the LDS-resident ones
    const size_t o_first = take((N + 1) * 8);
    const uint64_t nb = std::max(p3::resolve_blocks(S), p3::ovl::resolve_blocks(S)) + 2;
    const size_t o_desc = take(6 * nb * 8);
    (void)hipFree(ws_);
    ws_ = nullptr;
    ws_spans_ = 0;
    ws_streams_ = 0;
    HIP_TRY(hipMalloc(&ws_, off));
    ++ws_gen_;
    ws_bytes_ = off;
    ws_spans_ = S;
    ws_streams_ = N;
    char *b = static_cast<char *>(ws_);
    for (int k = 0; k < kSlots; ++k) {
        FastSlot &f = fs_[k];
        f.cand.cap = (uint32_t)cap;
        f.cand.count = reinterpret_cast<uint32_t *>(b + o_count[k]);
        f.cand.pos = reinterpret_cast<uint32_t *>(b + o_pos[k]);
        f.d_ptrs = reinterpret_cast<const uint8_t **>(b + o_ptrs[k]);
        f.d_lens = reinterpret_cast<uint64_t *>(b + o_lens[k]);
        f.d_sb = reinterpret_cast<uint64_t *>(b + o_sb[k]);
        f.d_tails = reinterpret_cast<uint64_t *>(b + o_tails[k]);
        f.stats = reinterpret_cast<uint64_t *>(b + o_stats[k]);
        f.tables.clear();
    }
    cand_ = fs_[0].cand;
    d_first_ = reinterpret_cast<uint64_t *>(b + o_first);
    d_ptrs_ = fs_[0].d_ptrs;  // (the fixed-size path)
    d_lens_ = fs_[0].d_lens;
    d_span_base_ = fs_[0].d_sb;
    ch3_.smax = (uint32_t)smax;
    ch3_.starts = reinterpret_cast<uint64_t *>(b + o_starts);
    uint64_t *desc = reinterpret_cast<uint64_t *>(b + o_desc);
    rs3_ = p3::Resolve{desc, desc + nb, desc + 2 * nb, desc + 3 * nb, desc + 4 * nb, desc + 5 * nb, 0};
    HIP_TRY(hipMemset(desc, 0, 6 * nb * 8));  // no stale status word can carry a live generation
    d_tails_ = fs_[0].d_tails;
    return CDC_OK;
}

int64_t Engine::chunk_batch_device(size_t n, const uint8_t *const *d_streams,
                                   const uint64_t *lens, cdc_chunk_t *d_out,
                                   size_t out_cap, uint64_t *first,
                                   hipStream_t stream) {
    return batch_device(n, d_streams, lens, d_out, out_cap, first, stream, false);
}

int64_t Engine::chunk_batch_device_async(size_t n, const uint8_t *const *d_streams, const uint64_t *lens,
                                         cdc_chunk_t *d_out, size_t out_cap, uint64_t *first,
                                         hipStream_t stream) {
    return batch_device(n, d_streams, lens, d_out, out_cap, first, stream, true);
}

int64_t Engine::batch_sync() {
    HIP_TRY(hipSetDevice(device_));
    if (fb_any_) {
        held_valid_ = false;
        return fast_drain();
    }
    if (held_valid_) {  // an implicit drain already completed them: its result
        held_valid_ = false;
        return held_;
    }
    return 0;
}

// A drain that another call makes on the caller's behalf (any call on the
// handle completes the async batches first): its result -- the last batch's
// chunk count, or the error of a failed collection -- is what the next
// cdc_batch_sync returns.
int64_t Engine::drain_implicit() {
    if (!fb_any_) return 0;
    held_ = fast_drain();
    held_valid_ = true;
    return held_;
}

// Batch k of the async walk pipeline goes to context k % walk_ctx_ (2 by
// default), once that context's previous batch is done; a failure of that batch fails this
// call (after the other context is drained), as FastCDC's collection does.
int64_t Engine::walk_submit(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                            size_t out_cap, uint64_t *first) {
    const int c = (int)(wk_seq_ % (uint64_t)walk_ctx_);
    if (!ww_[c]) {
        Engine *e = nullptr;
        int rc = create_walk(algo_, seq_cfg_, min_, avg_, max_, device_, &e);
        if (rc) return rc;
        e->walk_async_ = false;
        if (rabin_poly_) rc = e->set_rabin_poly(rabin_poly_);
        if (rc) {
            delete e;
            return rc;
        }
        std::unique_ptr<WalkWorker> w(new WalkWorker());
        w->ctx = e;
        w->device = device_;
        WalkWorker *wp = w.get();
        w->th = std::thread([wp] { wp->loop(); });
        ww_[c] = std::move(w);
    }
    WalkWorker &w = *ww_[c];
    {
        std::unique_lock<std::mutex> lk(w.m);
        w.wait_done(lk);
        if (w.fresh && w.rc < 0) {
            const int64_t rc = w.rc;
            const std::string msg = w.err;
            lk.unlock();
            (void)walk_drain();
            set_error(msg);
            return rc;
        }
        w.ptrs.assign(d_streams, d_streams + n);
        w.lens.assign(lens, lens + n);
        w.out = d_out;
        w.cap = out_cap;
        w.first = first;
        w.seq = wk_seq_;
        w.rc = 0;
        w.err.clear();
        w.done = false;
        w.fresh = true;
        w.has_job = true;
    }
    w.cv.notify_all();
    ++wk_seq_;
    wk_any_ = true;
    fb_any_ = true;
    return 0;
}

// Every walk batch in flight completed: the last one's chunk count (its
// context's timing becomes this handle's), or the first failure.
int64_t Engine::walk_drain() {
    int64_t res = 0, err = 0;
    std::string msg;
    uint64_t last = 0;
    bool any = false;
    for (auto &wp : ww_) {
        if (!wp) continue;
        WalkWorker &w = *wp;
        std::unique_lock<std::mutex> lk(w.m);
        w.wait_done(lk);
        if (!w.fresh) continue;
        w.fresh = false;
        if (w.rc < 0 && !err) {
            err = w.rc;
            msg = w.err;
        }
        if (!any || w.seq > last) {
            any = true;
            last = w.seq;
            res = w.rc;
            timing_ = w.ctx->timing_;
        }
    }
    wk_any_ = false;
    fb_any_ = false;
    if (err) {
        set_error(msg);
        return err;
    }
    return res;
}

int64_t Engine::batch_device(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                             size_t out_cap, uint64_t *first, hipStream_t stream, bool async) {
    if (n && (!d_streams || !lens || !first)) {
        set_error("cdc_chunk_batch_device: NULL argument");
        return CDC_EINVAL;
    }
    if (n > 0xFFFFFFFEull) {
        set_error("too many streams");
        return CDC_EINVAL;
    }
    HIP_TRY(hipSetDevice(device_));
    hipStream_t s = stream ? stream : own_stream_;
    uint64_t bytes = 0, need = 0;
    for (size_t i = 0; i < n; ++i) {
        bytes += lens[i];
        need += lens[i] / min_chunk() + 1;
        if (lens[i] && !d_streams[i]) {
            set_error("NULL stream pointer with non-zero length");
            return CDC_EINVAL;
        }
        // Every content-defined kernel reads streams with 16-byte vector loads
        // (FastCDC scan, walk-engine bitmap pass and LDS windows).
        if (lens[i] && algo_ != CDC_ALGO_FIXED && (reinterpret_cast<uintptr_t>(d_streams[i]) & 15)) {
            set_error("device stream pointers must be 16-byte aligned");
            return CDC_EINVAL;
        }
    }
    if (need > out_cap) {
        set_error("out_cap < cdc_batch_max_chunks()");
        return CDC_EINVAL;
    }
    // FastCDC multi-megabyte batches are pipelined; everything else runs to
    // completion here, after the batches in flight.
    if (async && is_walk() && walk_async_ && n > 0 && bytes > kSmallBatch)
        return walk_submit(n, d_streams, lens, d_out, out_cap, first);
    const bool pipe = algo_ == CDC_ALGO_FASTCDC && n > 0 && bytes > kSmallBatch;
    if (!pipe && fb_any_) {
        const int64_t r = drain_implicit();
        if (r < 0) return r;
    }
    if (pipe) {
        // (async batches: the start / split / end events that cdc_last_timing
        // reads are recorded on every event_every_-th batch only -- each
        // event costs the stream ~4 us, r05t)
        const int64_t r = fast_submit(n, d_streams, lens, d_out, out_cap, first, bytes, s,
                                      !async || fb_seq_ % event_every_ == 0, async && ovl_on_);
        if (r < 0 || async) return r;
        return fast_drain();
    }
    const double hash_ms = timing_.hash_ms;  // (reported with the batch it hashed)
    timing_pending_ = false;                 // (a new batch re-records the events)
    timing_ = cdc_timing_t{};
    timing_.hash_ms = hash_ms;
    timing_.bytes = bytes;
    timing_.path = CDC_PATH_EMPTY;
    out_cap_ = out_cap;
    if (n == 0) {
        if (first) first[0] = 0;
        return 0;
    }
    int rc = ensure_host_staging(n);
    if (rc) return rc;
    if (algo_ == CDC_ALGO_FASTCDC && n == 1 && !small_skip_ && small_ok(lens[0])) {
        rc = run_small(d_streams[0], lens[0], d_out, out_cap, first, s);
        if (rc == CDC_OK) {
            timing_.path = CDC_PATH_SMALL;  // (no events on the call path: timed stays 0)
            return (int64_t)first[1];
        }
        if (rc < 0) return rc;
        // (kSmallFallback: the regular pipeline below)
    }
    if (algo_ == CDC_ALGO_FASTCDC) {  // small batches: one scan + resolve, waited for here
        const int64_t r = fast_submit(n, d_streams, lens, d_out, out_cap, first, bytes, s, true, false);
        if (r < 0) return r;
        return fast_drain();
    }
    uint64_t *h = static_cast<uint64_t *>(h_stage_);
    uint64_t *h_ptrs = h, *h_lens = h + h_stage_streams_, *h_sb = h + 2 * h_stage_streams_;
    const uint32_t sl2 = is_walk() ? seg_log2_ : 0;
    uint64_t spans = 0;
    for (size_t i = 0; i < n; ++i) {
        h_ptrs[i] = reinterpret_cast<uint64_t>(d_streams[i]);
        h_lens[i] = lens[i];
        h_sb[i] = spans;
        if (is_walk()) spans += (lens[i] + (1ull << sl2) - 1) >> sl2;  // segments
    }
    h_sb[n] = spans;
    if (algo_ != CDC_ALGO_FIXED && spans == 0) {  // every stream is empty
        for (size_t i = 0; i <= n; ++i) first[i] = 0;
        return 0;
    }
    rc = is_walk() ? ensure_walk_workspace(spans, n) : ensure_workspace(spans, n);
    if (rc) return rc;
    // Small batches (the host path's per-segment calls) read the tables from
    // the pinned staging block itself: the kernels' few table loads cross
    // PCIe, but no copy sits on the call's critical path.  Larger batches
    // re-upload the three per-stream tables only when they change (repeated
    // batches over the same device buffers skip the H2D copies).
    const bool zero_copy = bytes <= kSmallBatch && n <= kZeroCopyStreams;
    const bool same = zero_copy || (ws_gen_ == tables_gen_ && tables_.size() == 2 * n &&
                                    std::memcmp(tables_.data(), h_ptrs, n * 8) == 0 &&
                                    std::memcmp(tables_.data() + n, h_lens, n * 8) == 0);
    if (!same) {
        HIP_TRY(hipMemcpyAsync(d_ptrs_, h_ptrs, n * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_lens_, h_lens, n * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_span_base_, h_sb, (n + 1) * 8, hipMemcpyHostToDevice, s));
        tables_.assign(h_ptrs, h_ptrs + n);
        tables_.insert(tables_.end(), h_lens, h_lens + n);
        tables_gen_ = ws_gen_;
    }
    StreamTable st{};
    st.ptrs = zero_copy ? reinterpret_cast<const uint8_t *const *>(h_ptrs) : d_ptrs_;
    st.lens = zero_copy ? h_lens : d_lens_;
    st.span_base = zero_copy ? h_sb : d_span_base_;
    st.n = (uint32_t)n;
    st.span_log2 = sl2;
    st.total_spans = spans;
    rc = is_walk() ? run_walk(st, d_out, n, first, s) : run_fixed(st, n, lens, d_out, first, s);
    if (rc) return rc;
    return (int64_t)first[n];
}

// One FastCDC batch enqueued: its tables into the batch's slots, the scan and
// the resolve launches; no host wait.  The host collects it (fast_collect)
// when its stats block is needed again or at fast_drain().
int64_t Engine::fast_submit(size_t n, const uint8_t *const *d_streams, const uint64_t *lens, cdc_chunk_t *d_out,
                            size_t out_cap, uint64_t *first, uint64_t bytes, hipStream_t s, bool timed, bool ovl) {
    if (fb_any_ && (s != fb_stream_ || ovl != fb_ovl_)) {  // one pipeline per stream (and kernel set)
        const int64_t r = drain_implicit();
        if (r < 0) return r;
    }
    if (ovl && !res_stream_) {
        HIP_TRY(hipStreamCreateWithFlags(&res_stream_, hipStreamNonBlocking));
        for (auto &ev : scan_ev_) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&res_ev_, hipEventDisableTiming));
        for (auto &ev : res_done_) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (!std::getenv("CHUNKFS_AMD_NO_PREWARM")) {
            // The first ~100 two-stream batches of a process ran 10-20 % slower
            // than later ones, whichever handle ran them (profiles/r06/r06y_*):
            // the cross-stream event pattern, rehearsed once here with 4-byte
            // fills.
            void *d = nullptr;
            HIP_TRY(hipMalloc(&d, 256));
            for (int i = 0; i < 256; ++i) {
                HIP_TRY(hipMemsetAsync(d, i, 4, s));
                HIP_TRY(hipEventRecord(scan_ev_[i % kSlots], s));
                HIP_TRY(hipStreamWaitEvent(res_stream_, scan_ev_[i % kSlots], 0));
                HIP_TRY(hipMemsetAsync(static_cast<char *>(d) + 128, i, 4, res_stream_));
                HIP_TRY(hipEventRecord(res_done_[i % 3], res_stream_));
            }
            HIP_TRY(hipStreamSynchronize(res_stream_));
            HIP_TRY(hipStreamSynchronize(s));
            HIP_TRY(hipFree(d));
        }
    }
    const uint32_t sl2 = bytes <= kSmallBatch ? small_span_log2_ : span_log2_;
    uint64_t spans = 0;
    for (size_t i = 0; i < n; ++i) spans += (lens[i] + (1ull << sl2) - 1) >> sl2;
    const bool zero_copy = bytes <= kSmallBatch && n <= kZeroCopyStreams;
    const bool grow = !(h_stage_ && h_stage_streams_ >= n) || !(ws_ && spans <= ws_spans_ && n <= ws_streams_);
    if (fb_any_ && (zero_copy || grow)) {  // (buffers the batches in flight use)
        const int64_t r = drain_implicit();
        if (r < 0) return r;
    }
    const uint64_t seq = fb_seq_;
    if (fb_[seq % 3].live) {  // batch seq-3: its host block is this batch's
        const int rc = fast_collect((int)(seq % 3));
        if (rc) {
            (void)fast_drain();
            return rc;
        }
    }
    int rc = ensure_host_staging(n);
    if (rc) return rc;
    rc = ensure_workspace(spans ? spans : 1, n);
    if (rc) return rc;
    const int slot = (int)(seq % kSlots);
    FastSlot &f = fs_[slot];
    uint64_t *hb = static_cast<uint64_t *>(h_stage_) + (seq % kHostSlots) * h_stage_per_;
    uint64_t *h_ptrs = hb, *h_lens = hb + h_stage_streams_, *h_sb = hb + 2 * h_stage_streams_;
    uint64_t *h_tails = hb + 3 * h_stage_streams_;
    bool same = !zero_copy && f.tables_gen == ws_gen_ && f.tables.size() == 2 * n;
    for (size_t i = 0; same && i < n; ++i)
        same = f.tables[i] == reinterpret_cast<uint64_t>(d_streams[i]) && f.tables[n + i] == lens[i];
    {
        // this batch's tables in its own host block (its collection reads the
        // lengths); the device slot's copies are re-uploaded when they differ
        uint64_t sp = 0;
        uint32_t nt = 0;
        for (size_t i = 0; i < n; ++i) {
            h_ptrs[i] = reinterpret_cast<uint64_t>(d_streams[i]);
            h_lens[i] = lens[i];
            h_sb[i] = sp;
            sp += (lens[i] + (1ull << sl2) - 1) >> sl2;
            if (lens[i] & ((1ull << sl2) - 1)) h_tails[nt++] = sp - 1;  // ragged last span
        }
        h_sb[n] = sp;
        if (same && nt != f.n_tails) same = false;  // (cannot differ for equal tables; a guard)
        f.n_tails = nt;
    }
    if (!same) {
        f.tables.clear();
        if (!zero_copy) {
            HIP_TRY(hipMemcpyAsync(f.d_ptrs, h_ptrs, n * 8, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(f.d_lens, h_lens, n * 8, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(f.d_sb, h_sb, (n + 1) * 8, hipMemcpyHostToDevice, s));
            if (f.n_tails) HIP_TRY(hipMemcpyAsync(f.d_tails, h_tails, f.n_tails * 8, hipMemcpyHostToDevice, s));
            f.tables.assign(h_ptrs, h_ptrs + n);
            f.tables.insert(f.tables.end(), h_lens, h_lens + n);
            f.tables_gen = ws_gen_;
        }
    }
    StreamTable st{};
    st.ptrs = zero_copy ? reinterpret_cast<const uint8_t *const *>(h_ptrs) : f.d_ptrs;
    st.lens = zero_copy ? h_lens : f.d_lens;
    st.span_base = zero_copy ? h_sb : f.d_sb;
    st.n = (uint32_t)n;
    st.span_log2 = sl2;
    st.total_spans = spans;
    uint64_t *h_misc = hb + 4 * h_stage_streams_;  // stats ++ first[n+1], written by the device
    const p3::Compact cp{f.stats, h_misc, h_misc + p3::kStatWords};
    h_misc[p3::kStatDone] = ~0ull;  // sentinel: overwritten by the resolve's last block
    if (!spans) {  // every stream is empty: nothing to launch
        h_misc[p3::kStatDone] = 1;
        h_misc[p3::kStatError] = 0;
        for (size_t i = 0; i <= n; ++i) cp.h_first[i] = 0;
    }
    p3::Resolve rs = rs3_;
    rs.gen = ++res_gen_;
    FastBatch &rec = fb_[seq % 3];
    rec = FastBatch{};  // (live only once every launch is enqueued, below)
    rec.resolved = true;
    rec.ovl = ovl;
    rec.slot = slot;
    rec.h = hb;
    rec.n = n;
    rec.first = first;
    rec.seq = seq;
    rec.bytes = bytes;
    rec.spans = spans;
    hipEvent_t *ev = tev_[seq % kTimeRing];
    tev_timed_[seq % kTimeRing] = timed;
    rec.timed = timed;
    if (timed) HIP_TRY(hipEventRecord(ev[0], s));
    if (!ovl) {
        if (spans)
            HIP_TRY(p3::launch_scan(st, fp_, d_gear_, f.cand, cp, zero_copy ? h_tails : f.d_tails, f.n_tails,
                                    num_cus_, s));
        if (timed) HIP_TRY(hipEventRecord(ev[1], s));
        if (spans) HIP_TRY(p3::launch_resolve(st, fp_, d_gear_, f.cand, ch3_, cp, rs, d_out, out_cap, s));
        if (timed) HIP_TRY(hipEventRecord(ev[2], s));
    } else {
        // The resolve goes to the second stream behind this scan's event, so
        // it runs beside the NEXT batch's scan (the overlap set fits one
        // resolve block next to each CU's scan block).  Resolves stay in order
        // on that stream (the look-back descriptors and the spilled chunk
        // starts are shared).  No wait guards the device slot: its previous
        // user, batch seq - kSlots, is complete -- batch seq - kHostSlots was
        // collected above (or by a drain), and resolves retire in order.
        static_assert(kSlots > kHostSlots, "device slots must outlast the host blocks");
        if (spans && ovl_std_)
            HIP_TRY(p3::launch_scan(st, fp_, d_gear_, f.cand, cp, zero_copy ? h_tails : f.d_tails, f.n_tails,
                                    num_cus_, s));
        else if (spans)
            HIP_TRY(p3::ovl::launch_scan(st, fp_, d_gear_, f.cand, cp, zero_copy ? h_tails : f.d_tails, f.n_tails,
                                         num_cus_, s));
        if (timed) HIP_TRY(hipEventRecord(ev[1], s));
        HIP_TRY(hipEventRecord(scan_ev_[slot], s));
        HIP_TRY(hipStreamWaitEvent(res_stream_, scan_ev_[slot], 0));
        if (spans && ovl_std_)
            HIP_TRY(p3::launch_resolve(st, fp_, d_gear_, f.cand, ch3_, cp, rs, d_out, out_cap, res_stream_));
        else if (spans)
            HIP_TRY(p3::ovl::launch_resolve(st, fp_, d_gear_, f.cand, ch3_, cp, rs, d_out, out_cap, res_stream_));
        if (timed) HIP_TRY(hipEventRecord(ev[2], res_stream_));
        // (an untimed batch's own end marker on the resolve stream, where an
        // event costs the scans nothing: a slow collection waits for this
        // batch, not for the later resolves already queued behind it)
        else HIP_TRY(hipEventRecord(res_done_[seq % 3], res_stream_));
    }
    rec.live = true;
    fb_seq_ = seq + 1;
    fast_batches_ = fb_seq_;
    fb_any_ = true;
    fb_stream_ = s;
    fb_ovl_ = ovl;
    cand_ = f.cand;
    last_spans_ = spans;
    return 0;
}

// Every batch in flight collected in order.  Returns the last batch's chunk
// count.
int64_t Engine::fast_drain() {
    if (!fb_any_) return 0;
    if (wk_any_) return walk_drain();
    const uint64_t last = fb_seq_ - 1;
    int rc = CDC_OK;
    int64_t total = 0;
    for (uint64_t q = last >= 2 ? last - 2 : 0; q <= last; ++q) {
        FastBatch &b = fb_[q % 3];
        if (!b.live || b.seq != q) continue;
        const int r = rc ? rc : fast_collect((int)(q % 3));
        b.live = false;
        if (r && !rc) rc = r;
        if (q == last && !rc) total = (int64_t)b.first[b.n];
    }
    if (fb_ovl_) {
        // later work on the caller's stream is ordered after the resolves
        if (!rc && hipEventRecord(res_ev_, res_stream_) == hipSuccess)
            (void)hipStreamWaitEvent(fb_stream_, res_ev_, 0);
        else
            (void)hipStreamSynchronize(res_stream_);
    }
    if (rc) (void)hipStreamSynchronize(fb_stream_);  // (nothing of a failed pipeline stays in flight)
    fb_any_ = false;
    return rc ? rc : total;
}

// Wait for batch record k's resolve (its last block writes the done word into
// coherent pinned memory after a system-scope fence: spin on it, then the
// batch's end event), check it and hand first[] to the caller.
int Engine::fast_collect(int k) {
    FastBatch &b = fb_[k];
    if (!b.resolved) {
        set_error("internal: FastCDC batch collected before its resolve was enqueued");
        return CDC_EDEVICE;
    }
    uint64_t *h_misc = b.h + 4 * h_stage_streams_;
    {
        const volatile uint64_t *done = h_misc + p3::kStatDone;
        // (two streams: a batch's resolve runs after the NEXT batch's scan, so
        // its done word comes about a step later)
        const uint64_t us = b.ovl ? std::min<uint64_t>(4000, std::max<uint64_t>(200, b.bytes / 1000000))
                                  : std::min<uint64_t>(2000, std::max<uint64_t>(100, b.bytes / 2000000));
        const auto budget = std::chrono::microseconds(us);
        const auto t_spin = std::chrono::steady_clock::now();
        while (*done == ~0ull && std::chrono::steady_clock::now() - t_spin < budget) __builtin_ia32_pause();
    }
    if (h_misc[p3::kStatDone] == ~0ull) {  // (slow batch or a failure: wait for the stream itself)
        if (b.timed) HIP_TRY(hipEventSynchronize(tev_[b.seq % kTimeRing][2]));
        else if (b.ovl) HIP_TRY(hipEventSynchronize(res_done_[b.seq % 3]));
        else HIP_TRY(hipStreamSynchronize(fb_stream_));
    }
    b.live = false;
    if (h_misc[p3::kStatDone] != 1 || h_misc[p3::kStatError] != 0) {
        set_error(h_misc[p3::kStatDone] != 1 ? "resolve kernel did not report back"
                                             : "chain overflow, output bound or look-back timeout (internal error)");
        return CDC_EDEVICE;
    }
    if (fp_.diag & 64) {  // resolve block spans (100 MHz stamps -> us)
        const uint64_t *d = h_misc + p3::kStatDiag0;
        const uint64_t s0 = ~d[0], s1 = d[1], e1 = d[2], e0 = ~d[3];
        const double blocks =
            (double)(b.ovl && !ovl_std_ ? p3::ovl::resolve_blocks(b.spans) : p3::resolve_blocks(b.spans));
        std::fprintf(stderr, "resolve blocks, us: scan's last block end -> first start %.2f  starts spread %.2f  "
                             "first start -> first end %.2f  -> last end %.2f  longest block %.2f  mean block %.2f\n",
                     ((double)s0 - (double)d[6]) / 100.0, (s1 - s0) / 100.0, (e0 - s0) / 100.0, (e1 - s0) / 100.0,
                     d[4] / 100.0, d[5] / 100.0 / (blocks ? blocks : 1.0));
    } else if (fp_.diag & 128) {
        const double waves = b.ovl && !ovl_std_ ? (double)p3::ovl::resolve_blocks(b.spans) * 4
                                                : (double)p3::resolve_blocks(b.spans) * 8;
        std::fprintf(stderr, (fp_.diag & 8192) ? "resolve link passes, us per wave (records: issue trunc link; "
                                                 "virtual: issue trunc link; -; -):"
                                               : "resolve phases, us per wave (meta recs settle+wait virtual-links "
                                                 "record-links walk lookback(w0) out):");
        for (int i = 0; i < p3::kStatDiagN; ++i)
            std::fprintf(stderr, " %.2f", (double)h_misc[p3::kStatDiag0 + i] / 100.0 / (waves ? waves : 1.0));
        std::fprintf(stderr, "\n");
    }
    // Zero-length streams own no span: their first[] is the next stream's.
    const uint64_t *lens = b.h + h_stage_streams_;
    uint64_t *hf = h_misc + p3::kStatWords;
    for (size_t i = b.n; i-- > 0;)
        if (lens[i] == 0) hf[i] = hf[i + 1];
    std::memcpy(b.first, hf, (b.n + 1) * 8);
    const double hash_ms = timing_.hash_ms;
    timing_ = cdc_timing_t{};
    timing_.hash_ms = hash_ms;
    timing_.bytes = b.bytes;
    timing_.candidates = h_misc[p3::kStatCand];
    timing_.overflow_spans = (uint32_t)h_misc[p3::kStatOvf];
    timing_.fixup_iterations = (uint32_t)h_misc[p3::kStatRewalk];
    timing_.walk_fallback_steps = h_misc[p3::kStatOnDemand];
    timing_.path = CDC_PATH_PIPELINE;
    timing_.timed = b.timed ? 1u : 0u;
    timing_pending_ = true;
    timing_seq_ = b.seq;
    return CDC_OK;
}

bool Engine::small_ok(uint64_t len) const {
    // ~len / 2^pmin records expected: keep well inside the kernel's record budget
    return small_on_ && len > 0 && len <= small::kMaxBytes && (len >> small_pmin_) <= small::kRecCap * 5 / 8;
}

int Engine::run_small(const uint8_t *data, uint64_t len, cdc_chunk_t *d_out, size_t out_cap, uint64_t *first,
                      hipStream_t s, bool host_input, const uint8_t *feed_src, uint8_t *feed_dst,
                      uint32_t feed_slot) {
    if (!small_mem_) {
        HIP_TRY(hipMalloc(&small_mem_, small::scratch_bytes() + small::copy_bytes() + small::bstamp_bytes()));
        HIP_TRY(hipMemset(small_mem_, 0, small::scratch_bytes()));  // the ticket starts at 0
        uint32_t *b = static_cast<uint32_t *>(small_mem_);
        small_ws_.brec = reinterpret_cast<uint64_t *>(b);
        small_ws_.bcnt = b + 2 * small::kMaxBlocks * small::kBlockRecCap;
        small_ws_.ticket = small_ws_.bcnt + small::kMaxBlocks;
        small_ws_.stamp = reinterpret_cast<uint64_t *>(static_cast<char *>(small_mem_) + small::scratch_bytes() - 64);
        small_ws_.bpub = small_ws_.stamp - small::kMaxBlocks;
        small_ws_.copy = static_cast<uint8_t *>(small_mem_) + small::scratch_bytes();
        small_ws_.bstamp = reinterpret_cast<uint64_t *>(small_ws_.copy + small::copy_bytes());
    }
    uint64_t *h = static_cast<uint64_t *>(h_stage_);
    uint64_t *h_misc = h + 4 * h_stage_streams_;  // (the regular path's stats ++ first[] area)
    uint64_t *h_first = h_misc + p3::kStatWords;
    volatile uint64_t *done = h_misc + small::kWordDone;
    *done = 0;
    small_seq_ = small_seq_ % 0xFFFFFFFEull + 1;  // 1 .. 2^32 - 2 (tags: seq << 32 | count)
    const small::Feed feed{feed_src ? h_ready_dev_ + (size_t)feed_slot * small::kFeedPieces : nullptr, small_seq_};
    auto feed_copy = [&]() {
        const auto tc = std::chrono::steady_clock::now();
        volatile uint64_t *ready = h_ready_ + (size_t)feed_slot * small::kFeedPieces;
        if (small_feed_pool_) {
            // the calling thread and whichever copy-pool helpers are awake
            // claim the pieces (work stealing: never a wait for a sleeper)
            pool_->copy_feed(feed_dst, feed_src, len, size_t(1) << small::kFeedLog2, ready, small_seq_);
        } else {
            // (A/B: the calling thread alone)
            const uint64_t piece = 1ull << small::kFeedLog2;
            for (uint64_t off = 0; off < len; off += piece) {
                std::memcpy(feed_dst + off, feed_src + off, std::min(piece, len - off));
                std::atomic_thread_fence(std::memory_order_release);  // (x86: stores stay in order)
                ready[off >> small::kFeedLog2] = small_seq_;
            }
        }
        small_copy_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - tc).count();
    };
    if (feed_src && small_feed_ == 2) feed_copy();  // (A/B: the feed copy first)
    HIP_TRY(small::launch_small(data, len, fp_, d_gear_, small_ws_, d_out, out_cap, h_misc, h_first, host_input,
                                feed, s));
    ++small_calls_;
    if (feed_src && small_feed_ != 2) {
        // The kernel is on its way (launch latency overlaps the copy): the
        // copy pool writes the bytes piece by piece, each announced by its
        // feed word once in memory.
        feed_copy();
    }
    // The last block writes the done word after a system-scope release: spin on
    // it (a call is ~20-60 us of device time), then the stream sync confirms.
    const auto t_spin = std::chrono::steady_clock::now();
    while (*done == 0 && std::chrono::steady_clock::now() - t_spin < std::chrono::microseconds(2000))
        __builtin_ia32_pause();
    if (*done == 0) HIP_TRY(hipStreamSynchronize(s));
    if (*done != 1) {
        set_error("small FastCDC kernel did not report back");
        return CDC_EDEVICE;
    }
    timing_pending_ = false;
    timing_.candidates = h_misc[small::kWordRecords];
    timing_.overflow_spans = 0;
    timing_.fixup_iterations = 0;
    timing_.walk_fallback_steps = 0;
    if (fp_.diag & small::kDiagStamps) {
        const uint64_t *t = h_misc + small::kWordStamp0;
        std::fprintf(stderr, "small: %llu B, us from block 0's start: last block %.2f, records %.2f, links %.2f "
                             "(%llu rounds), walk %.2f, output %.2f\n",
                     (unsigned long long)len, (t[1] - t[0]) / 100.0, (t[2] - t[0]) / 100.0, (t[3] - t[0]) / 100.0,
                     (unsigned long long)t[7], (t[4] - t[0]) / 100.0, (t[5] - t[0]) / 100.0);
        std::fprintf(stderr, "  round 0 max cycles per lane: load+trunc %llu, link %llu, successor %llu; rounds end at",
                     (unsigned long long)(t[6] & 0x1FFFFF), (unsigned long long)((t[6] >> 21) & 0x1FFFFF),
                     (unsigned long long)(t[6] >> 42));
        for (int k = 0; k < 4; ++k)
            if (h_first[2 + k]) std::fprintf(stderr, " %.2f", (h_first[2 + k] - t[0]) / 100.0);
        if (feed_src) std::fprintf(stderr, "; block 0 fed at %.2f; host copy %.2f us", (h_first[6] - t[0]) / 100.0,
                                   small_copy_s_ * 1e6);
        std::fprintf(stderr, "; round 0 added %llu entries, round 1 worked on %llu", (unsigned long long)(h_first[7] & 0xFFFF),
                     (unsigned long long)(h_first[7] >> 16));
        std::fprintf(stderr, "\n");
        // per-block stamps: min / median / max of start, fed, bytes in LDS, ticket
        const uint32_t G = (uint32_t)((len + small::kBlockBytes - 1) / small::kBlockBytes);
        std::vector<uint64_t> bs((size_t)G * 8);
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(hipMemcpy(bs.data(), small_ws_.bstamp, bs.size() * 8, hipMemcpyDeviceToHost));
        const char *nm[6] = {"fed", "loaded", "hashed(w0)", "tinfo(w0)", "drained", "ticket"};
        std::fprintf(stderr, "  blocks (%u):", G);
        for (int k = 0; k < 6; ++k) {
            std::vector<double> v;
            for (uint32_t b = 0; b < G; ++b) v.push_back(((double)bs[b * 8 + k] - (double)t[0]) / 100.0);
            std::sort(v.begin(), v.end());
            std::fprintf(stderr, " %s %.2f/%.2f/%.2f", nm[k], v.front(), v[v.size() / 2], v.back());
        }
        std::fprintf(stderr, "\n");
    }
    if (h_misc[small::kWordFallback]) {
        ++small_fallbacks_;
        return kSmallFallback;
    }
    first[0] = 0;
    first[1] = h_first[1];
    return CDC_OK;
}

// FastCDC batch events: [0] before its scan launch, [1] after it (before the
// resolve), [2] after the resolve.
const cdc_timing_t &Engine::timing() {
    if (fb_any_) (void)drain_implicit();  // (a failure is held for the next cdc_batch_sync)
    if (timing_pending_) {
        timing_pending_ = false;
        (void)timing_back((uint32_t)(fast_batches_ - 1 - timing_seq_), timing_);
    }
    return timing_;
}

int Engine::timing_back(uint32_t back, cdc_timing_t &out) {
    if (fb_any_) (void)drain_implicit();
    if (algo_ != CDC_ALGO_FASTCDC || back >= kTimeRing || back >= fast_batches_) {
        set_error("cdc_debug_timing_back: no such FastCDC batch in the event ring");
        return CDC_EINVAL;
    }
    if (&out != &timing_) out = timing_;
    hipEvent_t *ev = tev_[(fast_batches_ - 1 - back) % kTimeRing];
    float t01 = 0, t12 = 0, t02 = 0;
    HIP_TRY(hipSetDevice(device_));
    out.path = CDC_PATH_PIPELINE;
    out.timed = tev_timed_[(fast_batches_ - 1 - back) % kTimeRing] ? 1u : 0u;
    if (!out.timed) {  // an async batch recorded without events
        out.scan_ms = out.resolve_ms = out.total_ms = 0;
        return CDC_OK;
    }
    HIP_TRY(hipEventSynchronize(ev[2]));
    HIP_TRY(hipEventElapsedTime(&t01, ev[0], ev[1]));
    HIP_TRY(hipEventElapsedTime(&t12, ev[1], ev[2]));
    HIP_TRY(hipEventElapsedTime(&t02, ev[0], ev[2]));
    out.scan_ms = t01;
    out.resolve_ms = t12;
    out.total_ms = t02;
    return CDC_OK;
}

int Engine::run_fixed(const StreamTable &st, size_t n, const uint64_t *lens,
                      cdc_chunk_t *d_out, uint64_t *first, hipStream_t s) {
    uint64_t *h = static_cast<uint64_t *>(h_stage_);
    uint64_t *h_first = h + 4 * h_stage_streams_;
    uint64_t t = 0;
    for (size_t i = 0; i < n; ++i) {
        h_first[i] = t;
        t += (lens[i] + min_ - 1) / min_;  // fixed_size.rs:35-40: ceil(len/cs) chunks
    }
    h_first[n] = t;
    HIP_TRY(hipEventRecord(ev_[0], s));
    HIP_TRY(hipMemcpyAsync(d_first_, h_first, (n + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_fixed(st, min_, d_first_, d_out, t, s));
    HIP_TRY(hipEventRecord(ev_[3], s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(first, h_first, (n + 1) * 8);
    float t03 = 0;
    HIP_TRY(hipEventElapsedTime(&t03, ev_[0], ev_[3]));
    timing_.total_ms = t03;
    timing_.scan_ms = t03;
    timing_.path = CDC_PATH_FIXED;
    timing_.timed = 1;
    return CDC_OK;
}

int64_t Engine::fs_write(const uint8_t *data, size_t len, size_t seg_size, std::vector<uint64_t> &spans,
                         double *seconds) {
    spans.clear();
    if (seg_size == 0) {
        set_error("cdc_fs_write: seg_size must be > 0");
        return CDC_EINVAL;
    }
    if (len && !data) {
        set_error("cdc_fs_write: data is NULL");
        return CDC_EINVAL;
    }
    // ChunkStorage::write (storage.rs:84-100): StorageWriter::write per
    // seg_size slice, then flush -- through the streaming write path.
    int rc = write_begin();
    if (rc) return rc;  // (e.g. a streaming write in progress: left alone)
    for (size_t off = 0; !rc && off < len; off += seg_size)
        rc = write_segment(data + off, std::min(seg_size, len - off));
    if (rc) {
        wr_.active = false;
        return rc;
    }
    return write_finish(spans, seconds);
}

int Engine::sha256_device(const uint8_t *d_data, const cdc_chunk_t *d_chunks, size_t n,
                          uint8_t *d_digests, hipStream_t s) {
    const uint64_t first[2] = {0, n};
    return sha256_batch(1, &d_data, first, d_chunks, d_digests, s);
}

// One launch over every chunk of every stream (sha256.hip); the stream table
// (first[], bases) goes up through a pinned block with one H2D copy.
int Engine::sha256_batch(size_t n, const uint8_t *const *d_streams, const uint64_t *first,
                         const cdc_chunk_t *d_chunks, uint8_t *d_digests, hipStream_t s) {
    if (n == 0) return CDC_OK;
    if (!d_streams || !first) {
        set_error("cdc_sha256_batch_device: NULL stream table");
        return CDC_EINVAL;
    }
    if (first[0] != 0) {
        set_error("cdc_sha256_batch_device: first[0] must be 0");
        return CDC_EINVAL;
    }
    for (size_t i = 0; i < n; ++i) {
        if (first[i + 1] < first[i]) {
            set_error("cdc_sha256_batch_device: first[] must be non-decreasing");
            return CDC_EINVAL;
        }
        if (first[i + 1] > first[i] && !d_streams[i]) {
            set_error("cdc_sha256_batch_device: NULL stream with chunks");
            return CDC_EINVAL;
        }
    }
    const uint64_t total = first[n];
    if (total >= (1ull << 32)) {
        set_error("cdc_sha256_batch_device: more than 2^32 - 1 chunks in one batch");
        return CDC_EINVAL;
    }
    if (total && (!d_chunks || !d_digests)) {
        set_error("cdc_sha256_chunks_device: NULL argument");
        return CDC_EINVAL;
    }
    HIP_TRY(hipSetDevice(device_));
    if (fb_any_) {  // (the chunks it hashes are usually the last batch's)
        const int64_t r = drain_implicit();
        if (r < 0) return (int)r;
    }
    hipStream_t st = s ? s : own_stream_;
    (void)timing();  // the last batch's events, before ev_[2] is re-recorded
    if (total == 0) {
        timing_.hash_ms = 0;
        return CDC_OK;
    }
    const size_t words = 2 * n + 1;
    if (sha_tab_cap_ < words) {
        (void)hipFree(d_sha_tab_);
        (void)hipHostFree(h_sha_tab_);
        d_sha_tab_ = h_sha_tab_ = nullptr;
        sha_tab_cap_ = 0;
        const size_t want = words + 64;
        HIP_TRY(hipMalloc(&d_sha_tab_, want * 8));
        HIP_TRY(hipHostMalloc(&h_sha_tab_, want * 8, hipHostMallocDefault));
        sha_tab_cap_ = want;
    }
    std::memcpy(h_sha_tab_, first, (n + 1) * 8);
    for (size_t i = 0; i < n; ++i) h_sha_tab_[n + 1 + i] = reinterpret_cast<uint64_t>(d_streams[i]);
    HIP_TRY(hipMemcpyAsync(d_sha_tab_, h_sha_tab_, words * 8, hipMemcpyHostToDevice, st));
    ShaBatch b{};
    b.chunks = reinterpret_cast<const cdc_chunk_pod *>(d_chunks);
    b.n_chunks = total;
    b.first = d_sha_tab_;
    b.base = d_sha_tab_ + n + 1;
    b.n_streams = (uint32_t)n;
    b.digests = reinterpret_cast<uint32_t *>(d_digests);
    b.counter = d_counter_;
    if (sha_order_cap_ < total) {
        (void)hipFree(d_sha_order_);
        d_sha_order_ = nullptr;
        sha_order_cap_ = 0;
        const uint64_t want = total + total / 8 + 1024;
        HIP_TRY(hipMalloc(&d_sha_order_, want * sizeof(uint32_t)));
        sha_order_cap_ = want;
    }
    b.order = d_sha_order_;
    HIP_TRY(hipEventRecord(ev_[3], st));
    HIP_TRY(launch_sha256(b, num_cus_, st));
    HIP_TRY(hipEventRecord(ev_[2], st));
    HIP_TRY(hipStreamSynchronize(st));  // (also: the pinned table may be rewritten by the next call)
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ev_[3], ev_[2]));
    timing_.hash_ms = ms;
    return CDC_OK;
}

int64_t Engine::debug_copy(int what, void *out, size_t max_bytes) {
    if (fb_any_) {
        const int64_t r = drain_implicit();
        if (r < 0) return r;
    }
    if (algo_ != CDC_ALGO_FASTCDC || !ws_) {
        set_error("debug_copy: no FastCDC batch yet");
        return CDC_EINVAL;
    }
    const void *src = nullptr;
    size_t bytes = 0;
    if (what == 0) {
        src = cand_.count;
        bytes = last_spans_ * 4;
    } else if (what == 1) {
        src = cand_.pos;
        bytes = last_spans_ * cap_ * 4;
    } else {
        set_error("debug_copy: unknown array");
        return CDC_EINVAL;
    }
    if (bytes > max_bytes) bytes = max_bytes;
    HIP_TRY(hipSetDevice(device_));
    HIP_TRY(hipStreamSynchronize(own_stream_));
    if (bytes) HIP_TRY(hipMemcpy(out, src, bytes, hipMemcpyDeviceToHost));
    return (int64_t)bytes;
}

int Engine::read_bw(const uint8_t *d_buf, size_t len, int reps, double *ms) {
    HIP_TRY(hipSetDevice(device_));
    if (fb_any_) {
        const int64_t r = drain_implicit();
        if (r < 0) return (int)r;
    }
    uint64_t *d_acc = nullptr;
    const size_t words = (size_t)num_cus_ * 8;
    HIP_TRY(hipMalloc(&d_acc, words * 8));
    hipError_t e = hipMemsetAsync(d_acc, 0, words * 8, own_stream_);
    if (e == hipSuccess) e = launch_read_reduce(d_buf, len, d_acc, num_cus_, own_stream_);  // (warm-up)
    if (e == hipSuccess) e = hipEventRecord(ev_[0], own_stream_);
    for (int r = 0; e == hipSuccess && r < reps; ++r) e = launch_read_reduce(d_buf, len, d_acc, num_cus_, own_stream_);
    if (e == hipSuccess) e = hipEventRecord(ev_[3], own_stream_);
    if (e == hipSuccess) e = hipEventSynchronize(ev_[3]);
    float t = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, ev_[0], ev_[3]);
    (void)hipFree(d_acc);
    if (e != hipSuccess) {
        set_error(std::string("read_bw: ") + hipGetErrorString(e));
        return CDC_EDEVICE;
    }
    *ms = (double)t / reps;
    return CDC_OK;
}

int Engine::fill_splitmix64(uint8_t *d_buf, size_t len, uint64_t seed, hipStream_t s) {
    HIP_TRY(hipSetDevice(device_));
    hipStream_t st = s ? s : own_stream_;
    HIP_TRY(launch_fill_splitmix64(d_buf, len, seed, st));
    HIP_TRY(hipStreamSynchronize(st));
    return CDC_OK;
}

// ---- Rabin / UltraCDC / LeapCDC / SeqCDC: the segment-walk engine ----------

namespace {
// GF(2) remainder modulo the Rabin polynomial (host-side table build).
uint64_t gf2_mod(uint64_t x, uint64_t p) {
    const int dp = 63 - __builtin_clzll(p);
    while (x) {
        const int dx = 63 - __builtin_clzll(x);
        if (dx < dp) break;
        x ^= p << (dx - dp);
    }
    return x;
}

uint64_t splitmix_word(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
}  // namespace

int Engine::create_seq(const uint32_t seq[4], uint32_t min, uint32_t avg, uint32_t max, int device,
                       Engine **out) {
    if (!seq) {
        set_error("cdc_create_seq: config is NULL");
        return CDC_EINVAL;
    }
    return create_walk(CDC_ALGO_SEQ, seq, min, avg, max, device, out);
}

int Engine::create_walk(cdc_algo_t algo, const uint32_t seq[4], uint32_t min, uint32_t avg, uint32_t max,
                        int device, Engine **out) {
    if (!out) {
        set_error("cdc_create: out is NULL");
        return CDC_EINVAL;
    }
    *out = nullptr;
    // Size rules (oracle_cdc_check): 0 < min <= avg <= max, and the
    // bytes each rule reads before the first tested position.
    if (min == 0 || min > avg || avg > max || (algo == CDC_ALGO_ULTRA && min < 8) ||
        (algo == CDC_ALGO_LEAP && min < 32) || (algo == CDC_ALGO_RABIN && avg < 2)) {
        set_error("invalid sizes: need 0 < min <= avg <= max (UltraCDC min >= 8, LeapCDC min >= 32)");
        return CDC_EINVAL;
    }
    if (algo == CDC_ALGO_SEQ && (seq[0] > 1 || seq[1] == 0 || seq[2] == 0 || seq[3] == 0)) {
        set_error("invalid SeqCDC config: mode 0/1, seq_length > 0, jump_trigger > 0, jump_size > 0");
        return CDC_EINVAL;
    }
    Engine *e = new Engine();
    e->algo_ = algo;
    e->min_ = min;
    e->avg_ = avg;
    e->max_ = max;
    e->device_ = device;
    const char *name = algo == CDC_ALGO_RABIN ? "RabinCDC" : algo == CDC_ALGO_ULTRA ? "UltraCDC"
                     : algo == CDC_ALGO_LEAP ? "LeapCDC" : "SeqCDC";
    char buf[256];
    // impl Debug (rabin.rs:28-32, ultra.rs:24-28, leap.rs:24-28, seq.rs:34-38)
    if (algo == CDC_ALGO_SEQ)
        std::snprintf(buf, sizeof buf, "%s, sizes: SizeParams { min: %u, avg: %u, max: %u }, mode: %s [MI355X gfx950]",
                      name, min, avg, max, seq[0] ? "Decreasing" : "Increasing");
    else
        std::snprintf(buf, sizeof buf, "%s, sizes: SizeParams { min: %u, avg: %u, max: %u } [MI355X gfx950]", name,
                      min, avg, max);
    e->describe_ = buf;
    for (int i = 0; i < 4; ++i) e->seq_cfg_[i] = seq[i];
    if (const char *v = std::getenv("CHUNKFS_AMD_WALK_ASYNC")) e->walk_async_ = std::atoi(v) != 0;
    if (const char *v = std::getenv("CHUNKFS_AMD_WALK_CTX")) e->walk_ctx_ = std::max(2, std::min(kWalkCtxMax, std::atoi(v)));
    int rc = e->init();
    if (rc == CDC_OK) rc = e->init_walk(seq);
    if (rc != CDC_OK) {
        delete e;
        return rc;
    }
    *out = e;
    return CDC_OK;
}

int Engine::init_walk(const uint32_t *seq) {
    walk::WalkParams &wp = wp_;
    wp.algo = (uint32_t)algo_;
    wp.min = min_;
    wp.avg = avg_;
    wp.max = max_;
    wp.rabin_mask = (1ull << cdc_log2_round(avg_)) - 1;

    const uint64_t lspan = avg_ > min_ ? (uint64_t)(avg_ - min_) : 1;
    const uint32_t lb = cdc_log2_round(lspan);
    wp.leap_thr = CDC_LEAP_THRESHOLD[lb > 32 ? 32 : lb];
    wp.seq_mode = seq[0];
    wp.seq_len = seq[1];
    wp.seq_trig = seq[2];
    wp.seq_jump = seq[3];
    // Segments of 2^seg_log2 bytes (one lane each) and a warm-up of `warm`
    // bytes; CHUNKFS_AMD_WALK="seg_log2,warm_over_avg" overrides (experiments).
    // Defaults (tools/walk_bench.py sweeps on MI355X): segments of
    // 32 KiB whatever the average (at avg 64 KiB, 32 KiB segments beat 256 KiB
    // ones for every rule: more lanes, a shorter walk per lane and cheaper
    // fix-up re-walks; profiles/r02ak_walk_avg64k_segments.log), a warm-up of
    // 8 avg (a chain from an arbitrary start merges with the true one within a
    // few content-defined cuts).
    // Bitmap mode: Rabin when every tested digest is a full
    // window (min >= 48), UltraCDC, LeapCDC, and SeqCDC when its run length
    // fits a 64-bit step (seq_length <= 63).  CHUNKFS_AMD_WALK_BYTES=1 forces
    // the byte walks (A/B experiments).
    wp.nbm = algo_ == CDC_ALGO_RABIN ? (min_ >= CDC_RABIN_WINDOW ? 1u : 0u)
           : algo_ == CDC_ALGO_ULTRA ? 3u : algo_ == CDC_ALGO_LEAP ? 2u
           : (wp.seq_len <= 63 ? 1u : 0u);
    if (const char *b = std::getenv("CHUNKFS_AMD_WALK_BYTES"))
        if (std::atoi(b) != 0) wp.nbm = 0;
    // Wave-cooperative walks (walk.hip wwalk_kernel, one wave per segment)
    // for every rule in bitmap mode.  CHUNKFS_AMD_WAVE=0 disables.
    wp.wave = wp.nbm ? 1u : 0u;
    if (const char *v = std::getenv("CHUNKFS_AMD_WAVE")) wp.wave = wp.wave && std::atoi(v) != 0;
    // Lane walks: 32 KiB segments whatever the average (profiles/r02ak).
    // Wave walks: 128 KiB (Rabin, Leap) / 256 KiB segments, 8 avg warm-up
    // (profiles/r03_walk/r03w_walk_seg_sweep.txt: a wave walks thousands of
    // positions per step, so fewer, longer segments cut the warm-up share).
    // Warm-up, in averages: chains from an arbitrary start merge within a few
    // content-defined cuts.  Lane walks: 8 avg, SeqCDC 16
    // (profiles/r02ag_walk_warm_sweep.log).  Wave walks: Rabin 8, UltraCDC and
    // SeqCDC 16, LeapCDC 24 (its chains merge slowest; the fix-up rounds a
    // shorter warm-up leaves cost more than the walk it saves,
    // profiles/r03_walk/r03ab_walk_warm_ahead_sweep.txt).
    uint64_t warm_mult = !wp.wave ? (algo_ == CDC_ALGO_SEQ ? 16 : 8)
                       : algo_ == CDC_ALGO_RABIN ? 8 : algo_ == CDC_ALGO_LEAP ? 24 : 16;
    // Segments: lane walks 32 KiB whatever the average (profiles/r02ak).  Wave
    // walks: at least 128 KiB (Rabin) / 256 KiB and at least the warm-up, so
    // that the warm-up stays a fraction of each wave's walk (a wave walks
    // thousands of positions per step; r03w_walk_seg_sweep.txt), up to 4 MiB.
    seg_log2_ = !wp.wave ? 15 : algo_ == CDC_ALGO_RABIN ? 17 : 18;
    if (wp.wave) {
        const uint32_t wl = ceil_log2(warm_mult * avg_);
        if (wl > seg_log2_) seg_log2_ = wl < 22 ? wl : 22;
    }
    // The per-segment start list holds segment/min + 2 entries: keep it <= ~4k
    // (tiny min), and segments >= 4 KiB.
    const uint32_t lmin = 63 - (uint32_t)__builtin_clzll((uint64_t)min_) + 12;
    if (seg_log2_ > lmin) seg_log2_ = lmin < 12 ? 12 : lmin;
    if (const char *w = std::getenv("CHUNKFS_AMD_WALK")) {
        unsigned a = 0, b = 0;
        if (std::sscanf(w, "%u,%u", &a, &b) == 2 && a >= 10 && a <= 30) {
            seg_log2_ = a;
            warm_mult = b;
        }
    }
    wp.warm = warm_mult * avg_;
    // CHUNKFS_AMD_AHEAD="after,max" overrides the run-ahead schedule (experiments).
    if (const char *a = std::getenv("CHUNKFS_AMD_AHEAD")) {
        unsigned x = 0, y = 0;
        if (std::sscanf(a, "%u,%u", &x, &y) == 2 && y >= 1) {
            ahead_after_ = x;
            ahead_max_ = y;
        }
    }
    wp.ahead = 1;
    wp.bits_fine = 1;
    if (const char *f = std::getenv("CHUNKFS_AMD_BITS_FINE")) wp.bits_fine = std::atoi(f) != 0 ? 1u : 0u;
    if (const char *f = std::getenv("CHUNKFS_AMD_WALK_FUSED")) walk_fused_ = std::atoi(f) != 0;
    wp.cap = (uint32_t)((1ull << seg_log2_) / min_ + 2);
    // Link mode (Rabin, UltraCDC, LeapCDC): candidate lists of ~4x
    // the expected count per segment -- Rabin hits 2^-round(log2 avg) per
    // position, UltraCDC mask_l hits ~2^-11 (Hamming distance 16..19 of 64),
    // LeapCDC eligible-window runs ~2^-round(log2(avg - min));
    // CHUNKFS_AMD_LINKS=0 disables.  (SeqCDC's candidates -- completed runs --
    // are too dense: it keeps direct walks.)
    // Default on where it measured faster (1 GiB, 4/8/16 KiB: UltraCDC 223 ->
    // 252 GiB/s; Rabin 573 -> 520 and LeapCDC 153 -> 143 lose).
    const bool linkable = algo_ == CDC_ALGO_RABIN || algo_ == CDC_ALGO_ULTRA || algo_ == CDC_ALGO_LEAP;
    wp.links = algo_ == CDC_ALGO_ULTRA ? 1u : 0u;
    if (const char *l = std::getenv("CHUNKFS_AMD_LINKS")) wp.links = std::atoi(l) != 0 && linkable;
    {
        const uint32_t dens = algo_ == CDC_ALGO_RABIN ? cdc_log2_round(avg_) : algo_ == CDC_ALGO_ULTRA ? 10u : lb;
        const uint64_t expect = ((1ull << seg_log2_) >> dens) + 1;
        uint64_t cc = 16;
        while (cc < 4 * expect && cc < 1024) cc <<= 1;
        wp.ccap = (uint32_t)cc;
    }
    if (!wp.nbm) wp.links = 0;  // links are computed over the bitmaps
    if (wp.wave) wp.links = 0;  // the wave walks replace link mode
    wp.seg_words = (uint32_t)((1ull << seg_log2_) / 64);
    wp.piece_log2 = seg_log2_ < 15 ? seg_log2_ : 15;  // data-parallel passes: 32 KiB pieces
    wp.bm = nullptr;
    HIP_TRY(hipMalloc(&d_wtabs_, 768 * sizeof(uint64_t)));
    wp.tabs = d_wtabs_;
    return load_walk_tables(CDC_RABIN_POLY);
}

// Tables: Rabin mod/out of polynomial P (appending a byte; sliding one out of
// the window), LeapCDC window-hash table; and the digest's top-byte shift.
int Engine::load_walk_tables(uint64_t P) {
    uint64_t t[768];
    const int deg = 63 - __builtin_clzll(P);
    for (uint64_t b = 0; b < 256; ++b) {
        t[b] = gf2_mod(b << deg, P) | (b << deg);
        uint64_t h = b;
        for (uint32_t i = 1; i < CDC_RABIN_WINDOW; ++i) h = gf2_mod(h << 8, P);
        t[256 + b] = h;
        t[512 + b] = splitmix_word(CDC_LEAP_SEED + (b + 1) * 0x9E3779B97F4A7C15ull);
    }
    HIP_TRY(hipSetDevice(device_));
    HIP_TRY(hipMemcpy(d_wtabs_, t, sizeof t, hipMemcpyHostToDevice));
    wp_.rabin_shift = (uint32_t)deg - 8;
    return CDC_OK;
}

int Engine::set_rabin_poly(uint64_t P) {
    if (algo_ != CDC_ALGO_RABIN) {
        set_error("cdc_set_rabin_poly: not a RabinChunker handle");
        return CDC_EINVAL;
    }
    const int deg = P ? 63 - __builtin_clzll(P) : -1;
    if (deg < 9 || deg > 56) {
        set_error("cdc_set_rabin_poly: polynomial degree must be 9..56");
        return CDC_EINVAL;
    }
    if (wr_.active) {  // windows already chunked used the old polynomial: a write never mixes two
        set_error("cdc_set_rabin_poly: a streaming write is in progress (cdc_write_finish it first)");
        return CDC_EINVAL;
    }
    HIP_TRY(hipSetDevice(device_));
    if (fb_any_) {  // the batches in flight finish with the polynomial they were submitted with
        const int64_t r = drain_implicit();
        if (r < 0) return (int)r;
    }
    HIP_TRY(hipStreamSynchronize(own_stream_));
    rabin_poly_ = P;
    for (auto &w : ww_) w.reset();  // (the contexts are made again, with this polynomial)
    // The degree decides the bitmap kernel and whether it writes the quiet-run
    // summary (walk::bits_write_summary): the workspace is laid out again.
    (void)hipFree(wws_);
    wws_ = nullptr;
    wws_segs_ = 0;
    wws_streams_ = 0;
    return load_walk_tables(P);
}

int Engine::ensure_walk_workspace(uint64_t segs, size_t n) {
    if (wws_ && segs <= wws_segs_ && n <= wws_streams_) return CDC_OK;
    const uint64_t S = segs > wws_segs_ ? segs + segs / 4 + 16 : wws_segs_;
    const size_t N = n > wws_streams_ ? n + 64 : wws_streams_;
    const uint64_t nb = S / walk::kScanBlock + 2;
    const size_t A = 256;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align_up(off + bytes, A);
        return o;
    };
    const size_t oE = take(S * 8), oX = take(S * 8), oXs = take(S * 8), oEs = take(S * 8), oP = take((S + 1) * 8);
    const size_t oN = take(S * 4), oL = take(S * (size_t)wp_.cap * 8), oB = take((nb + 1) * 8);
    const size_t oF = take((N + 1) * 8), oG = take((4 + 4 * walk::kMaxFixRounds) * 8), oGo = take(16);
    const size_t oBM = take(S * (size_t)wp_.seg_words * wp_.nbm * 8);  // predicate bitmaps
    const bool jt = algo_ == CDC_ALGO_LEAP && wp_.wave;
    const size_t oJT = take(jt ? S * (size_t)wp_.seg_words * 24 : 0);  // LeapCDC word tables
    const size_t oJ8 = take(jt ? S * (size_t)wp_.seg_words * 6 : 0);   // and 512-position block tables
    bool rsum = walk::bits_write_summary(wp_);  // quiet runs (CHUNKFS_AMD_QUIET=0: off, A/B)
    if (const char *q = std::getenv("CHUNKFS_AMD_QUIET")) rsum = rsum && std::atoi(q) != 0;
    const size_t oRS = take(rsum ? S * (size_t)wp_.seg_words / 8 * (algo_ == CDC_ALGO_RABIN ? 2 : 1) : 0);  // quiet-run summary
    const size_t oQS = take(rsum ? S : 0);  // and per segment
    const size_t cc = wp_.links ? wp_.ccap : 0;                          // link mode
    const size_t oCN = take(S * 4), oCP = take(S * cc * 4), oLN = take(S * cc * 8), oLI = take(S * cc * 4);
    const size_t vc = wp_.links ? S * 8 : 0;
    const size_t oVC = take((2 * walk::kVirtRounds + 2) * 8), oVP = take(vc * 8), oVS = take(vc * 4),
                 oVN = take(vc * 8), oVI = take(vc * 4);
    const size_t o_ptrs = take(N * 8), o_lens = take(N * 8), o_sb = take((N + 1) * 8);
    (void)hipFree(wws_);
    wws_ = nullptr;
    wws_segs_ = 0;
    wws_streams_ = 0;
    HIP_TRY(hipMalloc(&wws_, off));
    ++ws_gen_;  // the stream tables move: re-upload them
    wws_segs_ = S;
    wws_streams_ = N;
    char *b = static_cast<char *>(wws_);
    wst_.E = reinterpret_cast<uint64_t *>(b + oE);
    wst_.X = reinterpret_cast<uint64_t *>(b + oX);
    wst_.Xs = reinterpret_cast<uint64_t *>(b + oXs);
    wst_.Es = reinterpret_cast<uint64_t *>(b + oEs);
    wst_.P = reinterpret_cast<uint64_t *>(b + oP);
    wst_.N = reinterpret_cast<uint32_t *>(b + oN);
    wst_.list = reinterpret_cast<uint64_t *>(b + oL);
    wst_.bsum = reinterpret_cast<uint64_t *>(b + oB);
    wst_.first = reinterpret_cast<uint64_t *>(b + oF);
    wst_.flags = reinterpret_cast<unsigned long long *>(b + oG);
    walk_go_ = reinterpret_cast<uint64_t *>(b + oGo);
    walk_flags_clean_ = false;  // (fresh memory: the next call initialises the flag blocks)
    wp_.bm = wp_.nbm ? reinterpret_cast<uint64_t *>(b + oBM) : nullptr;
    wp_.jt = jt ? reinterpret_cast<uint8_t *>(b + oJT) : nullptr;
    wp_.jt8 = jt ? reinterpret_cast<uint16_t *>(b + oJ8) : nullptr;
    wp_.rsum = rsum ? reinterpret_cast<uint64_t *>(b + oRS) : nullptr;
    wp_.qseg = rsum ? reinterpret_cast<uint8_t *>(b + oQS) : nullptr;
    wp_.ccnt = reinterpret_cast<uint32_t *>(b + oCN);
    wp_.cpos = reinterpret_cast<uint32_t *>(b + oCP);
    wp_.lnext = reinterpret_cast<uint64_t *>(b + oLN);
    wp_.lidx = reinterpret_cast<uint32_t *>(b + oLI);
    wp_.vcap = (uint32_t)vc;
    wp_.vcnt = reinterpret_cast<unsigned long long *>(b + oVC);
    wp_.vpos = reinterpret_cast<uint64_t *>(b + oVP);
    wp_.vseg = reinterpret_cast<uint32_t *>(b + oVS);
    wp_.vnext = reinterpret_cast<uint64_t *>(b + oVN);
    wp_.vidx = reinterpret_cast<uint32_t *>(b + oVI);
    d_ptrs_ = reinterpret_cast<const uint8_t **>(b + o_ptrs);
    d_lens_ = reinterpret_cast<uint64_t *>(b + o_lens);
    d_span_base_ = reinterpret_cast<uint64_t *>(b + o_sb);
    return CDC_OK;
}

int Engine::run_walk(const StreamTable &st, cdc_chunk_t *d_out, size_t n, uint64_t *first, hipStream_t s) {
    uint64_t *h = static_cast<uint64_t *>(h_stage_);
    uint64_t *h_first = h + 4 * h_stage_streams_ + 4;  // first[n+1]
    uint64_t *h_flags = h + 5 * h_stage_streams_ + 32;  // flags[4] ++ the round blocks, one copy
    uint64_t *h_rf = h_flags + 4;
    const uint32_t R = max_rounds_ < walk::kMaxFixRounds ? max_rounds_ : walk::kMaxFixRounds;
    HIP_TRY(hipEventRecord(ev_[0], s));
    // (the previous call's end kernel resets the flag blocks when it ends
    // the call: then no init launch here)
    if (!walk_flags_clean_) HIP_TRY(walk::launch_flags_init(wst_.flags, R, s));
    walk_flags_clean_ = false;
    static const bool diag = std::getenv("CHUNKFS_AMD_WALKDIAG") != nullptr;  // phase times + candidates
    auto lap = [&](const char *what) -> int {
        if (!diag) return CDC_OK;
        static auto t_last = std::chrono::steady_clock::now();
        HIP_TRY(hipStreamSynchronize(s));
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  walkdiag %-6s %9.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
        return CDC_OK;
    };
    (void)lap("start");
    HIP_TRY(walk::launch_bits(st, wp_, s));
    (void)lap("bits");
    HIP_TRY(walk::launch_links(st, wp_, s));
    (void)lap("links");
    if (diag && wp_.links) {
        std::vector<uint32_t> cn(st.total_spans);
        HIP_TRY(hipMemcpy(cn.data(), wp_.ccnt, cn.size() * 4, hipMemcpyDeviceToHost));
        uint64_t tot = 0, ovf = 0, mx = 0;
        for (uint32_t c : cn) {
            tot += c;
            ovf += c > wp_.ccap;
            mx = c > mx ? c : mx;
        }
        std::fprintf(stderr, "  walkdiag candidates %llu (%.2f per segment, max %llu, cap %u, overflowed %llu of %zu)\n",
                     (unsigned long long)tot, (double)tot / cn.size(), (unsigned long long)mx, wp_.ccap,
                     (unsigned long long)ovf, cn.size());
    }
    HIP_TRY(walk::launch_walk(st, wp_, wst_, s));
    (void)lap("walk");
    HIP_TRY(hipEventRecord(ev_[1], s));
    // Jacobi rounds: re-walk every segment whose entry is not its predecessor's
    // exit, until none is.  Rounds are launched in groups without a host sync:
    // round r counts into its own flag block (rf + 4 r) and returns at once on
    // the device when round r-1 changed no exit (WalkState::gate), so the host
    // waits once per group instead of once per round.
    // The output is queued right behind the first group, gated on the device
    // by the same rule (walk::launch_emit's egate): when that group settles
    // -- the common case -- the call needs one host wait, not two.
    // The first group is one round: on random data the first round settles
    // every segment (its re-walks meet the old chains), and the gated no-op
    // rounds after it cost ~14 us each (snapshot + fix launches).
    constexpr uint32_t kGroup = 4;
    unsigned long long *rf = wst_.flags + 4;
    uint64_t rewalked = 0, round_errors = 0;
    bool settled = false, quiet_stop = false, queued = false, fused = false;
    uint32_t launched = 0, last_round = 0;
    while (launched < R && !settled) {
        const uint32_t grp = launched == 0 ? walk::kFirstGroupRounds : kGroup;
        const uint32_t end = launched + grp < R ? launched + grp : R;
        for (uint32_t r = launched; r < end; ++r) {
            // Plain Jacobi for the first ahead_after_ rounds, then run-ahead
            // re-walks (walk.hip fix_kernel) so long non-merging stretches
            // settle before the serial pass would be needed.
            wp_.ahead = r < ahead_after_ ? 1u : ahead_max_;
            walk::WalkState ws = wst_;
            ws.flags = rf + 4 * r;
            ws.gate = r ? rf + 4 * (r - 1) : nullptr;
            const auto t0 = std::chrono::steady_clock::now();
            HIP_TRY(walk::launch_fix(st, wp_, ws, s, r != 0));  // (round 0's snapshot: written by the walk)
            if (diag) {
                HIP_TRY(hipStreamSynchronize(s));
                std::fprintf(stderr, "  walkdiag round %u %.3f ms\n", r,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            }
        }
        queued = launched == 0 && !diag;
        launched = end;
        // Fused end (walk::launch_finish_emit): the prefix, first[] and the
        // flag blocks go straight into the host staging block -- no D2H
        // copies -- and the flags are reset for the next call when it ends
        // this one.
        fused = queued && walk_fused_ && walk::finish_fits(st);
        if (fused) {
            HIP_TRY(walk::launch_finish_emit(st, wp_, wst_, d_out, out_cap_, s, rf, launched, launched, walk_go_,
                                             h_first, h_flags));
        } else {
            if (queued) {
                HIP_TRY(walk::launch_emit(st, wp_, wst_, d_out, out_cap_, s, rf, launched));
                HIP_TRY(hipMemcpyAsync(h_first, wst_.first, (n + 1) * 8, hipMemcpyDeviceToHost, s));
            }
            HIP_TRY(hipMemcpyAsync(h_flags, wst_.flags, (4 + (size_t)launched * 4) * 8, hipMemcpyDeviceToHost, s));
        }
        if (queued) HIP_TRY(hipEventRecord(ev_[2], s));
        HIP_TRY(hipStreamSynchronize(s));
        // The first round that settled everything, or whose changed exits
        // were mostly quiet-run re-walks (zero-filled / constant regions:
        // chains there keep their phase, so each round moves the true one a
        // single segment; the in-order pass takes such a region in one go).
        // Later rounds of the group returned at once on the device (the same
        // rule, walk.hip round_stops).
        for (uint32_t r = 0; r < launched; ++r) {
            const int v = walk::round_verdict(h_rf[4 * r], h_rf[4 * r + 3] >> 32);  // (walk.hpp: shared rule)
            if (v == walk::kRoundSettled) {
                settled = true;
                break;
            }
            if (v == walk::kRoundQuiet) {
                last_round = r;
                quiet_stop = true;
                break;
            }
        }
        if (quiet_stop) break;
    }
    for (uint32_t r = 0; r < launched; ++r) {
        round_errors += h_rf[4 * r + 1];
        rewalked += h_rf[4 * r + 3] & 0xFFFFFFFFull;
    }
    if (diag) {
        std::fprintf(stderr, "  walkdiag rounds %u settled %d:", launched, (int)settled);
        for (uint32_t r = 0; r < launched && r < 24; ++r)
            std::fprintf(stderr, " %llu/%llu", (unsigned long long)h_rf[4 * r + 3], (unsigned long long)h_rf[4 * r]);
        std::fprintf(stderr, "\n");
    }
    // Chains that never merge (periodic data): one exact in-order pass from
    // the lowest segment the last round changed.
    if (!settled) {
        const uint32_t lr = quiet_stop ? last_round : launched - 1;  // the last round that ran
        HIP_TRY(hipMemcpyAsync(wst_.flags + 2, rf + 4 * lr + 2, 8, hipMemcpyDeviceToDevice, s));
        HIP_TRY(walk::launch_serial(st, wp_, wst_, s));
    }
    (void)lap("fixup");
    // The gated output queued after the first group ran on the device exactly
    // when that group settled by the same rule (emit_skips), i.e. when the
    // loop stopped after it: launched == kFirstGroupRounds.
    const bool gated_ran = queued && settled && launched == walk::kFirstGroupRounds;
    walk_flags_clean_ = gated_ran && fused;  // (finish_kernel reset them)
    if (!gated_ran) {  // (else the gated output already ran)
        HIP_TRY(walk::launch_emit(st, wp_, wst_, d_out, out_cap_, s));
        HIP_TRY(hipMemcpyAsync(h_flags, wst_.flags, 4 * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h_first, wst_.first, (n + 1) * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(ev_[2], s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (h_flags[1] + round_errors != 0) {
        set_error("segment walk: chunk list or output bound exceeded (internal error)");
        return CDC_EDEVICE;
    }
    std::memcpy(first, h_first, (n + 1) * 8);
    float t01 = 0, t12 = 0, t02 = 0;
    HIP_TRY(hipEventElapsedTime(&t01, ev_[0], ev_[1]));
    HIP_TRY(hipEventElapsedTime(&t12, ev_[1], ev_[2]));
    HIP_TRY(hipEventElapsedTime(&t02, ev_[0], ev_[2]));
    timing_.scan_ms = t01;
    timing_.resolve_ms = t12;
    timing_.total_ms = t02;
    timing_.fixup_iterations = (uint32_t)rewalked;
    timing_.overflow_spans = settled ? 0u : 1u;
    timing_.path = CDC_PATH_WALK;
    timing_.timed = 1;
    return CDC_OK;
}

}  // namespace cdc
