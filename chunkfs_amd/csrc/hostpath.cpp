// hostpath.cpp -- the host-memory boundary of the engine:
// Chunker::chunk_data on a host buffer (reference src/lib.rs:80, called by
// StorageWriter::write, src/system/storage.rs:302-357) and the write path of
// one file (ChunkStorage::write / write_from_stream, storage.rs:78-137) as a
// streaming, overlapped upload.
//
//   upload       pageable caller bytes -> handle-owned pinned ring (CPU memcpy,
//                one slot per piece) -> async H2D on the engine stream; the
//                copy of piece k+1 runs while piece k's DMA is in flight
//   chunk_host   upload + the device pipeline; the chunk list is written by
//                the kernels straight into host-mapped pinned memory (no D2H
//                copy, no extra sync)
//   write_*      StorageWriter over a stream of segments: bytes accumulate in
//                a device window (double-buffered) while later segments
//                upload; a full window is chunked on the device, every chunk
//                but the last becomes a span and the last one is carried into
//                the next window in HBM (the reference's `rest`, storage.rs:
//                309-322); finish = flush (storage.rs:360-383).
//
// The spans equal the reference's per-segment loop for any segment sizes: every
// chunker here restarts at each chunk boundary and looks only forward, so a
// window's chunks other than its last are the whole write's (SURVEY.md A.4,
// tests/test_gpu_hostpath.py).
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <sstream>

#include "engine.hpp"

#include <atomic>

namespace cdc {

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));      \
            return CDC_EDEVICE;                                                \
        }                                                                      \
    } while (0)

namespace {
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

// ---- host placement ---------------------------------------------------------------
//
// The host side of a call is a memcpy into a pinned ring slot that the device
// then reads over PCIe, so both belong on the GPU's NUMA node: the pinned
// buffers are allocated with that node preferred (hipHostMallocNumaUser under
// a thread-local MPOL_PREFERRED) and the copy helpers run on that node's CPUs
// (those of them this process may use).  CHUNKFS_AMD_COPY_NUMA=0 turns both
// off (A/B).  Linux sysfs gives the node and the link; a box without them
// (node -1) keeps the default placement.

namespace {
std::string read_line(const std::string &path) {
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return "";
    char buf[256] = {0};
    const char *r = std::fgets(buf, sizeof buf, f);
    std::fclose(f);
    std::string s = r ? buf : "";
    while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
    return s;
}

std::vector<int> parse_cpulist(const std::string &s) {  // "0-63,128-191"
    std::vector<int> v;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        if (part.empty()) continue;
        const size_t d = part.find('-');
        const int a = std::atoi(part.c_str());
        const int b = d == std::string::npos ? a : std::atoi(part.c_str() + d + 1);
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c) v.push_back(c);
    }
    return v;
}

constexpr int kMpolDefault = 0, kMpolPreferred = 1;
constexpr unsigned long kMpolFNode = 1, kMpolFAddr = 2;

bool numa_enabled() {
    const char *e = std::getenv("CHUNKFS_AMD_COPY_NUMA");
    return !e || std::atoi(e) != 0;
}
}  // namespace

HostPlacement HostPlacement::probe(int device) {
    HostPlacement p;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return p;
    std::string id = bus;
    for (auto &c : id) c = (char)std::tolower((unsigned char)c);
    p.pci = id;
    const std::string dir = "/sys/bus/pci/devices/" + id + "/";
    const std::string node = read_line(dir + "numa_node");
    p.node = node.empty() ? -1 : std::atoi(node.c_str());
    p.link = read_line(dir + "current_link_speed") + " x" + read_line(dir + "current_link_width");
    p.link_max = read_line(dir + "max_link_speed") + " x" + read_line(dir + "max_link_width");
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0) {
        p.allowed = CPU_COUNT(&allowed);
        if (p.node >= 0)
            for (int c : parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(p.node) +
                                                 "/cpulist")))
                if (CPU_ISSET(c, &allowed)) p.cpus.push_back(c);
    }
    p.enabled = numa_enabled() && p.node >= 0 && !p.cpus.empty();
    return p;
}

// Pinned host memory on the placement's node (when enabled): the calling
// thread's policy prefers that node for this one allocation.
hipError_t HostPlacement::host_malloc(void **ptr, size_t bytes, unsigned flags) const {
    if (!enabled || node < 0 || node >= 1024) return hipHostMalloc(ptr, bytes, flags);
    int old_mode = kMpolDefault;
    unsigned long old_mask[16] = {0};
    const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, 1024ul, nullptr, 0ul) == 0;
    unsigned long mask[16] = {0};
    mask[node / 64] = 1ul << (node % 64);
    const bool set = syscall(SYS_set_mempolicy, kMpolPreferred, mask, 1024ul) == 0;
    const hipError_t e = hipHostMalloc(ptr, bytes, flags | (set ? hipHostMallocNumaUser : 0u));
    if (set) {
        if (saved)
            syscall(SYS_set_mempolicy, old_mode, old_mode == kMpolDefault ? nullptr : old_mask, 1024ul);
        else
            syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0ul);
    }
    return e;
}

int HostPlacement::node_of(const void *addr) {
    if (!addr) return -1;
    int n = -1;
    if (syscall(SYS_get_mempolicy, &n, nullptr, 0ul, addr, kMpolFNode | kMpolFAddr) != 0) return -1;
    return n;
}

// ---- copy pool ----------------------------------------------------------------

CopyPool::CopyPool(unsigned threads, unsigned spin_us, const std::vector<int> &cpus) : spin_us_(spin_us) {
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    for (unsigned i = 1; i < threads; ++i) {
        th_.emplace_back([this, i] { run(i); });
        if (!cpus.empty() && pthread_setaffinity_np(th_.back().native_handle(), sizeof set, &set) == 0) pinned_ += 1;
    }
}

// One pool per NUMA node, shared by every handle whose device sits on it
// (helpers capped at 16 threads per node whatever the number of handles):
// CHUNKFS_AMD_COPY_THREADS threads (default 4, the caller's included),
// helpers pinned to `cpus` (the node's CPUs this process may use; empty: not
// pinned) and spinning CHUNKFS_AMD_COPY_SPIN_US microseconds (default 200) for
// the next job before they sleep.  Handles of one node share its pool, one
// job at a time.
CopyPool &CopyPool::for_node(int node, const std::vector<int> &cpus) {
    static std::mutex m;
    static std::map<int, std::unique_ptr<CopyPool>> pools;
    std::lock_guard<std::mutex> g(m);
    auto &p = pools[node];
    if (!p) {
        const char *e = std::getenv("CHUNKFS_AMD_COPY_THREADS");
        const unsigned threads = (unsigned)std::max(1, std::min(e ? std::atoi(e) : 4, 16));
        const char *sp = std::getenv("CHUNKFS_AMD_COPY_SPIN_US");
        const unsigned spin = (unsigned)std::max(0, std::min(sp ? std::atoi(sp) : 200, 100000));
        p.reset(new CopyPool(threads, spin, node >= 0 ? cpus : std::vector<int>{}));
    }
    return *p;
}

CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> g(m_);
        stop_.store(true);
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
}

// Work stealing: a job is n bytes in pieces; the caller and every helper
// that is awake claim pieces from one counter, so a call never waits for a
// sleeping helper (in StorageWriter's loop the helpers sleep between calls:
// hashing and index inserts take longer than their spin).  A helper joins
// only while the job is open; the caller closes it once every piece is done
// and returns when no helper is still inside.
void CopyPool::work() {
    const size_t np = np_;
    for (size_t p; (p = next_.fetch_add(1, std::memory_order_relaxed)) < np;) {
        const size_t a = p * piece_;
        // (plain stores: the ring slot stays in the CPU caches, where the
        // device's PCIe reads snoop it -- non-temporal stores measured 2-3x
        // slower for 1 MiB calls)
        std::memcpy(dst_ + a, src_ + a, std::min(piece_, n_ - a));
        if (ready_) {
            std::atomic_thread_fence(std::memory_order_release);  // (x86: stores stay in order)
            ready_[p] = seq_;
        }
        done_.fetch_add(1, std::memory_order_release);
    }
}

void CopyPool::run(unsigned) {
    uint64_t seen = 0;
    for (;;) {
        // spin briefly for the next job (a streaming write hands over a
        // segment every ~50 us; a sleeping helper takes ~100 us to wake), then
        // sleep
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t g = gen_.load(std::memory_order_acquire);
        while (g == seen && !stop_.load(std::memory_order_relaxed) &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us_)) {
            __builtin_ia32_pause();
            g = gen_.load(std::memory_order_acquire);
        }
        if (g == seen) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_.load() || gen_.load(std::memory_order_acquire) != seen; });
            g = gen_.load(std::memory_order_acquire);
        }
        if (stop_.load()) return;
        seen = g;
        active_.fetch_add(1, std::memory_order_seq_cst);
        if (open_.load(std::memory_order_seq_cst)) work();  // (a closed job: nothing to touch)
        active_.fetch_sub(1, std::memory_order_seq_cst);
    }
}

void CopyPool::job(void *dst, const void *src, size_t n, size_t piece, volatile uint64_t *ready, uint64_t seq) {
    std::lock_guard<std::mutex> jl(job_m_);  // one job at a time (handles on several threads share the pool)
    dst_ = static_cast<uint8_t *>(dst);
    src_ = static_cast<const uint8_t *>(src);
    n_ = n;
    piece_ = piece;
    np_ = (n + piece - 1) / piece;
    ready_ = ready;
    seq_ = seq;
    next_.store(0, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    if (!th_.empty() && np_ > 1) {
        {
            std::lock_guard<std::mutex> g(m_);  // (pairs with the sleepers' predicate check)
            open_.store(true, std::memory_order_seq_cst);
            gen_.fetch_add(1, std::memory_order_acq_rel);
        }
        cv_.notify_all();
    }
    work();
    while (done_.load(std::memory_order_acquire) < np_) __builtin_ia32_pause();  // pieces a helper holds
    open_.store(false, std::memory_order_seq_cst);
    while (active_.load(std::memory_order_seq_cst) != 0) __builtin_ia32_pause();
}

void CopyPool::copy(void *dst, const void *src, size_t n) {
    if (n < (size_t(256) << 10) || th_.empty()) {  // not worth a hand-off
        std::memcpy(dst, src, n);
        return;
    }
    job(dst, src, n, size_t(256) << 10, nullptr, 0);
}

void CopyPool::copy_feed(void *dst, const void *src, size_t n, size_t piece, volatile uint64_t *ready,
                         uint64_t seq) {
    job(dst, src, n, piece, ready, seq);
}

// ---- host boundary --------------------------------------------------------------

const HostPlacement &Engine::placement() {
    if (!place_probed_) {
        place_ = HostPlacement::probe(device_);
        place_probed_ = true;
    }
    return place_;
}

int Engine::ensure_ring() {
    if (h_ring_) return CDC_OK;
    const HostPlacement &pl = placement();
    if (!pool_) pool_ = &CopyPool::for_node(pl.enabled ? pl.node : -1, pl.cpus);
    // Coherent (fine-grained): the small kernel reads a slot while the host is
    // still filling it (streamed input), so the device must never cache it.
    HIP_TRY(pl.host_malloc(&h_ring_, kRingSlots * kRingSlot, hipHostMallocCoherent));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_ring_dev_), h_ring_, 0));
    HIP_TRY(pl.host_malloc(reinterpret_cast<void **>(&h_ready_), kRingSlots * small::kFeedPieces * 8,
                           hipHostMallocCoherent));
    std::memset(h_ready_, 0, kRingSlots * small::kFeedPieces * 8);
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_ready_dev_), h_ready_, 0));
    for (auto &e : ring_ev_) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&copy_done_, hipEventDisableTiming));
    return CDC_OK;
}

int Engine::ensure_host_out(size_t chunks) {
    if (h_out_ && h_out_cap_ >= chunks) return CDC_OK;
    (void)hipHostFree(h_out_);
    h_out_ = nullptr;
    d_hout_ = nullptr;
    h_out_cap_ = 0;
    const size_t want = round_up(chunks + chunks / 8 + 64, 4096);
    // Coherent: the host reads the chunk list as soon as the kernel's done
    // word says so, with no stream synchronisation in between; in plain mapped
    // memory the device's writes did not always reach lines the CPU had read
    // in the previous call (9 of 27k calls returned a stale last chunk,
    // tools/tails_repro.py).
#ifndef CDC_HOUT_COHERENT
#define CDC_HOUT_COHERENT 1
#endif
    HIP_TRY(placement().host_malloc(reinterpret_cast<void **>(&h_out_), want * sizeof(cdc_chunk_t),
                                    hipHostMallocMapped | (CDC_HOUT_COHERENT ? hipHostMallocCoherent : 0u)));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_hout_), h_out_, 0));
    h_out_cap_ = want;
    return CDC_OK;
}

int Engine::ensure_device_data(size_t len) {
    if (d_data_bytes_ >= len) return CDC_OK;
    (void)hipFree(d_data_);
    d_data_ = nullptr;
    d_data_bytes_ = 0;
    const size_t want = round_up(len + len / 8, size_t(1) << 20);
    HIP_TRY(hipMalloc(&d_data_, want));
    d_data_bytes_ = want;
    return CDC_OK;
}

// Pageable host bytes -> pinned ring slot -> async H2D (stream s).  Pieces of
// `piece` bytes (<= kRingSlot); a slot is reused once its previous DMA is done.
int Engine::upload(const uint8_t *src, size_t len, uint8_t *dst, hipStream_t s, size_t piece) {
    for (size_t off = 0; off < len;) {
        const size_t n = std::min(piece, len - off);
        const uint32_t k = ring_next_;
        ring_next_ = (ring_next_ + 1) % kRingSlots;
        HIP_TRY(hipEventSynchronize(ring_ev_[k]));  // (an event never recorded is complete)
        uint8_t *slot = static_cast<uint8_t *>(h_ring_) + (size_t)k * kRingSlot;
        pool_->copy(slot, src + off, n);
        HIP_TRY(hipMemcpyAsync(dst + off, slot, n, hipMemcpyHostToDevice, s));
        HIP_TRY(hipEventRecord(ring_ev_[k], s));
        off += n;
    }
    return CDC_OK;
}

int64_t Engine::chunk_host(const uint8_t *data, size_t len, cdc_chunk_t *out, size_t cap, uint8_t *digests) {
    if (len && !data) {
        set_error("cdc_chunk_data: data is NULL");
        return CDC_EINVAL;
    }
    if (cap && !out) {
        set_error("cdc_chunk_data: out is NULL");
        return CDC_EINVAL;
    }
    if (len == 0) return 0;  // FastCDC iterator yields nothing; FSChunker loop never runs
    HIP_TRY(hipSetDevice(device_));
    if (fb_any_) {  // async batches first: the small path reuses host staging block 0
        const int64_t r = drain_implicit();
        if (r < 0) return r;
    }
    const double t0 = now_s();
    int rc = ensure_ring();
    if (!rc) rc = ensure_device_data(len);
    const size_t need = max_chunks(len);
    if (!rc) rc = ensure_host_out(need);
    if (rc) return rc;
    int64_t count = -1;
    double t1 = t0;
    bool small_tried = false;
    // FastCDC calls of the reference's size (StorageWriter's 1 MiB segments +
    // the carried chunk): the one-launch small kernel is launched first and
    // reads the bytes over PCIe from a pinned ring slot that this thread fills
    // meanwhile, 128 KiB at a time, each piece announced by a feed word -- the
    // copy overlaps the launch and the reads; no DMA, no second kernel on the
    // call's critical path (small.hip).  A call the kernel's budgets cannot
    // take falls through to the regular upload + pipeline.
    if (algo_ == CDC_ALGO_FASTCDC && small_zc_ && !digests && small_ok(len) && len <= kRingSlot) {
        rc = ensure_host_staging(1);
        if (rc) return rc;
        const uint32_t k = ring_next_;
        ring_next_ = (ring_next_ + 1) % kRingSlots;
        HIP_TRY(hipEventSynchronize(ring_ev_[k]));
        uint8_t *slot = static_cast<uint8_t *>(h_ring_) + (size_t)k * kRingSlot;
        uint64_t first[2] = {0, 0};
        if (small_feed_) {
            rc = run_small(h_ring_dev_ + (size_t)k * kRingSlot, len, d_hout_, need, first, own_stream_, true, data,
                           slot, k);
            t1 = t0 + small_copy_s_;
        } else {  // (A/B: the whole copy, then the launch)
            pool_->copy(slot, data, len);
            t1 = now_s();
            rc = run_small(h_ring_dev_ + (size_t)k * kRingSlot, len, d_hout_, need, first, own_stream_, true);
        }
        HIP_TRY(hipEventRecord(ring_ev_[k], own_stream_));  // the slot is free once the kernel retires
        if (rc < 0) return rc;
        if (rc == CDC_OK) count = (int64_t)first[1];
        small_tried = true;
    }
    // Small calls (the reference's 1 MiB segments) go through the pinned ring
    // in 256 KiB pieces, so that the CPU copy of one piece overlaps the DMA of
    // the previous one; large buffers take HIP's own pageable path, which
    // stages with several threads (measured 51 vs 31 GiB/s for the single-
    // thread ring on 1 GiB).
    if (count >= 0) {
        // (chunked by the small kernel from the ring slot)
    } else if (len <= kRingDirect) {
        // (4 MiB pieces, each copied by the pool and moved by one DMA: one
        // 1 MiB call is one hand-off and one hipMemcpyAsync)
        rc = upload(data, len, d_data_, own_stream_, kRingSlot);
        if (rc) return rc;
    } else {
        HIP_TRY(hipMemcpyAsync(d_data_, data, len, hipMemcpyHostToDevice, own_stream_));
    }
    if (count < 0) {
        t1 = now_s();
        const uint8_t *p = d_data_;
        const uint64_t l = len;
        uint64_t first[2] = {0, 0};
        small_skip_ = small_tried;  // (the small kernel already declined these bytes)
        count = chunk_batch_device(1, &p, &l, reinterpret_cast<cdc_chunk_t *>(d_hout_), need, first, own_stream_);
        small_skip_ = false;
        if (count < 0) return count;
    }
    const size_t copy = (size_t)count < cap ? (size_t)count : cap;
    if (digests && copy) {
        if (d_out_cap_ < (size_t)count) {  // the SHA-256 kernel reads the chunk list from HBM
            (void)hipFree(d_out_);
            d_out_ = nullptr;
            d_out_cap_ = 0;
            const size_t want = (size_t)count + (size_t)count / 8 + 64;
            HIP_TRY(hipMalloc(&d_out_, want * sizeof(cdc_chunk_t)));
            d_out_cap_ = want;
        }
        if (d_dig_cap_ < (size_t)count) {
            (void)hipFree(d_dig_);
            d_dig_ = nullptr;
            d_dig_cap_ = 0;
            const size_t want = (size_t)count + (size_t)count / 8 + 64;
            HIP_TRY(hipMalloc(&d_dig_, want * 32));
            d_dig_cap_ = want;
        }
        HIP_TRY(hipMemcpyAsync(d_out_, h_out_, (size_t)count * sizeof(cdc_chunk_t), hipMemcpyHostToDevice,
                               own_stream_));
        rc = sha256_device(d_data_, d_out_, (size_t)count, d_dig_, own_stream_);
        if (rc) return rc;
        HIP_TRY(hipMemcpy(digests, d_dig_, copy * 32, hipMemcpyDeviceToHost));
    }
    if (copy) std::memcpy(out, h_out_, copy * sizeof(cdc_chunk_t));
    host_.calls += 1;
    host_.upload_s += t1 - t0;
    host_.total_s += now_s() - t0;
    return count;
}

// ---- streaming write path ---------------------------------------------------

int Engine::write_begin() {
    HIP_TRY(hipSetDevice(device_));
    if (wr_.active) {  // (never silently drop a write in progress)
        set_error("cdc_write_begin: a write is already in progress on this handle (cdc_write_finish ends it)");
        return CDC_EINVAL;
    }
    int rc = ensure_ring();
    if (rc) return rc;
    // A window holds the carried chunk (<= max bytes) at offset 0, then the
    // new bytes: its start stays 16-byte aligned for the scan's vector loads.
    const size_t reserve = round_up(std::max(max_, min_) + 16, 256);  // FSChunker: max_ = 0
    if (!ws_win_[0]) {
        for (auto &w : ws_win_) HIP_TRY(hipMalloc(reinterpret_cast<void **>(&w), reserve + kWriteWindow + 64));
        HIP_TRY(hipEventCreateWithFlags(&ws_ev_, hipEventDisableTiming));
    }
    wr_ = WriteState{};
    wr_.reserve = reserve;
    wr_.active = true;
    wr_.t0 = now_s();
    return CDC_OK;
}

// Chunk the current window [0, carry + fill) on the device;
// all chunks but the last (all of them at the end of the write) are spans.
int Engine::write_window(bool final) {
    WriteState &W = wr_;
    const size_t n = W.carry + W.fill;
    if (n == 0) return CDC_OK;
    uint8_t *base = ws_win_[W.cur];
    // The window's uploads ran on the copy stream: the chunking waits for them.
    HIP_TRY(hipEventRecord(copy_done_, copy_stream_));
    HIP_TRY(hipStreamWaitEvent(own_stream_, copy_done_, 0));
    const size_t need = max_chunks(n);
    int rc = ensure_host_out(need);
    if (rc) return rc;
    const uint8_t *p = base;
    const uint64_t l = n;
    uint64_t first[2] = {0, 0};
    const double tc = now_s();
    const int64_t c = chunk_batch_device(1, &p, &l, reinterpret_cast<cdc_chunk_t *>(d_hout_), need, first,
                                         own_stream_);
    if (c < 0) return (int)c;
    W.chunk_s += now_s() - tc;
    const cdc_chunk_t *ch = h_out_;
    const int64_t keep = final ? c : c - 1;
    for (int64_t i = 0; i < keep; ++i) W.spans.push_back(ch[i].length);
    if (!final && c > 0) {
        // storage.rs:322: the last chunk is carried (`rest`), here in HBM, to the
        // front of the other window (it is <= max bytes: the reserve).
        const size_t r = (size_t)ch[c - 1].length;
        uint8_t *dst = ws_win_[1 - W.cur];
        HIP_TRY(hipMemcpyAsync(dst, base + ch[c - 1].offset, r, hipMemcpyDeviceToDevice, own_stream_));
        // new uploads into that window wait for the carry copy (same region's
        // neighbourhood; cheap)
        HIP_TRY(hipEventRecord(ws_ev_, own_stream_));
        HIP_TRY(hipStreamWaitEvent(copy_stream_, ws_ev_, 0));
        W.carry = r;
    } else {
        W.carry = 0;
    }
    W.cur = 1 - W.cur;
    W.fill = 0;
    return CDC_OK;
}

int Engine::write_segment(const uint8_t *data, size_t len) {
    if (!wr_.active) {
        set_error("cdc_write_segment: no write in progress (cdc_write_begin)");
        return CDC_EINVAL;
    }
    if (wr_.failed) {
        set_error("cdc_write_segment: an earlier call of this write failed (cdc_write_finish ends it)");
        return CDC_EINVAL;
    }
    if (len && !data) {
        set_error("cdc_write_segment: data is NULL");
        return CDC_EINVAL;
    }
    // Any failure past this point leaves the window state unknown: the write
    // is marked failed and cdc_write_finish reports an error, never spans.
    if (hipSetDevice(device_) != hipSuccess) {
        wr_.failed = true;
        set_error("cdc_write_segment: hipSetDevice failed");
        return CDC_EDEVICE;
    }
    WriteState &W = wr_;
    while (len) {
        if (W.fill == kWriteWindow) {
            const int rc = write_window(false);
            if (rc) {
                W.failed = true;
                return rc;
            }
        }
        const size_t n = std::min(len, kWriteWindow - W.fill);
        const int rc = upload(data, n, ws_win_[W.cur] + W.carry + W.fill, copy_stream_, kRingSlot);
        if (rc) {
            W.failed = true;
            return rc;
        }
        W.fill += n;
        W.bytes += n;
        data += n;
        len -= n;
    }
    W.segments += 1;
    return CDC_OK;
}

int64_t Engine::write_finish(std::vector<uint64_t> &spans, double *seconds) {
    if (!wr_.active) {
        set_error("cdc_write_finish: no write in progress (cdc_write_begin)");
        return CDC_EINVAL;
    }
    wr_.active = false;
    if (wr_.failed) {
        set_error("cdc_write_finish: a cdc_write_segment of this write failed; its spans are unknown");
        return CDC_EDEVICE;
    }
    HIP_TRY(hipSetDevice(device_));
    const int rc = write_window(true);  // StorageWriter::flush: the rest is the last span
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(copy_stream_));
    spans.assign(wr_.spans.begin() + (ptrdiff_t)wr_.drained, wr_.spans.end());
    if (seconds) *seconds = now_s() - wr_.t0;
    return (int64_t)spans.size();
}

// Spans final so far (file order), oldest first, that no drain has returned:
// every chunk of a chunked device window but its last.  The caller may
// release the bytes those spans cover.
int64_t Engine::write_drain(uint64_t *out, size_t cap) {
    if (!wr_.active) {
        set_error("cdc_write_drain: no write in progress (cdc_write_begin)");
        return CDC_EINVAL;
    }
    if (cap && !out) {
        set_error("cdc_write_drain: span_lengths is NULL");
        return CDC_EINVAL;
    }
    const size_t k = std::min(cap, wr_.spans.size() - wr_.drained);
    std::memcpy(out, wr_.spans.data() + wr_.drained, k * sizeof(uint64_t));
    wr_.drained += k;
    return (int64_t)k;
}

// JSON: the device's PCI address, NUMA node and link, where the pinned ring
// landed and how the copy helpers were placed (bench.py host_path.numa).
int64_t Engine::host_placement_json(char *out, size_t cap) {
    int rc = ensure_ring();
    if (rc) return rc;
    const HostPlacement &p = placement();
    std::ostringstream o;
    o << "{\"pci\": \"" << p.pci << "\", \"gpu_node\": " << p.node << ", \"link\": \"" << p.link
      << "\", \"link_max\": \"" << p.link_max << "\", \"numa_placement\": " << (p.enabled ? "true" : "false")
      << ", \"ring_node\": " << HostPlacement::node_of(h_ring_)
      << ", \"chunk_list_node\": " << HostPlacement::node_of(h_out_)
      << ", \"allowed_cpus\": " << p.allowed << ", \"node_cpus_allowed\": " << p.cpus.size()
      << ", \"copy_threads\": " << pool_->threads() << ", \"helpers_pinned\": " << pool_->pinned() << "}";
    const std::string s = o.str();
    if (out && cap) {
        const size_t k = std::min(cap - 1, s.size());
        std::memcpy(out, s.data(), k);
        out[k] = 0;
    }
    return (int64_t)s.size();
}

int Engine::host_stats(double *v, size_t n) const {
    const double s[7] = {(double)host_.calls, host_.upload_s, host_.total_s, wr_.chunk_s, (double)wr_.segments,
                         (double)small_calls_, (double)small_fallbacks_};
    for (size_t i = 0; i < n && i < 7; ++i) v[i] = s[i];
    return CDC_OK;
}

}  // namespace cdc
