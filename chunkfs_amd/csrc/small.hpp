// small.hpp -- one-launch FastCDC for a small single stream (small.hip): the
// host path's per-call chunk_data (StorageWriter's 1 MiB segments,
// reference src/system/storage.rs:302-357).
#pragma once
#include "cdc_kernels.hpp"

namespace cdc {
namespace small {

constexpr uint64_t kBlockBytes = 32768;  // 8 waves x 4 KiB per block
constexpr uint32_t kMaxBlocks = 128;     // streams up to 4 MiB
constexpr uint64_t kMaxBytes = kBlockBytes * kMaxBlocks;
constexpr uint32_t kBlockRecCap = 256;   // records per block region
constexpr uint32_t kRecCap = 2048;       // records the last block holds: streams of up to
                                         // kRecCap / 2 expected hits take this path

// Host-coherent words written by the kernel's last block.
constexpr int kWordRecords = 0;   // records (windowed mask_s / mask_l hits)
constexpr int kWordFallback = 1;  // 1: a budget was exceeded, run the regular pipeline
constexpr int kWordDone = 7;      // 1 once everything above and first[] are written

// Device scratch: per-block record regions and counts, the arrival ticket
// (zero between launches: the last block resets it).
struct Scratch {
    uint64_t *brec;    // [kMaxBlocks * kBlockRecCap]: record | truncated results << 32
    uint32_t *bcnt;    // [kMaxBlocks]
    uint32_t *ticket;  // [1]
    uint64_t *bpub;    // [kMaxBlocks]: launch seq << 32 | record count, once a block's records are out
    uint64_t *stamp;   // [8] phase timestamps (FastParams.diag & 4096 only)
    uint8_t *copy;     // [kMaxBytes + 64]: device copy of a host-memory input (stage)
    uint64_t *bstamp;  // [kMaxBlocks * 8] per-block stamps: fed, loaded, hashed, tinfo, drained, ticket (diag)
};

inline size_t scratch_bytes() {
    return (size_t)(2 * kMaxBlocks * kBlockRecCap + kMaxBlocks + 64) * 4 + kMaxBlocks * 8 + 8 * 8;
}
inline size_t copy_bytes() { return kMaxBytes + 64; }
inline size_t bstamp_bytes() { return kMaxBlocks * 8 * 8; }

// Streamed input (the host path): the kernel is launched before the host has
// copied the bytes into the pinned ring slot; the host copies them in pieces
// of 2^kFeedLog2 bytes and, after each, stores the launch's seq into
// ready[piece] (pinned, coherent).  A block starts loading once every piece
// its bytes (and the 64 before them) lie in is ready.  ready == nullptr: the
// bytes are complete at launch.
#ifndef CDC_FEED_LOG2
#define CDC_FEED_LOG2 17
#endif
constexpr uint32_t kFeedLog2 = CDC_FEED_LOG2;
constexpr uint32_t kFeedPieces = (uint32_t)(kMaxBytes >> kFeedLog2);
struct Feed {
    const uint64_t *ready;  // [kFeedPieces] (device address of pinned host words), or nullptr
    uint64_t seq;           // this launch's sequence number (also tags bpub)
};

// Diagnostics (CHUNKFS_AMD_DIAG & 4096): s_memrealtime stamps (100 MHz) in
// h_stats[kWordStamp0 + k]: block 0's start, the last block's arrival, records
// gathered, links done (rounds in kWordStamp0 + 7), chain walked, output written.
constexpr int kWordStamp0 = 8;
constexpr uint32_t kDiagStamps = 4096;

hipError_t launch_small(const uint8_t *data, uint64_t n, const FastParams &fp, const uint64_t *d_gear,
                        const Scratch &ws, void *out, uint64_t out_cap, uint64_t *h_stats, uint64_t *h_first,
                        bool stage, const Feed &feed, hipStream_t s);

}  // namespace small
}  // namespace cdc
