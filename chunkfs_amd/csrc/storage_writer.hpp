// storage_writer.hpp -- host mirror of chunkfs's write path for one write call.
//
// ChunkStorage::write (reference src/system/storage.rs:78-103) slices the
// written data into SEG_SIZE (1 MiB, src/lib.rs:39) pieces and feeds each to a
// StorageWriter (storage.rs:302-357): buffer = rest ++ slice; chunks =
// chunk_data(buffer); the LAST chunk is always carried over as the new rest
// (storage.rs:322) and the others become spans; flush (storage.rs:360-383)
// emits the final rest as one span.  Chunk time is the sum of the intervals
// around chunk_data only (storage.rs:314-316).
#pragma once
#include <chrono>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/chunkfs_amd.h"

namespace cdc {

// ChunkFn: int64_t(const uint8_t *buf, size_t len, std::vector<cdc_chunk_t> &out)
// returning the chunk count (out resized to it) or a negative error code.
template <class ChunkFn>
int64_t storage_write_spans(ChunkFn &&chunk_data, const uint8_t *data, size_t len,
                            size_t seg_size, std::vector<uint64_t> &spans,
                            double *chunk_seconds) {
    spans.clear();
    if (seg_size == 0) return CDC_EINVAL;
    std::vector<uint8_t> buffer;
    std::vector<cdc_chunk_t> chunks;
    size_t rest = 0;  // bytes of the carried-over chunk at the front of `buffer`
    double t_chunk = 0.0;
    for (size_t cur = 0; cur < len;) {
        const size_t take = len - cur < seg_size ? len - cur : seg_size;
        buffer.resize(rest + take);
        std::memcpy(buffer.data() + rest, data + cur, take);
        cur += take;
        const auto t0 = std::chrono::steady_clock::now();
        const int64_t n = chunk_data(buffer.data(), buffer.size(), chunks);
        t_chunk += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (n < 0) return n;
        if (n == 0) {  // storage.rs:318-320: nothing chunked, rest unchanged
            rest = buffer.size();
            continue;
        }
        for (int64_t i = 0; i + 1 < n; ++i) spans.push_back(chunks[i].length);
        const cdc_chunk_t last = chunks[n - 1];
        std::memmove(buffer.data(), buffer.data() + last.offset, last.length);
        rest = last.length;
    }
    if (rest) spans.push_back(rest);  // flush
    if (chunk_seconds) *chunk_seconds = t_chunk;
    return (int64_t)spans.size();
}

}  // namespace cdc
