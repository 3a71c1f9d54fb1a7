// chunkfs_amd.hpp -- header-only C++ mirror of chunkfs's chunking interface,
// built ON the C ABI of chunkfs_amd.h (link with libchunkfs_amd.so).
//
//   reference (Rust, src/lib.rs, src/chunkers)      here
//   struct Chunk {offset, length}   lib.rs:43-66    chunkfs_amd::Chunk
//   trait Chunker                   lib.rs:74-86    chunkfs_amd::Chunker
//   SizeParams {min, avg, max}      chunkers/mod.rs chunkfs_amd::SizeParams
//   FastChunker                     chunkers/fast.rs        chunkfs_amd::FastChunker
//   FSChunker                       chunkers/fixed_size.rs  chunkfs_amd::FSChunker
//   Rabin/Ultra/Leap/SeqChunker     chunkers/{rabin,ultra,leap,seq}.rs  same names
//   ChunkStorage::write spans       system/storage.rs:78-103  Chunker::write_spans
//
// The reference panics on invalid sizes; here constructors throw
// chunkfs_amd::Error (carrying the CDC_E* code and cdc_last_error()).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "chunkfs_amd.h"

namespace chunkfs_amd {

constexpr size_t KB = 1024;
constexpr size_t MB = 1024 * KB;
constexpr size_t GB = 1024 * MB;
constexpr size_t SEG_SIZE = MB;  // src/lib.rs:39

class Error : public std::runtime_error {
  public:
    Error(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

  private:
    int code_;
};

inline int64_t check(int64_t rc) {
    if (rc < 0) throw Error((int)rc, std::string("chunkfs_amd: ") + cdc_last_error());
    return rc;
}

// Chunk (src/lib.rs:41-66): offset and length only.
struct Chunk {
    size_t offset_ = 0;
    size_t length_ = 0;
    Chunk() = default;
    Chunk(size_t offset, size_t length) : offset_(offset), length_(length) {}
    size_t offset() const { return offset_; }
    size_t length() const { return length_; }
    size_t range_begin() const { return offset_; }
    size_t range_end() const { return offset_ + length_; }
    bool operator==(const Chunk &o) const { return offset_ == o.offset_ && length_ == o.length_; }
};

// cdc_chunkers::SizeParams (re-exported at src/chunkers/mod.rs:1).
struct SizeParams {
    size_t min, avg, max;
};

// The Chunker trait (src/lib.rs:74-86).  Not thread-safe: the reference
// serialises every call through Arc<Mutex<dyn Chunker>> (lib.rs:89-90).
class Chunker {
  public:
    virtual ~Chunker() { cdc_destroy(h_); }
    Chunker(const Chunker &) = delete;
    Chunker &operator=(const Chunker &) = delete;

    // chunk_data(&mut self, data, empty) -> Vec<Chunk> (lib.rs:80).
    std::vector<Chunk> chunk_data(const uint8_t *data, size_t len, std::vector<Chunk> empty = {}) {
        std::vector<cdc_chunk_t> raw(cdc_max_chunk_count(h_, len));
        const int64_t n = check(cdc_chunk_data(h_, data, len, raw.data(), raw.size()));
        empty.reserve(empty.size() + (size_t)n);
        for (int64_t i = 0; i < n; ++i) empty.emplace_back(raw[i].offset, raw[i].length);
        return empty;
    }
    std::vector<Chunk> chunk_data(const std::vector<uint8_t> &data, std::vector<Chunk> empty = {}) {
        return chunk_data(data.data(), data.size(), std::move(empty));
    }

    // estimate_chunk_count (lib.rs:85): the reference's own formula.
    size_t estimate_chunk_count(size_t len) const { return cdc_estimate_chunk_count(h_, len); }

    // impl Debug.
    std::string debug() const { return cdc_describe(h_); }

    // ChunkStorage::write + StorageWriter (storage.rs:78-103, 302-383): span
    // lengths of one write call; *chunk_seconds = time inside chunk_data.
    std::vector<uint64_t> write_spans(const uint8_t *data, size_t len, double *chunk_seconds = nullptr,
                                      size_t seg_size = SEG_SIZE) {
        std::vector<uint64_t> spans(cdc_max_chunk_count(h_, len) + 1);
        const int64_t n = check(cdc_fs_write(h_, data, len, seg_size, spans.data(), spans.size(), chunk_seconds));
        spans.resize((size_t)n);
        return spans;
    }

    // ChunkStorage::write_from_stream (storage.rs:105-137) through the
    // streaming write path: begin, one write_segment per StorageWriter::write,
    // finish = flush; returns the span lengths.
    void write_begin() { check(cdc_write_begin(h_)); }
    void write_segment(const uint8_t *data, size_t len) {
        check(cdc_write_segment(h_, data, len));
        written_ += len;
    }
    std::vector<uint64_t> write_finish(double *seconds = nullptr) {
        std::vector<uint64_t> spans(cdc_max_chunk_count(h_, written_) + 1);
        written_ = 0;
        const int64_t n = check(cdc_write_finish(h_, spans.data(), spans.size(), seconds));
        spans.resize((size_t)n);
        return spans;
    }

    cdc_handle_t *handle() { return h_; }

  protected:
    Chunker() = default;
    Chunker(cdc_algo_t algo, size_t min, size_t avg, size_t max, int device) {
        check(cdc_create(algo, (uint32_t)min, (uint32_t)avg, (uint32_t)max, device, &h_));
    }
    cdc_handle_t *h_ = nullptr;
    size_t written_ = 0;
};

// FastChunker (src/chunkers/fast.rs): FastCDC 2020, default 8/16/64 KiB.
class FastChunker : public Chunker {
  public:
    explicit FastChunker(SizeParams sizes = {8 * KB, 16 * KB, 64 * KB}, int device = 0)
        : Chunker(CDC_ALGO_FASTCDC, sizes.min, sizes.avg, sizes.max, device), sizes_(sizes) {}
    const SizeParams &sizes() const { return sizes_; }

  private:
    SizeParams sizes_;
};

// FSChunker (src/chunkers/fixed_size.rs): fixed size, default 4096.
class FSChunker : public Chunker {
  public:
    explicit FSChunker(size_t chunk_size = 4096, int device = 0)
        : Chunker(CDC_ALGO_FIXED, chunk_size, 0, 0, device), chunk_size_(chunk_size) {}
    size_t chunk_size() const { return chunk_size_; }

  private:
    size_t chunk_size_;
};

// RabinChunker / UltraChunker / LeapChunker (src/chunkers/{rabin,ultra,leap}.rs):
// published algorithms, parity unpinned (cdc-chunkers 0.1.3 absent); sizes are
// explicit because the crate's SizeParams::*_default() values are unknown.
class RabinChunker : public Chunker {
  public:
    explicit RabinChunker(SizeParams sizes, int device = 0)
        : Chunker(CDC_ALGO_RABIN, sizes.min, sizes.avg, sizes.max, device) {}
};

class UltraChunker : public Chunker {
  public:
    explicit UltraChunker(SizeParams sizes, int device = 0)
        : Chunker(CDC_ALGO_ULTRA, sizes.min, sizes.avg, sizes.max, device) {}
};

class LeapChunker : public Chunker {
  public:
    explicit LeapChunker(SizeParams sizes, int device = 0)
        : Chunker(CDC_ALGO_LEAP, sizes.min, sizes.avg, sizes.max, device) {}
};

// seq::OperationMode and seq::Config (re-exported at src/chunkers/seq.rs:3).
enum class OperationMode : uint32_t { Increasing = 0, Decreasing = 1 };
struct SeqConfig {
    uint32_t seq_length = 5, jump_trigger = 50, jump_size = 256;
};

// SeqChunker::new(mode, sizes, config) (src/chunkers/seq.rs:16-24).
class SeqChunker : public Chunker {
  public:
    SeqChunker(OperationMode mode, SizeParams sizes, SeqConfig config = {}, int device = 0) : Chunker() {
        check(cdc_create_seq((uint32_t)mode, config.seq_length, config.jump_trigger, config.jump_size,
                             (uint32_t)sizes.min, (uint32_t)sizes.avg, (uint32_t)sizes.max, device, &h_));
    }
};

// ChunkerRef (src/lib.rs:89): shared handle to one chunker.
using ChunkerRef = std::shared_ptr<Chunker>;

}  // namespace chunkfs_amd
