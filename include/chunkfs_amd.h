/*
 * chunkfs_amd.h -- C ABI of the MI355X content-defined-chunking engine.
 *
 * This is the drop-in boundary for chunkfs's chunking hot path,
 * `Chunker::chunk_data` (reference src/lib.rs:74-86).  Every entry point below
 * names the reference item it replaces.  The signatures use plain pointers and
 * sizes only, so a Rust `impl Chunker`, ctypes or any other FFI
 * can bind them.
 *
 * Threading: one handle is NOT thread-safe (the reference serialises all calls
 * through ChunkerRef = Arc<Mutex<dyn Chunker>>, src/lib.rs:89-90).  Different
 * handles may be used concurrently, e.g. one per GPU.
 *
 * Errors: the reference's signatures are infallible and panic on bad sizes
 * (fastcdc's size assert!s).  Here every call returns CDC_OK / a count >= 0,
 * or a negative CDC_E* code, with a message from cdc_last_error().
 */
#ifndef CHUNKFS_AMD_H
#define CHUNKFS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: cdc_last_timing takes the caller's sizeof(cdc_timing_t) (the struct
 *    may grow; fields are only ever appended); cdc_abi_version().
 * 3: cdc_timing_t.path / .timed appended; cdc_chunk_batch_device_async,
 *    cdc_batch_sync.
 * 4: cdc_sha256_batch_device. */
#define CHUNKFS_AMD_ABI_VERSION 4

/* Chunk{offset,length} -- reference src/lib.rs:43-47 (usize fields; u64 here). */
typedef struct cdc_chunk {
    uint64_t offset;
    uint64_t length;
} cdc_chunk_t;

/* Algorithms of reference src/chunkers/mod.rs:3-9. */
typedef enum cdc_algo {
    CDC_ALGO_FASTCDC = 0, /* FastChunker  (src/chunkers/fast.rs)        */
    CDC_ALGO_FIXED = 1,   /* FSChunker    (src/chunkers/fixed_size.rs)  */
    CDC_ALGO_RABIN = 2,   /* RabinChunker (src/chunkers/rabin.rs)    -- parity unpinned */
    CDC_ALGO_SUPER = 3,   /* SuperChunker (src/chunkers/supercdc.rs) -- CDC_ENOTSUP */
    CDC_ALGO_ULTRA = 4,   /* UltraChunker (src/chunkers/ultra.rs)    -- parity unpinned */
    CDC_ALGO_LEAP = 5,    /* LeapChunker  (src/chunkers/leap.rs)     -- leap structure of the paper,
                             stand-in eligibility function (chunkfs_amd_cdc_params.h) */
    CDC_ALGO_SEQ = 6      /* SeqChunker   (src/chunkers/seq.rs)      -- parity unpinned */
} cdc_algo_t;

#define CDC_OK 0
#define CDC_EINVAL (-1)  /* bad sizes / arguments (reference: fastcdc assert! panic) */
#define CDC_ENOMEM (-2)  /* device or host allocation failed */
#define CDC_EDEVICE (-3) /* HIP runtime error, or no usable gfx950 device */
#define CDC_ENOTSUP (-4) /* algorithm not implemented */

typedef struct cdc_handle cdc_handle_t;

/* Create a chunker bound to one GPU.
 *   CDC_ALGO_FASTCDC: FastChunker::new(SizeParams{min,avg,max}) (fast.rs:11-15);
 *                     v2020 FastCDC, Level1 normalization (fast.rs:37).
 *   CDC_ALGO_FIXED:   FSChunker::new(min) (fixed_size.rs:19-23); avg/max ignored.
 *   CDC_ALGO_RABIN / _ULTRA / _LEAP: RabinChunker / UltraChunker / LeapChunker
 *                     ::new(SizeParams{min,avg,max}) (rabin.rs:13-20,
 *                     ultra.rs:12-16, leap.rs:12-16).  The reference's crate
 *                     (cdc-chunkers 0.1.3) is absent: Rabin / Ultra restate the
 *                     published algorithms, parity unpinned; Leap
 *                     keeps the paper's leap structure with a STAND-IN window
 *                     eligibility function (not the published one).
 *                     Sizes: 0 < min <= avg <= max; Ultra min >= 8, Leap min >= 32.
 *   CDC_ALGO_SEQ:     SeqChunker with OperationMode::Increasing and the default
 *                     Config (cdc_create_seq for the full constructor).
 *   CDC_ALGO_SUPER:   CDC_ENOTSUP.
 * Returns CDC_OK and *out, or a negative code. */
int cdc_create(cdc_algo_t algo, uint32_t min, uint32_t avg, uint32_t max,
               int device, cdc_handle_t **out);

/* SeqChunker::new(mode, sizes, config) (seq.rs:16-24): mode 0 = Increasing,
 * 1 = Decreasing; config = seq_length (pairs in the mode's direction that
 * end a chunk), jump_trigger (opposing pairs before a jump), jump_size
 * (bytes skipped); defaults 5 / 50 / 256 (include/chunkfs_amd_cdc_params.h). */
int cdc_create_seq(uint32_t mode, uint32_t seq_length, uint32_t jump_trigger,
                   uint32_t jump_size, uint32_t min, uint32_t avg, uint32_t max,
                   int device, cdc_handle_t **out);

/* Drop(Chunker). */
void cdc_destroy(cdc_handle_t *h);

/* Chunker::chunk_data(&mut self, data: &[u8], empty: Vec<Chunk>) -> Vec<Chunk>
 * (src/lib.rs:80).  `data` is HOST memory (borrowed for the call, any alignment,
 * len may be 0).  Writes min(count, cap) chunks to `out` and returns the full
 * chunk count (snprintf convention: a return > cap means `out` was too small;
 * cdc_max_chunk_count() is always enough), or a negative CDC_E* code.
 * The chunks tile [0, len) exactly, in order. */
int64_t cdc_chunk_data(cdc_handle_t *h, const uint8_t *data, size_t len,
                       cdc_chunk_t *out, size_t cap);

/* Chunker::estimate_chunk_count (src/lib.rs:85): the reference's own formula,
 * len/min for FastCDC (fast.rs:47-49), Rabin, Ultra, Leap (rabin.rs:53-55,
 * ultra.rs:41-43, leap.rs:41-43), len/avg for Seq (seq.rs:52-54), len/size + 1
 * for fixed (fixed_size.rs:45-47). */
size_t cdc_estimate_chunk_count(const cdc_handle_t *h, size_t len);

/* A strict upper bound on the chunk count of `len` bytes (len/min + 1). */
size_t cdc_max_chunk_count(const cdc_handle_t *h, size_t len);

/* impl Debug for the chunker (fast.rs:52-56, fixed_size.rs:12-16), with the
 * engine suffix, e.g. "FastCDC (2020), sizes: SizeParams { min: 4096, avg:
 * 8192, max: 16384 } [MI355X gfx950]".  Owned by the handle. */
const char *cdc_describe(const cdc_handle_t *h);

/* Message for the last failing call on this thread ("" if none). */
const char *cdc_last_error(void);

/* Install a 256-entry GEAR table (fastcdc v2020 `GEAR`) for FastCDC handles.
 * The built-in table is a placeholder (include/chunkfs_amd_tables.h); a
 * maintainer pins parity with the Rust crate by passing the crate's table.
 * CDC_EINVAL while a streaming write (cdc_write_begin) is in progress on the
 * handle: one write never mixes two tables. */
int cdc_set_gear(cdc_handle_t *h, const uint64_t gear[256]);

/* Install the Rabin polynomial of a CDC_ALGO_RABIN handle (the reference's
 * RabinChunker carries its ChunkerParams tables, rabin.rs:34-51; the crate's
 * polynomial is absent offline, include/chunkfs_amd_cdc_params.h holds a
 * stand-in).  Degree 9..56 (the 48-byte window digest shifted by a byte stays
 * inside 64 bits); the tables are rebuilt for the handle.  CDC_EINVAL for
 * another algorithm or degree, and while a streaming write is in progress on
 * the handle (one write never mixes two polynomials). */
int cdc_set_rabin_poly(cdc_handle_t *h, uint64_t poly);

/* ---- Device-resident batch API (configs 2, 4, 5: inputs already in HBM) --
 * Chunk n independent streams in one pass.  d_streams[i] are DEVICE pointers
 * (16-byte aligned), lens[i] their byte lengths (host arrays of n entries).
 * The chunks of all streams are written to the DEVICE array d_out (offsets
 * relative to each stream's start), stream i occupying
 * d_out[first[i] .. first[i+1]); `first` is a HOST array of n+1 entries filled
 * by the call.  out_cap must be >= cdc_batch_max_chunks().  hip_stream is a
 * hipStream_t (NULL = the handle's own stream); the call returns after the
 * chunks are final (it synchronises that stream).  Returns the total chunk
 * count or a negative code.  No collective: multi-GPU runs give each rank its
 * own handle and its own streams (weak scaling). */
int64_t cdc_chunk_batch_device(cdc_handle_t *h, size_t n,
                               const uint8_t *const *d_streams,
                               const uint64_t *lens, cdc_chunk_t *d_out,
                               size_t out_cap, uint64_t *first,
                               void *hip_stream);

/* The same batch, enqueued: returns 0 once the batch is submitted, and
 * `first` (kept by the library until then) is filled by cdc_batch_sync.
 * FastCDC batches of more than 8 MiB are enqueued back to back with no host
 * round trip between them, their results collected later: the scans on
 * hip_stream, each resolve on a second stream of the handle behind its scan,
 * beside the next scan (CHUNKFS_AMD_OVERLAP=0 keeps both on hip_stream);
 * cdc_batch_sync orders hip_stream after the resolves.  d_streams' bytes and
 * d_out must stay untouched until cdc_batch_sync.
 * Consecutive async batches of one handle must use one hip_stream (another
 * stream first completes the batches in flight).  Rabin / Ultra / Leap / Seq
 * batches of more than 8 MiB alternate between two internal contexts of the
 * handle (own streams, own host worker threads), so one batch's walks run
 * beside the next one's bitmap pass; they are complete (host-synchronised)
 * when cdc_batch_sync returns (CHUNKFS_AMD_WALK_ASYNC=0: inside this call).
 * Smaller batches and FSChunker complete inside this call (first filled on
 * return).
 * Any other call on the handle first completes the batches in flight. */
int64_t cdc_chunk_batch_device_async(cdc_handle_t *h, size_t n,
                                     const uint8_t *const *d_streams,
                                     const uint64_t *lens, cdc_chunk_t *d_out,
                                     size_t out_cap, uint64_t *first,
                                     void *hip_stream);

/* Completes every batch enqueued by cdc_chunk_batch_device_async (their
 * first[] arrays are filled); returns the last batch's total chunk count (0
 * when none was in flight) or a negative code. */
int64_t cdc_batch_sync(cdc_handle_t *h);

size_t cdc_batch_max_chunks(const cdc_handle_t *h, size_t n,
                            const uint64_t *lens);

/* Per-phase device time of the last batch (HIP events on the launch
 * stream), milliseconds.  scan = the gear candidate scan kernel (the HBM-bound
 * kernel the roofline is quoted on); resolve = truncated-region precompute +
 * the single-pass resolve (chain walk, look-back, output); compact = 0 (fused
 * into resolve); total = all of it. */
typedef struct cdc_timing {
    double scan_ms;
    double resolve_ms;
    double compact_ms;
    double total_ms;
    uint32_t fixup_iterations; /* spans whose speculative chain was re-walked */
    uint32_t overflow_spans; /* spans whose candidate list overflowed */
    uint64_t candidates;     /* candidate positions emitted by the scan */
    uint64_t bytes;          /* input bytes of the batch */
    double hash_ms;          /* last cdc_sha256_chunks_device / _batch_device / cdc_chunk_and_hash kernel time */
    uint64_t walk_fallback_steps; /* chain-walk steps without a precomputed record link */
    uint32_t path;           /* CDC_PATH_*: which engine path ran the batch */
    uint32_t timed;          /* 1: the *_ms fields were measured (HIP events); 0: not timed */
} cdc_timing_t;

/* cdc_timing_t.path */
#define CDC_PATH_PIPELINE 0 /* FastCDC scan + resolve */
#define CDC_PATH_SMALL 1    /* FastCDC one-launch small-stream kernel (not timed: no events on its call path) */
#define CDC_PATH_WALK 2     /* Rabin / Ultra / Leap / Seq segment-walk engine */
#define CDC_PATH_FIXED 3    /* FSChunker */
#define CDC_PATH_EMPTY 4    /* a batch of no streams */

/* Kernel times (HIP events) of the last batch; a batch enqueued by
 * cdc_chunk_batch_device_async carries events one in four (0 ms otherwise).
 * Copies min(t_size, sizeof(cdc_timing_t)) bytes: pass sizeof(cdc_timing_t)
 * of the header the caller was built with, so an older (shorter) struct is
 * never overrun when fields are appended in a later version. */
int cdc_last_timing(const cdc_handle_t *h, cdc_timing_t *t, size_t t_size);

/* ---- Write path ---------------------------------------
 * ChunkStorage::write (storage.rs:78-103) + StorageWriter::{write,flush}
 * (storage.rs:302-383) for ONE write call: seg_size slices (1 MiB in the
 * reference), carry-over of the last chunk of every segment, flush of the
 * rest.  Writes the span lengths in file order (min(count, cap) of them) and
 * returns the span count.  Runs the streaming path below with seg_size
 * segments.  *chunk_seconds (may be NULL) receives the wall time of the whole
 * call (host copy into pinned memory + H2D + chunking + chunk list), i.e. NOT
 * the reference's summed chunk_data time (storage.rs:314-316), which excludes
 * the copies: compare it with the reference's write time. */
int64_t cdc_fs_write(cdc_handle_t *h, const uint8_t *data, size_t len,
                     size_t seg_size, uint64_t *span_lengths, size_t cap,
                     double *chunk_seconds);

/* Streaming form of the same write (ChunkStorage::write_from_stream,
 * storage.rs:105-137: segments of any size, short reads included): begin,
 * then one cdc_write_segment per StorageWriter::write, then finish (=
 * StorageWriter::flush) returns the spans exactly as the reference's loop over
 * the same segments would.  A segment is copied into a handle-owned pinned
 * ring and uploaded asynchronously while the caller goes on; the device
 * chunks 256 MiB windows of the file, carrying each window's last chunk to the
 * next one in HBM.  The caller's bytes are not retained after a call returns.
 * One write per handle at a time: cdc_write_begin on a handle whose write is
 * in progress returns CDC_EINVAL.  A failing cdc_write_segment marks the write
 * failed: later segments return CDC_EINVAL and cdc_write_finish returns an
 * error (never spans of unknown correctness) and ends the write. */
int cdc_write_begin(cdc_handle_t *h);
int cdc_write_segment(cdc_handle_t *h, const uint8_t *data, size_t len);
/* Spans that became final since the last drain, oldest first: moves
 * min(pending, cap) of them into span_lengths and returns how many it moved
 * (0: none pending).  Spans become final each time a device window has been
 * chunked, i.e. every 256 MiB of uploaded bytes, so a caller that hashes and
 * stores each span as StorageWriter::write does (storage.rs:324-350) needs to
 * keep only the bytes from the end of the last drained span on: at most one
 * window (256 MiB) + the segment in hand + max bytes, as the reference's
 * write_from_stream keeps SEG_SIZE + max. */
int64_t cdc_write_drain(cdc_handle_t *h, uint64_t *span_lengths, size_t cap);
/* The spans no cdc_write_drain returned (min(count, cap) written), returns
 * their count; *seconds (may be NULL) = wall time since cdc_write_begin. */
int64_t cdc_write_finish(cdc_handle_t *h, uint64_t *span_lengths, size_t cap,
                         double *seconds);

/* ---- Chunk fingerprints -------------------------------
 * Sha256Hasher::hash (src/hashers.rs:20-36), applied to every chunk as
 * StorageWriter::write does (storage.rs:324-329).  DEVICE arrays:
 * d_digests[32*i .. 32*i+32) = SHA-256(d_data[d_chunks[i].offset .. +length)).
 * Synchronises hip_stream (NULL = the handle's stream) before returning. */
int cdc_sha256_chunks_device(cdc_handle_t *h, const uint8_t *d_data,
                             const cdc_chunk_t *d_chunks, size_t n_chunks,
                             uint8_t *d_digests, void *hip_stream);

/* The same over a batch of streams in one launch -- e.g. the output of
 * cdc_chunk_batch_device: stream i's chunks are d_chunks[first[i] ..
 * first[i+1]) with offsets relative to d_streams[i]; first[0] must be 0.
 * d_streams (n_streams device pointers, 4-byte aligned) and first
 * (n_streams + 1 entries) are HOST arrays; d_chunks / d_digests are DEVICE
 * arrays of first[n_streams] entries (32-byte digests, chunk order).  Each
 * stream's chunks must lie inside its buffer.  Synchronises hip_stream. */
int cdc_sha256_batch_device(cdc_handle_t *h, size_t n_streams,
                            const uint8_t *const *d_streams, const uint64_t *first,
                            const cdc_chunk_t *d_chunks, uint8_t *d_digests,
                            void *hip_stream);

/* chunk_data + SHA-256 of each chunk on a HOST buffer: as cdc_chunk_data, and
 * digests[32*i ..] for the first min(count, cap) chunks. */
int64_t cdc_chunk_and_hash(cdc_handle_t *h, const uint8_t *data, size_t len,
                           cdc_chunk_t *out, uint8_t *digests, size_t cap);

/* ---- Dedup index --------------------------------------
 * The chunk Database of the reference keyed by SHA-256 digest
 * (src/system/database.rs:74-87: HashMap, `entry(key).or_insert`, i.e. the
 * FIRST insert of a digest wins) and the storage statistics built on it
 * (src/system/storage.rs:193-240), as a device hash set. */
typedef struct cdc_index cdc_index_t;

typedef struct cdc_index_stats {
    uint64_t chunks_written;  /* chunks inserted so far */
    uint64_t bytes_written;   /* size_written: bytes of all inserted chunks */
    uint64_t unique_chunks;   /* distinct digests */
    uint64_t unique_bytes;    /* total_cdc_size: bytes of the first chunk of each digest */
} cdc_index_stats_t;
/* cdc_dedup_ratio = bytes_written / unique_bytes (storage.rs:203-205);
 * average_chunk_size = unique_bytes / unique_chunks (storage.rs:208-220). */

/* Index on `device` for up to `capacity` distinct digests. */
int cdc_index_create(int device, size_t capacity, cdc_index_t **out);
void cdc_index_destroy(cdc_index_t *ix);
/* Database::clear + size_written = 0 (storage.rs:236-240). */
int cdc_index_clear(cdc_index_t *ix);
/* Database::insert of n (digest, chunk) pairs in chunk order (DEVICE arrays:
 * 32-byte digests, cdc_chunk_t records).  d_new (nullable, DEVICE u8[n])
 * receives 1 where the chunk's digest was not in the index before it.
 * Returns the number of new digests (CDC_ENOMEM past capacity). */
int64_t cdc_index_insert_device(cdc_index_t *ix, const uint8_t *d_digests,
                                const cdc_chunk_t *d_chunks, size_t n,
                                uint8_t *d_new, void *hip_stream);
int cdc_index_stats(const cdc_index_t *ix, cdc_index_stats_t *out);

/* ---- Synthetic data -----------------------------------------
 * Fill a DEVICE buffer with the splitmix64 stream: little-endian u64 words,
 * word i = mix64(seed + (i+1) * 0x9E3779B97F4A7C15). */
int cdc_fill_splitmix64_device(uint8_t *d_buf, size_t len, uint64_t seed,
                               void *hip_stream);

/* Engine build info, e.g. "chunkfs_amd 0.5 gfx950 abi 3". */
const char *cdc_version(void);

/* CHUNKFS_AMD_ABI_VERSION of the loaded library (compare with the header's). */
uint32_t cdc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CHUNKFS_AMD_H */
