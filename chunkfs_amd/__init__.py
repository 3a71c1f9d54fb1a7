"""chunkfs_amd -- MI355X-native content-defined chunking behind chunkfs's Chunker API.

Host-side mirror of the reference's chunking surface, over the C ABI in
include/chunkfs_amd.h (libchunkfs_amd.so, hand-written HIP for gfx950):

    reference (Rust)                          here
    Chunk            src/lib.rs:43-66         Chunk
    Chunker trait    src/lib.rs:74-86         Chunker.chunk_data / estimate_chunk_count
    SizeParams       src/chunkers/mod.rs:1    SizeParams
    FastChunker      src/chunkers/fast.rs     FastChunker
    FSChunker        src/chunkers/fixed_size  FSChunker
    Rabin/Ultra/Leap/Seq src/chunkers/*.rs    RabinChunker, UltraChunker, LeapChunker,
                                              SeqChunker (published algorithms; parity
                                              unpinned: cdc-chunkers 0.1.3 absent)
    SuperChunker                              raises NotImplementedError
    ChunkStorage::write  system/storage.rs    write_spans()

Every call runs on the GPU.  There is no CPU fallback: without the built
library or a gfx950 device the constructors raise.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import ALGO, CdcError, cdc_chunk_t, cdc_timing_t, check, lib

KB = 1024
MB = 1024 * KB
GB = 1024 * MB
SEG_SIZE = MB  # src/lib.rs:39

__all__ = [
    "KB", "MB", "GB", "SEG_SIZE", "Chunk", "SizeParams", "Chunker", "FastChunker",
    "FSChunker", "RabinChunker", "SuperChunker", "UltraChunker", "LeapChunker",
    "SeqChunker", "OperationMode", "SeqConfig", "CdcError", "write_spans", "StreamWriter", "version",
]


class Chunk:
    """A chunk of processed data: offset and length only (src/lib.rs:41-66)."""

    __slots__ = ("_offset", "_length")

    def __init__(self, offset, length):
        self._offset = int(offset)
        self._length = int(length)

    def offset(self):
        return self._offset

    def length(self):
        return self._length

    def range(self):
        return range(self._offset, self._offset + self._length)

    def __eq__(self, other):
        return isinstance(other, Chunk) and (self._offset, self._length) == (other._offset, other._length)

    def __hash__(self):
        return hash((self._offset, self._length))

    def __repr__(self):
        return f"Chunk {{ offset: {self._offset}, length: {self._length} }}"


class SizeParams:
    """cdc_chunkers::SizeParams {min, avg, max} (re-exported at src/chunkers/mod.rs:1)."""

    __slots__ = ("min", "avg", "max")

    def __init__(self, min, avg, max):  # noqa: A002 -- reference field names
        self.min, self.avg, self.max = int(min), int(avg), int(max)

    def __repr__(self):
        return f"SizeParams {{ min: {self.min}, avg: {self.avg}, max: {self.max} }}"

    def __eq__(self, other):
        return isinstance(other, SizeParams) and (self.min, self.avg, self.max) == (other.min, other.avg, other.max)


def _as_buffer(data):
    """(pointer, length, keepalive) for bytes / bytearray / numpy / memoryview."""
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    else:
        arr = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    return arr.ctypes.data_as(ctypes.c_void_p), arr.size, arr


class Chunker:
    """The Chunker trait (src/lib.rs:74-86), backed by one GPU handle.

    Not thread-safe, like the reference's Mutex-serialised ChunkerRef.
    """

    _algo = None

    def __init__(self, algo, min, avg, max, device=0):  # noqa: A002
        L = lib()
        h = ctypes.c_void_p()
        rc = L.cdc_create(ALGO[algo], min, avg, max, device, ctypes.byref(h))
        if rc == -4:
            raise NotImplementedError(L.cdc_last_error().decode())
        check(rc)
        self._h = h
        self._pending = []  # first[] arrays of enqueued batches (chunk_batch_device_async)
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().cdc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- trait methods -------------------------------------------------------
    def chunk_array(self, data):
        """chunk_data as an (n, 2) uint64 array of (offset, length)."""
        ptr, n, keep = _as_buffer(data)
        cap = lib().cdc_max_chunk_count(self._h, n)
        out = np.empty((max(cap, 1), 2), dtype=np.uint64)
        cnt = check(lib().cdc_chunk_data(self._h, ptr, n,
                                         out.ctypes.data_as(ctypes.POINTER(cdc_chunk_t)), cap))
        self._drained()
        del keep
        assert cnt <= cap
        return out[:cnt]

    def chunk_and_hash(self, data):
        """chunk_data plus Sha256Hasher::hash (src/hashers.rs:20-36) of every
        chunk, as StorageWriter::write computes them (storage.rs:324-329).
        Returns ((n, 2) uint64 chunks, (n, 32) uint8 SHA-256 digests)."""
        ptr, n, keep = _as_buffer(data)
        cap = lib().cdc_max_chunk_count(self._h, n)
        out = np.empty((max(cap, 1), 2), dtype=np.uint64)
        dig = np.empty((max(cap, 1), 32), dtype=np.uint8)
        cnt = check(lib().cdc_chunk_and_hash(self._h, ptr, n,
                                             out.ctypes.data_as(ctypes.POINTER(cdc_chunk_t)),
                                             dig.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap))
        self._drained()
        del keep
        assert cnt <= cap
        return out[:cnt], dig[:cnt]

    def sha256_chunks_device(self, d_data, d_chunks, n_chunks, d_digests, stream=None):
        """SHA-256 of n_chunks chunks of one device-resident stream (device pointers)."""
        check(lib().cdc_sha256_chunks_device(self._h, ctypes.c_void_p(d_data), ctypes.c_void_p(d_chunks),
                                             n_chunks, ctypes.c_void_p(d_digests),
                                             None if stream is None else ctypes.c_void_p(stream)))

    def sha256_batch_device(self, d_ptrs, first, d_chunks, d_digests, stream=None):
        """SHA-256 of every chunk of a multi-stream batch in one launch
        (cdc_sha256_batch_device): stream i's chunks are d_chunks[first[i] ..
        first[i+1]), offsets relative to d_ptrs[i]."""
        ptrs = np.ascontiguousarray(np.asarray(d_ptrs, dtype=np.uint64))
        fa = np.ascontiguousarray(np.asarray(first, dtype=np.uint64))
        assert fa.size == ptrs.size + 1
        check(lib().cdc_sha256_batch_device(self._h, int(ptrs.size), ctypes.c_void_p(ptrs.ctypes.data),
                                            ctypes.c_void_p(fa.ctypes.data), ctypes.c_void_p(int(d_chunks)),
                                            ctypes.c_void_p(int(d_digests)),
                                            None if stream is None else ctypes.c_void_p(stream)))
        self._drained()

    def chunk_data(self, data, empty=None):
        """Chunker::chunk_data (src/lib.rs:80): chunks tiling `data`, appended to `empty`."""
        chunks = [] if empty is None else empty
        chunks.extend(Chunk(int(o), int(l)) for o, l in self.chunk_array(data))
        return chunks

    def estimate_chunk_count(self, data):
        """Chunker::estimate_chunk_count (src/lib.rs:85) -- the reference formula."""
        if isinstance(data, int):
            n = data
        elif isinstance(data, np.ndarray):
            n = data.nbytes
        else:
            n = memoryview(data).nbytes
        return lib().cdc_estimate_chunk_count(self._h, n)

    def max_chunk_count(self, n):
        return lib().cdc_max_chunk_count(self._h, n)

    def __repr__(self):  # impl Debug
        return lib().cdc_describe(self._h).decode()

    # -- device-resident batch (configs 2, 4) --------------------------------
    def chunk_batch_device(self, d_ptrs, lens, d_out_ptr, out_cap, stream=0):
        """Chunk n streams already in HBM.  Returns the host array first[n+1].
        `d_ptrs` / `lens` may be uint64 numpy arrays (no per-call conversion)."""
        ptrs = np.ascontiguousarray(np.asarray(d_ptrs, dtype=np.uint64))
        lens_a = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        n = int(lens_a.size)
        first = np.empty(n + 1, dtype=np.uint64)
        check(lib().cdc_chunk_batch_device(self._h, n, ctypes.c_void_p(ptrs.ctypes.data),
                                           ctypes.c_void_p(lens_a.ctypes.data), ctypes.c_void_p(int(d_out_ptr)),
                                           out_cap, ctypes.c_void_p(first.ctypes.data),
                                           ctypes.c_void_p(int(stream))))
        self._drained()
        return first

    def chunk_batch_device_async(self, d_ptrs, lens, d_out_ptr, out_cap, stream=0):
        """cdc_chunk_batch_device_async: enqueue the batch (FastCDC batches of
        more than 8 MiB run back to back with no host wait between them).
        Returns its first[n+1] array, filled by batch_sync()."""
        ptrs = np.ascontiguousarray(np.asarray(d_ptrs, dtype=np.uint64))
        lens_a = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        n = int(lens_a.size)
        first = np.zeros(n + 1, dtype=np.uint64)
        pend = self.__dict__.setdefault("_pending", [])
        pend.append(first)  # the library writes it when the batch is collected
        check(lib().cdc_chunk_batch_device_async(self._h, n, ctypes.c_void_p(ptrs.ctypes.data),
                                                 ctypes.c_void_p(lens_a.ctypes.data),
                                                 ctypes.c_void_p(int(d_out_ptr)), out_cap,
                                                 ctypes.c_void_p(first.ctypes.data), ctypes.c_void_p(int(stream))))
        # At most 3 batches are in flight (a submit collects the batch 3 before
        # it), so older arrays are already written: keep only those 3.
        del pend[:-3]
        return first

    def _drained(self):
        """Every library call but an async submit completes the batches in
        flight first (include/chunkfs_amd.h): their first[] arrays are written."""
        self.__dict__["_pending"] = []

    def batch_sync(self):
        """cdc_batch_sync: complete every enqueued batch; the last one's chunk count."""
        r = check(lib().cdc_batch_sync(self._h))
        self._drained()
        return r

    def batch_max_chunks(self, lens):
        n = len(lens)
        lens_a = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in lens])
        return lib().cdc_batch_max_chunks(self._h, n, lens_a)

    def last_timing(self):
        t = cdc_timing_t()
        check(lib().cdc_last_timing(self._h, ctypes.byref(t), ctypes.sizeof(t)))
        self._drained()
        return {f: getattr(t, f) for f, _ in cdc_timing_t._fields_}

    def timing_back(self, back):
        """Kernel times of the FastCDC batch `back` calls before the last one
        (0 = last, <= 63; include/chunkfs_amd_debug.h cdc_debug_timing_back)."""
        t = cdc_timing_t()
        check(lib().cdc_debug_timing_back(self._h, back, ctypes.byref(t), ctypes.sizeof(t)))
        return {f: getattr(t, f) for f, _ in cdc_timing_t._fields_}

    def set_gear(self, gear):
        g = np.ascontiguousarray(gear, dtype=np.uint64)
        assert g.shape == (256,)
        check(lib().cdc_set_gear(self._h, g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))


class FastChunker(Chunker):
    """FastCDC 2020 (src/chunkers/fast.rs); default sizes 8/16/64 KiB (fast.rs:17-27)."""

    def __init__(self, sizes=None, device=0):
        sizes = sizes or SizeParams(8 * KB, 16 * KB, 64 * KB)
        self.sizes = sizes
        super().__init__("fast", sizes.min, sizes.avg, sizes.max, device)

    @classmethod
    def default(cls):
        return cls()


class FSChunker(Chunker):
    """Fixed-size chunking (src/chunkers/fixed_size.rs); default 4096 (fixed_size.rs:26-30)."""

    def __init__(self, chunk_size=4096, device=0):
        self.chunk_size = chunk_size
        super().__init__("fixed", chunk_size, 0, 0, device)

    @classmethod
    def default(cls):
        return cls()


class _SizedChunker(Chunker):
    """Common constructor of the chunkers built on the segment-walk engine.

    The reference's Default sizes (SizeParams::{rabin,ultra,leap,seq}_default)
    live in cdc-chunkers 0.1.3, absent offline, so sizes are always explicit.
    Cut rules restate the published algorithms: parity unpinned."""

    _name = None

    def __init__(self, sizes, device=0):
        if sizes is None:
            raise TypeError(f"{self._name}: pass SizeParams explicitly (the crate's defaults are unknown here)")
        self.sizes = sizes
        super().__init__(self._algo, sizes.min, sizes.avg, sizes.max, device)


class RabinChunker(_SizedChunker):
    """Rabin CDC (src/chunkers/rabin.rs:34-56): 48-byte window fingerprint modulo
    a degree-53 polynomial, cut where digest & (2^round(log2 avg) - 1) == 0."""
    _algo, _name = "rabin", "RabinChunker"

    def set_poly(self, poly):
        """Install another polynomial (cdc_set_rabin_poly; degree 9..56): the
        one-call hook for the crate's ChunkerParams once its source exists."""
        check(lib().cdc_set_rabin_poly(self._h, int(poly)))


class UltraChunker(_SizedChunker):
    """UltraCDC (src/chunkers/ultra.rs:30-44): 8-byte Hamming distance to 0xAA..,
    two masks around the normal size, low-entropy (LEST) early cut."""
    _algo, _name = "ultra", "UltraChunker"


class LeapChunker(_SizedChunker):
    """Leap-shaped CDC for LeapChunker (src/chunkers/leap.rs:30-44): 24 eligible
    windows before a cut, leaping past a failing window, as in the Leap-based
    CDC paper.  The window eligibility function is a STAND-IN (a seeded table
    hash against a threshold, include/chunkfs_amd_cdc_params.h), not the
    published one the crate builds from random draws: parity unpinned."""
    _algo, _name = "leap", "LeapChunker"


class OperationMode:
    """seq::OperationMode (re-exported at src/chunkers/seq.rs:3)."""
    Increasing = 0
    Decreasing = 1


class SeqConfig:
    """seq::Config (re-exported at src/chunkers/seq.rs:3); defaults of
    include/chunkfs_amd_cdc_params.h (the crate's field names are unknown)."""

    __slots__ = ("seq_length", "jump_trigger", "jump_size")

    def __init__(self, seq_length=5, jump_trigger=50, jump_size=256):
        self.seq_length, self.jump_trigger, self.jump_size = int(seq_length), int(jump_trigger), int(jump_size)

    def __repr__(self):
        return (f"Config {{ seq_length: {self.seq_length}, jump_trigger: {self.jump_trigger}, "
                f"jump_size: {self.jump_size} }}")


class SeqChunker(Chunker):
    """SeqCDC (src/chunkers/seq.rs:40-55): SeqChunker::new(mode, sizes, config).
    estimate_chunk_count is len / avg (seq.rs:52-54), unlike the others."""

    _algo = "seq"

    def __init__(self, mode=OperationMode.Increasing, sizes=None, config=None, device=0):
        if sizes is None:
            raise TypeError("SeqChunker: pass SizeParams explicitly (the crate's defaults are unknown here)")
        self.mode, self.sizes = int(mode), sizes
        self.config = config or SeqConfig()
        L = lib()
        h = ctypes.c_void_p()
        check(L.cdc_create_seq(self.mode, self.config.seq_length, self.config.jump_trigger,
                               self.config.jump_size, sizes.min, sizes.avg, sizes.max, device, ctypes.byref(h)))
        self._h = h
        self.device = device


class SuperChunker(Chunker):
    """SuperCDC (src/chunkers/supercdc.rs:35-57): NOT implemented.  Its cut rule
    and the cross-call `records` map live in cdc-chunkers 0.1.3, absent offline;
    the constructor raises NotImplementedError (CDC_ENOTSUP)."""

    _algo = "super"

    def __init__(self, sizes=None, device=0):
        s = sizes or SizeParams(2 * KB, 8 * KB, 64 * KB)
        super().__init__("super", s.min, s.avg, s.max, device)


def write_spans(chunker, data, seg_size=SEG_SIZE):
    """ChunkStorage::write (storage.rs:78-103) for one write call (seg_size
    segments through the streaming write path).

    Returns (span lengths in file order, wall seconds of the whole call: host
    copy + H2D + chunking, not the reference's chunk_data-only time).
    """
    ptr, n, keep = _as_buffer(data)
    cap = chunker.max_chunk_count(n) + 1  # spans are chunks: all but the last are >= min
    out = np.empty(max(cap, 1), dtype=np.uint64)
    secs = ctypes.c_double(0.0)
    cnt = check(lib().cdc_fs_write(chunker._h, ptr, n, seg_size,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap,
                                   ctypes.byref(secs)))
    del keep
    assert cnt <= cap
    return out[:cnt], secs.value


class StreamWriter:
    """One file write through the streaming write path (cdc_write_begin /
    cdc_write_segment / cdc_write_finish): ChunkStorage::write_from_stream
    (storage.rs:105-137) with StorageWriter::write per segment and
    StorageWriter::flush at the end (storage.rs:302-383).  Segments are copied
    into a pinned ring and uploaded while the caller continues; drain()
    returns the spans that became final so far (each chunked 256 MiB device
    window), finish() the rest and the wall seconds since begin."""

    def __init__(self, chunker):
        self._ch = chunker
        self._bytes = 0
        check(lib().cdc_write_begin(chunker._h))

    def write(self, segment):
        ptr, n, keep = _as_buffer(segment)
        check(lib().cdc_write_segment(self._ch._h, ptr, n))
        del keep
        self._bytes += n

    def drain(self):
        """Span lengths final since the last drain (cdc_write_drain), file order."""
        cap = self._ch.max_chunk_count(self._bytes) + 1
        out = np.empty(max(cap, 1), dtype=np.uint64)
        cnt = check(lib().cdc_write_drain(self._ch._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap))
        return out[:cnt]

    def finish(self):
        cap = self._ch.max_chunk_count(self._bytes) + 1
        out = np.empty(max(cap, 1), dtype=np.uint64)
        secs = ctypes.c_double(0.0)
        cnt = check(lib().cdc_write_finish(self._ch._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap,
                                           ctypes.byref(secs)))
        assert cnt <= cap
        return out[:cnt], secs.value


def host_stats(chunker):
    """cdc_debug_host_stats: chunk_data calls, upload s, total s; streaming
    write chunking s and segments; one-launch small-stream calls and how many
    of them fell back to the regular pipeline."""
    v = (ctypes.c_double * 7)()
    check(lib().cdc_debug_host_stats(chunker._h, v, 7))
    return {"calls": int(v[0]), "upload_s": v[1], "total_s": v[2], "write_chunk_s": v[3], "write_segments": int(v[4]),
            "small_calls": int(v[5]), "small_fallbacks": int(v[6])}


def host_placement(chunker):
    """cdc_debug_host_placement: the device's PCI address, NUMA node and link;
    the node the pinned ring and chunk list landed on; copy-helper pinning."""
    import json
    buf = ctypes.create_string_buffer(1024)
    n = lib().cdc_debug_host_placement(chunker._h, buf, 1024)
    check(n)
    return json.loads(buf.value.decode())


class DedupIndex:
    """The reference's chunk Database keyed by SHA-256 digest (database.rs:74-87,
    first insert wins) with its storage statistics (storage.rs:193-240), as a
    device hash set on one GPU."""

    def __init__(self, capacity, device=0):
        h = ctypes.c_void_p()
        check(lib().cdc_index_create(device, capacity, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().cdc_index_destroy(h)
            self._h = None

    def insert_device(self, d_digests, d_chunks, n, d_new=None, stream=None):
        """Database::insert of n (digest, chunk) pairs (device pointers), in chunk
        order.  Returns the number of new digests; d_new (optional u8[n]) marks them."""
        return check(lib().cdc_index_insert_device(
            self._h, ctypes.c_void_p(d_digests), ctypes.c_void_p(d_chunks), n,
            None if d_new is None else ctypes.c_void_p(d_new),
            None if stream is None else ctypes.c_void_p(stream)))

    def clear(self):
        check(lib().cdc_index_clear(self._h))

    def stats(self):
        s = _lib.cdc_index_stats_t()
        check(lib().cdc_index_stats(self._h, ctypes.byref(s)))
        d = {f: getattr(s, f) for f, _ in _lib.cdc_index_stats_t._fields_}
        d["cdc_dedup_ratio"] = d["bytes_written"] / d["unique_bytes"] if d["unique_bytes"] else float("nan")
        d["average_chunk_size"] = d["unique_bytes"] // d["unique_chunks"] if d["unique_chunks"] else 0
        return d


def version():
    return lib().cdc_version().decode()
