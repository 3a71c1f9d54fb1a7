"""ctypes binding of libchunkfs_amd.so (include/chunkfs_amd.h).

Loading fails loudly: there is no CPU fallback anywhere in the product.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# CHUNKFS_AMD_LIB: an experiment build of the same sources (tools/scan_variants.sh)
LIB_PATH = os.environ.get("CHUNKFS_AMD_LIB") or os.path.join(HERE, "libchunkfs_amd.so")

CDC_OK = 0
CDC_EINVAL = -1
CDC_ENOMEM = -2
CDC_EDEVICE = -3
CDC_ENOTSUP = -4

ALGO = {"fast": 0, "fixed": 1, "rabin": 2, "super": 3, "ultra": 4, "leap": 5, "seq": 6}

# Every symbol include/chunkfs_amd.h declares (tests check the export table).
EXPORTS = [
    "cdc_create", "cdc_create_seq", "cdc_destroy", "cdc_chunk_data", "cdc_estimate_chunk_count",
    "cdc_max_chunk_count", "cdc_describe", "cdc_last_error", "cdc_set_gear", "cdc_set_rabin_poly",
    "cdc_chunk_batch_device", "cdc_chunk_batch_device_async", "cdc_batch_sync", "cdc_batch_max_chunks",
    "cdc_last_timing",
    "cdc_fs_write", "cdc_write_begin", "cdc_write_segment", "cdc_write_drain", "cdc_write_finish",
    "cdc_sha256_chunks_device", "cdc_sha256_batch_device", "cdc_chunk_and_hash",
    "cdc_index_create", "cdc_index_destroy", "cdc_index_clear", "cdc_index_insert_device",
    "cdc_index_stats",
    "cdc_fill_splitmix64_device", "cdc_version", "cdc_abi_version",
]
# include/chunkfs_amd_debug.h (diagnostics, not part of the drop-in boundary)
DEBUG_EXPORTS = ["cdc_debug_pipeline", "cdc_debug_record_cap", "cdc_debug_copy", "cdc_debug_host_stats",
                 "cdc_debug_read_bw", "cdc_debug_host_placement",
                 "cdc_debug_timing_back"]


class CdcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"chunkfs_amd error {code}: {msg}")
        self.code = code


class cdc_chunk_t(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("length", ctypes.c_uint64)]


class cdc_index_stats_t(ctypes.Structure):
    _fields_ = [("chunks_written", ctypes.c_uint64), ("bytes_written", ctypes.c_uint64),
                ("unique_chunks", ctypes.c_uint64), ("unique_bytes", ctypes.c_uint64)]


class cdc_timing_t(ctypes.Structure):
    _fields_ = [
        ("scan_ms", ctypes.c_double),
        ("resolve_ms", ctypes.c_double),
        ("compact_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("fixup_iterations", ctypes.c_uint32),
        ("overflow_spans", ctypes.c_uint32),
        ("candidates", ctypes.c_uint64),
        ("bytes", ctypes.c_uint64),
        ("hash_ms", ctypes.c_double),
        ("walk_fallback_steps", ctypes.c_uint64),
        ("path", ctypes.c_uint32),   # CDC_PATH_*: 0 pipeline, 1 small kernel, 2 walk, 3 fixed, 4 empty
        ("timed", ctypes.c_uint32),  # 1: the *_ms fields are HIP-event measurements
    ]


_lib = None


def lib():
    """Load and type the shared library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP engine is the only implementation; there is no CPU fallback)")
    # PyTorch-ROCm wheels bundle their own libamdhip64 (same SONAME
    # libamdhip64.so.7 as /opt/rocm's).  If ours were loaded first, a later
    # `import torch` would map a SECOND HIP runtime into the process and fail
    # ("No HIP GPUs are available").  Importing torch first makes our NEEDED
    # libamdhip64.so.7 resolve to the already-loaded copy: one runtime, shared
    # device pointers and streams.  Without torch the system runtime is used.
    if "torch" not in sys.modules and not os.environ.get("CHUNKFS_AMD_NO_TORCH"):
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    sz = ctypes.c_size_t
    L.cdc_create.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                             ctypes.c_int, ctypes.POINTER(P)]
    L.cdc_create.restype = ctypes.c_int
    u32 = ctypes.c_uint32
    L.cdc_create_seq.argtypes = [u32, u32, u32, u32, u32, u32, u32, ctypes.c_int, ctypes.POINTER(P)]
    L.cdc_create_seq.restype = ctypes.c_int
    L.cdc_destroy.argtypes = [P]
    L.cdc_destroy.restype = None
    L.cdc_chunk_data.argtypes = [P, P, sz, ctypes.POINTER(cdc_chunk_t), sz]
    L.cdc_chunk_data.restype = ctypes.c_int64
    L.cdc_estimate_chunk_count.argtypes = [P, sz]
    L.cdc_estimate_chunk_count.restype = sz
    L.cdc_max_chunk_count.argtypes = [P, sz]
    L.cdc_max_chunk_count.restype = sz
    L.cdc_describe.argtypes = [P]
    L.cdc_describe.restype = ctypes.c_char_p
    L.cdc_last_error.argtypes = []
    L.cdc_last_error.restype = ctypes.c_char_p
    L.cdc_set_gear.argtypes = [P, u64p]
    L.cdc_set_gear.restype = ctypes.c_int
    L.cdc_set_rabin_poly.argtypes = [P, ctypes.c_uint64]
    L.cdc_set_rabin_poly.restype = ctypes.c_int
    L.cdc_chunk_batch_device.argtypes = [P, sz, P, P, P, sz, P, P]
    L.cdc_chunk_batch_device.restype = ctypes.c_int64
    L.cdc_chunk_batch_device_async.argtypes = [P, sz, P, P, P, sz, P, P]
    L.cdc_chunk_batch_device_async.restype = ctypes.c_int64
    L.cdc_batch_sync.argtypes = [P]
    L.cdc_batch_sync.restype = ctypes.c_int64
    L.cdc_batch_max_chunks.argtypes = [P, sz, u64p]
    L.cdc_batch_max_chunks.restype = sz
    L.cdc_last_timing.argtypes = [P, ctypes.POINTER(cdc_timing_t), sz]
    L.cdc_last_timing.restype = ctypes.c_int
    L.cdc_fs_write.argtypes = [P, P, sz, sz, u64p, sz, ctypes.POINTER(ctypes.c_double)]
    L.cdc_fs_write.restype = ctypes.c_int64
    L.cdc_write_begin.argtypes = [P]
    L.cdc_write_begin.restype = ctypes.c_int
    L.cdc_write_segment.argtypes = [P, P, sz]
    L.cdc_write_segment.restype = ctypes.c_int
    L.cdc_write_drain.argtypes = [P, u64p, sz]
    L.cdc_write_drain.restype = ctypes.c_int64
    L.cdc_write_finish.argtypes = [P, u64p, sz, ctypes.POINTER(ctypes.c_double)]
    L.cdc_write_finish.restype = ctypes.c_int64
    L.cdc_debug_host_stats.argtypes = [P, ctypes.POINTER(ctypes.c_double), sz]
    L.cdc_debug_host_stats.restype = ctypes.c_int
    L.cdc_debug_timing_back.argtypes = [P, ctypes.c_uint32, ctypes.POINTER(cdc_timing_t), sz]
    L.cdc_debug_timing_back.restype = ctypes.c_int
    L.cdc_sha256_chunks_device.argtypes = [P, P, P, sz, P, P]
    L.cdc_sha256_chunks_device.restype = ctypes.c_int
    L.cdc_sha256_batch_device.argtypes = [P, sz, P, P, P, P, P]
    L.cdc_sha256_batch_device.restype = ctypes.c_int
    L.cdc_chunk_and_hash.argtypes = [P, P, sz, ctypes.POINTER(cdc_chunk_t), u8p, sz]
    L.cdc_chunk_and_hash.restype = ctypes.c_int64
    L.cdc_index_create.argtypes = [ctypes.c_int, sz, ctypes.POINTER(P)]
    L.cdc_index_create.restype = ctypes.c_int
    L.cdc_index_destroy.argtypes = [P]
    L.cdc_index_destroy.restype = None
    L.cdc_index_clear.argtypes = [P]
    L.cdc_index_clear.restype = ctypes.c_int
    L.cdc_index_insert_device.argtypes = [P, P, P, sz, P, P]
    L.cdc_index_insert_device.restype = ctypes.c_int64
    L.cdc_index_stats.argtypes = [P, ctypes.POINTER(cdc_index_stats_t)]
    L.cdc_index_stats.restype = ctypes.c_int
    L.cdc_fill_splitmix64_device.argtypes = [P, sz, ctypes.c_uint64, P]
    L.cdc_fill_splitmix64_device.restype = ctypes.c_int
    L.cdc_debug_pipeline.argtypes = [P]
    L.cdc_debug_pipeline.restype = ctypes.c_int
    L.cdc_debug_record_cap.argtypes = [P]
    L.cdc_debug_record_cap.restype = ctypes.c_uint32
    L.cdc_debug_read_bw.argtypes = [P, P, sz, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.cdc_debug_read_bw.restype = ctypes.c_int
    L.cdc_debug_host_placement.argtypes = [P, ctypes.c_char_p, sz]
    L.cdc_debug_host_placement.restype = ctypes.c_int64
    L.cdc_debug_copy.argtypes = [P, ctypes.c_int, P, sz]
    L.cdc_debug_copy.restype = ctypes.c_int64
    L.cdc_version.argtypes = []
    L.cdc_version.restype = ctypes.c_char_p
    L.cdc_abi_version.argtypes = []
    L.cdc_abi_version.restype = ctypes.c_uint32
    del u8p
    _lib = L
    return L


def check(rc):
    """Raise CdcError for a negative return code, else return rc."""
    if rc < 0:
        raise CdcError(rc, lib().cdc_last_error().decode())
    return rc
