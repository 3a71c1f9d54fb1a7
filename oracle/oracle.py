"""ctypes wrapper of the CPU oracle (oracle/libcdc_oracle.so) + a pure-Python twin.

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product (chunkfs_amd/).

Parity status: FastCDC "parity unpinned" vs the fastcdc 3.1.0 crate (the GEAR
table is a placeholder, see include/chunkfs_amd_tables.h); FSChunker and the
1 MiB write-path segmentation are pinned by the reference's known answers
(tests/filesystem.rs:135-166, src/system/storage.rs:471-485).
"""
import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libcdc_oracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_fastcdc_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                           u64p, u64p, ctypes.c_uint64]
        L.oracle_fastcdc_chunk.restype = ctypes.c_int64
        L.oracle_fixed_chunk.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64]
        L.oracle_fixed_chunk.restype = ctypes.c_int64
        L.oracle_fs_write.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                      u64p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double)]
        L.oracle_fs_write.restype = ctypes.c_int64
        L.oracle_fill_splitmix64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_fill_splitmix64.restype = None
        L.oracle_fastcdc_masks.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u64p, u64p]
        L.oracle_fastcdc_masks.restype = ctypes.c_int
        L.oracle_time_fastcdc.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_time_fastcdc.restype = ctypes.c_double
        L.oracle_cdc_chunk.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, u64p, u64p,
                                       ctypes.c_uint64]
        L.oracle_cdc_chunk.restype = ctypes.c_int64
        L.oracle_cdc_chunk_p.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, u64p,
                                         u64p, ctypes.c_uint64]
        L.oracle_cdc_chunk_p.restype = ctypes.c_int64
        L.oracle_cdc_check.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_cdc_check.restype = ctypes.c_int
        L.oracle_leap_threshold.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_leap_threshold.restype = ctypes.c_uint32
        L.oracle_cdc_tables.argtypes = [u64p, u64p, u64p]
        L.oracle_cdc_tables.restype = None
        L.oracle_time_cdc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_time_cdc.restype = ctypes.c_double
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def splitmix64_bytes(n, seed):
    buf = np.empty(n, dtype=np.uint8)
    lib().oracle_fill_splitmix64(_ptr(buf), n, seed)
    return buf


def masks(mn, avg, mx):
    s, l = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().oracle_fastcdc_masks(mn, avg, mx, ctypes.byref(s), ctypes.byref(l))
    if rc:
        raise ValueError("invalid FastCDC sizes")
    return s.value, l.value


def fastcdc(data, mn, avg, mx, gear=None):
    """(n, 2) uint64 array of (offset, length): FastCDC v2020 over the whole buffer."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n = data.size
    cap = n // max(2 * (mn // 2), 1) + 2
    off = np.empty(cap, dtype=np.uint64)
    ln = np.empty(cap, dtype=np.uint64)
    g = None if gear is None else np.ascontiguousarray(gear, dtype=np.uint64)
    cnt = lib().oracle_fastcdc_chunk(_ptr(data), n, mn, avg, mx, None if g is None else _ptr(g),
                                     _u64p(off), _u64p(ln), cap)
    if cnt < 0:
        raise ValueError("invalid FastCDC sizes")
    assert cnt <= cap
    return np.stack([off[:cnt], ln[:cnt]], axis=1)


def fixed(n, cs):
    cap = n // cs + 2
    off = np.empty(cap, dtype=np.uint64)
    ln = np.empty(cap, dtype=np.uint64)
    cnt = lib().oracle_fixed_chunk(n, cs, _u64p(off), _u64p(ln), cap)
    return np.stack([off[:cnt], ln[:cnt]], axis=1)


# cdc_algo_t numbering (include/chunkfs_amd.h).
ALGOS = {"fast": 0, "fixed": 1, "rabin": 2, "ultra": 4, "leap": 5, "seq": 6}


def cdc(algo, data, mn, avg, mx, seqcfg=None, rabin_poly=None):
    """(n, 2) uint64 (offset, length) of Rabin / Ultra / Leap / Seq over the whole
    buffer (oracle/cdc_oracle.c; parity unpinned, see the header there).
    seqcfg = (mode, seq_length, jump_trigger, jump_size) for "seq"; rabin_poly
    = a Rabin polynomial other than the built-in one (cdc_set_rabin_poly)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n = data.size
    cap = n // mn + 2
    off = np.empty(cap, dtype=np.uint64)
    ln = np.empty(cap, dtype=np.uint64)
    cfg = None if seqcfg is None else np.ascontiguousarray(seqcfg, dtype=np.uint32)
    cnt = lib().oracle_cdc_chunk_p(ALGOS[algo], _ptr(data), n, mn, avg, mx,
                                   None if cfg is None else _ptr(cfg), int(rabin_poly or 0), _u64p(off),
                                   _u64p(ln), cap)
    if cnt < 0:
        raise ValueError("invalid sizes")
    assert cnt <= cap
    return np.stack([off[:cnt], ln[:cnt]], axis=1)


def time_cdc(algo, data, mn, avg, mx):
    """Single-thread wall seconds of one whole-buffer pass (cpu_baseline)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cnt = ctypes.c_int64(0)
    t = lib().oracle_time_cdc(ALGOS[algo], _ptr(data), data.size, mn, avg, mx, ctypes.byref(cnt))
    return t, cnt.value


def fs_write(algo, data, mn, avg=0, mx=0, seg_size=1 << 20, gear=None):
    """StorageWriter mirror: span lengths of one write call, and summed chunk_data seconds."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = data.size // max(2 * (mn // 2), 1) + 2
    out = np.empty(cap, dtype=np.uint64)
    secs = ctypes.c_double(0.0)
    g = None if gear is None else np.ascontiguousarray(gear, dtype=np.uint64)
    cnt = lib().oracle_fs_write(ALGOS[algo], _ptr(data), data.size, mn, avg, mx,
                                None if g is None else _ptr(g), seg_size, _u64p(out), cap,
                                ctypes.byref(secs))
    if cnt < 0:
        raise ValueError("invalid arguments")
    return out[:cnt], secs.value


def time_fastcdc_threads(data, mn, avg, mx, threads, seconds):
    """Aggregate CPU rate with `threads` workers, each chunking its own slice of
    `data` as an independent stream (one thread per stream on
    the host cores).  The C oracle runs without the GIL (ctypes).  Returns
    (bytes processed, wall seconds)."""
    import threading
    import time as _t
    data = np.ascontiguousarray(data, dtype=np.uint8)
    per = data.size // threads
    slices = [data[i * per:(i + 1) * per] for i in range(threads)]
    done = [0] * threads
    stop = _t.perf_counter() + seconds

    def work(i):
        while True:
            time_fastcdc(slices[i], mn, avg, mx)
            done[i] += slices[i].size
            if _t.perf_counter() >= stop:
                return

    t0 = _t.perf_counter()
    ws = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    return sum(done), _t.perf_counter() - t0


def time_fastcdc(data, mn, avg, mx):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    c = ctypes.c_int64()
    t = lib().oracle_time_fastcdc(_ptr(data), data.size, mn, avg, mx, ctypes.byref(c))
    return t, c.value


# ---------------------------------------------------------------------------
# Pure-Python twin (small inputs only): an independent restatement of
# SURVEY.md Appendix A.2 in the BYTE-WISE form  h = (h << 1) + GEAR[b],
# tested against the mask at every position -- a different code shape from the
# C oracle's two-bytes-per-iteration loop, so the two cross-check each other.

def _tables():
    path = os.path.join(ROOT, "include", "chunkfs_amd_tables.h")
    txt = open(path).read()
    import re
    def grab(name):
        body = txt.split(name, 1)[1].split("{", 1)[1].split("}", 1)[0]
        return [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]+)ULL", body)]
    return grab("CHUNKFS_AMD_GEAR["), grab("CHUNKFS_AMD_MASKS[")


def py_fastcdc(data, mn, avg, mx, gear=None):
    g, M = _tables()
    if gear is not None:
        g = [int(x) for x in gear]
    bits = int(round(math.log2(avg)))
    ms, ml = M[bits + 1], M[bits - 1]
    data = bytes(bytearray(np.asarray(data, dtype=np.uint8)))
    out = []
    pos = 0
    n = len(data)
    M64 = (1 << 64) - 1
    while pos < n:
        rem = n - pos
        if rem <= mn:
            cut = rem
        else:
            center = avg
            if rem > mx:
                rem = mx
            elif rem < center:
                center = rem
            a0, ce, re_ = (mn // 2) * 2, (center // 2) * 2, (rem // 2) * 2
            h = 0
            cut = rem
            for p in range(a0, re_):
                h = ((h << 1) + g[data[pos + p]]) & M64
                if h & (ms if p < ce else ml) == 0:
                    cut = p
                    break
        out.append((pos, cut))
        pos += cut
    return np.array(out, dtype=np.uint64).reshape(-1, 2)


# ---------------------------------------------------------------------------
# Pure-Python twins of the Rabin / Ultra / Leap / Seq restatements (small
# inputs only).  Different code shapes from the C oracle: Rabin by direct
# GF(2) polynomial arithmetic (no tables), Ultra with the 8-byte distance
# recomputed at every tested position (C keeps it incrementally).

def _cdc_params():
    path = os.path.join(ROOT, "include", "chunkfs_amd_cdc_params.h")
    txt = open(path).read()
    import re
    d = {}
    for k, v in re.findall(r"#define (CDC_[A-Z_]+) (0x[0-9A-Fa-f]+|[0-9]+)", txt):
        d[k] = int(v, 0)
    body = txt.split("CDC_LEAP_THRESHOLD[33]", 1)[1].split("{", 1)[1].split("}", 1)[0]
    d["THR"] = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]+)u", body)]
    return d


def _log2_round(x):
    b = x.bit_length() - 1
    if 0 < b < 63 and x - (1 << b) >= (1 << b) // 2:
        b += 1
    return b


def _polmod(x, p):
    dp = p.bit_length() - 1
    while x and x.bit_length() - 1 >= dp:
        x ^= p << (x.bit_length() - 1 - dp)
    return x


def _mix64(z):
    M = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def _py_cut(algo, d, s, n, mn, avg, mx, P, cfg):
    if n <= mn:
        return n
    end = min(n, mx)
    if algo == "rabin":
        W, poly = P["CDC_RABIN_WINDOW"], P["CDC_RABIN_POLY"]
        xw = _polmod(1 << (8 * W), poly)  # x^(8W) mod P
        mask = (1 << _log2_round(avg)) - 1
        start = mn - W if mn >= W else 0
        h = 0
        for i in range(start, end):
            o = d[s + i - W] if i >= start + W else 0
            h = (h << 8) ^ d[s + i]
            # subtract o * x^(8W): multiply o by xw in GF(2)
            t = 0
            for bit in range(8):
                if (o >> bit) & 1:
                    t ^= xw << bit
            h = _polmod(h ^ t, poly)
            if i + 1 >= mn and (h & mask) == 0:
                return i + 1
        return end
    if algo == "ultra":
        pat = P["CDC_ULTRA_PATTERN"]
        normal = avg
        end = n
        if n >= mx:
            end = mx
        elif n <= normal:
            normal = n
        lec = 0
        i = mn
        while i + 8 <= end:
            blk_in, blk_out = d[s + i:s + i + 8], d[s + i - 8:s + i]
            if blk_in == blk_out:
                lec += 1
                if lec >= P["CDC_ULTRA_LEST"]:
                    return i + 8
                i += 8
                continue
            lec = 0
            mask = P["CDC_ULTRA_MASK_L"] if i >= normal else P["CDC_ULTRA_MASK_S"]
            for j in range(8):
                q = s + i + j
                dist = sum(bin(b ^ pat).count("1") for b in d[q - 8:q])
                if dist & mask == 0:
                    return i + j
            i += 8
        return end
    if algo == "leap":
        M = (1 << 64) - 1
        E = [_mix64((P["CDC_LEAP_SEED"] + (b + 1) * 0x9E3779B97F4A7C15) & M) for b in range(256)]
        thr = P["THR"][min(_log2_round(max(avg - mn, 1)), 32)]

        def h(p):
            v = 0
            for j in range(P["CDC_LEAP_WSIZE"]):
                e, r = E[d[s + p - j]], (11 * j) % 64
                v = (v + (((e << r) | (e >> (64 - r))) & M if r else e)) & M
            return v
        c = mn
        while c <= end:
            k = 0
            while k < P["CDC_LEAP_WINDOWS"]:
                v = h(c - 1 - k)
                v = v >> 32 if k < P["CDC_LEAP_PRIMARY"] else v & 0xFFFFFFFF
                if v >= thr:
                    break
                k += 1
            if k == P["CDC_LEAP_WINDOWS"]:
                return c
            c += P["CDC_LEAP_WINDOWS"] - k
        return end
    if algo == "seq":
        mode, length, trig, jump = cfg
        cnt = opp = 0
        i = mn
        while i < end:
            a, b = d[s + i - 1], d[s + i]
            if (b < a) if mode else (b > a):
                cnt += 1
                if cnt >= length:
                    return i + 1
            else:
                cnt = 0
                opp += 1
                if opp >= trig:
                    opp = 0
                    i += jump
                    continue
            i += 1
        return end
    raise ValueError(algo)


def py_cdc(algo, data, mn, avg, mx, seqcfg=None):
    P = _cdc_params()
    cfg = tuple(seqcfg) if seqcfg is not None else (0, P["CDC_SEQ_LENGTH"], P["CDC_SEQ_JUMP_TRIGGER"],
                                                     P["CDC_SEQ_JUMP_SIZE"])
    d = bytes(bytearray(np.asarray(data, dtype=np.uint8)))
    out, pos = [], 0
    while pos < len(d):
        cut = _py_cut(algo, d, pos, len(d) - pos, mn, avg, mx, P, cfg)
        out.append((pos, cut))
        pos += cut
    return np.array(out, dtype=np.uint64).reshape(-1, 2)
