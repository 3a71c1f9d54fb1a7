"""Executable model of the GPU decomposition (DESIGN.md "Pipeline and kernels"),
checked against the sequential oracle on the CPU.

The GPU replaces the reference's sequential cut loop (fastcdc v2020
`cut_gear`) by: a windowed-hash candidate scan; per-record
links to the next chunk start; per-span speculative chain walks from a
warm-up start, settled against the previous span's exit (fastcdc.hip
resolve_kernel).  This model restates those steps in numpy/Python with the same
span size, warm-up, regime and record semantics, so a flaw in the
decomposition itself (not in its HIP code) shows up here, on CPU.
"""
import numpy as np
import pytest

import oracle

SPAN = 1 << 16
M64 = (1 << 64) - 1


def _params(mn, avg, mx):
    gear, masks = oracle._tables()
    bits = int(round(np.log2(avg)))
    return np.array(gear, dtype=np.uint64), masks[bits + 1], masks[bits - 1]


def windowed_hash(data, gear):
    """W[i] = sum_{k<48} GEAR[b[i-k]] << k  (mod 2^64): bits 0..47 of the
    in-chunk hash at i whenever the chunk's hash started >= 48 bytes earlier."""
    g = gear[data]
    W = np.zeros(data.size, dtype=np.uint64)
    for k in range(48):
        W[k:] += g[:data.size - k] << np.uint64(k)
    return W


def regime(s, n, mn, avg, mx):
    rem = n - s
    center = avg
    if rem > mx:
        rem = mx
    elif rem < center:
        center = rem
    a0, ce, re_ = (mn // 2) * 2, (center // 2) * 2, (rem // 2) * 2
    return rem, a0, ce, re_


class Model:
    def __init__(self, data, mn, avg, mx):
        self.d = np.ascontiguousarray(data, dtype=np.uint8)
        self.n = self.d.size
        self.mn, self.avg, self.mx = mn, avg, mx
        self.gear, self.ms, self.ml = _params(mn, avg, mx)
        top = max(int(self.ms | self.ml).bit_length() - 1, 0)
        self.trunc = top
        W = windowed_hash(self.d, self.gear)
        cm = np.uint64(self.ms & self.ml)
        self.rec = np.nonzero((W & cm) == 0)[0]  # candidate records (scan_kernel)
        self.hit_s = (W[self.rec] & np.uint64(self.ms)) == 0
        self.hit_l = (W[self.rec] & np.uint64(self.ml)) == 0
        self.idx = {int(p): i for i, p in enumerate(self.rec)}
        self.nxt = {}

    def step(self, s):
        """Start of the chunk after the one starting at s (an exact step)."""
        n = self.n
        if n - s <= self.mn:
            return n
        rem, a0, ce, re_ = regime(s, n, self.mn, self.avg, self.mx)
        tl = min(a0 + self.trunc, re_)
        h = 0
        for p in range(a0, tl):  # truncated positions: exact in-chunk hash
            h = ((h << 1) + int(self.gear[self.d[s + p]])) & M64
            if h & (self.ms if p < ce else self.ml) == 0:
                return s + p
        if tl >= re_:
            return s + rem
        j = np.searchsorted(self.rec, s + tl)
        while j < self.rec.size and self.rec[j] < s + re_:
            c = int(self.rec[j])
            if (self.hit_s[j] if c - s < ce else self.hit_l[j]):
                return c
            j += 1
        return s + rem

    def link(self, s):
        """the precomputed link when s is a record, else a lane step."""
        if s in self.idx:
            if s not in self.nxt:
                self.nxt[s] = self.step(s)
            return self.nxt[s]
        return self.step(s)

    def walk(self, s, off, end):
        starts = []
        while s < end:
            if s >= off:
                starts.append(s)
            s = self.link(s)
        return starts, s

    def chunks(self, warm_spans=2):
        n = self.n
        spans = []
        for off in range(0, n, SPAN):
            end = min(off + SPAN, n)
            w0 = max(off - warm_spans * self.mx, 0)
            st, ex = self.walk(w0, off, end)
            spans.append([off, end, st, ex, st[0] if st else ex])
        # settle: a span whose entry differs from its predecessor's exit re-walks
        # from it (the walk kernel does this in-wave, then across waves).
        changed, passes = True, 0
        while changed:
            changed, passes = False, passes + 1
            for i in range(1, len(spans)):
                off, end, st, ex, entry = spans[i]
                pe = spans[i - 1][3]
                if entry != pe:
                    st, ex = self.walk(pe, off, end)
                    spans[i] = [off, end, st, ex, pe]
                    changed = True
        starts = [s for sp in spans for s in sp[2]]
        lengths = np.diff(np.array(starts + [n], dtype=np.int64))
        return np.stack([np.array(starts, dtype=np.uint64), lengths.astype(np.uint64)], axis=1)


@pytest.mark.parametrize("sizes,n,seed", [
    ((4096, 8192, 16384), 1 << 20, 1),
    ((4096, 8192, 16384), (1 << 20) + 54321, 2),
    ((2048, 8192, 65536), 3 << 19, 3),
    ((8192, 16384, 65536), 1 << 20, 4),
    ((1000, 3000, 9000), 700_001, 5),
])
def test_decomposition_matches_sequential_oracle(sizes, n, seed):
    data = oracle.splitmix64_bytes(n, seed)
    got = Model(data, *sizes).chunks()
    ref = oracle.fastcdc(data, *sizes)
    assert got.shape == ref.shape and (got == ref).all()


def test_windowed_hash_equals_in_chunk_hash_after_47_positions():
    """The identity the scan rests on: 48+ positions after a chunk's hash
    reset, the windowed hash agrees with the in-chunk hash on bits 0..47."""
    data = oracle.splitmix64_bytes(4096, 9)
    gear, ms, ml = _params(4096, 8192, 16384)
    W = windowed_hash(data, gear)
    h = 0
    for i in range(1000, 2000):
        h = ((h << 1) + int(gear[data[i]])) & M64
        if i - 1000 >= 47:
            assert (h ^ int(W[i])) & ((1 << 48) - 1) == 0
