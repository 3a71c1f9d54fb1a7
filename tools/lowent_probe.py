#!/usr/bin/env python3
"""Diagnostics (GPU): time the walk rules on the bench's low-entropy inputs
(zeros, random with 1-32 MiB zero regions), a few calls each, for a
rocprofv3 kernel split.  usage: tools/lowent_probe.py [algo ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402
import oracle  # noqa: E402

n = 256 << 20
runs = torch.from_numpy(oracle.splitmix64_bytes(n, 17)).to("cuda:0")
rng = np.random.default_rng(17)
pos = int(rng.integers(1, 1 << 20))
while pos < n:
    ln = int(rng.integers(1 << 20, 32 << 20))
    runs[pos:pos + ln] = 0
    pos += ln + int(rng.integers(1 << 16, 8 << 20))
sp = c.SizeParams(4096, 8192, 16384)
for name in sys.argv[1:] or ["rabin", "ultra", "leap", "seq"]:
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(name)
    ch = cls(sp) if cls else c.SeqChunker(0, sp)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ch.chunk_batch_device([runs.data_ptr()], [n], out.data_ptr(), cap)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    t = ch.last_timing()
    print(f"{name} zero_runs {n / el / 2**30:.1f} GiB/s  {el * 1e3:.2f} ms  rewalked {t['fixup_iterations']}"
          f"  in_order {bool(t['overflow_spans'])}", flush=True)
    ch.close()
