#!/usr/bin/env python3
"""Segment-walk engine on low-entropy inputs (diagnostics only): every walk rule
(Rabin / Ultra / Leap / Seq) over device-resident zeros, a 61-byte period and
splitmix64 bytes, at the bench sizes and config 5's size triples; device time,
fix-up statistics (re-walked segments, serial pass taken) and parity vs the
oracle.

Usage: python3 tools/lowent_probe.py [bytes] [inputs,comma,separated]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402
import oracle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["zeros", "periodic61", "splitmix64"]
sizes = [(4096, 8192, 16384), (512, 2048, 16384), (2048, 8192, 65536), (16384, 65536, 524288)]
inputs = {
    "zeros": np.zeros(n, dtype=np.uint8),
    "periodic61": np.resize(oracle.splitmix64_bytes(61, 7), n),
    "splitmix64": oracle.splitmix64_bytes(n, 1),
}
for inp in which:
    host = inputs[inp]
    dev = torch.from_numpy(host).to("cuda:0")
    for sz in sizes:
        for name in ("rabin", "ultra", "leap", "seq"):
            cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(name)
            s = c.SizeParams(*sz)
            ch = cls(s) if cls else c.SeqChunker(0, s)
            cap = ch.batch_max_chunks([n])
            out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
            t0 = time.perf_counter()
            first = ch.chunk_batch_device([dev.data_ptr()], [n], out.data_ptr(), cap)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            t = ch.last_timing()
            got = out[:int(first[1])].cpu().numpy().view(np.uint64)
            t1 = time.perf_counter()
            ref = oracle.cdc(name, host, *sz)
            t_cpu = time.perf_counter() - t1
            ok = bool(got.shape == ref.shape and (got == ref).all())
            print(f"{inp:10s} {name:5s} {sz!s:22s} {n / el / 2**30:8.2f} GiB/s  walk {t['scan_ms']:8.3f} ms  "
                  f"rest {t['resolve_ms']:9.3f} ms  rewalked {t['fixup_iterations']:6d}  serial {t['overflow_spans']}"
                  f"  chunks {int(first[1]):8d}  parity {ok}  cpu {n / t_cpu / 2**30:.2f} GiB/s", flush=True)
            ch.close()
            del out
    del dev
