"""Config-4 scan-rate probe (verdict r05 item 2): the same FastCDC batch step
over stream layouts that separate data size from buffer count.
    python tools/c4_probe.py VARIANT [steps]
VARIANT: c2      1 x 1 GiB buffer (config 2)
         c4      1024 x 64 MiB separate buffers (config 4)
         c4one   1024 x 64 MiB slices of ONE 64 GiB buffer
         g16     16 x 64 MiB separate buffers (1 GiB in config 4's buffers)
         big1    1 x 64 GiB buffer, one stream
Prints ms/step, scan ms (HIP events) and scan GB/s per step."""
import ctypes
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

MB = 1 << 20


def fill(ptr, n, seed):
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(ptr), n, seed, None))


def main():
    v = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    keep = []
    if v == "c2":
        lens = [1 << 30]
    elif v in ("c4", "c4one"):
        lens = [64 * MB] * 1024
    elif v == "g16":
        lens = [64 * MB] * 16
    elif v == "big1":
        lens = [64 << 30]
    else:
        sys.exit("variant?")
    if v == "c4one":
        big = torch.empty(sum(lens), dtype=torch.uint8, device="cuda")
        keep.append(big)
        ptrs = [big.data_ptr() + i * 64 * MB for i in range(len(lens))]
    else:
        for n in lens:
            keep.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
        ptrs = [b.data_ptr() for b in keep]
    for i, (p, n) in enumerate(zip(ptrs, lens)):
        fill(p, n, 1000 + i)
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    pa, la = np.array(ptrs, dtype=np.uint64), np.array(lens, dtype=np.uint64)
    for _ in range(2):
        ch.chunk_batch_device(pa, la, out.data_ptr(), cap)
    torch.cuda.synchronize()
    res = []
    for _ in range(steps):
        t0 = time.perf_counter()
        ch.chunk_batch_device(pa, la, out.data_ptr(), cap)  # synchronous: every step timed by events
        el = time.perf_counter() - t0
        t = ch.last_timing()
        res.append((el * 1e3, t["scan_ms"], t["resolve_ms"]))
    tot = sum(lens)
    ms = sorted(r[0] for r in res)[len(res) // 2]
    scan = sorted(r[1] for r in res)[len(res) // 2]
    res_ms = sorted(r[2] for r in res)[len(res) // 2]
    print(json.dumps({"variant": v, "streams": len(lens), "bytes": tot, "ms_per_step": ms, "scan_ms": scan,
                      "resolve_ms": res_ms, "scan_GBps": tot / (scan * 1e-3) / 1e9,
                      "scan_ms_per_GiB": scan / (tot / (1 << 30)),
                      "scan_ms_all": [round(r[1], 4) for r in res]}), flush=True)


if __name__ == "__main__":
    main()
