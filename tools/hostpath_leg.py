#!/usr/bin/env python3
"""The bench's host_path leg alone (bench.host_path_leg) on a 256 MiB
splitmix64 stream: the whole-buffer cdc_chunk_data rate, the reference's
1 MiB chunk_data loop (timed inside the C library and by Python) and the
streaming write.  Diagnostics only.  usage: tools/hostpath_leg.py [MiB]"""
import json
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd.synthetic import splitmix64_bytes  # noqa: E402

n = (int(sys.argv[1]) if len(sys.argv) > 1 else 256) << 20
buf = torch.from_numpy(splitmix64_bytes(n, 1)).to("cuda:0")
eng = SimpleNamespace(ch=c.FastChunker(c.SizeParams(4096, 8192, 16384)), sizes=(4096, 8192, 16384))
w = SimpleNamespace(bufs=[buf], lens=[n])
hp = bench.host_path_leg(eng, w)
print(json.dumps(hp["chunk_data_1MiB_calls"]))
print(json.dumps({k: v for k, v in hp["write_stream_1MiB_segments"].items() if k != "metric"}))
