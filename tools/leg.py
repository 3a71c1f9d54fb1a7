"""Run one bench.py leg by itself on the GPU box (A/B and profiling runs):
    python tools/leg.py config3|algos|lowent|config5_1gpu|config4|host [bench args...]
Prints the leg's JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    leg, argv = sys.argv[1], sys.argv[2:]
    args = bench.parse(argv)
    import torch
    torch.cuda.set_device(0)
    if leg == "config3":
        out = bench.config3_line(args, 0)
    else:
        eng = bench.DeviceEngine(args, 0)
        from chunkfs_amd import sharding
        shard = sharding.stream_shard(0, 1, args.stream_bytes)
        w = eng.prepare(shard.lens, shard.seeds)
        bench._SETTLE.append((eng, w, args.settle_ms))
        if leg == "algos":
            out = bench.algo_lines(args, eng, w, 3)
        elif leg == "lowent":
            out = bench.lowentropy_walk_lines(args, eng)
        elif leg == "config5_1gpu":
            out = bench.config5_lines(args, eng, w)
        elif leg == "config4":
            del w
            out = bench.config4_leg(args, eng, 0, 1, None)
        elif leg == "host":
            out = bench.host_path_leg(eng, w)
        else:
            sys.exit(f"unknown leg {leg}")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
