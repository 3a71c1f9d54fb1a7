#!/usr/bin/env python3
"""bench.py -- device-resident FastCDC throughput on MI355X (BASELINE.json metric).

A "step" = one full pass of the chunking hot path (scan -> resolve -> compact,
final Chunk{offset,length} list in HBM) over the rank's synthetic input, which
is already resident in HBM when the timed region starts.

Workload at N=1 (BASELINE.json configs[1]): one 1 GiB
stream of splitmix64(seed=1) bytes, FastCDC min/avg/max = 4/8/16 KiB.  At N>1
every rank chunks its own 1 GiB stream (seed 1+rank): independent streams,
no data-path collective, weak scaling.  `--workload batch`
runs config 4 instead: 1024 streams of 64 MiB (stream i: seed 1000+i) split
into contiguous blocks across the ranks, strong scaling
(chunkfs_amd/sharding.py).  `host_path` records the PCIe-inclusive rate of
the host-buffer entry point beside `value` (never as it).

Rank 0 prints ONE JSON line.  `roofline` is for the scan kernel (the only
HBM-bound kernel): achieved = input bytes per launch / average scan-kernel
duration measured with HIP events around that launch on its own stream.
`cpu_baseline` times the oracle's scalar C restatement (oracle/cdc_oracle.c)
on a bounded sample on this host, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["stream", "batch"], default="stream")
    p.add_argument("--stream-bytes", type=int, default=1 << 30)
    p.add_argument("--batch-streams", type=int, default=1024,
                   help="config 4: total streams, split across ranks (strong scaling)")
    p.add_argument("--batch-stream-bytes", type=int, default=64 << 20)
    p.add_argument("--min", type=int, default=4096)
    p.add_argument("--avg", type=int, default=8192)
    p.add_argument("--max", type=int, default=16384)
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline budget (rank 0, N=1 only); 0 disables")
    p.add_argument("--cpu-threads", type=int, default=16,
                   help="also time the oracle on this many host threads (one stream each); 0 disables")
    p.add_argument("--no-parity", action="store_true", help="skip the one-off oracle check")
    p.add_argument("--hash", action="store_true", help="also report the SHA-256 fingerprint rate (§8f row 2)")
    p.add_argument("--no-host-path", action="store_true",
                   help="skip the one-off host-buffer (PCIe-inclusive) rate")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_pmc_traffic.json"))
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import chunkfs_amd as cfa
    from chunkfs_amd import _lib, sharding

    ch = cfa.FastChunker(cfa.SizeParams(args.min, args.avg, args.max), device=local)

    if args.workload == "stream":
        shard = sharding.stream_shard(rank, world, args.stream_bytes)
    else:
        shard = sharding.batch_shard(rank, world, args.batch_streams, args.batch_stream_bytes)
    lens, seeds = shard.lens, shard.seeds
    bufs = []
    for n, s in zip(lens, seeds):
        b = torch.empty(n, dtype=torch.uint8, device=dev)
        _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, s, None))
        bufs.append(b)
    ptrs = [b.data_ptr() for b in bufs]
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def step():
        return ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)

    for _ in range(args.warmup):
        first = step()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    scan_ms = []
    total_ms = []
    rewalked = []
    resolve_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        first = step()
        t = ch.last_timing()
        scan_ms.append(t["scan_ms"])
        total_ms.append(t["total_ms"])
        rewalked.append(t["fixup_iterations"])  # spans whose speculative chain was re-walked
        resolve_ms.append(t["resolve_ms"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = sharding.max_over_ranks(time.perf_counter() - t0, dev)

    bytes_rank = sum(lens)
    total_bytes = sharding.sum_over_ranks(bytes_rank, dev) * args.steps
    value = sharding.aggregate_gibps(total_bytes, elapsed)
    scan_avg_ms = sum(scan_ms) / len(scan_ms)
    achieved = bytes_rank / (scan_avg_ms * 1e-3) / 1e9  # GB/s, algorithmic bytes of one launch
    nchunks = int(first[-1])

    # SHA-256 of every chunk of stream 0 (device-resident),
    # reported beside the chunking metric (not part of `value`).
    fingerprint = None
    if args.hash and lens and lens[0]:
        n0 = int(first[1]) - int(first[0])
        dig = torch.empty((max(n0, 1), 32), dtype=torch.uint8, device=dev)
        hms = []
        for _ in range(3):
            ch.sha256_chunks_device(bufs[0].data_ptr(), out.data_ptr(), n0, dig.data_ptr())
            hms.append(ch.last_timing()["hash_ms"])
        hm = sorted(hms)[1]
        fingerprint = {"algo": "SHA-256 per chunk (Sha256Hasher)", "chunks": n0, "kernel_ms": hm,
                       "GiBps": lens[0] / (hm * 1e-3) / (1 << 30)}

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("workload_bytes") == bytes_rank and tj.get("kernel", "").startswith("scan_kernel"):
                traffic = tj.get("hbm_read_bytes_per_launch")
        except Exception:
            traffic = None

    # PCIe-inclusive rate of the host boundary (cdc_chunk_data on a pageable
    # host buffer: H2D, pipeline, D2H of the chunk list).  Recorded beside
    # `value`, never as it.
    host_path = None
    if rank == 0 and world == 1 and not args.no_host_path:
        hb = bufs[0].cpu().numpy()
        ch.chunk_array(hb)  # warm the host-path staging
        reps, t_h = 3, time.perf_counter()
        for _ in range(reps):
            hc = ch.chunk_array(hb)
        t_h = (time.perf_counter() - t_h) / reps
        host_path = {"GiBps": hb.size / t_h / (1 << 30), "bytes": int(hb.size), "chunks": int(hc.shape[0]),
                     "entry": "cdc_chunk_data (pageable host buffer -> H2D -> pipeline -> D2H chunks)"}
        # The reference harness's own path (src/bench/mod.rs:93-140): the
        # StorageWriter loop over 1 MiB segments, throughput = bytes / summed
        # chunk_data time (storage.rs:314-316).
        fs_bytes = min(hb.size, 256 << 20)
        spans, chunk_s = cfa.write_spans(ch, hb[:fs_bytes])
        host_path["fs_write_1MiB_segments"] = {
            "GiBps": fs_bytes / chunk_s / (1 << 30), "bytes": int(fs_bytes), "spans": int(spans.size),
            "metric": "bytes / summed chunk_data seconds, as CDCFixture::measure"}

    parity = None
    cpu_baseline = None
    if rank == 0 and world == 1 and (not args.no_parity or args.cpu_seconds > 0):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        host = [b.cpu().numpy() for b in bufs[:1]]
        if not args.no_parity:
            got = out[:int(first[1])].cpu().numpy().view(np.uint64)
            ref = oracle.fastcdc(host[0], args.min, args.avg, args.max)
            parity = bool(got.shape == ref.shape and (got == ref).all())
        if args.cpu_seconds > 0:
            secs, passes, done = 0.0, 0, 0
            while passes == 0 or secs < args.cpu_seconds:
                t, _ = oracle.time_fastcdc(host[0], args.min, args.avg, args.max)
                secs += t
                passes += 1
                done += host[0].size
            cpu_baseline = {
                "value": done / secs / (1 << 30),
                "unit": "GiB/s",
                "cores": 1,
                "kind": "port",
                "sample": f"{passes} whole-buffer pass(es) over stream 0 ({host[0].size} B) of this workload; "
                          "oracle/cdc_oracle.c scalar C restatement of fastcdc v2020 (gcc -O3), single thread",
            }
            if args.cpu_threads > 1:
                thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
                nb, wall = oracle.time_fastcdc_threads(host[0], args.min, args.avg, args.max, thr,
                                                       args.cpu_seconds / 2)
                cpu_baseline["multi_thread"] = {
                    "value": nb / wall / (1 << 30), "unit": "GiB/s", "cores": thr,
                    "sample": f"{thr} threads, each chunking its own {host[0].size // thr} B slice of stream 0 "
                              f"as an independent stream for ~{args.cpu_seconds / 2:.0f} s"}

    if rank == 0:
        line = {
            "metric": "GiB/s chunked device-resident, FastCDC 4/8/16 KiB avg, at 1/2/4/8 MI355X",
            "value": value,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": shard.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {
                "workload": ("config2: 1 x 1 GiB stream per GPU" if args.workload == "stream"
                             else f"config4: {args.batch_streams} x {args.batch_stream_bytes} B streams "
                                  f"split across {world} GPU(s)"),
                "algo": "FastCDC v2020 (Level1)", "min": args.min, "avg": args.avg, "max": args.max,
                "bytes_per_gpu": bytes_rank, "streams_per_gpu": len(lens), "chunks_per_gpu": nchunks,
                "parallelism": f"independent streams x{world}, no collective",
                "pipeline": int(os.environ.get("CHUNKFS_AMD_PIPELINE", "1")),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "scan_kernel (gear candidate scan)", "kernel_ms": scan_avg_ms,
            },
            "cpu_baseline": cpu_baseline,
            "host_path": host_path,
            "fingerprint": fingerprint,
            "phase_ms": {"scan": scan_avg_ms, "total_device": sum(total_ms) / len(total_ms),
                         "resolve": sum(resolve_ms) / len(resolve_ms),
                         "rewalked_spans": max(rewalked)},
            "parity_vs_oracle": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
