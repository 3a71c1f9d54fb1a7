#!/usr/bin/env python3
"""bench.py -- device-resident FastCDC throughput on MI355X (BASELINE.json metric).

A "step" = one full pass of the chunking hot path (candidate scan -> chain
resolve -> Chunk{offset,length} list in HBM) over the rank's synthetic input,
which is already resident in HBM when the timed region starts.

Workloads:
  * `value` (default `--workload stream`, every N): BASELINE configs[1] /
    config 2 -- one 1 GiB stream of splitmix64(seed=1+rank) bytes per GPU,
    FastCDC 4/8/16 KiB, weak scaling: the per-GPU work is the same at every N,
    so the driver's N=1 line is the matching denominator of its 1->8 curve.
  * `config5` sub-object (every N, unless --no-config5): config 5 -- 16 x 1 GiB
    streams (stream i: seed 5000+i) split across the ranks, UltraCDC / LeapCDC
    (+ Rabin, SeqCDC) at avg 2 / 8 / 64 KiB, strong scaling, no collective.
  * `config4` sub-object (every N, unless --no-config4): config 4 -- 1024
    independent 64 MiB streams (stream i: seed 1000+i) split into contiguous
    blocks across the ranks, strong scaling, no data-path collective
    (chunkfs_amd/sharding.py).  At N > 1 rank 0 also times the whole 1024-
    stream batch alone in the same run, the N=1 denominator of that line's
    strong-scaling efficiency.  `--workload batch` makes config 4 `value`.

Launch: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
environment starts `torch.distributed.run` with N ranks as a CHILD process
(this process never touches the GPU) and exits with its status.  Under an
external launcher WORLD_SIZE must equal --gpus.

Rank 0 prints ONE JSON line.  `roofline` is for the scan kernel (the only
HBM-bound kernel): achieved = input bytes per launch / average scan-kernel
duration measured with HIP events around that launch on the engine's stream,
over the synchronous calls of latency_leg (rank 0, N=1), where each scan has
the chip to itself: the headline's two-stream schedule starts each scan while
the previous resolve still holds CUs, so its event span includes that wait
(reported beside it as `kernel_ms_in_pipeline`; at N > 1 the roofline uses
it).
`roofline.traffic` comes from a PMC file under profiles/ only when that
file's recorded source digest equals this build's (chunkfs_amd.build).
`cpu_baseline` times the oracle's scalar C restatement (oracle/cdc_oracle.c)
on a bounded sample on this host, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, HBM section)
METRIC = "GiB/s chunked device-resident, FastCDC 4/8/16 KiB avg, at 1/2/4/8 MI355X"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--settle-ms", type=float, default=60.0,
                   help="device warm-up before the warmup steps: untimed steps of the workload for this long "
                        "(clocks and the two-stream schedule settle over the first ~20 ms of load); 0 = none")
    p.add_argument("--workload", choices=["stream", "batch"], default="stream",
                   help="what `value` measures: stream = config 2 per GPU (weak), batch = config 4 (strong)")
    p.add_argument("--stream-bytes", type=int, default=1 << 30)
    p.add_argument("--batch-streams", type=int, default=1024,
                   help="config 4: total streams, split across ranks (strong scaling)")
    p.add_argument("--batch-stream-bytes", type=int, default=64 << 20)
    p.add_argument("--no-config4", action="store_true",
                   help="skip the config-4 (1024 x 64 MiB, strong scaling) sub-object")
    p.add_argument("--config4-steps", type=int, default=5)
    p.add_argument("--min", type=int, default=4096)
    p.add_argument("--avg", type=int, default=8192)
    p.add_argument("--max", type=int, default=16384)
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline budget (rank 0, N=1 only); 0 disables")
    p.add_argument("--cpu-threads", type=int, default=-1,
                   help="threads for the multi-thread CPU leg (-1: every usable host core, 0: off)")
    p.add_argument("--no-parity", action="store_true", help="skip the one-off oracle check")
    p.add_argument("--no-sweep", action="store_true",
                   help="skip the avg 4/16 KiB and low-entropy lines (N=1)")
    p.add_argument("--no-algos", action="store_true",
                   help="skip the Rabin / Ultra / Leap / Seq lines (N=1)")
    p.add_argument("--hash", action="store_true", help="also report the SHA-256 fingerprint rate (§8f row 2)")
    p.add_argument("--no-host-path", action="store_true",
                   help="skip the one-off host-buffer (PCIe-inclusive) rates")
    p.add_argument("--config5-bytes", type=int, default=1 << 30,
                   help="bytes of the bench stream the config-5 size sweep chunks")
    p.add_argument("--no-config5", action="store_true",
                   help="skip the config-5 (16 GiB, walk rules at 2/8/64 KiB, strong scaling) sub-object")
    p.add_argument("--config5-streams", type=int, default=16,
                   help="config 5: total streams, split across ranks (strong scaling)")
    p.add_argument("--config5-stream-bytes", type=int, default=1 << 30, help="config 5: bytes per stream")
    p.add_argument("--config5-check", type=int, default=-1,
                   help="config 5: bytes of the checked streams compared with the oracle (-1: whole streams)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)  # CPU launcher test only
    # Multi-rank rehearsal on a box with fewer GPUs than ranks (tests only):
    # ranks mapped onto the visible devices round-robin, and every rank checks
    # its own first streams against the oracle.
    # The only collectives are the barrier and the scalar timing / byte-count
    # reductions (no data-path collective): gloo on the host by
    # default; nccl (= RCCL) reduces on the devices instead.
    p.add_argument("--dist-backend", choices=["gloo", "nccl"], default="gloo",
                   help="backend of the barrier and the scalar reductions (default gloo)")
    p.add_argument("--share-device", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--rank-parity", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


# ---------------------------------------------------------------------------
# Launcher

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """Start args.gpus ranks under torch.distributed.run as a child process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------
# Engines: the HIP engine, and a CPU stub (fixed-size cuts in numpy) that lets
# tests/test_bench_launcher.py exercise the launcher and the reductions with
# gloo on a machine without a GPU.  The stub is never a product path.

class Work:
    """One workload resident on the rank's device: streams, output, capacity."""

    def __init__(self, lens):
        self.lens = list(lens)
        self.bufs, self.out = [], None


class DeviceEngine:
    def __init__(self, args, local):
        import torch
        import chunkfs_amd as cfa
        from chunkfs_amd import _lib
        self.torch, self.cfa, self._lib = torch, cfa, _lib
        self.dev = torch.device("cuda", local)
        self.local = local
        self.ch = cfa.FastChunker(cfa.SizeParams(args.min, args.avg, args.max), device=local)
        self.sizes = (args.min, args.avg, args.max)

    def prepare(self, lens, seeds):
        import numpy as np
        torch = self.torch
        w = Work(lens)
        for n, s in zip(lens, seeds):
            b = torch.empty(max(n, 16), dtype=torch.uint8, device=self.dev)
            self._lib.check(self._lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, s, None))
            w.bufs.append(b)
        w.ptrs_a = np.array([b.data_ptr() for b in w.bufs], dtype=np.uint64)  # converted once, not per step
        w.lens_a = np.array(w.lens, dtype=np.uint64)
        w.cap = self.ch.batch_max_chunks(w.lens)
        w.out = torch.empty((max(w.cap, 1), 2), dtype=torch.int64, device=self.dev)
        torch.cuda.synchronize()
        return w

    def step(self, w):
        """Enqueue one pass (cdc_chunk_batch_device_async): back-to-back FastCDC
        batches run with no host round trip between them, and sync() completes
        them; the returned first[] is filled then."""
        return self.ch.chunk_batch_device_async(w.ptrs_a, w.lens_a, w.out.data_ptr(), w.cap)

    def timing(self):
        return self.ch.last_timing()

    def read_bw(self, w, reps=10):
        """Measured-achievable HBM read rate: a read-only reduction over the same
        bytes (cdc_debug_read_bw), GB/s."""
        ms = ctypes.c_double()
        self._lib.check(self._lib.lib().cdc_debug_read_bw(self.ch._h, ctypes.c_void_p(w.bufs[0].data_ptr()),
                                                         int(w.lens[0]), reps, ctypes.byref(ms)))
        return w.lens[0] / (ms.value * 1e-3) / 1e9, ms.value

    def timings(self, k):
        """HIP-event timings of the last k batches (oldest first), read after
        the timed loop from the engine's event ring (no per-step event wait
        inside the loop; include/chunkfs_amd_debug.h).  Async batches carry
        events one in four (CHUNKFS_AMD_EVENT_EVERY; an event costs the stream
        ~4 us): the timed steps' sampled batches."""
        allt = [self.ch.timing_back(b) for b in range(min(k, 64) - 1, -1, -1)]
        return [t for t in allt if t["timed"]]  # (may be empty: callers report the timing as unavailable)

    def sync_step(self, w):
        """One synchronous batch (cdc_chunk_batch_device): submit, wait, first[]
        filled on return -- the single-batch latency, nothing pipelined."""
        return self.ch.chunk_batch_device(w.ptrs_a, w.lens_a, w.out.data_ptr(), w.cap)

    def sync(self):
        self.ch.batch_sync()
        self.torch.cuda.synchronize()

    def settle(self, w, ms):
        """Device warm-up before the warmup steps: untimed back-to-back steps
        of the workload for >= ms of wall time, then a drain.  MI355X clocks
        ramp over the first tens of ms of load: with 3 warmup steps and no
        settle the timed steps ran at 0.322 ms, after 60 ms of read-only
        passes at 0.276 (profiles/r05/r05ac_*); the two-stream schedule's
        step keeps falling for ~70 steps (~20 ms) of its own load whatever ran
        before it (0.32 -> 0.255 ms, profiles/r06/r06z_*), so the settle runs
        the workload itself.  `sustained` (>= 150 ms of timed steps) checks
        that the figure holds."""
        if not w.lens or not w.lens[0]:
            return
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            self.step(w)
        self.sync()

class StubEngine:
    def __init__(self, args, local):
        import torch
        self.torch = torch
        self.dev = torch.device("cpu")
        self.cs = args.avg

    def prepare(self, lens, seeds):
        return Work(lens)

    def step(self, w):
        first = [0]
        for n in w.lens:
            first.append(first[-1] + -(-n // self.cs))
        return first

    def timing(self):
        return {"scan_ms": 0.0, "total_ms": 0.0, "resolve_ms": 0.0, "fixup_iterations": 0, "walk_fallback_steps": 0,
                "timed": 1}

    def sync_step(self, w):
        return self.step(w)

    def timings(self, k):
        return [self.timing() for _ in range(min(k, 64))]

    def sync(self):
        pass

    def read_bw(self, w, reps=10):
        return None, None

    def settle(self, w, ms):
        pass


_SETTLE = []  # [(engine, workload, ms)] once main() has its workload: _settle() warms the device


def _settle():
    """Device warm-up before a leg's timed region (each leg follows CPU-side
    oracle checks, during which the clocks drop back)."""
    if _SETTLE:
        eng, w, ms = _SETTLE[0]
        eng.settle(w, ms)


def timed_steps(eng, w, steps, warmup, world, red_dev, settle_ms=0.0):
    """Device settle (read-only passes, settle_ms), W untimed + K timed steps
    of workload w, bracketed by a barrier and a device sync on both sides;
    returns (max-over-ranks seconds, last first[], per-step engine timings)."""
    import torch.distributed as dist
    from chunkfs_amd import sharding
    first = None
    if settle_ms > 0:
        eng.settle(w, settle_ms)
    for _ in range(warmup):
        first = eng.step(w)
    if world > 1:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        first = eng.step(w)
    eng.sync()
    el = time.perf_counter() - t0
    tims = eng.timings(steps)  # HIP events of the timed steps (the last <= 64 of them)
    if world > 1:
        dist.barrier()
        el = sharding.max_over_ranks(el, red_dev)
    return el, first, tims


def latency_leg(eng, w, reps=20):
    """Synchronous single-batch latency of the headline workload: one
    cdc_chunk_batch_device call (tables, scan, resolve, host wait; nothing
    pipelined), wall time per call, beside the pipelined `value`."""
    eng.sync()
    for _ in range(3):
        eng.sync_step(w)
    ts, scans = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.sync_step(w)
        ts.append(time.perf_counter() - t0)
        scans.append(eng.timing()["scan_ms"])  # (events on every synchronous batch)
    ts.sort()
    t = eng.timing()
    return {"definition": "one synchronous cdc_chunk_batch_device call on the headline stream(s), wall time",
            "calls": reps, "median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3,
            "GiBps_at_median": sum(w.lens) / ts[len(ts) // 2] / (1 << 30),
            "last_call_scan_ms": t["scan_ms"], "last_call_resolve_ms": t["resolve_ms"],
            "scan_ms_mean": sum(scans) / len(scans) if scans else None}


def sustained_leg(eng, w, ms_per_step, target_ms=150.0):
    """The headline workload timed over >= target_ms of back-to-back steps
    (the headline's 100 steps are ~28 ms): shows whether clocks or power droop
    under sustained load."""
    steps = max(200, int(target_ms / max(ms_per_step, 1e-3)) + 1)
    el, _, tims = timed_steps(eng, w, steps, 5, 1, None)
    scan = sum(t["scan_ms"] for t in tims) / len(tims) if tims else None
    return {"steps": steps, "timed_ms": el * 1e3, "ms_per_step": el / steps * 1e3,
            "GiBps": sum(w.lens) * steps / el / (1 << 30), "scan_ms": scan,
            "scan_batches_timed": len(tims)}


def config4_leg(args, eng, rank, world, red_dev):
    """Config 4 (BASELINE configs[3]): 1024 x 64 MiB streams split across the
    ranks (strong scaling, no data-path collective); at N > 1 rank 0 also times
    the whole batch alone in this run (the N=1 denominator)."""
    import torch.distributed as dist
    from chunkfs_amd import sharding
    shard = sharding.batch_shard(rank, world, args.batch_streams, args.batch_stream_bytes)
    w = eng.prepare(shard.lens, shard.seeds)
    steps = max(1, args.config4_steps)
    _settle()
    el, first, tims = timed_steps(eng, w, steps, 2, world, red_dev)
    total = sharding.sum_over_ranks(sum(shard.lens), red_dev) * steps
    scan = sum(t["scan_ms"] for t in tims) / len(tims) if tims else 0.0
    out = {"workload": f"config4: {args.batch_streams} x {args.batch_stream_bytes} B streams split across "
                       f"{world} GPU(s)", "scaling": "strong", "steps": steps,
           "value": sharding.aggregate_gibps(total, el), "unit": "GiB/s", "ms_per_step": el / steps * 1e3,
           "streams_per_gpu": len(shard.lens), "bytes_per_gpu": sum(shard.lens),
           "chunks_total": sharding.sum_over_ranks(int(first[-1]) if first is not None else 0, red_dev),
           "scan_ms": scan if tims else None,  # (None: no timed batch among the steps)
           "scan_frac_of_hbm": (sum(shard.lens) / (scan * 1e-3) / 1e9 / HBM_PEAK_GBS) if scan > 0 else None}
    if not args.no_parity and not args.stub and rank == 0 and len(shard.lens):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np
        import oracle
        ok = True
        for i in range(min(len(shard.lens), 2)):
            got = w.out[int(first[i]):int(first[i + 1])].cpu().numpy().view(np.uint64)
            ref = oracle.fastcdc(w.bufs[i][:shard.lens[i]].cpu().numpy(), args.min, args.avg, args.max)
            ok &= bool(got.shape == ref.shape and (got == ref).all())
        out["parity_vs_oracle"] = ok
    del w
    if world > 1:
        n1 = None
        if rank == 0:
            whole = sharding.batch_shard(0, 1, args.batch_streams, args.batch_stream_bytes)
            w1 = eng.prepare(whole.lens, whole.seeds)
            _settle()
            el1, _, _ = timed_steps(eng, w1, steps, 2, 1, None)
            n1 = sum(whole.lens) * steps / el1 / (1 << 30)
            del w1
        dist.barrier()
        if rank == 0:
            out["n1_value_rank0_alone"] = n1
            out["strong_scaling_efficiency"] = out["value"] / (world * n1)
    return out


def config5_leg(args, eng, rank, world, red_dev):
    """Config 5 (BASELINE configs[4]) at every N: 16 GiB of synthetic data as
    16 independent 1 GiB streams (--config5-streams x --config5-stream-bytes;
    stream i: seed 5000+i) split across the ranks
    (strong scaling, no collective), UltraCDC and LeapCDC (plus Rabin and
    SeqCDC) at avg 2 / 8 / 64 KiB, min = avg/4, max = 8 avg.
    Per (rule, sizes): one warm-up pass, then one pass bracketed by a barrier
    and a device sync on both sides; value = 16 GiB / max-over-ranks time.
    After the timed pass, rank 0's first stream -- and at N > 1 also the
    first stream of the last rank -- is checked against the oracle, whole
    (or its first --config5-check bytes: all chunks but the oracle's last
    there, since these rules look only forward), the verdict a min over
    ranks.  SuperCDC is not implemented (CDC_ENOTSUP)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import chunkfs_amd as cfa
    from chunkfs_amd import sharding
    nst, sbytes = args.config5_streams, args.config5_stream_bytes
    shard = sharding.batch_shard(rank, world, nst, sbytes)
    dev = eng.dev
    bufs = []
    for n, sd in zip(shard.lens, shard.seeds):
        b = torch.empty(n, dtype=torch.uint8, device=dev)
        eng._lib.check(eng._lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 4000 + sd, None))
        bufs.append(b)
    torch.cuda.synchronize()
    ptrs, lens = [b.data_ptr() for b in bufs], list(shard.lens)
    total = sharding.sum_over_ranks(sum(lens), red_dev)
    oracle = None
    checker = rank == 0 or rank == world - 1  # rank 0 and, at N > 1, the last rank
    whole = args.config5_check < 0 or (lens and args.config5_check >= lens[0])
    if checker and not args.no_parity and lens:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        host0 = bufs[0][:lens[0] if whole else args.config5_check].cpu().numpy()
    res = {}
    for avg in (2048, 8192, 65536):
        sz = cfa.SizeParams(avg // 4, avg, avg * 8)
        for name in ("ultra", "leap", "rabin", "seq"):
            cls = {"rabin": cfa.RabinChunker, "ultra": cfa.UltraChunker, "leap": cfa.LeapChunker}.get(name)
            ch = cls(sz, device=eng.local) if cls else cfa.SeqChunker(0, sz, device=eng.local)
            cap = ch.batch_max_chunks(lens) if lens else 1
            out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
            first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap) if lens else [0]
            _settle()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if lens:
                first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if world > 1:
                dist.barrier()
                el = sharding.max_over_ranks(el, red_dev)
            line = {"sizes": [sz.min, sz.avg, sz.max], "GiBps": total / el / (1 << 30),
                    "frac_of_hbm": total / el / 1e9 / HBM_PEAK_GBS / world,
                    "chunks_total": sharding.sum_over_ranks(int(first[-1]), red_dev)}
            ok = 1
            if oracle is not None:
                ref = oracle.cdc(name, host0, sz.min, sz.avg, sz.max)
                if not whole:
                    ref = ref[:-1]
                    got = out[:len(ref)].cpu().numpy().view(np.uint64) if len(ref) else np.zeros((0, 2), np.uint64)
                else:
                    got = out[int(first[0]):int(first[1])].cpu().numpy().view(np.uint64)
                ok = int(got.shape == ref.shape and bool((got == ref).all()))
            if not args.no_parity and lens:
                if world > 1:
                    ok = sharding.min_over_ranks(ok, red_dev)
                line["parity_vs_oracle"] = bool(ok)
            res[f"{name}_avg{avg // 1024}k"] = line
            ch.close()
            del out
    del bufs
    return {"workload": f"config5: {nst} x {sbytes} B synthetic streams split across {world} GPU(s)",
            "scaling": "strong",
            "streams_per_gpu": len(lens), "bytes_per_gpu": sum(lens),
            "frac_definition": "per-GPU bytes / max-over-ranks time / 8 TB/s",
            "parity_definition": (None if args.no_parity else
                                  ("the whole first stream of rank 0" + (f" and of rank {world - 1}" if world > 1 else "")
                                   + f" ({lens[0] if lens else 0} B each)") if whole else
                                  f"rank 0 (and rank {world - 1}), stream 0, the chunks inside its first "
                                  f"{args.config5_check} B"),
            "lines": res}


# ---------------------------------------------------------------------------
# Host facts for the CPU baseline

def host_facts():
    facts = {"nproc": os.cpu_count()}
    try:
        facts["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        facts["affinity"] = os.cpu_count()
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    facts["cgroup_cpu_quota"] = quota
    try:
        for ln in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if ln.startswith("Model name:"):
                facts["cpu_model"] = ln.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    usable = facts["affinity"] or 1
    if quota:
        usable = max(1, min(usable, int(quota)))
    facts["usable_cores"] = usable
    return facts


def cpu_baseline_leg(args, host0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    secs, passes, done = 0.0, 0, 0
    while passes == 0 or secs < args.cpu_seconds:
        t, _ = oracle.time_fastcdc(host0, args.min, args.avg, args.max)
        secs += t
        passes += 1
        done += host0.size
    facts = host_facts()
    out = {
        "value": done / secs / (1 << 30), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{passes} whole-buffer pass(es) over stream 0 ({host0.size} B) of this workload; "
                  "oracle/cdc_oracle.c scalar C restatement of fastcdc v2020 (gcc -O3), single thread",
        "host": facts,
    }
    thr = facts["usable_cores"] if args.cpu_threads < 0 else args.cpu_threads
    if thr > 1:
        nb, wall = oracle.time_fastcdc_threads(host0, args.min, args.avg, args.max, thr, args.cpu_seconds / 2)
        out["multi_thread"] = {
            "value": nb / wall / (1 << 30), "unit": "GiB/s", "cores": thr,
            "sample": f"{thr} threads (every usable host core), each chunking its own "
                      f"{host0.size // thr} B slice of stream 0 as an independent stream for "
                      f"~{args.cpu_seconds / 2:.0f} s"}
    return out


def traffic_for_build(path, bytes_rank):
    """HBM bytes per scan launch from a PMC JSON of THIS build (same source
    digest and workload), else None."""
    if not os.path.exists(path):
        return None, None
    try:
        from chunkfs_amd import build as b
        tj = json.load(open(path))
        if tj.get("workload_bytes") == bytes_rank and tj.get("source_digest") == b.source_digest():
            return tj.get("hbm_read_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        pass
    return None, None


def sweep_lines(args, eng, w, steps):
    """Extra single-GPU lines: avg 4 KiB and 16 KiB (min = avg/2, max = 2*avg)
    on the same 1 GiB stream, and 1 GiB of low-entropy data (zeros; a 61-byte
    period) at 4/8/16 KiB, each with an oracle parity check after timing."""
    import numpy as np
    import torch
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    n = w.lens[0]
    base = w.bufs[0]
    period = torch.from_numpy(oracle.splitmix64_bytes(61, 7)).to(eng.dev)
    inputs = {
        "splitmix64": base,
        "zeros": torch.zeros(n, dtype=torch.uint8, device=eng.dev),
        "periodic61": period.repeat(-(-n // 61))[:n].contiguous(),
    }
    cases = [("avg4k", (2048, 4096, 8192), "splitmix64"), ("avg16k", (8192, 16384, 32768), "splitmix64"),
             ("zeros", (4096, 8192, 16384), "zeros"), ("periodic61", (4096, 8192, 16384), "periodic61")]
    res = {}
    for name, sizes, inp in cases:
        buf = inputs[inp]
        ch = cfa.FastChunker(cfa.SizeParams(*sizes), device=eng.local)
        cap = ch.batch_max_chunks([n])
        out = torch.empty((cap, 2), dtype=torch.int64, device=eng.dev)
        for _ in range(2):
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
        _settle()
        torch.cuda.synchronize()
        scan, tot = [], []
        t0 = time.perf_counter()
        for _ in range(steps):
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            t = ch.last_timing()
            scan.append(t["scan_ms"])
            tot.append(t["total_ms"])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        got = out[:int(first[1])].cpu().numpy().view(np.uint64)
        parity = None
        if not args.no_parity:
            ref = oracle.fastcdc(buf.cpu().numpy(), *sizes)
            parity = bool(got.shape == ref.shape and (got == ref).all())
        res[name] = {"sizes": list(sizes), "data": inp, "GiBps": n * steps / el / (1 << 30),
                     "ms_per_step": el / steps * 1e3, "scan_ms": sum(scan) / len(scan),
                     "device_total_ms": sum(tot) / len(tot), "chunks": int(first[1]), "parity_vs_oracle": parity}
        ch.close()
        del out
    return res


def algo_lines(args, eng, w, steps):
    """Rabin / UltraCDC / LeapCDC / SeqCDC (segment-walk engine) over the same
    1 GiB stream at the bench sizes: device GiB/s, the walk / fix-up split,
    bit-exactness against the oracle on the whole stream, and the oracle's
    single-thread rate on the same bytes (parity vs the crate is unpinned)."""
    import numpy as np
    import torch
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    n = w.lens[0]
    buf = w.bufs[0]
    sizes = cfa.SizeParams(args.min, args.avg, args.max)
    host = buf[:n].cpu().numpy() if not args.no_parity else None
    res = {}
    for name in ("rabin", "ultra", "leap", "seq"):
        ch = {"rabin": cfa.RabinChunker, "ultra": cfa.UltraChunker, "leap": cfa.LeapChunker}.get(name)
        ch = ch(sizes, device=eng.local) if ch else cfa.SeqChunker(cfa.OperationMode.Increasing, sizes,
                                                                  device=eng.local)
        cap = ch.batch_max_chunks([n])
        out = torch.empty((cap, 2), dtype=torch.int64, device=eng.dev)
        first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
        _settle()
        torch.cuda.synchronize()
        walk, tot, rew = [], [], []
        t0 = time.perf_counter()
        for _ in range(steps):
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            t = ch.last_timing()
            walk.append(t["scan_ms"])
            tot.append(t["total_ms"])
            rew.append(t["fixup_iterations"])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # back-to-back async batches (cdc_chunk_batch_device_async: two
        # contexts, one batch's walks beside the next one's bitmap pass),
        # alternate output buffers
        outs = [out, torch.empty((cap, 2), dtype=torch.int64, device=eng.dev)]
        ka = max(8, 4 * steps)
        for i in range(2):
            ch.chunk_batch_device_async([buf.data_ptr()], [n], outs[i % 2].data_ptr(), cap)
        ch.batch_sync()
        _settle()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(ka):
            fa = ch.chunk_batch_device_async([buf.data_ptr()], [n], outs[i % 2].data_ptr(), cap)
        ch.batch_sync()
        torch.cuda.synchronize()
        ela = time.perf_counter() - t0
        line = {"sizes": [args.min, args.avg, args.max], "GiBps": n * ka / ela / (1 << 30),
                "ms_per_step": ela / ka * 1e3, "steps": ka,
                "definition": "back-to-back async batches of the 1 GiB stream (two walk contexts)",
                "GiBps_sync": n * steps / el / (1 << 30), "ms_per_step_sync": el / steps * 1e3,
                "walk_ms": sum(walk) / len(walk),
                "device_total_ms": sum(tot) / len(tot), "rewalked_segments": max(rew), "chunks": int(first[1]),
                "frac_of_hbm": n * ka / ela / 1e9 / HBM_PEAK_GBS}
        if host is not None:
            assert int(fa[1]) == int(first[1])
            got = outs[(ka - 1) % 2][:int(first[1])].cpu().numpy().view(np.uint64)
            secs = time.perf_counter()
            ref = oracle.cdc(name, host, args.min, args.avg, args.max)
            secs = time.perf_counter() - secs
            line["parity_vs_oracle"] = bool(got.shape == ref.shape and (got == ref).all())
            line["cpu_single_thread_GiBps"] = n / secs / (1 << 30)
        res[name] = line
        ch.close()
        del out, outs
    return res


def lowentropy_walk_lines(args, eng, nbytes=256 << 20):
    """Rabin / UltraCDC / LeapCDC / SeqCDC on low-entropy device streams of
    `nbytes` (zeros; a 61-byte period; random bytes with 1-32 MiB zero-filled
    regions at unaligned offsets; random bytes with a dozen 64-512 KiB zero
    islands), bench sizes: chains from different
    starts never merge on such data, so these lines time the fix-up rounds
    and the in-order pass (one wave per stream) that the splitmix64 lines
    never reach.  Device GiB/s, the re-walk statistics and bit-exactness vs
    the oracle (parity vs the crate is unpinned)."""
    import numpy as np
    import torch
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    n = nbytes
    period = torch.from_numpy(oracle.splitmix64_bytes(61, 7)).to(eng.dev)
    # a sparse-image shape: random bytes with zero-filled regions of 1-32 MiB at
    # unaligned offsets (chains enter each region at an arbitrary phase)
    runs = torch.from_numpy(oracle.splitmix64_bytes(n, 17)).to(eng.dev)
    rng = np.random.default_rng(17)
    pos = int(rng.integers(1, 1 << 20))
    while pos < n:
        ln = int(rng.integers(1 << 20, 32 << 20))
        runs[pos:pos + ln] = 0
        pos += ln + int(rng.integers(1 << 16, 8 << 20))
    # random bytes with a few small zero islands (64-512 KiB): the fix-up
    # rounds' quiet hand-off must not fire on such mostly random data
    isl = torch.from_numpy(oracle.splitmix64_bytes(n, 19)).to(eng.dev)
    for _ in range(12):
        a = int(rng.integers(0, n - (1 << 19)))
        isl[a:a + int(rng.integers(1 << 16, 1 << 19))] = 0
    inputs = {"zeros": torch.zeros(n, dtype=torch.uint8, device=eng.dev),
              "periodic61": period.repeat(-(-n // 61))[:n].contiguous(),
              "zero_runs": runs, "zero_islands": isl}
    sizes = cfa.SizeParams(args.min, args.avg, args.max)
    res = {}
    for inp, buf in inputs.items():
        host = buf.cpu().numpy() if not args.no_parity else None
        for name in ("rabin", "ultra", "leap", "seq"):
            cls = {"rabin": cfa.RabinChunker, "ultra": cfa.UltraChunker, "leap": cfa.LeapChunker}.get(name)
            ch = cls(sizes, device=eng.local) if cls else cfa.SeqChunker(0, sizes, device=eng.local)
            cap = ch.batch_max_chunks([n])
            out = torch.empty((cap, 2), dtype=torch.int64, device=eng.dev)
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            _settle()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            t = ch.last_timing()
            line = {"GiBps": n / el / (1 << 30), "chunks": int(first[1]),
                    "rewalked_segments": t["fixup_iterations"], "in_order_pass": bool(t["overflow_spans"])}
            if host is not None:
                got = out[:int(first[1])].cpu().numpy().view(np.uint64)
                ref = oracle.cdc(name, host, args.min, args.avg, args.max)
                line["parity_vs_oracle"] = bool(got.shape == ref.shape and (got == ref).all())
            res[f"{name}_{inp}"] = line
            ch.close()
            del out
    return {"bytes": int(n), "sizes": [args.min, args.avg, args.max], "lines": res}


def config5_lines(args, eng, w, steps=2):
    """Config 5's size sweep (BASELINE.json configs[4]) on one GPU: UltraCDC and
    LeapCDC (plus Rabin and Seq) at avg 2 / 8 / 64 KiB, min = avg/4, max = 8 avg
    (SURVEY.md §8d), over the first --config5-bytes of the bench stream (default
    the whole 1 GiB; config 5's share per GPU at 8 GPUs is 2 GiB, and the
    segment-walk engine needs the bytes for lanes: at avg 64 KiB a segment is
    256 KiB, so 256 MiB would be only 1024 lanes); device GiB/s,
    fraction of HBM peak, bit-exactness vs the oracle.  SuperCDC is not
    implemented (CDC_ENOTSUP)."""
    import numpy as np
    import torch
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    n = min(args.config5_bytes, w.lens[0])
    buf = w.bufs[0]
    host = buf[:n].cpu().numpy() if not args.no_parity else None
    res = {}
    for avg in (2048, 8192, 65536):
        sz = cfa.SizeParams(avg // 4, avg, avg * 8)
        for name in ("ultra", "leap", "rabin", "seq"):
            cls = {"rabin": cfa.RabinChunker, "ultra": cfa.UltraChunker, "leap": cfa.LeapChunker}.get(name)
            ch = cls(sz, device=eng.local) if cls else cfa.SeqChunker(0, sz, device=eng.local)
            cap = ch.batch_max_chunks([n])
            out = torch.empty((cap, 2), dtype=torch.int64, device=eng.dev)
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            _settle()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / steps
            line = {"sizes": [sz.min, sz.avg, sz.max], "GiBps": n / el / (1 << 30),
                    "frac_of_hbm": n / el / 1e9 / HBM_PEAK_GBS, "chunks": int(first[1]),
                    "rewalked_segments": ch.last_timing()["fixup_iterations"]}
            if host is not None:
                got = out[:int(first[1])].cpu().numpy().view(np.uint64)
                ref = oracle.cdc(name, host, sz.min, sz.avg, sz.max)
                line["parity_vs_oracle"] = bool(got.shape == ref.shape and (got == ref).all())
            res[f"{name}_avg{avg // 1024}k"] = line
            ch.close()
            del out
    return {"bytes": int(n), "lines": res}


def config3_line(args, local, base_bytes=256 << 20, versions=16):
    """Config 3 (BASELINE.json configs[2]): RabinChunker 2/4/8 KiB over a
    versioned archive at SURVEY.md §8d's size (256 MiB base + 15 edited
    copies, ~4 GiB; chunkfs_amd.synthetic); every version is one file write (a fresh StorageWriter,
    storage.rs:79).  GPU: chunk -> SHA-256 per chunk -> dedup index, all
    device-resident; dedup ratio = size_written / unique bytes (storage.rs:
    203-205).  CPU: the oracle's chunks, hashlib SHA-256 and a dict (first
    insert wins, database.rs:76), single thread."""
    import hashlib
    import numpy as np
    import torch
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from chunkfs_amd.synthetic import versioned_archive
    sizes = (2048, 4096, 8192)
    files = versioned_archive(base_bytes, versions)
    total = sum(f.size for f in files)
    dev = torch.device("cuda", local)
    bufs = [torch.from_numpy(f).to(dev) for f in files]
    ch = cfa.RabinChunker(cfa.SizeParams(*sizes), device=local)
    lens = [f.size for f in files]
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    dig = torch.empty((cap, 32), dtype=torch.uint8, device=dev)

    ptrs = [b.data_ptr() for b in bufs]
    ix = cfa.DedupIndex(cap + 64, device=local)  # (sized once; cleared per pass: Database::clear)
    phase = {}

    def gpu_pass():
        # one launch per stage over all versions: chunk every file, hash every
        # chunk (cdc_sha256_batch_device), insert every digest in file order
        # (the reference's sequential writes: first insert wins)
        ix.clear()
        t0 = time.perf_counter()
        first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
        t1 = time.perf_counter()
        ch.sha256_batch_device(ptrs, first, out.data_ptr(), dig.data_ptr())
        t2 = time.perf_counter()
        ix.insert_device(dig.data_ptr(), out.data_ptr(), int(first[-1]))
        st = ix.stats()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        phase.update(chunk_ms=(t1 - t0) * 1e3, sha256_ms=(t2 - t1) * 1e3, index_ms=(t3 - t2) * 1e3,
                     sha256_kernel_ms=ch.last_timing()["hash_ms"])
        return first, st

    gpu_pass()
    _settle()
    t0 = time.perf_counter()
    first, st = gpu_pass()
    t_gpu = time.perf_counter() - t0
    got = out[:int(first[-1])].cpu().numpy().view(np.uint64)
    t0 = time.perf_counter()
    db, written, parity = {}, 0, True
    for i, f in enumerate(files):
        ref = oracle.cdc("rabin", f, *sizes)
        parity &= bool(np.array_equal(got[int(first[i]):int(first[i + 1])], ref))
        for o, ln in ref:
            d = hashlib.sha256(f[int(o):int(o) + int(ln)].tobytes()).digest()
            db.setdefault(d, int(ln))
            written += int(ln)
    t_cpu = time.perf_counter() - t0
    cpu_ratio = written / sum(db.values())
    ch.close()
    del ix
    return {"workload": f"config3 substitute: {versions} versions of a {base_bytes} B splitmix64 base, "
                        "~1 % seeded overwrites/inserts/deletes per version (gcc tarball unavailable offline)",
            "algo": "RabinCDC (parity unpinned)", "sizes": list(sizes), "bytes": int(total),
            "chunks": int(first[-1]), "gpu_dedup_ratio": st["cdc_dedup_ratio"], "cpu_dedup_ratio": cpu_ratio,
            "dedup_ratio_equal": bool(abs(st["cdc_dedup_ratio"] - cpu_ratio) < 1e-12),
            "chunks_bit_exact": parity, "unique_chunks": st["unique_chunks"],
            "gpu_GiBps": total / t_gpu / (1 << 30),
            "gpu_definition": "device-resident: Rabin chunking + SHA-256 per chunk + dedup index inserts, wall time",
            "gpu_phase_ms": phase,
            "sha256_GiBps": total / (phase["sha256_kernel_ms"] * 1e-3) / (1 << 30) if phase.get("sha256_kernel_ms") else None,
            "cpu_GiBps": total / t_cpu / (1 << 30),
            "cpu_definition": "oracle Rabin (C) + hashlib SHA-256 + dict, single thread"}


def host_path_leg(eng, w):
    """PCIe-inclusive rates of the host boundary, recorded beside `value`,
    never as it:
      * cdc_chunk_data on the whole 1 GiB host buffer;
      * chunk_data_1MiB_calls: the Rust shim's own loop -- StorageWriter::write
        per 1 MiB segment (buffer = rest ++ segment, chunk_data, rest = last
        chunk; storage.rs:302-357) timed like the reference, Sum of the
        chunk_data calls only (storage.rs:314-316, report.rs:168-175);
      * write_stream_1MiB_segments: the same write through the streaming path
        (cdc_write_segment per 1 MiB segment, wall time begin -> finish).
    Spans are checked against the oracle's StorageWriter loop."""
    import numpy as np
    import chunkfs_amd as cfa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ch = eng.ch
    numa = cfa.host_placement(ch)
    # The caller's thread joins the copy: run it (and place the source buffer)
    # on the GPU's node too, as a NUMA-aware application would
    # (CHUNKFS_AMD_COPY_NUMA=0: leave both where they are, A/B).
    old_aff = os.sched_getaffinity(0)
    if numa.get("numa_placement"):
        try:
            with open(f"/sys/devices/system/node/node{numa['gpu_node']}/cpulist") as f:
                near = set(_parse_cpulist(f.read())) & old_aff
            if near:
                os.sched_setaffinity(0, near)
                numa["caller_pinned_cpus"] = len(near)
        except OSError:
            pass
    try:
        return _host_path_leg(eng, w, ch, numa)
    finally:
        os.sched_setaffinity(0, old_aff)


def _parse_cpulist(s):
    out = []
    for part in s.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out += range(int(a), int(b or a) + 1)
    return out


def _host_path_leg(eng, w, ch, numa):
    import numpy as np
    import chunkfs_amd as cfa
    import oracle
    hb = w.bufs[0][:w.lens[0]].cpu().numpy()  # (first touched by this thread: on its node)
    ch.chunk_array(hb)
    reps, t_h = 3, time.perf_counter()
    for _ in range(reps):
        hc = ch.chunk_array(hb)
    t_h = (time.perf_counter() - t_h) / reps
    hp = {"GiBps": hb.size / t_h / (1 << 30), "bytes": int(hb.size), "chunks": int(hc.shape[0]),
          "entry": "cdc_chunk_data (pageable host buffer -> pinned ring -> H2D -> pipeline -> host-mapped chunk list)"}
    hp["numa"] = numa  # (re-read after the calls below: the chunk list is allocated by the first one)
    fs_bytes = min(hb.size, 256 << 20)
    seg = 1 << 20
    ref_spans, ref_secs = oracle.fs_write("fast", hb[:fs_bytes], *eng.sizes)
    # the reference loop through cdc_chunk_data
    for rnd in range(2):  # (round 0 warms the buffers)
        _settle()
        spans, rest, chunk_s = [], np.empty(0, dtype=np.uint8), 0.0
        st0 = cfa.host_stats(ch)
        for off in range(0, fs_bytes, seg):
            buf = np.concatenate([rest, hb[off:off + seg]])
            t0 = time.perf_counter()
            chunks = ch.chunk_array(buf)
            chunk_s += time.perf_counter() - t0
            spans += [int(x) for x in chunks[:-1, 1]]
            o, ln = (int(x) for x in chunks[-1])
            rest = buf[o:o + ln]
        spans.append(int(rest.size))
        st1 = cfa.host_stats(ch)
    calls = st1["calls"] - st0["calls"]
    chunk_c = st1["total_s"] - st0["total_s"]  # seconds inside cdc_chunk_data, timed by the library itself
    hp["chunk_data_1MiB_calls"] = {
        "GiBps": fs_bytes / chunk_c / (1 << 30), "bytes": int(fs_bytes), "calls": calls,
        "us_per_call": chunk_c / calls * 1e6,
        "GiBps_python_wall": fs_bytes / chunk_s / (1 << 30),
        "us_per_call_python_wall": chunk_s / calls * 1e6,
        "upload_us_per_call": (st1["upload_s"] - st0["upload_s"]) / calls * 1e6,
        "spans_equal_oracle_fs_write": spans == [int(x) for x in ref_spans],
        "cpu_oracle_same_loop_GiBps": fs_bytes / ref_secs / (1 << 30),
        "metric": "bytes / summed seconds inside cdc_chunk_data over the reference's 1 MiB StorageWriter loop "
                  "(what CDCFixture::measure reports as chunk throughput), timed inside the C library as the oracle's "
                  "loop is timed inside C (the *_python_wall fields add this harness's ctypes / numpy overhead); "
                  "each call = the one-launch small kernel launched, the bytes copied into a pinned ring slot it "
                  "reads over PCIe as they arrive, chunk list in host-mapped memory"}
    # the streaming write path over the whole 1 GiB
    for rnd in range(2):
        _settle()
        sw = cfa.StreamWriter(ch)
        for off in range(0, hb.size, seg):
            sw.write(hb[off:off + seg])
        sspans, ssecs = sw.finish()
    whole = hc[:, 1]
    hp["write_stream_1MiB_segments"] = {
        "GiBps": hb.size / ssecs / (1 << 30), "bytes": int(hb.size), "spans": int(sspans.size),
        "spans_equal_whole_stream": bool(sspans.shape == whole.shape and (sspans == whole).all()),
        "metric": "bytes / wall seconds cdc_write_begin -> cdc_write_finish, 1 MiB cdc_write_segment calls "
                  "(CPU copy into the pinned ring, async H2D, device chunking of 256 MiB windows, carried chunk "
                  "in HBM)"}
    hp["numa"] = {**numa, **cfa.host_placement(ch)}
    return hp


def summary(line, read_gbs):
    """The line's headline figures in one small object (printed last)."""
    g = lambda *ks: _dig(line, ks)  # noqa: E731
    out = {"value_GiBps": line.get("value"), "ms_per_step": line.get("ms_per_step"),
           "sustained_ms_per_step": g("sustained", "ms_per_step"), "sync_latency_ms": g("latency_sync", "median_ms"),
           "parity_vs_oracle": line.get("parity_vs_oracle"),
           "scan_frac_of_hbm": g("roofline", "frac"), "scan_frac_of_achievable": g("roofline", "frac_of_achievable"),
           "achievable_read_GBps": read_gbs, "end_to_end_frac_of_hbm": g("roofline", "end_to_end", "frac"),
           "host_chunk_data_1MiB_us_per_call": g("host_path", "chunk_data_1MiB_calls", "us_per_call"),
           "host_chunk_data_1MiB_x_cpu_single_thread": g("host_path", "chunk_data_1MiB_calls", "x_cpu_single_thread"),
           "host_chunk_data_spans_equal_oracle_fs_write":
               g("host_path", "chunk_data_1MiB_calls", "spans_equal_oracle_fs_write"),
           "host_write_stream_GiBps": g("host_path", "write_stream_1MiB_segments", "GiBps"),
           "host_numa": g("host_path", "numa"),
           "cpu_baseline_GiBps_1core": g("cpu_baseline", "value")}
    oc = line.get("other_chunkers") or {}
    out["walk_frac_of_hbm"] = {k: v.get("frac_of_hbm") for k, v in oc.items()}
    out["walk_parity"] = all(v.get("parity_vs_oracle", False) for v in oc.values()) if oc else None
    c3 = line.get("config3") or {}
    if c3:
        out["config3"] = {"GiBps": c3.get("gpu_GiBps"), "dedup_ratio_equal": c3.get("dedup_ratio_equal"),
                          "chunks_bit_exact": c3.get("chunks_bit_exact")}
    c4 = line.get("config4") or {}
    if c4:
        out["config4"] = {"GiBps": c4.get("value"), "scan_frac_of_hbm": c4.get("scan_frac_of_hbm"),
                          "parity_vs_oracle": c4.get("parity_vs_oracle"),
                          "strong_scaling_efficiency": c4.get("strong_scaling_efficiency")}
    c5 = (line.get("config5") or {}).get("lines") or {}
    if c5:
        out["config5"] = {"GiBps": {k: round(v["GiBps"], 1) for k, v in c5.items()},
                          "parity": all(v.get("parity_vs_oracle", True) for v in c5.values()),
                          "parity_definition": (line.get("config5") or {}).get("parity_definition")}
    return out


def _dig(d, ks):
    for k in ks:
        if not isinstance(d, dict):
            return None
        d = d.get(k)
    return d


# ---------------------------------------------------------------------------

def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist
    from chunkfs_amd import sharding

    if args.stub:
        eng = StubEngine(args, local)
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if args.share_device:
            local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if world > 1:
            if args.dist_backend == "gloo":
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        eng = DeviceEngine(args, local)
    dev = eng.dev
    red_dev = None if (args.stub or args.dist_backend == "gloo") else dev  # where reductions run

    if args.workload == "stream":
        shard = sharding.stream_shard(rank, world, args.stream_bytes)
    else:
        shard = sharding.batch_shard(rank, world, args.batch_streams, args.batch_stream_bytes)
    w = eng.prepare(shard.lens, shard.seeds)
    if args.settle_ms > 0:
        _SETTLE.append((eng, w, args.settle_ms))
    elapsed, first, tims = timed_steps(eng, w, args.steps, args.warmup, world, red_dev, args.settle_ms)

    bytes_rank = sum(shard.lens)
    read_gbs, read_ms = eng.read_bw(w) if shard.lens and shard.lens[0] else (None, None)
    total_bytes = sharding.sum_over_ranks(bytes_rank, red_dev) * args.steps
    value = sharding.aggregate_gibps(total_bytes, elapsed)
    tims = tims or [dict(scan_ms=0.0, total_ms=0.0, resolve_ms=0.0, fixup_iterations=0, timed=0)]  # (none timed)
    scan_avg_ms = sum(t["scan_ms"] for t in tims) / len(tims)
    nchunks = int(first[-1])
    total_chunks = sharding.sum_over_ranks(nchunks, red_dev)
    ms_per_step = elapsed / args.steps * 1e3
    achieved = bytes_rank / (scan_avg_ms * 1e-3) / 1e9 if scan_avg_ms > 0 else None
    e2e = bytes_rank / (ms_per_step * 1e-3) / 1e9  # per-GPU bytes / wall step time

    extras = {}
    pipe_scan_ms = scan_avg_ms
    if rank == 0 and world == 1 and not args.stub and shard.lens and shard.lens[0]:
        extras["sustained"] = sustained_leg(eng, w, ms_per_step)
        extras["latency_sync"] = latency_leg(eng, w)
        if extras["latency_sync"]["scan_ms_mean"]:
            scan_avg_ms = extras["latency_sync"]["scan_ms_mean"]  # the scan alone (module docstring)
            achieved = bytes_rank / (scan_avg_ms * 1e-3) / 1e9
    if rank == 0 and world == 1 and not args.stub:
        if args.hash and shard.lens[0]:
            n0 = int(first[1]) - int(first[0])
            dig = torch.empty((max(n0, 1), 32), dtype=torch.uint8, device=dev)
            hms = []
            for _ in range(3):
                eng.ch.sha256_chunks_device(w.bufs[0].data_ptr(), w.out.data_ptr(), n0, dig.data_ptr())
                hms.append(eng.ch.last_timing()["hash_ms"])
            hm = sorted(hms)[1]
            extras["fingerprint"] = {"algo": "SHA-256 per chunk (Sha256Hasher)", "chunks": n0, "kernel_ms": hm,
                                     "GiBps": shard.lens[0] / (hm * 1e-3) / (1 << 30)}
        if not args.no_host_path:
            extras["host_path"] = host_path_leg(eng, w)
        if not args.no_parity:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            checked = []
            for i in range(min(len(shard.lens), 4)):
                got = w.out[int(first[i]):int(first[i + 1])].cpu().numpy().view(np.uint64)
                ref = oracle.fastcdc(w.bufs[i][:shard.lens[i]].cpu().numpy(), args.min, args.avg, args.max)
                checked.append(bool(got.shape == ref.shape and (got == ref).all()))
            extras["parity_vs_oracle"] = all(checked)
            extras["parity_streams_checked"] = len(checked)
        if not args.no_sweep and args.workload == "stream":
            extras["sweep"] = sweep_lines(args, eng, w, max(5, args.steps // 2))
        if not args.no_algos and args.workload == "stream":
            extras["other_chunkers"] = algo_lines(args, eng, w, 3)
            extras["other_chunkers_low_entropy"] = lowentropy_walk_lines(args, eng)
            extras["config3"] = config3_line(args, local)
            extras["config5_1gpu"] = config5_lines(args, eng, w)
        if args.cpu_seconds > 0:
            extras["cpu_baseline"] = cpu_baseline_leg(args, w.bufs[0][:shard.lens[0]].cpu().numpy())
            for k in ("chunk_data_1MiB_calls", "write_stream_1MiB_segments"):
                fw = extras.get("host_path", {}).get(k)
                if fw:
                    fw["x_cpu_single_thread"] = fw["GiBps"] / extras["cpu_baseline"]["value"]

    if args.rank_parity and not args.stub:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        ok = 1
        for i in range(min(len(shard.lens), 2)):
            got = w.out[int(first[i]):int(first[i + 1])].cpu().numpy().view(np.uint64)
            ref = oracle.fastcdc(w.bufs[i][:shard.lens[i]].cpu().numpy(), args.min, args.avg, args.max)
            ok &= int(got.shape == ref.shape and bool((got == ref).all()))
        extras["parity_all_ranks"] = bool(sharding.min_over_ranks(ok, red_dev)) if world > 1 else bool(ok)

    if not args.no_config4 and args.workload == "stream":
        del w
        c4 = config4_leg(args, eng, rank, world, red_dev)
        if rank == 0:
            extras["config4"] = c4
    if not args.no_config5 and not args.stub and args.workload == "stream":
        c5 = config5_leg(args, eng, rank, world, red_dev)
        if rank == 0:
            extras["config5"] = c5

    traffic, traffic_src = traffic_for_build(args.traffic_json, bytes_rank)
    # the same counter on the bare read kernel (tools/pmc.sh fetch_read): what
    # a pure streaming read of these bytes fetches on this part
    traffic_read, _ = traffic_for_build(os.path.join(os.path.dirname(args.traffic_json), "pmc_read_traffic.json"),
                                        bytes_rank)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,  # read-only passes before the warmup steps (and before each leg)
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": shard.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {
                "workload": ("config2: 1 x %d B stream per GPU" % args.stream_bytes if args.workload == "stream"
                             else f"config4: {args.batch_streams} x {args.batch_stream_bytes} B streams "
                                  f"split across {world} GPU(s)"),
                "algo": "FastCDC v2020 (Level1)", "min": args.min, "avg": args.avg, "max": args.max,
                "bytes_per_gpu": bytes_rank, "streams_per_gpu": len(shard.lens), "chunks_total": total_chunks,
                "parallelism": f"independent streams x{world}, no collective",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_read_kernel": traffic_read,
                "kernel": "scan_kernel (gear candidate scan)",
                "kernel_ms": scan_avg_ms, "algorithmic_bytes_per_launch": bytes_rank,
                "kernel_ms_source": ("latency_sync calls (scan alone on the chip)" if pipe_scan_ms != scan_avg_ms
                                     else "headline steps"),
                "kernel_ms_in_pipeline": pipe_scan_ms,
                "achievable_GBps": read_gbs,
                "frac_of_achievable": (achieved / read_gbs) if (achieved and read_gbs) else None,
                "achievable_definition": "read-only reduction kernel over the same bytes in this run "
                                         "(cdc_debug_read_bw, 10 launches, HIP events)",
                "end_to_end": {"achieved": e2e, "frac": e2e / HBM_PEAK_GBS,
                               "definition": "per-GPU input bytes / wall ms_per_step"},
            },
            "cpu_baseline": extras.pop("cpu_baseline", None),
            "phase_ms": {"scan": pipe_scan_ms, "scan_alone": scan_avg_ms,
                         "total_device": sum(t["total_ms"] for t in tims) / len(tims),
                         "resolve": sum(t["resolve_ms"] for t in tims) / len(tims),
                         "rewalked_spans": max(t["fixup_iterations"] for t in tims),
                         "walk_fallback_steps": max(t.get("walk_fallback_steps", 0) for t in tims)},
        }
        line.update(extras)
        line["summary"] = summary(line, read_gbs)  # last: the driver keeps the line's tail
        if args.stub:
            line["data"] = "stub engine (CPU launcher test; not a measurement)"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
