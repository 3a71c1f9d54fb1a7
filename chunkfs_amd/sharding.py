"""Multi-GPU sharding of independent streams.

Streams are independent in the reference -- every `write_to_file` starts a
fresh StorageWriter with an empty carry-over (src/system/storage.rs:79) -- so
the data path needs no collective: each rank chunks its own streams.  The
only cross-rank step is the timing reduction (max over ranks), which the
bench contract requires.  These helpers are device-agnostic so the N>1 path
is testable with the gloo backend on CPU (tests/test_distributed.py).
"""
from dataclasses import dataclass
from typing import List


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    lens: List[int]    # byte length of each stream this rank chunks
    seeds: List[int]   # splitmix64 seed of each stream (synthetic data)
    scaling: str       # "weak" (per-rank work fixed) or "strong" (total fixed)


def stream_shard(rank: int, world: int, stream_bytes: int) -> Shard:
    """Config 2 at N GPUs: one stream of `stream_bytes` per rank, seed 1+rank."""
    return Shard(rank, world, [stream_bytes], [1 + rank], "weak")


def batch_shard(rank: int, world: int, total_streams: int, stream_bytes: int) -> Shard:
    """Config 4: `total_streams` streams (stream i has seed 1000+i), split into
    contiguous blocks of ceil(total/world) per rank."""
    per = -(-total_streams // world)
    lo, hi = min(rank * per, total_streams), min((rank + 1) * per, total_streams)
    return Shard(rank, world, [stream_bytes] * (hi - lo), [1000 + i for i in range(lo, hi)], "strong")


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank float across the default process group (identity
    when torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, device=None) -> int:
    """Sum of a per-rank integer (bytes processed) across the process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def min_over_ranks(value: int, device=None) -> int:
    """Min of a per-rank integer (e.g. a 0/1 check) across the process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def aggregate_gibps(total_bytes: int, elapsed_max_s: float) -> float:
    """Whole-job throughput: bytes all ranks processed / max-over-ranks time."""
    return total_bytes / elapsed_max_s / (1 << 30)
