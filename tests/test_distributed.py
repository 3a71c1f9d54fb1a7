"""N>1 path on CPU with gloo, world_size 2.

The GPU data path has no collective; what the multi-rank bench adds is the
shard assignment and the max-over-ranks timing.  Each rank here chunks its
shard with the CPU oracle (standing in for the device, which this container
lacks), then the ranks reduce: the union of per-rank results must equal a
single-rank run over all streams, the time reduction must be the max, and
the byte count the sum.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from chunkfs_amd import sharding

STREAM = 1 << 20
TOTAL = 5  # odd: the last rank gets a short block


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _chunk_counts(shard):
    return [int(oracle.fastcdc(oracle.splitmix64_bytes(n, s), 4096, 8192, 16384).shape[0])
            for n, s in zip(shard.lens, shard.seeds)]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = sharding.batch_shard(rank, world, TOTAL, STREAM)
        counts = _chunk_counts(sh)
        gathered = [None] * world
        dist.all_gather_object(gathered, (sh.seeds, counts))
        t_max = sharding.max_over_ranks(0.25 + rank)  # rank r pretends to take 0.25+r s
        b_sum = sharding.sum_over_ranks(sum(sh.lens))
        q.put((rank, gathered, t_max, b_sum))
    finally:
        dist.destroy_process_group()


def test_stream_shard_is_weak_scaling():
    shards = [sharding.stream_shard(r, 4, 1 << 30) for r in range(4)]
    assert [s.seeds for s in shards] == [[1], [2], [3], [4]]
    assert all(s.lens == [1 << 30] and s.scaling == "weak" for s in shards)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_batch_shard_partitions_streams(world):
    shards = [sharding.batch_shard(r, world, 1024, 64 << 20) for r in range(world)]
    seeds = [s for sh in shards for s in sh.seeds]
    assert seeds == [1000 + i for i in range(1024)]  # contiguous, disjoint, complete
    assert max(len(sh.lens) for sh in shards) - min(len(sh.lens) for sh in shards) <= world


def test_two_rank_gloo_shards_match_single_rank():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    single = _chunk_counts(sharding.batch_shard(0, 1, TOTAL, STREAM))
    for rank, gathered, t_max, b_sum in res:
        seeds = [s for g in gathered for s in g[0]]
        counts = [c for g in gathered for c in g[1]]
        assert seeds == [1000 + i for i in range(TOTAL)]
        assert counts == single
        assert t_max == pytest.approx(1.25)
        assert b_sum == TOTAL * STREAM
    assert sharding.aggregate_gibps(TOTAL * STREAM, 1.25) == pytest.approx(TOTAL * STREAM / 1.25 / 2**30)
    assert np.all(np.array(single) > 0)
