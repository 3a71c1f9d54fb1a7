"""The N>1 bench path on the HIP engine (-m gpu): `bench.py --gpus 2` starts two
ranks itself; on a one-GPU box both share cuda:0 (--share-device) and the
timing / byte reductions run over gloo (--dist-backend gloo) -- on an 8-GPU node
the driver runs the same path with one GPU per rank over RCCL.  Each rank chunks
its own block of the config-4 batch with no data-path collective and checks its
first streams bit-exact against the oracle (--rank-parity, min over ranks)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_on_hip_engine():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--rank-parity", "--workload", "batch", "--batch-streams", "8",
                        "--batch-stream-bytes", str(8 << 20), "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["streams_per_gpu"] == 4
    assert line["parity_all_ranks"] is True
    assert line["value"] > 0


def test_two_ranks_default_stream_workload():
    """The driver's own N>1 command shape (`bench.py --gpus N`, default
    `--workload stream`, default gloo reductions) with small sizes: `value` is
    config 2 per GPU (weak), the config-4 leg runs its N>1 branch (rank 0 re-times
    the whole batch alone: the strong-scaling denominator) and the config-5 leg
    runs every walk rule at avg 2/8/64 KiB across both ranks, checked against
    the oracle."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--rank-parity", "--stream-bytes", str(64 << 20), "--batch-streams", "8",
                        "--batch-stream-bytes", str(8 << 20), "--config4-steps", "2", "--config5-streams", "4",
                        "--config5-stream-bytes", str(32 << 20), "--config5-check", str(8 << 20), "--steps", "2",
                        "--warmup", "1", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["config"]["workload"].startswith("config2")
    assert line["parity_all_ranks"] is True and line["value"] > 0
    c4 = line["config4"]
    assert c4["streams_per_gpu"] == 4 and c4["parity_vs_oracle"] is True
    assert c4["strong_scaling_efficiency"] > 0 and c4["n1_value_rank0_alone"] > 0
    c5 = line["config5"]
    assert c5["streams_per_gpu"] == 2 and len(c5["lines"]) == 12
    assert all(v["parity_vs_oracle"] is True for v in c5["lines"].values()), c5["lines"]


def test_eight_ranks_real_shard_counts():
    """The driver's 8-GPU shapes rehearsed on one GPU: `bench.py --gpus 8` with
    the real shard COUNTS (config 4: 1024 streams = 128 per rank; config 5: 16
    streams = 2 per rank) at small sizes, every rank sharing cuda:0, every
    rank's first streams checked against the oracle (min over ranks; config
    5: the whole first streams of ranks 0 and 7), the config-4 strong-scaling efficiency reported (rank 0 re-times the whole
    1024-stream batch alone)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--share-device",
                        "--rank-parity", "--stream-bytes", str(24 << 20), "--batch-streams", "1024",
                        "--batch-stream-bytes", str(1 << 20), "--config4-steps", "1", "--config5-streams", "16",
                        "--config5-stream-bytes", str(8 << 20), "--steps", "2",
                        "--warmup", "1", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 8 and line["scaling"] == "weak"
    assert line["parity_all_ranks"] is True and line["value"] > 0
    c4 = line["config4"]
    assert c4["streams_per_gpu"] == 128 and c4["parity_vs_oracle"] is True
    assert c4["strong_scaling_efficiency"] > 0 and c4["n1_value_rank0_alone"] > 0
    c5 = line["config5"]
    assert c5["streams_per_gpu"] == 2 and len(c5["lines"]) == 12
    assert all(v["parity_vs_oracle"] is True for v in c5["lines"].values()), c5["lines"]
    assert c5["parity_definition"].startswith("the whole first stream of rank 0 and of rank 7")
    assert "summary" in line and line["summary"]["value_GiBps"] == line["value"]
