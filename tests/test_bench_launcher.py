"""bench.py's own N-rank launcher (CPU, gloo): `bench.py --gpus 2` must start
two ranks itself when no external launcher set WORLD_SIZE, reduce over both
and print n_gpus 2.  The --stub engine replaces the GPU (fixed-size cuts in
numpy) so only the launch, barrier and max/sum reductions are exercised."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    return r


def test_bench_launches_two_ranks_itself():
    """Default: `value` is config 2 per GPU (weak scaling, the same per-GPU work
    as the N=1 line), plus the config-4 strong-scaling sub-object with rank 0's
    whole-batch time from the same run as its N=1 denominator."""
    r = _run(["--gpus", "2", "--stub", "--steps", "2", "--warmup", "1", "--stream-bytes", str(1 << 20),
              "--batch-streams", "6", "--batch-stream-bytes", "65536", "--config4-steps", "2", "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["workload"].startswith("config2")
    assert line["config"]["bytes_per_gpu"] == 1 << 20 and line["config"]["streams_per_gpu"] == 1
    assert line["config"]["chunks_total"] == 2 * ((1 << 20) // 8192)
    assert line["value"] > 0
    c4 = line["config4"]
    assert c4["scaling"] == "strong" and c4["workload"].startswith("config4")
    assert c4["streams_per_gpu"] == 3 and c4["chunks_total"] == 6 * (65536 // 8192)
    assert c4["value"] > 0 and c4["n1_value_rank0_alone"] > 0
    assert abs(c4["strong_scaling_efficiency"] - c4["value"] / (2 * c4["n1_value_rank0_alone"])) < 1e-9


def test_bench_batch_value_is_config4():
    r = _run(["--gpus", "2", "--stub", "--workload", "batch", "--steps", "2", "--warmup", "1",
              "--batch-streams", "6", "--batch-stream-bytes", "65536", "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stdout + r.stderr
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["scaling"] == "strong" and line["config"]["workload"].startswith("config4")
    assert line["config"]["streams_per_gpu"] == 3 and "config4" not in line


def test_bench_single_rank_has_config4():
    r = _run(["--gpus", "1", "--stub", "--steps", "2", "--warmup", "1", "--stream-bytes", str(1 << 20),
              "--batch-streams", "4", "--batch-stream-bytes", "65536", "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stdout + r.stderr
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["n_gpus"] == 1 and line["config4"]["streams_per_gpu"] == 4
    assert "strong_scaling_efficiency" not in line["config4"]


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--stub", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
