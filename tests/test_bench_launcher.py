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
    r = _run(["--gpus", "2", "--stub", "--steps", "2", "--warmup", "1", "--batch-streams", "6",
              "--batch-stream-bytes", "65536", "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["workload"].startswith("config4")
    assert line["config"]["streams_per_gpu"] == 3
    assert line["config"]["chunks_total"] == 6 * (65536 // 8192)
    assert line["value"] > 0


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--stub", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
