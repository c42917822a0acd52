"""bench.py's multi-rank path on the CPU: `--gpus N` spawns N ranks itself (no torchrun around it), each
rank joins a gloo process group, the timed region is max-over-ranks and the work is summed; rank 0 prints
one JSON line.  The GPU workloads take the same launcher / setup / timed_region / sum_max path with nccl."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env_extra=None):
    env = dict(os.environ, MUZ_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "selftest", *extra],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout      # only rank 0 prints
    return json.loads(lines[0])


def test_launcher_two_ranks_weak():
    r = _run("--gpus", "2", "--steps", "3", "--batch", "4096")
    assert r["n_gpus"] == 2
    assert r["units"] == 3 * (1 + 2) * 4096      # summed over both ranks
    assert r["elapsed"] >= 3 * 0.02 * 0.9        # the slower rank (rank 1 sleeps 20 ms a step) bounds the job
    assert r["scaling"] == "weak" and r["config"]["games_per_gpu"] == 4096
    assert r["config"]["parallelism"].startswith("dp2 weak")


def test_launcher_two_ranks_split():
    r = _run("--gpus", "2", "--steps", "2", "--batch", "4096", "--split")
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["games_per_gpu"] == 2048
    assert r["units"] == 2 * (1 + 2) * 2048
    assert r["config"]["parallelism"] == "dp2 strong: 4096 games split 2048/GPU"


def test_single_rank_unchanged():
    r = _run("--steps", "2", "--batch", "64")
    assert r["n_gpus"] == 1 and r["units"] == 2 * 64 and r["scaling"] == "weak"


def test_world_size_mismatch_fails():
    env = dict(os.environ, MUZ_BENCH_BACKEND="gloo", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "selftest", "--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
