"""bench.py contract on the CPU: ``--gpus N`` launches its own N ranks when started bare (no
WORLD_SIZE), and rank 0 prints exactly one JSON line.  Without a GPU the line is a gloo rehearsal of
the edge-cut plumbing (launcher, partition, halo all-to-all, max-over-ranks timing), marked as such."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_self_launches_n_ranks_without_world_size():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--graph", "S1", "--hidden", "8", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 1
    assert out["metric"] == "edges/sec SIRConv fwd+bwd, d_hidden=256, 1/2/4/8 MI355X"
    assert out["config"]["E"] == 10_000_000 and "edge-cut" in out["config"]["parallelism"]
    assert "rehearsal" in out                   # no GPU here: plumbing only, not a measurement


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_bench_cfg5_data_parallel_rehearsal_two_ranks():
    """``bench.py --gpus 2 --dist-backend gloo --workload cfg5``: two self-launched ranks, a different
    molecule batch per rank, DDP's gloo all-reduce, one JSON line (a rehearsal: no GPU here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--workload", "cfg5", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and "rehearsal" in out
    assert out["config"]["parallelism"] == "data-parallel x2" and out["config"]["graphs"] == 128
