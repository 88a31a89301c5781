"""bench.py's multi-rank launch contract, rehearsed on CPU (gloo, NLOSGR_BENCH_STUB=1).

`python bench.py --gpus N` without a launcher must start N ranks itself, and a
launcher whose WORLD_SIZE differs from --gpus must be refused rather than reported as N GPUs.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(NLOSGR_BENCH_STUB="1", NLOSGR_DIST_BACKEND="gloo", OMP_NUM_THREADS="1", **kw)
    return env


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT)


def test_gpus2_spawns_two_ranks():
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1"], _env())
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout           # rank 0 alone prints the job line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    assert out["dist"] == {"backend": "gloo", "world_size": 2}
    assert sorted(r["rank"] for r in out["ranks"]) == [0, 1]
    # the job time is the max over ranks
    assert out["ms_per_step"] >= max(r["ms_per_step"] for r in out["ranks"]) - 1e-6


def test_single_rank_default():
    p = _run(["--steps", "2", "--warmup", "0"], _env())
    assert p.returncode == 0, p.stderr
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1


def test_world_size_mismatch_refused():
    p = _run(["--gpus", "4", "--steps", "1", "--warmup", "0"],
             _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr and not p.stdout.strip()


def test_failing_rank_ends_the_job():
    """A rank that dies must not leave the others waiting at the barrier: the launcher ends them
    and exits non-zero."""
    p = _run(["--gpus", "2", "--steps", "2", "--warmup", "0"], _env(NLOSGR_BENCH_STUB_FAIL_RANK="1"),
             timeout=120)
    assert p.returncode != 0
