"""bench.py's multi-rank launch on the CPU (--dry-run: gloo ranks, the oracle episode as
the step): --gpus N starts N ranks itself, reports n_gpus = N and dpN, and a launcher
whose WORLD_SIZE disagrees with --gpus is refused instead of silently benchmarking one
rank."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=e, capture_output=True, text=True, timeout=300)


def _json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_dry_run_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json(r.stdout)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"].startswith("dp2")
    assert j["allgather_instances"] == 2 * j["config"]["batch_per_gpu"]
    assert j["value"] > 0 and j["scaling"] == "weak"


def test_dry_run_single_rank():
    r = _run(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json(r.stdout)
    assert j["n_gpus"] == 1 and j["config"]["parallelism"].startswith("dp1")


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1"], env={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)
