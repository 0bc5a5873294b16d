"""bench.py's driver contract on CPU: ``--gpus N`` launches N ranks itself (gloo rehearsal here),
prints exactly one JSON line, and a failing rank fails the whole command."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None, timeout=600):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["MS_DIST_BACKEND"] = "gloo"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def _json_lines(out: str) -> list[dict]:
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{\"metric\"")]


def test_bench_gpus_two_self_launches_two_ranks():
    p = _run("--gpus", "2", "--steps", "2", "--warmup", "1", "--map-size", "64", "--cells", "200")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    out = lines[0]
    assert out["ranks"] == 2 and out["config"]["ranks"] == 2
    assert out["config"]["parallelism"] == "spatial2"
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0
    assert len(out["devices"]) == 2


def test_bench_single_rank_unchanged():
    p = _run("--steps", "2", "--warmup", "1", "--map-size", "64", "--cells", "200")
    assert p.returncode == 0, p.stderr[-3000:]
    (out,) = _json_lines(p.stdout)
    assert out["ranks"] == 1 and out["config"]["parallelism"] == "single"
    assert "ranks" not in out["config"]


def test_bench_failing_rank_fails_the_command():
    # an impossible config on every rank: the launcher reports the failure with a non-zero code
    p = _run("--gpus", "2", "--steps", "1", "--warmup", "0", "--map-size", "64", "--cells", "200",
             "--chemistry", "synthetic:0:0")
    assert p.returncode != 0
    assert not _json_lines(p.stdout)
