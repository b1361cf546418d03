"""bench.py's own rank launcher: a plain ``python bench.py --gpus N`` -- the form the driver's
BENCH / SCALE runs use -- must run N ranks, not one.  Exercised on CPU with the ``--stub-step`` hook (gloo): the
parent starts a torch.distributed.run job before importing torch, every rank joins the group, rank 0 alone prints
the single JSON line, and a rank whose group size differs from ``--gpus`` refuses to run.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=env, cwd=str(ROOT))


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_bench_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--stub-step"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["ranks_reporting"] == 2 and line["steps"] == 3
    assert line["pid"] != os.getpid()
    # the DP diagnostics: per-rank step time, exposed all-reduce time and early-bucket lead
    # from the real GradAllReduce, with the max / min over ranks
    dp = line["dp"]
    assert [d["rank"] for d in dp["per_rank"]] == [0, 1]
    for d in dp["per_rank"]:
        assert d["step_ms"] > 0 and d["allreduce_exposed_ms"] >= 0 and d["early_bucket_lead_ms"] >= 0
        assert d["timed_steps"] == 3 and d["early_bucket_steps"] == 3
    for k in ("step_ms", "allreduce_exposed_ms", "early_bucket_lead_ms"):
        agg = dp["over_ranks"][k]
        assert agg["min"] <= agg["max"]
        assert agg["max"] == max(d[k] for d in dp["per_rank"])
    assert dp["bytes_allreduced_per_step"] == 4 * (64 * 64 + 64 + 64 * 8 + 8)


def test_bench_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--steps", "2", "--warmup", "0", "--stub-step"])
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 1 and line["ranks_reporting"] == 1


def test_bench_world_mismatch_refuses():
    """Under a 1-rank torchrun-style environment, --gpus 2 must fail loudly instead of reporting one GPU."""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--stub-step"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert not _json_lines(r.stdout)
    assert "--gpus 2" in r.stderr
