"""bench.py's process launch without a GPU: `python bench.py --gpus N` spawns N rank processes
itself (before any HIP call) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set and a private
ncclUniqueId file, relays rank 0's line, and refuses a WORLD_SIZE that differs from --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(SNPMI_BENCH_DRYRUN="1", **kw)
    return env


def test_spawns_n_ranks_and_relays_rank0():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--steps", "1"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 writes to stdout
    d = lines[0]
    assert d["RANK"] == "0" and d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "3"
    assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
    assert d["SNPMI_RCCL_ID_FILE"] and not os.path.exists(os.path.dirname(d["SNPMI_RCCL_ID_FILE"]))  # cleaned up
    others = [json.loads(x) for x in r.stderr.splitlines() if x.startswith("{")]
    assert sorted(o["RANK"] for o in others) == ["1", "2"]


def test_refuses_world_size_mismatch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="4", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=4" in r.stderr


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["RANK"] is None and d["WORLD_SIZE"] is None  # no launcher, no children


def test_rank_failure_propagates():
    # a child that cannot parse its arguments fails; the parent exits non-zero
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "x"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
