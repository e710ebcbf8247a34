"""bench.py's whole N > 1 control flow on ONE GPU: every rank of a world-2 / world-3 job runs on
the box's single device inside the host rehearsal group (SNPMI_DIST_HOST=1, pysnptools_amd.dist.
HostDist: gloo barriers and max-over-ranks, host-staged all-gather; RCCL refuses two ranks per
device).  Both launch paths the driver uses -- bench.py's own spawner (--gpus N) and
torch.distributed.run -- must end with exit 0 and exactly one JSON line from rank 0, the SNP
shards covering the matrix, the cfg5 block rebuilt bit-exactly by the all-gather and every parity
check passing.  Rank 0's rank-only legs (file, CPU baselines) run while the others wait at the
final barrier."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SMALL = ["--steps", "1", "--warmup", "0", "--n-iid", "4099", "--n-sid", "6000", "--grm-iid", "5000",
         "--grm-sid", "12000", "--grm-block", "5000", "--grm5-iid", "20000", "--grm5-sid", "2048",
         "--e2e-sid", "4096", "--e2e-passes", "1", "--cpu-seconds", "0.2", "--beta-iid", "5001",
         "--beta-sid", "6000", "--file-iid", "3001", "--file-sid", "5000", "--cpu-grm-iid", "3000",
         "--cpu-grm-sid", "64", "--dist-timeout", "120"]


def _check(out, world):
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["config"]["process_group"].startswith("host rehearsal")
    assert d["config"]["n_sid_per_gpu"] == 6000 // world and d["value"] > 0
    assert d["parity"]["bit_exact"] and d["beta"]["parity"]["pass"]
    for k in ("grm", "grm_f64"):
        assert d[k]["parity"]["pass"], d[k]["parity"]
        # configs[3]'s exchange is an all-reduce; the reduce is timed beside it
        assert "allreduce" in d[k]["collective"], d[k]["collective"]
        assert set(d[k]["collective_alone"]) >= {"reduce_ms", "allreduce_ms", "bytes"}
    sc = d["selfcheck"]
    assert sc["pass"] and sc["group_size_ok"] and sc["allreduce"]["every_rank_same_K"], sc
    assert sc["allgather_bit_exact"] and sc["rccl_same_calls_every_rank"], sc
    assert d["box"]["uuid"] and d["box"]["fill_GBps"] > 0
    g5 = d["grm5"]
    assert g5["parity"]["pass"] and g5["parity"]["gathered_block_bit_exact"], g5["parity"]
    assert "host all-gather" in g5["workload"]
    f = d["file"]
    assert f["read_kernel_f32"]["parity"]["pass"] and f["read_hbm"]["parity"]["bit_exact"]
    return d


def test_bench_spawned_world2_on_one_gpu():
    env = dict(os.environ, SNPMI_DIST_HOST="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL
    _check(subprocess.run(cmd, capture_output=True, text=True, timeout=290, env=env), 2)


def test_bench_torchrun_world3_on_one_gpu():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, SNPMI_DIST_HOST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "3"] + SMALL
    _check(subprocess.run(cmd, capture_output=True, text=True, timeout=290, env=env), 3)


def test_bench_spawned_world8_on_one_gpu():
    """The driver's largest scaling point (N = 8) rehearsed on one GPU: 8 ranks of bench.py's own
    spawner in the host group -- every rank owns one of the cfg5 plan's 8 parts and 1/8 of each
    block's all-gather, the cfg4 reduce combines 8 partial tile sets."""
    env = dict(os.environ, SNPMI_DIST_HOST="1")
    small = [a for a in SMALL]
    small[small.index("--n-sid") + 1] = "8000"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"] + small
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=290, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["n_sid_per_gpu"] == 1000
    for k in ("grm", "grm_f64"):
        assert d[k]["parity"]["pass"], d[k]["parity"]
    g5 = d["grm5"]
    assert g5["parts"] == 8 and g5["parity"]["pass"] and g5["parity"]["gathered_block_bit_exact"], g5["parity"]


def test_bench_watchdog_world3_stalled_rank():
    """Rank 1 hangs inside the cfg4 leg (SNPMI_BENCH_STALL) while ranks 0 and 2 wait for it at the
    leg's barrier: the whole job must exit 4 within the watchdog bound, every rank's diagnostic line
    on stderr and one partial JSON line (the legs measured before the stall) from rank 0."""
    env = dict(os.environ, SNPMI_DIST_HOST="1", SNPMI_BENCH_STALL="1:grm cfg4")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--watchdog", "20"] + SMALL
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=290, env=env)
    took = time.time() - t0
    assert out.returncode == 4, (out.returncode, out.stderr[-4000:])
    assert took < 240, took
    diags = {}
    for ln in out.stderr.splitlines():
        if ln.startswith("[watchdog] rank "):
            d = json.loads(ln.split(" ", 3)[3])
            diags[d["rank"]] = d
    assert sorted(diags) == [0, 1, 2], out.stderr[-4000:]
    assert all(d["leg"].startswith("grm cfg4") for d in diags.values()), diags
    assert all(d["group"] == "host" and d["group_ops"] > 0 for d in diags.values())
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    p = json.loads(lines[0])
    assert p["partial"] is True and "watchdog" in p["error"] and p["value"] > 0
    assert p["selfcheck"]["pass"] and p["watchdog"]["rank"] == 0


def test_bench_rccl_init_failure_falls_back_to_the_host_group():
    """World 2 WITHOUT the host group on a one-GPU box: RCCL's ncclCommInitRank refuses two ranks
    on one device ("invalid usage") on both ranks, and bench.py runs the job in the host group
    instead of printing nothing -- exit 0, one JSON line naming the RCCL error, every parity check
    passing."""
    env = {k: v for k, v in os.environ.items() if k != "SNPMI_DIST_HOST"}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--watchdog", "60"] + SMALL
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=290, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    c = d["config"]
    if "rccl_init_error" not in c:  # an RCCL that accepts two ranks per device ran the real collectives
        assert c["process_group"] == "rccl"
    else:
        assert "ncclCommInitRank" in c["rccl_init_error"] and c["process_group"].startswith("host rehearsal")
    assert d["selfcheck"]["pass"]
    for k in ("grm", "grm_f64"):
        assert d[k]["parity"]["pass"], d[k]["parity"]
    assert d["grm5"]["parity"]["pass"]
