"""pysnptools_amd.dist without a GPU: the rank layout from the launcher's environment, device
choice under per-rank HIP_VISIBLE_DEVICES, the ncclUniqueId hand-off between real processes,
the time limits, and the single-node refusal.  (The RCCL calls themselves run in the GPU tests.)"""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT
from pysnptools_amd import dist as D


def test_env_layout_defaults_and_torchrun_vars():
    assert D.env_layout({}) == (0, 1, 0, 1)
    env = {"RANK": "5", "WORLD_SIZE": "8", "LOCAL_RANK": "5", "LOCAL_WORLD_SIZE": "8"}
    assert D.env_layout(env) == (5, 8, 5, 8)
    # a launcher that sets only RANK / WORLD_SIZE: local rank = rank on one node
    assert D.env_layout({"RANK": "2", "WORLD_SIZE": "4"}) == (2, 4, 2, 4)
    with pytest.raises(ValueError):
        D.env_layout({"RANK": "4", "WORLD_SIZE": "4"})


def test_pick_device_narrowed_visibility():
    assert D.pick_device(3, 8) == 3  # all 8 GPUs visible: LOCAL_RANK
    assert D.pick_device(3, 1) == 0  # one GPU made visible per rank: it is device 0
    with pytest.raises(RuntimeError):
        D.pick_device(0, 0)


def test_multi_node_refused_without_shared_id_file():
    env = {"RANK": "0", "WORLD_SIZE": "16", "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "8"}
    with pytest.raises(RuntimeError, match="single-node"):
        D.init_from_env(env=env, set_current=False)


def test_id_file_is_private_per_launcher(monkeypatch):
    monkeypatch.delenv("SNPMI_RCCL_ID_FILE", raising=False)
    a = D.id_file({"MASTER_PORT": "1234"})
    b = D.id_file({"MASTER_PORT": "1235"})
    assert a != b and "1234" in a
    assert D.id_file({"SNPMI_RCCL_ID_FILE": "/x/y"}) == "/x/y"


def test_publish_never_overwrites(tmp_path):
    path = str(tmp_path / "rccl.id")
    D.publish_id(path, bytes(range(128)))
    with pytest.raises(FileExistsError):
        D.publish_id(path, bytes(128))
    assert D.wait_id(path, timeout=1) == bytes(range(128))
    assert [p for p in os.listdir(tmp_path)] == ["rccl.id"]  # no temporaries left


def test_wait_id_times_out(tmp_path):
    t0 = time.time()
    with pytest.raises(TimeoutError):
        D.wait_id(str(tmp_path / "never"), timeout=0.5)
    assert time.time() - t0 < 5


def test_run_bounded_times_out_and_reraises():
    with pytest.raises(TimeoutError):
        D._run_bounded(lambda: time.sleep(5), 0.3, "sleep")
    with pytest.raises(ZeroDivisionError):
        D._run_bounded(lambda: 1 / 0, 5, "div")
    assert D._run_bounded(lambda: 7, 5, "seven") == 7


def test_rccl_init_binds_the_helper_thread_to_the_rank_device(monkeypatch, tmp_path):
    """ncclCommInitRank runs on a helper thread (bounded wait) and the library's current device is
    per thread: the helper must select this rank's device itself before the init, or every rank's
    communicator would be built on device 0."""
    import threading

    from pysnptools_amd import _native as N

    calls = []
    monkeypatch.setattr(N, "device_count", lambda: 8)
    monkeypatch.setattr(N, "call", lambda name, *a: calls.append((name, a, threading.get_ident())))
    env = {"RANK": "0", "WORLD_SIZE": "4", "LOCAL_RANK": "3", "LOCAL_WORLD_SIZE": "4",
           "SNPMI_RCCL_ID_FILE": str(tmp_path / "rccl.id")}
    d = D.init_from_env(env=env, set_current=False, timeout=30)
    assert d.device == 3
    init = [c for c in calls if c[0] == "snpmi_rccl_init"]
    assert len(init) == 1
    helper = init[0][2]
    assert helper != threading.get_ident()
    on_helper = [c for c in calls if c[2] == helper]
    assert on_helper[0][0] == "snpmi_set_device" and on_helper[0][1] == (3,)
    assert on_helper[1][0] == "snpmi_rccl_init"


_WORKER = r"""
import os, sys
sys.path.insert(0, %r)
from pysnptools_amd import dist as D
rank = int(os.environ["RANK"])
path = D.id_file()
if rank == 0:
    D.publish_id(path, bytes([7] * 128))
else:
    assert D.wait_id(path, timeout=60) == bytes([7] * 128)
print("ok", rank)
"""


@pytest.mark.parametrize("world", [2, 4])
def test_id_handoff_between_processes(tmp_path, world):
    """Rank 0 publishes, the other ranks (started first) wait for the file and read the same id."""
    env = dict(os.environ, SNPMI_RCCL_ID_FILE=str(tmp_path / "rccl.id"), WORLD_SIZE=str(world))
    procs = []
    for r in list(range(1, world)) + [0]:
        procs.append(subprocess.Popen([sys.executable, "-c", _WORKER % ROOT], env=dict(env, RANK=str(r)),
                                      stdout=subprocess.PIPE, text=True))
        time.sleep(0.1)
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert sorted(o.strip() for o in outs) == sorted("ok %d" % r for r in range(world))


_HOST_WORKER = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np
from pysnptools_amd import dist as D
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
d = D.HostDist(rank, world, rank, 0, timeout=60)
assert d.world == world and d.n_gpus == world and not d.rccl
d.barrier()
assert d.max(rank * 1.5) == (world - 1) * 1.5
s = d.sum_host(np.arange(5, dtype=np.float32) * (rank + 1))
assert s.dtype == np.float32 and np.array_equal(s, np.arange(5) * sum(range(1, world + 1)))
parts = d.allgather_bytes(bytes([rank]) * (rank + 1000))
assert [len(p) for p in parts] == [r + 1000 for r in range(world)] and all(p[:1] == bytes([r]) for r, p in enumerate(parts))
# the host-staged reduce behind sum_dev: on every rank, or on one root only
tot = d._reduce_f64(np.full(3, rank + 1.0))
assert np.array_equal(tot, np.full(3, world * (world + 1) / 2.0))
for root in range(world):
    got = d._reduce_f64(np.full(2, float(rank)), root=root)
    assert (got is None) == (rank != root), (rank, root)
    if got is not None:
        assert np.array_equal(got, np.full(2, world * (world - 1) / 2.0))
e = d._reduce_f64(np.zeros(0))
assert e is not None and e.size == 0
assert d.can_reduce
d.barrier()
d.close()
print("ok", rank)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_host_rehearsal_group_collectives(tmp_path, world):
    """HostDist (SNPMI_DIST_HOST=1, the rehearsal group bench.py's N > 1 control flow runs on with
    every rank on one GPU): barrier, max-over-ranks, host sums and byte all-gathers across real
    processes through rank 0's socket hub (its port handed over in the id file)."""
    env = dict(os.environ, SNPMI_RCCL_ID_FILE=str(tmp_path / "hub.id"), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, "-c", _HOST_WORKER % ROOT], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = [p.communicate(timeout=180) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    assert sorted(o[0].strip() for o in outs) == sorted("ok %d" % r for r in range(world))
