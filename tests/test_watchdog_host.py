"""pysnptools_amd.dist.Watchdog without a GPU: a world-3 job in the host rehearsal group
(HostDist over local sockets) where one rank stalls inside a leg while the others wait for it in a
collective.  Every rank must exit non-zero within the bound, each with its one-line diagnostic
(rank, leg, detail, the group's last call, the library's collective trace), rank 0 with a partial
JSON line on stdout -- the failure mode of the driver's first multi-GPU run made bounded and
self-describing."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

_WORKER = r"""
import json, os, sys, time
sys.path.insert(0, %r)
from pysnptools_amd import dist as D
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = os.environ["WD_MODE"]
d = D.HostDist(rank, world, rank, 0, timeout=120)
d.watchdog_path = D.id_file() + ".watchdog"

def on_fire(diag):
    print(json.dumps({"metric": "m", "value": None, "partial": True, "watchdog": diag}), flush=True)

# "stall": every rank's bound is short; "peer": only the stalled rank's is, the others must learn of
# it through the abort file; "raise": rank 2 raises outside any collective and calls fail()
limit = 2.0 if mode == "stall" or (mode == "peer" and rank == 1) else 60.0
wd = D.Watchdog(d, limit=limit, on_fire=on_fire if rank == 0 else None, poll=0.1)
wd.mark("leg A")
d.barrier()
wd.mark("leg B", detail="block 7")
if mode in ("stall", "peer") and rank == 1:
    time.sleep(120)  # stuck inside leg B
if mode == "raise" and rank == 2:
    try:
        raise RuntimeError("boom")
    except RuntimeError as e:
        wd.fail("RuntimeError on rank 2: %%s" %% e)
try:
    d.barrier()  # the other ranks wait here for the stalled one
except Exception as e:  # a peer's exit closed the hub: report it the way bench.py does
    wd.fail("%%s on rank %%d: %%s" %% (type(e).__name__, rank, e))
print("unreachable", rank, flush=True)
"""


def _run(tmp_path, mode, world=3):
    env = dict(os.environ, SNPMI_RCCL_ID_FILE=str(tmp_path / "hub.id"), WORLD_SIZE=str(world), WD_MODE=mode)
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, "-c", _WORKER % ROOT], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = [p.communicate(timeout=90) for p in procs]
    return time.time() - t0, procs, outs


def _diag(err):
    lines = [ln for ln in err.splitlines() if ln.startswith("[watchdog] rank ")]
    assert len(lines) == 1, err[-2000:]
    return json.loads(lines[0].split(" ", 3)[3])


@pytest.mark.parametrize("mode", ["stall", "peer", "raise"])
def test_watchdog_bounds_a_stalled_rank(tmp_path, mode):
    took, procs, outs = _run(tmp_path, mode)
    assert took < 40, took
    assert all(p.returncode == 4 for p in procs), [(p.returncode, o[1][-1500:]) for p, o in zip(procs, outs)]
    diags = [_diag(err) for _, err in outs]
    assert [d["rank"] for d in diags] == [0, 1, 2]
    for d in diags:
        assert d["world"] == 3 and d["leg"] == "leg B" and d["detail"] == "block 7" and d["group"] == "host"
        assert d["group_ops"] >= 1 and d["group_last_op"] == "barrier"
        # the library's collective trace is readable from the watchdog thread (no RCCL here: zeros)
        assert isinstance(d["rccl_trace"], dict) and d["rccl_trace"]["calls"] == 0, d["rccl_trace"]
    if mode == "peer":  # only rank 1's own bound expired; ranks 0 and 2 fired on its abort file
        assert diags[1]["reason"].startswith("no progress")
        assert all(diags[r]["reason"].startswith("another rank") for r in (0, 2))
    if mode == "raise":
        assert diags[2]["reason"].startswith("RuntimeError on rank 2")
    # rank 0: exactly one partial JSON line on stdout, nobody reached the statement after the stall
    out0 = [ln for ln in outs[0][0].splitlines() if ln.strip()]
    assert len(out0) == 1 and json.loads(out0[0])["partial"] is True
    assert not any("unreachable" in o for o, _ in outs)


def test_watchdog_quiet_when_marked(tmp_path):
    """A rank that keeps marking never fires, and stop() ends the thread."""
    from pysnptools_amd import dist as D

    class G(object):
        rank, world, rccl, ops, last_op = 0, 1, False, 0, None

    wd = D.Watchdog(G(), limit=0.5, poll=0.05, path=str(tmp_path / "wd"))
    for _ in range(20):
        time.sleep(0.05)
        wd.mark("leg", detail=1)
    wd.stop()
    assert not os.path.exists(str(tmp_path / "wd"))
