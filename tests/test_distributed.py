"""world_size-2/3 gloo rehearsal of the multi-GPU GRM (no GPU): each rank computes the partial K
of its contiguous SNP span (shard.rank_span, the product's plan; oracle arithmetic stands in for
the MFMA kernel), the partials are all-reduced, the stats are combined by shard._sum_stats, and
every rank must hold the full-matrix K and the merged stats."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import DATA, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_grm_equals_single(tmp_path, world):
    from oracle import oracle as O
    from pysnptools_amd.shard import rank_span_blocks

    owned = sorted(b for r in range(world) for b in rank_span_blocks(1015, 97, r, world))
    assert sum(c for _, c in owned) == 1015  # every SNP exactly once
    assert all(a[0] + a[1] == b[0] for a, b in zip(owned, owned[1:]))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_dist_worker.py"), str(tmp_path),
                                       "97"], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    Kref, sref = O.grm_from_bed(O.read_bed_bytes(os.path.join(DATA, "n300.bed")), 300, 1015)
    for r in range(world):
        K = np.load(tmp_path / ("K%d.npy" % r))
        np.testing.assert_allclose(K, Kref, rtol=1e-10, atol=1e-8)
        np.testing.assert_array_equal(np.load(tmp_path / ("S%d.npy" % r)), sref)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_span_blocks_cover_once_balanced(world):
    """bench.py's cfg4 plan: contiguous equal SNP shards, each in blocks <= block_size."""
    from pysnptools_amd.shard import rank_span_blocks

    m, bs = 500_000, 10_000
    spans = [rank_span_blocks(m, bs, r, world) for r in range(world)]
    cover = sorted(s0 + i for sp in spans for s0, c in sp for i in (0, c - 1))
    assert sum(c for sp in spans for _, c in sp) == m
    flat = sorted((s0, c) for sp in spans for s0, c in sp)
    assert flat[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(flat, flat[1:]))
    assert all(0 < c <= bs for sp in spans for _, c in sp) and cover[-1] == m - 1
    per = [sum(c for _, c in sp) for sp in spans]
    assert max(per) - min(per) <= 1


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_k_read_over_gloo(tmp_path, world):
    """The partitioned K's sub-matrix read (PartitionedKernel: each rank's blocks in the library's
    layout, non-owned entries 0, summed over the group) rehearsed over gloo: every rank gets
    K[rows, cols] exactly, and the parts cover the 45 blocks of a 2300-iid K once."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_dist_worker.py"), str(tmp_path),
                                       "partitioned"], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    ref = np.load(tmp_path / "Pref.npy")
    assert sum(int(np.load(tmp_path / ("Pn%d.npy" % r))[0]) for r in range(world)) == 45
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("P%d.npy" % r)), ref)
