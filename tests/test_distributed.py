"""world_size-2 gloo rehearsal of the multi-GPU GRM (no GPU): each rank computes the
partial K of its SNP blocks (oracle arithmetic stands in for the MFMA kernel), the partials
are all-reduced, and every rank must hold the full-matrix K and the merged stats."""
import os
import socket

import numpy as np
import pytest

from conftest import DATA, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from oracle import oracle as O
    from pysnptools_amd.shard import merge_order, rank_blocks

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    body = O.read_bed_bytes(os.path.join(DATA, "n300.bed"))
    n, m, block = 300, 1015, 97
    K = np.zeros((n, n))
    stats = []
    for s0, c in rank_blocks(m, block, rank, world):
        Z = O.decode(body, n, m, sid_index=np.arange(s0, s0 + c))
        stats.append(O.standardize_native(Z))
        K += Z.dot(Z.T)
    t = torch.from_numpy(K)
    dist.all_reduce(t)
    gathered = [None] * world
    dist.all_gather_object(gathered, stats)
    merged = np.concatenate([gathered[r][i] for r, i in merge_order(m, block, world)])
    np.save(os.path.join(out_dir, "K%d.npy" % rank), t.numpy())
    np.save(os.path.join(out_dir, "S%d.npy" % rank), merged)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_grm_equals_single(tmp_path, world):
    import torch.multiprocessing as mp

    from oracle import oracle as O
    from pysnptools_amd.shard import rank_blocks, snp_blocks

    blocks = snp_blocks(1015, 97)
    owned = sorted(b for r in range(world) for b in rank_blocks(1015, 97, r, world))
    assert owned == blocks  # every block exactly once
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    Kref, sref = O.grm_from_bed(O.read_bed_bytes(os.path.join(DATA, "n300.bed")), 300, 1015)
    for r in range(world):
        K = np.load(tmp_path / ("K%d.npy" % r))
        np.testing.assert_allclose(K, Kref, rtol=1e-10, atol=1e-8)
        np.testing.assert_array_equal(np.load(tmp_path / ("S%d.npy" % r)), sref)
