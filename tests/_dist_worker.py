"""Worker of tests/test_distributed.py (run as a subprocess so the pytest process never
imports torch next to libsnpmi).  The product's SNP-sharded plan (pysnptools_amd/shard.py) with
the oracle's arithmetic standing in for the MFMA kernel: rank r owns the contiguous SNP span
``rank_span`` and streams it in blocks of at most ``block`` SNPs (``rank_span_blocks``) into a
partial K and per-SNP stats (zeros for SNPs it does not own); the partial K is all-reduced and
the stats are combined by the product's own ``_sum_stats`` -- over a gloo group instead of RCCL."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class GlooDist(object):
    """The part of pysnptools_amd.dist.Dist that shard.py's host-side combine uses, over gloo."""

    def __init__(self, rank, world):
        self.rank, self.world, self.rccl = rank, world, False

    def sum_host(self, arr):
        import torch
        import torch.distributed as dist

        a = np.asarray(arr)
        t = torch.from_numpy(np.array(a, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy().astype(a.dtype)


def main(out_dir, block):
    import torch.distributed as dist

    from oracle import oracle as O
    from pysnptools_amd.shard import _sum_stats, rank_span, rank_span_blocks

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = GlooDist(rank, world)
    body = O.read_bed_bytes(os.path.join(ROOT, "tests", "golden", "data", "n300.bed"))
    n, m = 300, 1015
    K = np.zeros((n, n))
    stats = np.zeros((m, 2))
    lo, hi = rank_span(m, rank, world)
    for s0, c in rank_span_blocks(m, block, rank, world):
        assert lo <= s0 and s0 + c <= hi
        Z = O.decode(body, n, m, sid_index=np.arange(s0, s0 + c))
        stats[s0:s0 + c] = O.standardize_native(Z)
        K += Z.dot(Z.T)
    K = d.sum_host(K)  # the tile all-reduce (ShardedGrm.combine) on the host
    stats = _sum_stats(d, stats, "allreduce", world)
    np.save(os.path.join(out_dir, "K%d.npy" % rank), K)
    np.save(os.path.join(out_dir, "S%d.npy" % rank), stats)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
