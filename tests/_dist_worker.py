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


def partitioned(out_dir):
    """cfg5's read of K[iid0, iid1] (kernelreader.PartitionedKernel) over gloo: each rank holds only
    the 256x256 blocks of its part (the library's layout, shard.part_coords), fills the entries of
    the requested sub-matrix that its blocks hold (0 elsewhere; NumPy standing in for
    k_part_extract) and the ranks' outputs are summed -- every rank must get the sub-matrix."""
    import torch.distributed as dist

    from pysnptools_amd.shard import part_coords

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = GlooDist(rank, world)
    n = 2300
    rng = np.random.default_rng(11)
    Z = rng.standard_normal((n, 40))
    K = Z.dot(Z.T)  # every rank builds the same K; each keeps only its blocks
    coords = part_coords(n, rank, world)
    slot = {(int(r0) // 256, int(c0) // 256): b for b, (r0, c0) in enumerate(coords)}
    nb = (n + 255) // 256
    blocks = np.zeros((len(coords), 256, 256))
    Kp = np.zeros((nb * 256, nb * 256))
    Kp[:n, :n] = K
    for (I, J), b in slot.items():
        blocks[b] = Kp[256 * I:256 * I + 256, 256 * J:256 * J + 256]
    rows, cols = rng.permutation(n)[:300], np.arange(n - 1, 0, -7)
    out = np.zeros((len(rows), len(cols)))
    for a, i in enumerate(rows):
        for c, j in enumerate(cols):
            lo, hi = min(i, j), max(i, j)
            b = slot.get((lo // 256, hi // 256))
            if b is not None:
                out[a, c] = blocks[b, lo % 256, hi % 256]
    out = d.sum_host(out)
    np.save(os.path.join(out_dir, "P%d.npy" % rank), out)
    np.save(os.path.join(out_dir, "Pref.npy"), K[np.ix_(rows, cols)])
    np.save(os.path.join(out_dir, "Pn%d.npy" % rank), np.array([len(coords)]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if sys.argv[2] == "partitioned":
        partitioned(sys.argv[1])
    else:
        main(sys.argv[1], int(sys.argv[2]))
