"""Worker of tests/test_distributed.py (run as a subprocess so the pytest process never
imports torch next to libsnpmi).  Rank r computes the GRM of its SNP blocks with the
oracle arithmetic, then the partials are all-reduced over gloo."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_dir, block):
    import torch
    import torch.distributed as dist

    from oracle import oracle as O
    from pysnptools_amd.shard import merge_order, rank_blocks

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    body = O.read_bed_bytes(os.path.join(ROOT, "tests", "golden", "data", "n300.bed"))
    n, m = 300, 1015
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


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
