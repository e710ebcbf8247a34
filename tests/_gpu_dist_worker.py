"""Worker of tests/test_gpu_dist_world.py: one rank of a world-2/3 job on the box's single GPU,
inside the host rehearsal group (SNPMI_DIST_HOST=1 -> pysnptools_amd.dist.HostDist, which the
package treats as any open process group: barriers, sums and all-gathers staged through host
memory because RCCL refuses two ranks per device).  It runs the reference's own entry points
under the group -- Bed.read_kernel (routed through shard.grm_sharded with the all-reduce),
grm_sharded with a reduce onto rank 1, DistributedBed via grm_pieces -- and the cfg5 plan
(shard.grm_partitioned: per-rank .bed shares + all-gather), and saves what every rank got."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "tests", "golden", "data")


def main(out):
    from pysnptools_amd import dist as D
    from pysnptools_amd import shard
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Beta, Unit

    d = D.init_from_env(timeout=120)
    assert D.current() is d and d.world > 1 and d.can_reduce
    r = d.rank

    def save(key, arr):
        if arr is not None:
            np.save(os.path.join(out, "%s.r%d.npy" % (key, r)), np.asarray(arr))

    for name in ("n300", "toydata"):
        bed = Bed(os.path.join(DATA, name + ".bed"), count_A1=False)
        for dt in (np.float32, np.float64):
            kd = bed.read_kernel(Unit(), dtype=dt)  # the reference's call, routed by the open group
            save("%s_readkernel_%s" % (name, np.dtype(dt).name), kd.val)
        K, trained, f = shard.grm_sharded(bed, Unit(), dtype=np.float64, collective="reduce", root=1,
                                          diag_k_to_n=True)
        save("%s_reduce1" % name, K)
        save("%s_reduce1_stats" % name, trained.stats)
        if K is not None:
            save("%s_reduce1_factor" % name, np.array([f]))
        n = bed.iid_count
        rows = np.arange(n - 1, 0, -2)
        for std, tag in ((Unit(), "unit"), (Beta(1, 25), "beta")):
            blocks, coords, tr = shard.grm_partitioned(bed[rows, :], std, block_size=97)
            save("%s_part_%s_blocks" % (name, tag), blocks)
            save("%s_part_%s_coords" % (name, tag), coords)
            save("%s_part_%s_stats" % (name, tag), tr.stats)
    d.barrier()
    d.close()
    print("ok", r)


if __name__ == "__main__":
    main(sys.argv[1])
