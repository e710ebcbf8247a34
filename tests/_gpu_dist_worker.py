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


SYNTH = (2300, 700)


def write_bed(path, n, m, seed):
    """A random .bed/.fam/.bim (codes 0..3, pad bits zero), written with NumPy."""
    rng = np.random.default_rng(seed)
    bpc = (n + 3) // 4
    codes = rng.choice(np.array([0, 1, 2, 3], dtype=np.uint8), size=(m, bpc * 4), p=[0.4, 0.05, 0.3, 0.25])
    codes[:, n:] = 0
    body = (codes[:, 0::4] | (codes[:, 1::4] << 2) | (codes[:, 2::4] << 4) | (codes[:, 3::4] << 6)).astype(np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(body.tobytes())
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))


def kernel_reader_api(out, save, path, name):
    """SnpKernel(bed, Unit())[rows, cols].read(), Bed.read_kernel, DiagKtoN and the persisted blocks,
    every K partitioned over the group (set_grm_partition("always"))."""
    from pysnptools_amd.kernelreader import PartitionedKernel, SnpKernel, set_grm_partition
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    set_grm_partition("always")
    try:
        bed = Bed(path, count_A1=False)
        rows, cols = pk_indices(bed.iid_count)
        for dt in (np.float32, np.float64):
            sk = SnpKernel(bed, Unit())
            save("%s_pk_sub_%s" % (name, np.dtype(dt).name), sk[rows, cols].read(dtype=dt).val)
            save("%s_pk_full_%s" % (name, np.dtype(dt).name), bed.read_kernel(Unit(), dtype=dt).val)
        kd, _, k_tr = SnpKernel(bed, Unit())._read_with_standardizing(True, return_trained=True)
        save("%s_pk_diag" % name, kd.val)
        save("%s_pk_factor" % name, np.array([k_tr.factor]))
        sk = SnpKernel(bed, Unit())
        sk[rows, cols].read(dtype=np.float32)
        pk = sk._partitioned(np.float32)
        pk.write(os.path.join(out, name + "_pk"))
        pk2 = PartitionedKernel.load(os.path.join(out, name + "_pk"))
        save("%s_pk_loaded" % name, pk2[rows, cols].read(dtype=np.float32).val)
    finally:
        set_grm_partition("auto")


def pk_indices(n):
    rng = np.random.default_rng(7)
    return rng.permutation(n)[:max(1, n // 3)], np.arange(n - 1, 0, -3)


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
        blocks, coords, tr = shard.grm_partitioned(bed[rows, :], Unit(), block_size=97, dtype=np.float64)
        save("%s_part_f64_blocks" % name, blocks)
        save("%s_part_f64_coords" % name, coords)
        save("%s_part_f64_stats" % name, tr.stats)
    # a K of 9 x 9 blocks, so every part of the plan owns some (the fixtures' K is one block)
    synth = os.path.join(out, "synth")
    if r == 0:
        write_bed(synth, SYNTH[0], SYNTH[1], 5)
    d.barrier()
    bed = Bed(synth, count_A1=False)
    for dt in (np.float32, np.float64):
        blocks, coords, tr = shard.grm_partitioned(bed, Unit(), block_size=200, dtype=dt)
        save("synth_part_%s_blocks" % np.dtype(dt).name, blocks)
        save("synth_part_%s_coords" % np.dtype(dt).name, coords)
    # the partitioned K through the reference's KernelReader API (forced partitioning)
    kernel_reader_api(out, save, os.path.join(DATA, "n300"), "n300")
    kernel_reader_api(out, save, synth, "synth")
    d.barrier()
    d.close()
    print("ok", r)


if __name__ == "__main__":
    main(sys.argv[1])
