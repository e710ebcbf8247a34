"""The partitioned K (cfg5) behind the reference's KernelReader API on one GPU
(pysnptools_amd/kernelreader/partitionedkernel.py; reference kernelreader.py:245-302, 342-350,
snpkernel.py:78-101):

* at configs[4]'s 500,000 iids, part 0 of the 8-part plan computed over SnpGen-shaped SNPs streamed
  from pinned host memory (shard.PartitionedGrm), then a 1024 x 1024 K sub-matrix read through
  ``PartitionedKernel[rows, cols].read()`` -- extracted on the device from the part's blocks --
  against the f64 oracle (stats over every iid), f32 and float64 (the reference's default dtype);
  a read that needs another part's blocks raises;
* one process with the partitioning forced (``set_grm_partition("always")``, one part): every
  KernelReader entry point on the reference fixtures vs the oracle, DiagKtoN, and the
  write / load round trip of the blocks."""
import os

import numpy as np
import pytest

from conftest import DATA, ROOT  # noqa: F401  (sys.path)
import bench
from oracle import oracle as O
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,tol", [(np.float32, 1e-5), (np.float64, 1e-12)])
def test_kernelreader_over_part0_at_500k_iids(dtype, tol):
    from pysnptools_amd.kernelreader import PartitionedKernel
    from pysnptools_amd.shard import PartitionedGrm

    n, m, P, seed, miss = 500_000, 8192, 8, 77, 0.218
    threads = bench.cpu_threads()
    pitch = N.lib().snpmi_packed_pitch(n)
    fill = bench.grm5_source(N, n, pitch, seed, miss, threads)
    g = PartitionedGrm(n, m, N.STD_UNIT, part=0, parts=P, block=4096, out="hbm", dtype=dtype)
    try:
        g.run(fill)
        blocks = g.finish()
        gpu_stats = g.stats()
    finally:
        g.close()
    iid = np.array([["f", "i%d" % i] for i in range(n)])
    pk = PartitionedKernel(iid, blocks, part=0, parts=P, dist=None)
    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(4096, size=1024, replace=False))  # supertile (0, 0) belongs to part 0
    cols = rng.permutation(4096)[:1024]
    K = pk[rows, cols].read(dtype=dtype).val
    assert K.shape == (1024, 1024) and K.dtype == np.dtype(dtype)
    with pytest.raises(ValueError, match="outside part 0"):
        pk[rows, np.array([n - 1])].read(dtype=dtype)
    del pk, blocks
    # oracle: the same SNPs regenerated on the host, stats over all 500k iids
    buf = np.empty((m, pitch), dtype=np.uint8)
    fill(N.ctypes.c_void_p(buf.ctypes.data), 0, m)
    body = np.ascontiguousarray(buf[:, :(n + 3) // 4]).reshape(-1)
    del buf
    stats = O.snp_stats(body, n, m)
    np.testing.assert_array_equal(stats.astype(dtype), gpu_stats)
    Zr = O.decode(body, n, m, iid_index=rows, dtype=np.float64)
    Zc = O.decode(body, n, m, iid_index=cols, dtype=np.float64)
    O.standardize_native(Zr, use_stats=True, stats=stats)
    O.standardize_native(Zc, use_stats=True, stats=stats)
    ref = Zr.dot(Zc.T)
    Zd = O.decode(body, n, m, iid_index=rows[:64], dtype=np.float64)
    O.standardize_native(Zd, use_stats=True, stats=stats)
    scale = float(np.max(np.einsum("ij,ij->i", Zd, Zd)))
    err = np.abs(K.astype(np.float64) - ref).max() / scale
    assert err <= tol, err


@pytest.mark.parametrize("name", ["n300", "toydata"])
def test_kernelreader_api_with_forced_partitioning(name, tmp_path):
    from pysnptools_amd.kernelreader import PartitionedKernel, SnpKernel, set_grm_partition
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    n, m = {"n300": (300, 1015), "toydata": (500, 10000)}[name]
    body = O.read_bed_bytes(os.path.join(DATA, name + ".bed"))
    Z = O.decode(body, n, m, dtype=np.float64)
    st = O.standardize_native(Z)
    Kref = Z.dot(Z.T)
    scale = np.abs(np.diag(Kref)).max()
    bed = Bed(os.path.join(DATA, name + ".bed"), count_A1=False)
    rows, cols = np.arange(n - 1, 0, -3), np.arange(0, n, 2)
    set_grm_partition("always")
    try:
        for dt, tol in ((np.float32, 1e-5), (np.float64, 1e-12)):
            sk = SnpKernel(bed, Unit())
            sub = sk[rows, cols].read(dtype=dt).val
            assert np.abs(sub - Kref[np.ix_(rows, cols)]).max() / scale <= tol
            assert any(v is not None for v in sk._pk.values())  # the blocks are reused by the next read
            sub2 = sk[cols, rows].read(dtype=dt, order="C").val
            np.testing.assert_array_equal(sub2, sub.T)
            full = bed.read_kernel(Unit(), dtype=dt).val
            assert np.abs(full - Kref).max() / scale <= tol and np.array_equal(full, full.T)
        kd, snp_tr, k_tr = SnpKernel(bed, Unit())._read_with_standardizing(True, return_trained=True)
        factor = n / np.trace(Kref)
        np.testing.assert_allclose(k_tr.factor, factor, rtol=1e-13)
        assert np.abs(kd.val - Kref * factor).max() / (scale * factor) <= 1e-12
        np.testing.assert_array_equal(snp_tr.stats, st)
        # FaST-LMM's other kernel standardizers: a trained factor and Identity apply as the
        # scale on extraction of the partitioned K; one it cannot apply falls back to the replicated K
        from pysnptools_amd.kernelstandardizer import DiagKtoNTrained, Identity as KIdentity

        sk = SnpKernel(bed, Unit())
        kd2, _, tr2 = sk._read_with_standardizing(True, DiagKtoNTrained(0.5), return_trained=True)
        assert tr2.factor == 0.5 and np.abs(kd2.val - Kref * 0.5).max() / (scale * 0.5) <= 1e-12
        assert any(v is not None for v in sk._pk.values())
        kd3, _, tr3 = sk._read_with_standardizing(True, KIdentity(), return_trained=True)
        assert isinstance(tr3, KIdentity) and np.abs(kd3.val - Kref).max() / scale <= 1e-12

        class Halve(object):  # a kernel standardizer the partitioned K does not know
            def standardize(self, kerneldata, return_trained=False, force_python_only=False, num_threads=None):
                kerneldata.val[...] *= 0.5
                return (kerneldata, self) if return_trained else kerneldata

        kd4 = SnpKernel(bed, Unit())._read_with_standardizing(True, Halve())
        assert np.abs(kd4.val - Kref * 0.5).max() / (scale * 0.5) <= 1e-12
        import pickle

        assert "_pk" not in pickle.loads(pickle.dumps(sk)).__dict__  # no HBM blocks in pickled state
        sk.release_partitioned()
        assert "_pk" not in sk.__dict__
        sk = SnpKernel(bed, Unit())
        pk = sk._partitioned(np.float64)
        path = str(tmp_path / "k")
        pk.write(path)
        pk2 = PartitionedKernel.load(path)
        np.testing.assert_array_equal(pk2[rows, cols].read().val, pk[rows, cols].read().val)
        assert pk2.iid_count == n and np.array_equal(pk2.iid, bed.iid)
    finally:
        set_grm_partition("auto")
