"""DistributedBed / _MergeSIDs against the reference-written
tests/datasets/distributed_bed_test1 pieces (distributedbed.py:285-300).  Host-only checks
here; reads, writes and GRMs through the GPU are in the gpu-marked tests below."""
import ctypes
import os
import tempfile

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from pysnptools_amd.shard import rank_pieces
from pysnptools_amd.snpreader import Bed, DistributedBed, _MergeSIDs

DIST = os.path.join(DATA, "distributed_bed_test1")


def dist_x():
    return Bed(os.path.join(DATA, "dist_x.bed"), count_A1=False)


def test_metadata_matches_single_bed():
    d = DistributedBed(DIST)
    x = dist_x()
    assert d.iid_count == 100 and d.sid_count == 100 and len(d.pieces) == 44
    assert np.array_equal(d.iid, x.iid)
    assert np.array_equal(np.sort(d.sid), np.sort(x.sid))
    assert repr(d) == "DistributedBed(LocalCache('%s'))" % DIST


def test_merge_sids_checks():
    x = dist_x()
    m = _MergeSIDs([x[:, :30], x[:, 30:]])
    assert np.array_equal(m.sid, x.sid) and m.iid_count == 100
    with pytest.raises(AssertionError):
        _MergeSIDs([x[:, :30], x[:, 20:40]]).sid  # duplicate SNPs
    with pytest.raises(AssertionError):
        _MergeSIDs([x[:50, :10], x[:, 10:20]]).sid  # different iids


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_pieces_partition(world):
    d = DistributedBed(DIST)
    d._run_once()
    sizes = d._merge.col_count_list
    owned = [rank_pieces(sizes, r, world) for r in range(world)]
    flat = sorted(k for o in owned for k in o)
    assert flat == list(range(len(sizes)))
    loads = [sum(int(sizes[k]) for k in o) for o in owned]
    assert max(loads) - min(loads) <= max(sizes)


# ------------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


@gpu
def test_read_equals_single_bed():
    """distributedbed.py:285-300: the pieces read back to distributed_bed_test1_X's values."""
    d = DistributedBed(DIST)
    x = dist_x()
    sd, sx = d.read(), x.read()
    order = {s: j for j, s in enumerate(sx.sid)}
    idx = np.array([order[s] for s in sd.sid])
    assert np.array_equal(sd.val, sx.val[:, idx], equal_nan=True)
    rows, cols = np.arange(99, 0, -3), np.arange(95, 3, -7)
    sub = d[rows, cols].read(order="C", dtype=np.float32).val
    assert np.array_equal(sub, sx.val[np.ix_(rows, idx[cols])].astype(np.float32), equal_nan=True)


@gpu
def test_write_reproduces_reference_pieces():
    """DistributedBed.write(SnpGen 100x100 -> pieces of 2) rewrites every .bed/.bim/.fam of the
    reference's own distributed_bed_test1 byte for byte (the HIP encoder, count_A1=True)."""
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "db")
        d = DistributedBed.write(out, dist_x(), piece_per_chrom_count=2)
        names = sorted(f for f in os.listdir(DIST) if not f.endswith(".npz"))
        assert names == sorted(f for f in os.listdir(out) if not f.endswith(".npz"))
        for f in names:
            assert open(os.path.join(out, f), "rb").read() == open(os.path.join(DIST, f), "rb").read(), f
        assert np.array_equal(d.read().val, DistributedBed(DIST).read().val, equal_nan=True)


@gpu
@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-5)])
def test_grm_over_pieces_vs_reference(dtype, tol):
    from pysnptools_amd.kernelreader import SnpKernel
    from pysnptools_amd.standardizer import Beta, Unit

    d = DistributedBed(DIST)
    x = dist_x()
    G = np.load(os.path.join(GOLDEN, "dist_x.npz"), allow_pickle=False)
    # K does not depend on SNP order
    K = d.read_kernel(Unit(), dtype=dtype).val
    scale = np.abs(np.diag(G["K_unit"])).max()
    assert np.abs(K - G["K_unit"]).max() / scale <= tol
    Kb = SnpKernel(d, Beta(1, 25)).read(dtype=dtype).val
    assert np.abs(Kb - G["K_beta"]).max() / np.abs(np.diag(G["K_beta"])).max() <= tol
    rows, cols = np.arange(0, 100, 3), np.arange(99, 10, -2)
    Ks, tr = d[rows, cols]._read_kernel(Unit(), dtype=dtype, return_trained=True)
    Kx, trx = x[rows, :][:, [list(x.sid).index(s) for s in d.sid[cols]]]._read_kernel(Unit(), dtype=dtype,
                                                                                      return_trained=True)
    assert np.abs(Ks - Kx).max() / np.abs(np.diag(Kx)).max() <= tol
    np.testing.assert_array_equal(tr.stats, trx.stats)


@gpu
def test_grm_pieces_rccl_world1():
    """shard.grm_pieces with a one-rank RCCL communicator equals the single-session GRM."""
    from pysnptools_amd import _native as N
    from pysnptools_amd.shard import grm_pieces
    from pysnptools_amd.standardizer import Unit

    d = DistributedBed(DIST)
    uid = (ctypes.c_uint8 * 256)()
    N.call("snpmi_rccl_unique_id", uid, 256)
    N.call("snpmi_rccl_init", 1, 0, uid, 256)
    try:
        K, tr, f = grm_pieces(d, Unit(), 0, 1, dtype="float64", diag_k_to_n=True)
    finally:
        N.call("snpmi_rccl_destroy")
    Kref, trref = d._read_kernel(Unit(), return_trained=True)
    Kd = Kref * (100 / np.trace(Kref))
    np.testing.assert_allclose(K, Kd, rtol=1e-12, atol=1e-10)
    np.testing.assert_array_equal(tr.stats, trref.stats)
    assert abs(f - 100 / np.trace(Kref)) < 1e-12
