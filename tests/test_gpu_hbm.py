"""Device-resident values (pysnptools_amd.hbm, ARRAY_MODULE='hbm'): the reference's array-module
seam (util/__init__.py:652-730; snpreader.py:638-643, pstdata.py:139-148, kerneldata.py:73,91,
unit.py:32-38).  Every result computed with val / K in HBM must equal the host-API result of the
same kernels bit for bit, and the goldens at the usual bars."""
import os
import tempfile

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from oracle import oracle as O
from pysnptools_amd import hbm
from pysnptools_amd.kernelreader import KernelData, SnpKernel
from pysnptools_amd.snpreader import Bed, SnpData
from pysnptools_amd.standardizer import Beta, DiagKtoN, Unit
from pysnptools_amd.util import asnumpy, get_array_module, sub_matrix

pytestmark = pytest.mark.gpu


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def bed(name):
    return Bed(os.path.join(DATA, name + ".bed"), count_A1=False)


def body(name):
    return O.read_bed_bytes(os.path.join(DATA, name + ".bed"))


@pytest.fixture
def hbm_env(monkeypatch):
    monkeypatch.setenv("ARRAY_MODULE", "hbm")


def test_hbm_array_round_trip_views_and_elements():
    rng = np.random.default_rng(1)
    for order in ("C", "F"):
        h = np.asarray(rng.standard_normal((37, 11)), order=order)
        d = hbm.asarray(h)
        assert d.order == order and d.shape == h.shape and d.flags[order + "_CONTIGUOUS"]
        assert np.array_equal(d.get(), h) and np.array_equal(asnumpy(d), h)
        assert get_array_module(d) is hbm
        assert d[3, 7] == h[3, 7] and d[-1, -2] == h[-1, -2]
        assert np.array_equal(d[2:5], h[2:5])
        t = d.T
        assert t.shape == (11, 37) and t.ptr == d.ptr and np.array_equal(t.get(), h.T)
        c = d.copy()
        assert c.ptr != d.ptr and np.array_equal(c.get(), h)
        f = hbm.asarray(h.astype(np.float32)).astype(np.float64, order="F")
        assert f.dtype == np.float64 and f.order == "F" and np.array_equal(f.get(), h.astype(np.float32))
        cai = d.__cuda_array_interface__
        assert cai["data"][0] == d.ptr and cai["shape"] == h.shape
    z = hbm.zeros((5, 3), dtype=np.float32)
    assert np.array_equal(z.get(), np.zeros((5, 3), np.float32))
    with pytest.raises(IndexError):
        z[5, 0]


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int8])
@pytest.mark.parametrize("order", ["F", "C"])
def test_read_decodes_into_hbm(dtype, order):
    """Bed.read(xp='hbm') decodes straight into HBM: bit-exact vs the oracle (direct decode when
    the columns are 16-B aligned, block buffer + device copy otherwise)."""
    b = bed("n300")
    full = O.decode(body("n300"), 300, 1015, dtype=dtype)
    for ri, ci in ((slice(None), slice(None)), (slice(None, None, -2), slice(1014, 0, -3)),
                   (np.arange(299), slice(5, 40)), (np.arange(296), [7, 3, 3])):
        d = b[ri, ci].read(order=order, dtype=dtype, xp="hbm", _require_float32_64=False)
        assert isinstance(d.val, hbm.HbmArray) and d.val.dtype == dtype and d.val.order == order
        rows, cols = np.arange(300)[ri], np.arange(1015)[ci]
        assert np.array_equal(d.val.get(), full[np.ix_(rows, cols)], equal_nan=True)


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_standardize_in_hbm(dtype, tol, order):
    G = g("n300")
    tag = "f64" if dtype == np.float64 else "f32"
    for std, key in ((Unit(), "unit"), (Beta(1, 25), "beta")):
        host, th = bed("n300").read(order=order, dtype=dtype).standardize(std, return_trained=True)
        d = bed("n300").read(order=order, dtype=dtype, xp="hbm")
        ptr = d.val.ptr
        d2, td = d.standardize(std, return_trained=True)
        assert isinstance(d2.val, hbm.HbmArray) and d2.val.ptr == ptr  # in place, in HBM
        assert np.array_equal(d2.val.get(), host.val)
        assert np.array_equal(td.stats, th.stats)
        np.testing.assert_allclose(d2.val.get(), G["%s_%s" % (key, tag)], rtol=tol, atol=tol)


def test_unit_moves_host_val_under_env(hbm_env):
    d = SnpData(iid=[["a", str(i)] for i in range(300)], sid=[str(j) for j in range(1015)],
                val=O.decode(body("n300"), 300, 1015, dtype=np.float64))
    assert isinstance(d.val, hbm.HbmArray)  # pstdata.py:146 under ARRAY_MODULE
    d.standardize(Unit())
    np.testing.assert_allclose(d.val.get(), g("n300")["unit_f64"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-5)])
@pytest.mark.parametrize("block_size", [None, 100])
def test_read_kernel_leaves_k_in_hbm(hbm_env, dtype, tol, block_size):
    G = g("n300")
    k = bed("n300").read_kernel(Unit(), block_size=block_size, dtype=dtype)
    assert isinstance(k.val, hbm.HbmArray) and k.val.dtype == dtype
    K = k.val.get()
    np.testing.assert_allclose(K, G["K_unit"], rtol=0, atol=tol * np.abs(np.diag(G["K_unit"])).max())
    kd, _, diag = SnpKernel(bed("n300"), Unit(), block_size=block_size)._read_with_standardizing(
        to_kerneldata=True, return_trained=True)
    assert isinstance(kd.val, hbm.HbmArray)
    np.testing.assert_allclose(diag.factor, G["diag_factor"], rtol=1e-12)
    np.testing.assert_allclose(kd.val.get(), G["K_unit_diag"], rtol=0, atol=1e-10)
    kf = bed("n300").read_kernel(Unit(), order="F", dtype=dtype).val
    assert kf.order == "F" and np.array_equal(kf.get(), K)


def test_kerneldata_diag_k_to_n_in_hbm():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((64, 64))
    Kh = x.dot(x.T)
    host = KernelData(iid=[["a", str(i)] for i in range(64)], val=Kh.copy())
    dev = KernelData(iid=[["a", str(i)] for i in range(64)], val=hbm.asarray(Kh), xp="hbm")
    ptr = dev.val.ptr
    _, th = host.standardize(DiagKtoN(), return_trained=True)
    _, td = dev.standardize(DiagKtoN(), return_trained=True)
    assert dev.val.ptr == ptr and th.factor == td.factor
    assert np.array_equal(dev.val.get(), host.val)


@pytest.mark.parametrize("order", ["F", "C"])
def test_dense_grm_from_device_snpdata(order):
    """SnpData.read_kernel with val in HBM (two-phase path at N >= 4096) == the host API."""
    rng = np.random.default_rng(7)
    n, m = 4200, 45
    v = rng.integers(0, 3, size=(n, m)).astype(np.float32)
    v[rng.random(v.shape) < 0.02] = np.nan
    v = np.asarray(v, order=order)
    iid, sid = [["f", str(i)] for i in range(n)], ["s%d" % j for j in range(m)]
    Kh = SnpData(iid=iid, sid=sid, val=v.copy(order="K")).read_kernel(Unit(), dtype=np.float32).val
    dev = SnpData(iid=iid, sid=sid, val=hbm.asarray(v), xp="hbm")
    Kd = dev.read_kernel(Unit(), dtype=np.float32).val
    assert isinstance(Kd, hbm.HbmArray)
    assert np.array_equal(Kd.get(), Kh)
    assert np.array_equal(dev.val.get(), v, equal_nan=True)  # the input val is left untouched
    # a subset of a device SnpData is gathered on the device (sub_matrix) and gives the same K
    rows = np.arange(n - 1, 0, -2)
    Ks = dev[rows, 3:40].read_kernel(Unit(), dtype=np.float32).val
    Ksh = SnpData(iid=iid, sid=sid, val=v.copy(order="K"))[rows, 3:40].read_kernel(Unit(), dtype=np.float32).val
    assert isinstance(Ks, hbm.HbmArray) and np.array_equal(Ks.get(), Ksh)


def test_generic_block_loop_in_hbm(hbm_env):
    """A reader outside the fused path (here a device SnpData standardized by Identity in
    blocks) accumulates K on the device session and returns it in HBM."""
    G = g("n300")
    d = bed("n300").read(dtype=np.float64).standardize(Unit())
    assert isinstance(d.val, hbm.HbmArray)
    from pysnptools_amd.standardizer import Identity

    K = d._read_kernel_blocks(Identity(), 200, "C", np.dtype(np.float64), False, None)[0]
    assert isinstance(K, hbm.HbmArray)
    np.testing.assert_allclose(K.get(), G["K_unit"], rtol=0, atol=1e-10 * np.abs(np.diag(G["K_unit"])).max())


def test_sub_matrix_on_device():
    rng = np.random.default_rng(5)
    for order in ("C", "F"):
        h = np.asarray(rng.standard_normal((50, 40)).astype(np.float32), order=order)
        rows, cols = rng.permutation(50)[:17], np.arange(39, 0, -3)
        for dtype in (np.float32, np.float64):
            got = sub_matrix(hbm.asarray(h), rows, cols, order="A", dtype=dtype)
            assert isinstance(got, hbm.HbmArray) and got.dtype == dtype
            assert np.array_equal(got.get(), sub_matrix(h, rows, cols, order="A", dtype=dtype))


def test_write_from_device_values():
    """Bed.write of a device SnpData: the encoder reads the values where they are (no host copy)."""
    v = O.decode(body("dist_x"), 100, 100, dtype=np.float64)
    d = SnpData(iid=[["f", str(i)] for i in range(100)], sid=["s%d" % j for j in range(100)], val=hbm.asarray(v))
    with tempfile.TemporaryDirectory() as tmp:
        b = Bed.write(os.path.join(tmp, "w.bed"), d, count_A1=False)
        assert np.array_equal(b.read().val, v, equal_nan=True)


def test_distributed_bed_and_subsets_in_hbm(hbm_env):
    """DistributedBed GRM (one GPU session over the 44 pieces) and SnpKernel subsets with K in HBM
    equal the host API (snpkernel.py:78-99; the subset of a device K is gathered on the device)."""
    import pysnptools_amd.util as U
    from pysnptools_amd.snpreader import DistributedBed

    dist = DistributedBed(os.path.join(DATA, "distributed_bed_test1"))
    Kd = dist.read_kernel(Unit(), dtype=np.float64).val
    assert isinstance(Kd, hbm.HbmArray)
    sub = SnpKernel(bed("toydata"), Unit())[::2, ::3].read(dtype=np.float32).val
    assert isinstance(sub, hbm.HbmArray) and sub.shape == (250, 167)
    os.environ["ARRAY_MODULE"] = "numpy"
    try:
        Kh = dist.read_kernel(Unit(), dtype=np.float64).val
        subh = SnpKernel(bed("toydata"), Unit())[::2, ::3].read(dtype=np.float32).val
    finally:
        os.environ["ARRAY_MODULE"] = "hbm"
    assert isinstance(Kh, np.ndarray) and np.array_equal(Kd.get(), Kh)
    assert np.array_equal(U.asnumpy(sub), subh)
    np.testing.assert_allclose(Kh, g("dist_x")["K_unit"], rtol=1e-10, atol=1e-8)
