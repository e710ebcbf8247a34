"""Dense standardize of float matrices (SnpData.standardize -> snpmi_standardize_*, the reference's
standardizer.py:90-133 call of bed-reader's standardize_f32/f64) through the round-4 kernels:
k_std_cols_f (F order; genotype-valued columns with the whole column in registers -- one HBM read
and one write --, a table lookup instead of a per-element f64 divide, other columns handed to the
general kernel) and k_std_cols_c16 (C order, 16-B row segments).

Every case is compared bit for bit with round 3's kernels (hook "std" = 1, the general path) and
with the oracle's restatement of bed-reader: the shapes hit every dispatch tier (256 x 4, 256 x 16,
1024 x 8, 1024 x 16 vectors per column, and the chunked two-read path beyond 64k f32 rows), columns
whose start is not 16-B aligned (odd row counts), NaN, -0.0, non-genotype values in some columns
(the flagged fallback), all-missing and constant columns, trained stats, Unit and Beta(1,25)."""
import numpy as np
import pytest

from oracle import oracle as O
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


def _std(val, beta=False, use_stats=False, stats=None):
    v = val.copy(order="K")
    order_c = 1 if v.flags["C_CONTIGUOUS"] and not v.flags["F_CONTIGUOUS"] else 0
    st = np.empty((v.shape[1], 2), dtype=v.dtype) if stats is None else np.array(stats, dtype=v.dtype)
    N.call("snpmi_standardize_" + N.suffix(v.dtype), N.ptr(v), v.shape[0], v.shape[1], order_c, int(beta),
           1.0 if beta else np.nan, 25.0 if beta else np.nan, 1, int(use_stats), N.ptr(st), 0)
    return v, st


def _old(val, **kw):
    N.call("snpmi_set_kernel_variant", b"std", 1)
    try:
        return _std(val, **kw)
    finally:
        N.call("snpmi_set_kernel_variant", b"std", 0)


def _matrix(rows, cols, dtype, order, seed, other_cols=(), negzero_cols=()):
    rng = np.random.default_rng(seed)
    p = rng.uniform(0.0, 0.5, cols)
    g = (rng.random((rows, cols)) < p).astype(np.int64) + (rng.random((rows, cols)) < p)
    val = g.astype(dtype)
    val[rng.random((rows, cols)) < 0.2] = np.nan
    if cols > 2:
        val[:, 1] = np.nan  # all missing
        val[:, 2] = 2.0     # constant (SNC)
    for j in other_cols:
        val[:, j] = rng.standard_normal(rows).astype(dtype)
        val[rng.random(rows) < 0.1, j] = np.nan
    for j in negzero_cols:
        val[val[:, j] == 0, j] = -0.0
    return np.asarray(val, order=order)


def _same(a, b):
    return np.array_equal(a.view(np.uint32 if a.dtype == np.float32 else np.uint64),
                          b.view(np.uint32 if b.dtype == np.float32 else np.uint64))


ROWS = [1, 3, 300, 4099, 16383, 40003, 50000, 65537, 131071]


@pytest.mark.parametrize("rows", ROWS)
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_f_order_unit_matches_round3_and_oracle(rows, dtype):
    cols = 7 if rows > 60000 else 11
    val = _matrix(rows, cols, dtype, "F", rows, other_cols=(4,) if cols > 4 else (), negzero_cols=(5,))
    got, st = _std(val)
    old, st_old = _old(val)
    assert _same(got, old) and _same(st, st_old)
    ref = val.copy(order="F")
    st_ref = O.standardize_native(ref)
    geno = [j for j in range(cols) if j not in (4,)]
    assert _same(got[:, geno], ref[:, geno]) and _same(st[geno], st_ref[geno])
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("rows", [300, 16383, 50000, 65537])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_f_order_beta_and_trained(rows, dtype):
    val = _matrix(rows, 9, dtype, "F", rows + 1, other_cols=(3,))
    got, st = _std(val, beta=True)
    old, st_old = _old(val, beta=True)
    assert _same(got, old) and _same(st, st_old)
    # trained (use_stats): the stats of a first pass applied to the same values
    got2, _ = _std(val, use_stats=True, stats=st)
    old2, _ = _old(val, use_stats=True, stats=st)
    assert _same(got2, old2)
    ref = val.copy(order="F")
    O.standardize_native(ref, use_stats=True, stats=st)
    geno = [j for j in range(9) if j != 3]
    assert _same(got2[:, geno], ref[:, geno])


@pytest.mark.parametrize("shape", [(300, 1015), (5000, 256), (4099, 257), (1001, 64)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_c_order_matches_round3(shape, dtype):
    rows, cols = shape
    val = _matrix(rows, cols, dtype, "C", cols, other_cols=(7,), negzero_cols=(9,))
    got, st = _std(val)
    old, st_old = _old(val)
    assert _same(got, old) and _same(st, st_old)
    ref = val.copy(order="C")
    st_ref = O.standardize_native(ref)
    geno = [j for j in range(cols) if j != 7]
    assert _same(got[:, geno], ref[:, geno]) and _same(st[geno], st_ref[geno])
    got_b, _ = _std(val, beta=True)
    old_b, _ = _old(val, beta=True)
    assert _same(got_b, old_b)


def test_hbm_resident_values_standardize_in_place():
    """Bed.read(xp='hbm').standardize(Unit()) shape: device values standardized in place equal the
    host path bit for bit."""
    from pysnptools_amd import hbm

    val = _matrix(50000, 33, np.float32, "F", 7)
    host, st = _std(val)
    d = hbm.asarray(val)
    st_d = np.empty((33, 2), dtype=np.float32)
    N.call("snpmi_standardize_f32", N.ptr(d), 50000, 33, 0, 0, np.nan, np.nan, 1, 0, N.ptr(st_d), 0)
    assert _same(d.get(), host) and _same(st_d, st)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("order", ["F", "C"])
def test_fused_read_standardize_equals_two_calls(dtype, order):
    """The reference's read().standardize() call sites (_as_snpdata, SnpKernel.read_snps,
    _read_with_standardizing) run as one fused native call on a Bed: values, stats and the trained
    standardizer are bit-identical to the two calls, for slices, Unit / Beta / trained, host or HBM."""
    import os

    from conftest import DATA
    from pysnptools_amd import hbm
    from pysnptools_amd.kernelreader import SnpKernel
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.snpreader.snpreader import _read_and_standardize
    from pysnptools_amd.standardizer import Beta, Unit

    bed = Bed(os.path.join(DATA, "n300.bed"), count_A1=False)
    for reader in (bed, bed[::-2, 5:900:3]):
        for std in (Unit(), Beta(1, 25)):
            two, tr2 = reader.read(order=order, dtype=dtype).standardize(std, return_trained=True)
            one, tr1 = _read_and_standardize(reader, std, order, dtype)
            assert _same(np.asarray(one.val), np.asarray(two.val)) and one.val.flags["C_CONTIGUOUS"] == (order == "C")
            assert _same(tr1.stats, tr2.stats) and type(tr1) is type(tr2) and str(one) == str(two)
            # trained: applies the given stats
            t1, _ = _read_and_standardize(reader[:100, :], tr1, order, dtype)
            t2 = reader[:100, :].read(order=order, dtype=dtype).standardize(tr2)
            assert _same(np.asarray(t1.val), np.asarray(t2.val))
    os.environ["ARRAY_MODULE"] = "hbm"
    try:
        one, _ = _read_and_standardize(bed, Unit(), order, dtype)
        assert isinstance(one.val, hbm.HbmArray)
    finally:
        del os.environ["ARRAY_MODULE"]
    two = bed.read(order=order, dtype=dtype).standardize(Unit())
    assert _same(one.val.get(order=order), two.val)
    k = SnpKernel(bed, Unit())
    assert _same(np.asarray(k.read_snps(order=order, dtype=dtype).val), two.val)
