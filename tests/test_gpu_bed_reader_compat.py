"""The reference-side binding (pysnptools_amd.bed_reader_compat) called exactly
the way PySnpTools calls bed-reader, checked against the reference's goldens:

  * open_bed(filepath, properties={... None ...}, skip_format_check, count_A1, num_threads,
    fam_filepath, bim_filepath)                                           snpreader/bed.py:119-145
  * .read(index=(uintp | None, uintp | None), order, dtype, force_python_only, num_threads)
                                                                          snpreader/bed.py:337-343
  * standardize_f32/f64(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads) with
    `stats` in the val's order (standardizer.py:96-121), train and apply
  * subset_f64_f64 / f32_f64 / f32_f32 on 3-D vals                        util/__init__.py:316-375
"""
import os

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from pysnptools_amd import bed_reader_compat as br

pytestmark = pytest.mark.gpu

SHAPES = {"n300": (300, 1015), "snpgen": (1000, 5), "dist_x": (100, 100)}


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def from_i8(v):
    out = v.astype(np.float64)
    out[v == -127] = np.nan
    return out


def _properties(iid=None, sid=None, pos=None):
    """bed.py:_open_bed_if_needed's dict: the pheno columns None, the rest from a prior read."""
    p = {"father": None, "mother": None, "sex": None, "pheno": None, "allele_1": None, "allele_2": None}
    if iid is not None:
        p["fid"], p["iid"] = iid[:, 0], iid[:, 1]
    if sid is not None:
        p["sid"] = sid
    if pos is not None:
        p["chromosome"], p["cm_position"], p["bp_position"] = pos[:, 0], pos[:, 1], pos[:, 2]
    return p


def _open(name, count_A1=False, with_props=False):
    path = os.path.join(DATA, name + ".bed")
    props = _properties()
    if with_props:
        fam = np.loadtxt(os.path.join(DATA, name + ".fam"), dtype=str, usecols=(0, 1), ndmin=2)
        bim = np.loadtxt(os.path.join(DATA, name + ".bim"), dtype=str, usecols=(0, 1, 2, 3), ndmin=2)
        props = _properties(fam, bim[:, 1], bim[:, [0, 2, 3]].astype(float))
    return br.open_bed(path, properties=props, skip_format_check=False, count_A1=count_A1, num_threads=None,
                       fam_filepath=os.path.join(DATA, name + ".fam"), bim_filepath=os.path.join(DATA, name + ".bim"))


def _uintp(idx):
    return np.ascontiguousarray(idx, dtype=np.uintp)


@pytest.mark.parametrize("name", sorted(SHAPES))
@pytest.mark.parametrize("dtype", ["float32", "float64", "int8"])
@pytest.mark.parametrize("order", ["F", "C"])
@pytest.mark.parametrize("sel", ["all", "iids", "sids", "both"])
def test_open_bed_read_as_bed_py(name, dtype, order, sel):
    n, m = SHAPES[name]
    exp_i8 = g(name)["val_i8"]
    rng = np.random.default_rng(n + m)
    ii = _uintp(rng.permutation(n)[: max(1, n // 3)]) if sel in ("iids", "both") else None
    si = _uintp(rng.permutation(m)[: max(1, m // 2)][::-1]) if sel in ("sids", "both") else None
    with _open(name, with_props=sel == "both") as ob:
        assert ob.iid_count == n and ob.sid_count == m
        val = ob.read(index=(ii, si), order=order, dtype=dtype, force_python_only=False, num_threads=None)
    exp = exp_i8[(slice(None) if ii is None else ii.astype(np.int64))][:, (slice(None) if si is None else si.astype(np.int64))]
    assert val.dtype == np.dtype(dtype)
    assert val.flags["F_CONTIGUOUS" if order == "F" else "C_CONTIGUOUS"]
    if dtype == "int8":
        assert np.array_equal(val, exp)
    else:
        assert np.array_equal(val, from_i8(exp).astype(dtype), equal_nan=True)


def test_open_bed_count_a1_and_metadata():
    with _open("n300", count_A1=True) as ob:
        val = ob.read(index=(None, None), order="F", dtype=np.int8, force_python_only=False, num_threads=2)
        assert np.array_equal(val, g("n300")["val_a1_i8"])
        fam = np.loadtxt(os.path.join(DATA, "n300.fam"), dtype=str, usecols=(0, 1))
        assert np.array_equal(ob.iid, fam[:, 1]) and np.array_equal(ob.fid, fam[:, 0])
        bim = np.loadtxt(os.path.join(DATA, "n300.bim"), dtype=str, usecols=(0, 1, 2, 3))
        assert np.array_equal(ob.sid, bim[:, 1]) and np.array_equal(ob.chromosome, bim[:, 0])
        assert np.array_equal(ob.bp_position, bim[:, 3].astype(float).astype(np.int32))


def test_open_bed_bad_index_raises():
    with _open("dist_x") as ob:
        with pytest.raises(IndexError):
            ob.read(index=(_uintp([0, 100]), None), order="F", dtype="float32")


def _stats_like(val):
    """standardizer.py:99-100: stats of the val's dtype and order."""
    return np.empty([val.shape[1], 2], dtype=val.dtype, order="F" if val.flags["F_CONTIGUOUS"] else "C")


@pytest.mark.parametrize("dtype,tol", [(np.float32, 1e-5), (np.float64, 1e-10)])
@pytest.mark.parametrize("order", ["F", "C"])
@pytest.mark.parametrize("kind", ["unit", "beta"])
def test_standardize_train_as_standardizer_py(dtype, tol, order, kind):
    gg = g("n300")
    tag = "f32" if dtype == np.float32 else "f64"
    val = np.array(from_i8(gg["val_i8"]), dtype=dtype, order=order)
    stats = _stats_like(val)
    fn = br.standardize_f32 if dtype == np.float32 else br.standardize_f64
    is_beta, a, b = (True, 1.0, 25.0) if kind == "beta" else (False, np.nan, np.nan)
    fn(val, is_beta, a, b, True, False, stats, None)
    assert stats.flags["F_CONTIGUOUS" if order == "F" else "C_CONTIGUOUS"]
    np.testing.assert_allclose(val, gg["%s_%s" % (kind, tag)], rtol=tol, atol=tol)
    np.testing.assert_allclose(stats, gg["%s_stats_%s" % (kind, tag)], rtol=tol, atol=0)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("order", ["F", "C"])
def test_standardize_stats_only_leaves_val(dtype, order):
    """apply_in_place=False: stats are computed, the values are left as they were."""
    gg = g("n300")
    val = np.array(from_i8(gg["val_i8"]), dtype=dtype, order=order)
    before = val.copy()
    stats = _stats_like(val)
    (br.standardize_f32 if dtype == np.float32 else br.standardize_f64)(val, False, np.nan, np.nan, False, False,
                                                                          stats, 4)
    assert np.array_equal(val, before, equal_nan=True)
    tol = 1e-5 if dtype == np.float32 else 1e-10
    np.testing.assert_allclose(stats, gg["unit_stats_" + ("f32" if dtype == np.float32 else "f64")], rtol=tol)


@pytest.mark.parametrize("kind", ["unit", "beta"])
@pytest.mark.parametrize("order", ["F", "C"])
def test_standardize_apply_trained_stats(kind, order):
    """UnitTrained/BetaTrained (unittrained.py:47-70): stats trained on iids 10.., applied with
    use_stats=True to iids 0..9 (standardizer.py:31-42 doctest); stats passed in the val's order."""
    gg = g("n300")
    raw = from_i8(gg["val_i8"])
    is_beta, a, b = (True, 1.0, 25.0) if kind == "beta" else (False, np.nan, np.nan)
    train = np.array(raw[10:], order=order)
    stats = _stats_like(train)
    br.standardize_f64(train, is_beta, a, b, False, False, stats, None)
    np.testing.assert_allclose(stats, gg[kind + "_train_stats"], rtol=1e-10)
    test = np.array(raw[:10], order=order)
    stats_in = np.array(gg[kind + "_train_stats"], order=order)
    br.standardize_f64(test, is_beta, a, b, True, True, stats_in, None)
    np.testing.assert_allclose(test, gg[kind + "_test"], rtol=1e-10, atol=1e-12)
    # f32 val with f32 stats
    test32 = np.array(raw[:10], dtype=np.float32, order=order)
    br.standardize_f32(test32, is_beta, a, b, True, True, np.array(stats_in, dtype=np.float32, order=order), None)
    np.testing.assert_allclose(test32, gg[kind + "_test"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag,dtype,tol", [("f64", np.float64, 1e-10), ("f32", np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
@pytest.mark.parametrize("kind", ["unit", "beta"])
def test_standardize_edge_goldens(tag, dtype, tol, order, kind):
    """SNC, missing and all-missing columns (Python-path semantics: NaN stats, zero column)."""
    e = g("edge")
    key = "%s_%s_%s" % (kind, tag, order)
    is_beta, a, b = (True, 2.0, 10.0) if kind == "beta" else (False, np.nan, np.nan)
    fn = br.standardize_f32 if dtype == np.float32 else br.standardize_f64
    x0 = np.array(e["x0"], dtype=dtype, order=order)
    stats = _stats_like(x0)
    fn(x0, is_beta, a, b, True, False, stats, None)
    np.testing.assert_allclose(x0, e[key + "_train"], rtol=tol, atol=tol)
    np.testing.assert_allclose(stats, e[key + "_stats"], rtol=tol, atol=0)
    x1 = np.array(e["x1"], dtype=dtype, order=order)
    fn(x1, is_beta, a, b, True, True, stats, None)
    np.testing.assert_allclose(x1, e[key + "_apply"], rtol=tol, atol=tol)


@pytest.mark.parametrize("fn,src,dst", [("subset_f64_f64", np.float64, np.float64),
                                        ("subset_f32_f64", np.float32, np.float64),
                                        ("subset_f32_f32", np.float32, np.float32)])
@pytest.mark.parametrize("in_order", ["F", "C"])
@pytest.mark.parametrize("out_order", ["F", "C"])
@pytest.mark.parametrize("k", [1, 3])
def test_subset_3d_as_sub_matrix(fn, src, dst, in_order, out_order, k):
    """util/__init__.py:316-375: val reshaped to 3-D (iid, sid, k), sub_val = np.full(..., NaN,
    order), row/col lists as uintp, written in place."""
    rng = np.random.default_rng(k)
    val = np.array(rng.standard_normal((37, 23, k)), dtype=src, order=in_order)
    rows = _uintp([5, 0, 36, 5, 12])
    cols = _uintp(rng.permutation(23)[:9])
    out = np.full((len(rows), len(cols), k), np.nan, dtype=dst, order=out_order)
    getattr(br, fn)(val, rows, cols, out, None)
    exp = val[rows.astype(np.int64)][:, cols.astype(np.int64)].astype(dst)
    assert np.array_equal(out, exp)
