"""Pin the CPU oracle (oracle/) to the reference: its fixtures, doctest digits and the
golden vectors tools/make_golden.py produced by running the reference's Python path."""
import os

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from oracle import oracle as O


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def body(name):
    return O.read_bed_bytes(os.path.join(DATA, name + ".bed"))


def from_i8(v):
    out = v.astype(np.float64)
    out[v == -127] = np.nan
    return out


@pytest.mark.parametrize("name,n_iid,n_sid", [("n300", 300, 1015), ("snpgen", 1000, 5),
                                               ("dist_x", 100, 100), ("toydata", 500, 10000),
                                               ("gen1", 190, 20), ("gen4", 198, 20)])
def test_shape_from_fam_bim(name, n_iid, n_sid):
    assert O.bed_shape(os.path.join(DATA, name + ".bed")) == (n_iid, n_sid)


@pytest.mark.parametrize("name", ["n300", "snpgen", "dist_x"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int8])
@pytest.mark.parametrize("order", ["F", "C"])
def test_decode_bit_exact(name, dtype, order):
    G = g(name)
    exp = G["val_i8"]
    n_iid, n_sid = exp.shape
    got = O.decode(body(name), n_iid, n_sid, order=order, dtype=dtype)
    assert got.flags[order + "_CONTIGUOUS"]
    if dtype == np.int8:
        assert np.array_equal(got, exp)
    else:
        assert np.array_equal(got, from_i8(exp).astype(dtype), equal_nan=True)


@pytest.mark.parametrize("name,n_iid", [("gen1", 190), ("gen4", 198)])
def test_decode_and_encode_writer_files(name, n_iid):
    """gen1/gen4.bed were written by the reference's Bed.write (util/generate.py:207-240) with
    N % 4 == 2: decode matches snp_gen's values and the encoder reproduces every byte."""
    exp = g("generate")[name + "_val_i8"]
    got = O.decode(body(name), n_iid, 20, dtype=np.int8)
    assert np.array_equal(got, exp)
    assert np.array_equal(O.encode(from_i8(exp)).reshape(-1), body(name))
    assert np.array_equal(O.encode(exp).reshape(-1), body(name))


def test_encode_reproduces_n300_file_and_a1_round_trip():
    v = g("n300")["val_i8"]
    assert np.array_equal(O.encode(from_i8(v)).reshape(-1), body("n300"))  # NaN -> 01
    for n in (1, 2, 3, 5, 297):
        x = from_i8(v[:n, :40])
        back = O.decode(O.encode(x, count_A1=True).reshape(-1), n, 40, count_A1=True)
        assert np.array_equal(back, x, equal_nan=True)
    with pytest.raises(ValueError):
        O.encode(np.array([[0.5]]))


def test_decode_count_a1():
    G = g("n300")
    got = O.decode(body("n300"), 300, 1015, count_A1=True, dtype=np.int8)
    assert np.array_equal(got, G["val_a1_i8"])
    a2 = from_i8(G["val_i8"])
    assert np.array_equal(from_i8(got), 2 - a2, equal_nan=True)  # test.py:226-232


def test_decode_gather_and_toydata10():
    t10 = O.decode(body("toydata"), 500, 10000, sid_index=np.arange(10))
    G = g("toydata")
    assert t10.shape == (500, 10)
    rows = np.arange(299, 0, -2)
    cols = np.arange(1014, 0, -2)
    full = from_i8(g("n300")["val_i8"])
    got = O.decode(body("n300"), 300, 1015, iid_index=rows, sid_index=cols, order="C")
    assert np.array_equal(got, full[np.ix_(rows, cols)], equal_nan=True)
    with pytest.raises(IndexError):
        O.decode(body("n300"), 300, 1015, iid_index=[300])
    assert G["K_rows"].shape == (64, 500)


@pytest.mark.parametrize("name", ["n300", "snpgen"])
@pytest.mark.parametrize("tag,dtype,tol", [("f64", np.float64, 1e-10), ("f32", np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_standardize_vs_reference_python(name, tag, dtype, tol, order):
    G = g(name)
    val = from_i8(G["val_i8"])
    for std, is_beta, a, b in (("unit", False, np.nan, np.nan), ("beta", True, 1, 25)):
        v = np.array(val, dtype=dtype, order=order)
        stats = O.standardize_native(v, is_beta, a, b)
        np.testing.assert_allclose(stats, G["%s_stats_%s" % (std, tag)], rtol=tol, atol=tol)
        np.testing.assert_allclose(v, G["%s_%s" % (std, tag)], rtol=tol, atol=tol)


def test_snp_stats_matches_standardize():
    st = O.snp_stats(body("n300"), 300, 1015)
    v = O.decode(body("n300"), 300, 1015)
    assert np.array_equal(st, O.standardize_native(v), equal_nan=True)


def test_fused_decode_standardize_equals_two_step():
    for dtype in (np.float64, np.float32):
        for is_beta in (False, True):
            v = O.decode(body("n300"), 300, 1015, dtype=dtype)
            st = O.standardize_native(v, is_beta, 1, 25)
            f, st2 = O.decode_standardize(body("n300"), 300, 1015, is_beta, 1, 25, dtype=dtype)
            assert np.array_equal(f, v) and np.array_equal(st, st2)


def test_doctest_digits_one_pass():
    """standardizer.py:17-42 doctests, reproduced by the one-pass native formula."""
    val = from_i8(g("n300")["val_i8"])
    v = val.copy(order="F")
    O.standardize_native(v)
    assert "%.6f" % v[0, 0] == "0.229416"
    tr = val[10:].copy(order="F")
    stats = O.standardize_native(tr)
    assert "%.6f" % tr[0, 0] == "0.233550"
    np.testing.assert_allclose(stats[0], [1.94827586, 0.22146953], atol=1e-8)
    te = val[:10].copy(order="F")
    O.standardize_native(te, use_stats=True, stats=stats)
    assert te[0, 0] == 0.23354968324845735  # bit-exact: pins the one-pass formula
    vb = val.copy(order="F")
    O.standardize_native(vb, True, 1, 25)
    assert "%.6f" % vb[0, 0] == "0.680802"  # beta.py:23


def test_trained_apply_vs_reference():
    G = g("n300")
    val = from_i8(G["val_i8"])
    for std, is_beta in (("unit", False), ("beta", True)):
        tr = val[10:].copy(order="F")
        st = O.standardize_native(tr, is_beta, 1, 25)
        np.testing.assert_allclose(st, G[std + "_train_stats"], rtol=1e-10)
        te = val[:10].copy(order="F")
        O.standardize_native(te, is_beta, 1, 25, use_stats=True, stats=st)
        np.testing.assert_allclose(te, G[std + "_test"], rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("tag,dtype,tol", [("f64", np.float64, 1e-10), ("f32", np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_edge_cases_vs_reference(tag, dtype, tol, order):
    """NaN, SNC and all-missing columns (kernelreader/test.py:56-111; NaNCNC test.py:1201-1358)."""
    G = g("edge")
    for std, is_beta, a, b in (("unit", False, np.nan, np.nan), ("beta", True, 2, 10)):
        key = "%s_%s_%s" % (std, tag, order)
        x0 = np.array(G["x0"], dtype=dtype, order=order)
        st = O.standardize_native(x0, is_beta, a, b)
        np.testing.assert_allclose(st, G[key + "_stats"], rtol=tol, atol=tol, equal_nan=True)
        np.testing.assert_allclose(x0, G[key + "_train"], rtol=tol, atol=tol)
        assert np.isinf(st[1, 1]) and np.all(x0[:, 1] == 0) and x0[0, 2] == 0
        assert np.all(np.isnan(st[5])) and np.all(x0[:, 5] == 0)
        x1 = np.array(G["x1"], dtype=dtype, order=order)
        O.standardize_native(x1, is_beta, a, b, use_stats=True, stats=st)
        np.testing.assert_allclose(x1, G[key + "_apply"], rtol=tol, atol=tol)


def test_beta_pdf_matches_scipy():
    from scipy.stats import beta

    for a, b in ((1, 25), (2, 10), (0.5, 0.5), (3.5, 1.2)):
        for x in (0.0, 1e-7, 0.001, 0.013, 0.25, 0.5):
            ref = beta.pdf(x, a, b)
            got = O.beta_pdf(x, a, b)
            if np.isinf(ref):
                assert np.isinf(got)
            else:
                np.testing.assert_allclose(got, ref, rtol=1e-12)


def test_grm_vs_reference_goldens():
    G = g("n300")
    K, stats = O.grm_from_bed(body("n300"), 300, 1015, block_size=100)
    np.testing.assert_allclose(K, G["K_unit"], rtol=1e-10, atol=1e-9)
    Kb, _ = O.grm_from_bed(body("n300"), 300, 1015, is_beta=True, a=1, b=25)
    np.testing.assert_allclose(Kb, G["K_beta"], rtol=1e-10, atol=1e-9)
    Kd, f = O.diag_k_to_n(K)
    np.testing.assert_allclose(f, G["diag_factor"], rtol=1e-12)
    np.testing.assert_allclose(Kd, G["K_unit_diag"], rtol=1e-10, atol=1e-12)
    D = g("dist_x")
    K, _ = O.grm_from_bed(body("dist_x"), 100, 100)
    np.testing.assert_allclose(K, D["K_unit"], rtol=1e-10, atol=1e-9)


def test_grm_toydata_fixture():
    T = g("toydata")
    K, _ = O.grm_from_bed(body("toydata"), 500, 10000, block_size=2500)
    assert "%.6f" % K[0, 0] == "9923.069928"  # standardizer.py:28 doctest
    np.testing.assert_allclose(K[:64], T["K_rows"], rtol=1e-10, atol=1e-8)
    np.testing.assert_allclose(np.diag(K), T["K_diag"], rtol=1e-12)
    np.testing.assert_allclose(K.sum(1), T["K_rowsum"], rtol=1e-9, atol=1e-6)


def test_subset_semantics():
    """sub_matrix doctest (util/__init__.py:296-304) and util/test.py:110-121."""
    np.random.seed(0)
    m = np.random.rand(12, 7)
    s = O.subset(m, [0, 2, 11], [6, 5, 4, 3, 2, 1, 0])
    assert s.shape == (3, 7) and m[2, 0] == s[1, 6]
    m3 = np.random.rand(5, 4, 3).astype(np.float32)
    s3 = O.subset(m3, [4, 0], [1, 3], dtype=np.float64)
    assert np.array_equal(s3, m3[np.ix_([4, 0], [1, 3])].astype(np.float64))
    mf = np.asfortranarray(m)
    assert O.subset(mf, [1], [2, 0]).flags["F_CONTIGUOUS"]


def test_synth_generator_properties():
    a = O.synth_bed(7, 1003, 0, 40, 0.01, pitch=256)
    b = O.synth_bed(7, 1003, 20, 20, 0.01, pitch=256)
    assert np.array_equal(a[20:], b)  # counter-based: columns regenerate independently
    val = O.decode(a.reshape(-1)[: 40 * 256].reshape(40, 256)[:, :251].reshape(-1), 1003, 40)
    miss = np.isnan(val).mean()
    assert 0.003 < miss < 0.02
    assert np.nanmax(val) <= 2 and np.nanmin(val) >= 0
    assert np.all(a[:, 251:] == 0)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 299, 300, 4099])
@pytest.mark.parametrize("count_A1", [False, True])
def test_snp_stats_matches_decode_then_standardize(n, count_A1):
    """oracle.snp_stats (code counts, whole bytes through a per-byte table) == the stats of decode +
    one-pass standardize, including the pad codes of a partial last byte and all-missing columns."""
    rng = np.random.default_rng(n)
    m = 23
    bpc = (n + 3) // 4
    body = rng.integers(0, 256, size=m * bpc, dtype=np.uint8)
    body[:bpc] = 0x55  # all missing (code 1)
    Z = O.decode(body, n, m, count_A1=count_A1, dtype=np.float64)
    st_dec = O.standardize_native(Z)
    st = O.snp_stats(body, n, m, count_A1=count_A1)
    np.testing.assert_array_equal(st, st_dec)
