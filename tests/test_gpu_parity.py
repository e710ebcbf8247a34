"""Parity of the HIP path (through the C ABI / mirrored API) with the oracle and the
reference goldens.  Bars: decode/indexing bit-exact; standardized values f32 within 1e-5
relative (f64 within 1e-10); GRM max|dK| / max diag(K_ref) <= 1e-5 (f32), 1e-10 (f64)."""
import ctypes
import os
import tempfile

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from oracle import oracle as O
from pysnptools_amd import _native as N
from pysnptools_amd.kernelreader import KernelData, SnpKernel
from pysnptools_amd.snpreader import Bed, SnpData
from pysnptools_amd.standardizer import Beta, BetaTrained, DiagKtoN, Identity, Unit, UnitTrained
from pysnptools_amd.util import sub_matrix

pytestmark = pytest.mark.gpu

SHAPES = {"n300": (300, 1015), "snpgen": (1000, 5), "dist_x": (100, 100), "toydata": (500, 10000)}


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def bed(name, count_A1=False):
    return Bed(os.path.join(DATA, name + ".bed"), count_A1=count_A1)


def body(name):
    return O.read_bed_bytes(os.path.join(DATA, name + ".bed"))


def from_i8(v):
    out = v.astype(np.float64)
    out[v == -127] = np.nan
    return out


def rel_close(got, exp, tol):
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    assert got.shape == exp.shape
    both_nan = np.isnan(got) & np.isnan(exp)
    with np.errstate(invalid="ignore"):
        d = np.abs(got - exp)
    bound = tol * np.maximum(np.abs(exp), 1e-30)
    bad = ~(both_nan | (got == exp) | (d <= bound) | ((exp == 0) & (d <= tol)))
    assert not bad.any(), "max rel err %g at %s" % ((d / np.maximum(np.abs(exp), 1e-30))[bad].max(), np.argwhere(bad)[:3])


def grm_close(K, Kref, tol):
    Kref = np.asarray(Kref, dtype=np.float64)
    scale = max(np.abs(np.diag(Kref)).max(), 1.0)
    err = np.abs(np.asarray(K, dtype=np.float64) - Kref).max() / scale
    assert err <= tol, "GRM max|dK|/max diag = %g > %g" % (err, tol)
    rel_close(np.diag(K), np.diag(Kref), tol)


def test_device_visible():
    assert N.device_count() >= 1


# ---------------------------------------------------------------------------------- decode
@pytest.mark.parametrize("name", ["n300", "snpgen", "dist_x", "toydata"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int8])
@pytest.mark.parametrize("order", ["F", "C"])
def test_decode_bit_exact(name, dtype, order):
    n, m = SHAPES[name]
    got = bed(name).read(order=order, dtype=dtype, _require_float32_64=False).val
    assert got.dtype == dtype and got.flags[order + "_CONTIGUOUS"] and got.shape == (n, m)
    exp = O.decode(body(name), n, m, order=order, dtype=dtype)
    if name != "toydata":
        assert np.array_equal(O.decode(body(name), n, m, dtype=np.int8), g(name)["val_i8"])
    assert np.array_equal(got, exp, equal_nan=True)


def test_decode_count_a1():
    got = bed("n300", count_A1=True).read(dtype=np.int8, _require_float32_64=False).val
    assert np.array_equal(got, g("n300")["val_a1_i8"])
    f = bed("n300", count_A1=True).read(dtype=np.float32).val
    assert np.array_equal(f, 2 - from_i8(g("n300")["val_i8"]).astype(np.float32), equal_nan=True)


@pytest.mark.parametrize("order", ["F", "C"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int8])
def test_decode_subsets(order, dtype):
    b = bed("n300")
    full = O.decode(body("n300"), 300, 1015, dtype=dtype)
    rng = np.random.default_rng(0)
    perm = rng.permutation(300)[:123]
    cases = [(slice(None, None, -2), slice(1014, 0, -2)), (perm, slice(3, 900, 7)), ([5], [7]),
             (np.arange(300) % 3 == 0, [-1, 0, 500]), (slice(10, 11), slice(None))]
    for ri, ci in cases:
        sub = b[ri, ci]
        got = sub.read(order=order, dtype=dtype, _require_float32_64=False).val
        rows = np.arange(300)[ri]
        cols = np.arange(1015)[ci]
        assert np.array_equal(got, full[np.ix_(np.atleast_1d(rows), np.atleast_1d(cols))], equal_nan=True)
    with pytest.raises(IndexError):
        b[[300], :].read()


@pytest.mark.parametrize("n_iid", [1, 2, 3, 5, 17, 297, 298, 299])
def test_decode_padding_round_trip(n_iid):
    """N % 4 != 0: the last byte's pad bits must be ignored (test.py:689-746)."""
    v = from_i8(g("n300")["val_i8"][:n_iid, :33])
    d = SnpData(iid=[["f", str(i)] for i in range(n_iid)], sid=["s%d" % j for j in range(33)], val=v)
    with tempfile.TemporaryDirectory() as tmp:
        b = Bed.write(os.path.join(tmp, "p.bed"), d, count_A1=False)
        for dtype in (np.float32, np.float64):
            for order in ("F", "C"):
                assert np.array_equal(b.read(order=order, dtype=dtype).val, v.astype(dtype), equal_nan=True)
        st = b.read(dtype=np.float64).standardize(Unit(), return_trained=True)[1].stats
        ref = v.copy(order="F")
        np.testing.assert_array_equal(st, O.standardize_native(ref))


# ---------------------------------------------------------------------------------- standardize
@pytest.mark.parametrize("name", ["n300", "snpgen"])
@pytest.mark.parametrize("tag,dtype,tol", [("f64", np.float64, 1e-10), ("f32", np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_standardize_vs_reference(name, tag, dtype, tol, order):
    G = g(name)
    for std, key in ((Unit(), "unit"), (Beta(1, 25), "beta")):
        d, tr = bed(name).read(order=order, dtype=dtype).standardize(std, return_trained=True)
        rel_close(d.val, G["%s_%s" % (key, tag)], tol)
        rel_close(tr.stats, G["%s_stats_%s" % (key, tag)], tol)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("order", ["F", "C"])
def test_unit_standardize_bit_exact_vs_oracle(dtype, order):
    v = O.decode(body("n300"), 300, 1015, dtype=dtype, order=order)
    st = O.standardize_native(v)
    d, tr = bed("n300").read(order=order, dtype=dtype).standardize(Unit(), return_trained=True)
    assert np.array_equal(d.val, v)
    assert np.array_equal(np.asarray(tr.stats), st)
    vb = O.decode(body("n300"), 300, 1015, dtype=dtype, order=order)
    O.standardize_native(vb, True, 1, 25)
    db = bed("n300").read(order=order, dtype=dtype).standardize(Beta(1, 25))
    rel_close(db.val, vb, 1e-12 if dtype == np.float64 else 1e-6)


def test_doctest_goldens():
    """standardizer.py:17-42, beta.py:23, snpkernel.py:41, kernelreader.py:293."""
    b = bed("n300")
    assert "%.6f" % b.read().standardize(Unit()).val[0, 0] == "0.229416"
    assert "%.6f" % b.read().standardize(Beta(1, 25)).val[0, 0] == "0.680802"
    train, tr = Unit().standardize(b[range(10, 300), :].read(), return_trained=True)
    assert "%.6f" % train.val[0, 0] == "0.233550"
    np.testing.assert_allclose(tr.stats[0], [1.94827586, 0.22146953], atol=1e-8)
    test = b[range(0, 10), :].read().standardize(tr)
    assert test.val[0, 0] == 0.23354968324845735
    k = bed("toydata").read_kernel(Unit())
    assert "%.6f" % k.val[0, 0] == "9923.069928"
    kd = SnpKernel(bed("toydata"), Unit()).read().standardize()
    assert "%.6f" % kd.val[0, 0] == "0.992307"


def test_trained_apply_vs_reference():
    G = g("n300")
    b = bed("n300")
    for std, key in ((Unit(), "unit"), (Beta(1, 25), "beta")):
        _, tr = b[10:, :].read().standardize(std, return_trained=True)
        rel_close(tr.stats, G[key + "_train_stats"], 1e-12)
        te = b[:10, :].read().standardize(tr)
        rel_close(te.val, G[key + "_test"], 1e-10)


@pytest.mark.parametrize("tag,dtype,tol", [("f64", np.float64, 1e-10), ("f32", np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_edge_cases(tag, dtype, tol, order):
    """NaN, SNC and all-missing columns; train then apply (kernelreader/test.py:56-111)."""
    G = g("edge")
    for std, key in ((Unit(), "unit"), (Beta(2, 10), "beta")):
        k = "%s_%s_%s" % (key, tag, order)
        x0 = SnpData(iid=[["a", str(i)] for i in range(3)], sid=[str(j) for j in range(20)],
                     val=np.array(G["x0"], dtype=dtype, order=order))
        x0, tr = x0.standardize(std, return_trained=True)
        rel_close(x0.val, G[k + "_train"], tol)
        rel_close(tr.stats, G[k + "_stats"], tol)
        assert np.isinf(tr.stats[1, 1]) and np.all(x0.val[:, 1] == 0) and x0.val[0, 2] == 0
        assert np.all(x0.val[:, 5] == 0)
        x1 = SnpData(iid=[["b", str(i)] for i in range(2)], sid=[str(j) for j in range(20)],
                     val=np.array(G["x1"], dtype=dtype, order=order))
        x1.standardize(tr)
        rel_close(x1.val, G[k + "_apply"], tol)


def test_fused_read_standardize_abi():
    """snpmi_bed_read_standardize_* == decode then standardize (oracle), bit-exact for Unit."""
    for dtype in (np.float32, np.float64):
        exp, st_exp = O.decode_standardize(body("n300"), 300, 1015, dtype=dtype)
        out = np.empty((300, 1015), dtype=dtype, order="F")
        st = np.empty((1015, 2), dtype=dtype)
        N.call("snpmi_bed_read_standardize_" + N.suffix(dtype), os.path.join(DATA, "n300.bed").encode(), 300, 1015, 0,
               None, 0, None, 0, 0, N.STD_UNIT, 0.0, 0.0, 0, N.ptr(st), N.ptr(out), 0)
        assert np.array_equal(out, exp) and np.array_equal(st, st_exp)


# ---------------------------------------------------------------------------------- subset
def test_sub_matrix():
    np.random.seed(0)
    m = np.random.rand(12, 7)
    s = sub_matrix(m, [0, 2, 11], [6, 5, 4, 3, 2, 1, 0])
    assert s.shape == (3, 7) and m[2, 0] == s[1, 6]
    for order in ("C", "F", "A"):
        for src in (m, np.asfortranarray(m), m.astype(np.float32)):
            for dt in (np.float32, np.float64):
                if src.dtype == np.float64 and dt == np.float32:
                    continue
                got = sub_matrix(src, [3, 1], [0, 6, 2], order=order, dtype=dt)
                assert np.array_equal(got, src[np.ix_([3, 1], [0, 6, 2])].astype(dt))
    m3 = np.random.rand(5, 4, 3)
    assert np.array_equal(sub_matrix(m3, [4, 0], [1, 3]), m3[np.ix_([4, 0], [1, 3])])


# ---------------------------------------------------------------------------------- GRM
@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-5)])
@pytest.mark.parametrize("block_size", [None, 100])
def test_grm_n300_vs_reference(dtype, tol, block_size, syrk_variant):
    G = g("n300")
    b = bed("n300")
    k = b.read_kernel(Unit(), block_size=block_size, dtype=dtype)
    assert k.val.dtype == dtype
    grm_close(k.val, G["K_unit"], tol)
    kb = b.read_kernel(Beta(1, 25), block_size=block_size, dtype=dtype)
    grm_close(kb.val, G["K_beta"], tol)
    kd, _, diag = SnpKernel(b, Unit(), block_size=block_size)._read_with_standardizing(to_kerneldata=True,
                                                                                       return_trained=True)
    np.testing.assert_allclose(diag.factor, G["diag_factor"], rtol=1e-12)
    grm_close(kd.val, G["K_unit_diag"], 1e-10)


def test_grm_symmetry_and_orders():
    b = bed("n300")
    for order in ("C", "F", "A"):
        for dtype in (np.float32, np.float64):
            v = b.read_kernel(Unit(), order=order, dtype=dtype).val
            assert v.dtype == dtype and np.array_equal(v, v.T)
            if order != "A":
                assert v.flags[order + "_CONTIGUOUS"]


def test_grm_dist_x_and_toydata(syrk_variant):
    D = g("dist_x")
    grm_close(bed("dist_x").read_kernel(Unit()).val, D["K_unit"], 1e-10)
    grm_close(bed("dist_x").read_kernel(Beta(1, 25), block_size=7).val, D["K_beta"], 1e-10)
    T = g("toydata")
    for dtype, tol in ((np.float64, 1e-10), (np.float32, 1e-5)):
        K = bed("toydata").read_kernel(Unit(), block_size=1000, dtype=dtype).val.astype(np.float64)
        scale = np.abs(T["K_diag"]).max()
        assert np.abs(K[:64] - T["K_rows"]).max() / scale <= tol
        rel_close(np.diag(K), T["K_diag"], tol)
        assert np.abs(K.sum(1) - T["K_rowsum"]).max() / (scale * 500) <= tol


def test_grm_identity_raw_values():
    """Identity standardizer on raw decoded values (NaN propagates as in NumPy dot)."""
    b = bed("n300")[:, :200]
    raw = O.decode(body("n300"), 300, 1015, sid_index=np.arange(200))
    K = b.read_kernel(Identity()).val
    ref = raw.dot(raw.T)
    grm_close(K, ref, 1e-12)


def test_grm_subsets_and_pushdown(syrk_variant):
    b = bed("toydata")
    whole = b.read_kernel(Unit()).val
    sub = SnpKernel(b, Unit())[::2, ::2].read().val   # kernelreader/test.py:235-247
    np.testing.assert_allclose(sub, whole[::2, ::2], rtol=1e-10, atol=1e-9)
    sub2 = SnpKernel(b, Unit())[::2].read().val
    np.testing.assert_allclose(sub2, whole[::2, ::2], rtol=1e-10, atol=1e-9)
    # iid subset read through the fused path (repack kernel) == oracle on the subset
    rows = np.arange(499, 0, -3)
    Ks = b[rows, 100:2100].read_kernel(Unit()).val
    # oracle over the SNP range 100:2100 only
    Z = O.decode(body("toydata"), 500, 10000, iid_index=rows, sid_index=np.arange(100, 2100))
    O.standardize_native(Z)
    grm_close(Ks, Z.dot(Z.T), 1e-10)
    # constant standardizer: the iid subset is pushed down
    _, tr = b.read().standardize(Unit(), return_trained=True)
    k3 = SnpKernel(b, tr)[[5, 1, 9]].read().val
    Z = O.decode(body("toydata"), 500, 10000, iid_index=[5, 1, 9])
    O.standardize_native(Z, use_stats=True, stats=np.asarray(tr.stats))
    grm_close(k3, Z.dot(Z.T), 1e-10)


def test_grm_dense_snpdata_vs_reference():
    G = g("edge")
    xr = G["xr"]
    for dtype, tol in ((np.float64, 1e-10), (np.float32, 1e-5)):
        for order in ("F", "C"):
            d = SnpData(iid=[["a", str(i)] for i in range(7)], sid=[str(j) for j in range(20)],
                        val=np.array(xr, dtype=dtype, order=order))
            for std, key in ((Unit(), "unit"), (Beta(1, 25), "beta")):
                k = d.read_kernel(std, block_size=1, dtype=dtype)
                grm_close(k.val, G["K_%s_xr" % key], tol)
            assert np.array_equal(d.val, np.array(xr, dtype=dtype), equal_nan=True)  # input untouched


def test_merge_std_block_size_invariance():
    """kernelreader/test.py:44-54: block_size=1 == block_size=None."""
    np.random.seed(0)
    val = np.array(np.random.randint(3, size=[3, 20]), dtype=np.float64, order="F")
    sd = SnpData(iid=[["0", "0"], ["1", "1"], ["2", "2"]], sid=[str(i) for i in range(20)], val=val)
    for std in (Beta(2, 10), Unit()):
        k0, t0, d0 = SnpKernel(sd, std, block_size=1)._read_with_standardizing(to_kerneldata=True, return_trained=True)
        k1, t1, d1 = SnpKernel(sd, std, block_size=None)._read_with_standardizing(to_kerneldata=True, return_trained=True)
        np.testing.assert_array_almost_equal(k0.val, k1.val, decimal=10)
        np.testing.assert_array_almost_equal(t0.stats, t1.stats, decimal=10)
        assert abs(d0.factor - d1.factor) < 1e-7


def test_kerneldata_diag_k_to_n():
    kd = KernelData(iid=[["0", "0"], ["1", "1"], ["2", "2"]], val=[[1, 2, 3], [4, 5, 6], [7, 8, 9]])
    kd = kd.standardize()
    assert abs(np.diag(kd.val).sum() - 3) < 1e-7  # kernelreader/test.py:221-229


@pytest.fixture(params=[0, 36, 20, 5], ids=["auto", "bf3", "f32mfma", "small128"])
def syrk_variant(request):
    """Run a test under each SYRK kernel the product library ships -- f32: 0 = the default chain
    (packed: the fp16x2-split kernel, 3 products on the fp16 MFMA pipe, with the bf16x3 kernel
    as its device-side range fallback; dense operand N >= 4096: fp16x2 LDS-DMA stage images,
    the f32-MFMA k_syrk256d as fallback), 36 = the bf16x3 kernel alone, 20 = the f32-MFMA
    kernels (two-phase decode to Z + glds SYRK at N >= 4096, the 128x128 kernel below), 5 =
    the 128x128 small-N kernels; f64: every variant runs the f64 kernels (0 / 20 / 36: the
    default fused / glds kernels).  The ablation variants of rounds 1-5 were deleted in round 6."""
    N.call("snpmi_set_kernel_variant", b"syrk", request.param)
    yield request.param
    N.call("snpmi_set_kernel_variant", b"syrk", 0)


def test_product_library_refuses_ablation_variants():
    for v in (4, 30, 41, 44, 49):
        with pytest.raises(ValueError):
            N.call("snpmi_set_kernel_variant", b"syrk", v)
    N.call("snpmi_set_kernel_variant", b"syrk", 0)


@pytest.mark.parametrize("n", [1, 127, 128, 129, 255, 256, 257, 383, 600, 4096, 4097, 4353])
def test_grm_tile_edges(n, syrk_variant):
    """Odd tile coverage: N not a multiple of the 128/256-iid tiles, 1 SNP .. several chunks.
    N >= 4096 under variant 0 runs the two-phase path (decode to Z + glds SYRK) over two Z
    sub-blocks (32 + 5 SNPs: a zero-filled tail stage)."""
    rng = np.random.default_rng(n)
    val = rng.integers(0, 3, size=(n, 37)).astype(np.float64)
    val[rng.random(val.shape) < 0.05] = np.nan
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(37)], val=val)
    for dtype, tol in ((np.float64, 1e-10), (np.float32, 1e-5)):
        Z = val.astype(dtype).copy(order="F")
        O.standardize_native(Z)
        ref = Z.astype(np.float64).dot(Z.astype(np.float64).T)
        grm_close(d.read_kernel(Unit(), dtype=dtype).val, ref, tol)
        with tempfile.TemporaryDirectory() as tmp:
            b = Bed.write(os.path.join(tmp, "t.bed"), d, count_A1=False)
            grm_close(b.read_kernel(Unit(), dtype=dtype).val, ref, tol)


@pytest.mark.parametrize("m", [1, 15, 16, 17, 31, 32, 33, 48, 49])
def test_grm_stage_counts(m, syrk_variant):
    """SNP counts around the 16-SNP LDS stage of the SYRK kernels: one stage, an exact multiple,
    and odd/even stage counts (the bf16x3 kernel runs its stages in pairs, so an odd count ends
    on a single stage); N = 513 gives diagonal, off-diagonal and 1-iid edge blocks."""
    n = 513
    rng = np.random.default_rng(m)
    val = rng.integers(0, 3, size=(n, m)).astype(np.float64)
    val[rng.random(val.shape) < 0.05] = np.nan
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(m)], val=val)
    with tempfile.TemporaryDirectory() as tmp:
        b = Bed.write(os.path.join(tmp, "t.bed"), d, count_A1=False)
        for dtype, tol in ((np.float64, 1e-10), (np.float32, 1e-5)):
            Z = val.astype(dtype).copy(order="F")
            O.standardize_native(Z)
            ref = Z.astype(np.float64).dot(Z.astype(np.float64).T)
            grm_close(b.read_kernel(Unit(), dtype=dtype).val, ref, tol)


@pytest.mark.parametrize("case", ["unit", "beta11", "beta125_common", "beta125_mixed", "one_carrier"])
def test_grm_h2_range_fallback(case, syrk_variant):
    """The fp16x2 SYRK holds f32 accuracy only while each SNP's largest |LUT value| is in
    [2^-2, 2^15): Unit and Beta(1,1) blocks stay on it (one_carrier: M_s ~ sqrt(n)); Beta(1,25)
    over common SNPs (weights ~1e-6, fp16 subnormals) and a block mixing rare and common SNPs
    must take the bf16x3 fallback -- all checked against the f64 oracle at 1e-5 of the largest
    diagonal, which the fp16 kernel alone misses by orders of magnitude on the common-SNP block."""
    rng = np.random.default_rng(7)
    n, m = 700, 53
    p = rng.uniform(0.3, 0.5, size=m) if case == "beta125_common" else rng.uniform(0.002, 0.5, size=m)
    val = (rng.random((n, m)) < p).astype(np.float64) + (rng.random((n, m)) < p)
    if case == "one_carrier":
        val[:] = 0
        val[rng.integers(0, n, size=m), np.arange(m)] = 1
    val[rng.random(val.shape) < 0.03] = np.nan
    is_beta, a, b = {"beta11": (True, 1, 1), "beta125_common": (True, 1, 25),
                     "beta125_mixed": (True, 1, 25)}.get(case, (False, np.nan, np.nan))
    std = Beta(a, b) if is_beta else Unit()
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(m)], val=val)
    Z = val.copy(order="F")
    O.standardize_native(Z, is_beta, a, b)
    ref = Z.dot(Z.T)
    with tempfile.TemporaryDirectory() as tmp:
        bd = Bed.write(os.path.join(tmp, "t.bed"), d, count_A1=False)
        K = bd.read_kernel(std, dtype=np.float32).val
        grm_close(K, ref, 1e-5)
        grm_close(bd.read_kernel(std, dtype=np.float32, block_size=16).val, ref, 1e-5)
    # f32-level accuracy, not just the 1e-5 bar: ~2^-21 of the largest diagonal for the split
    # kernels (fp16 subnormal residuals included), f32 MFMA rounding for the others
    err = np.abs(K.astype(np.float64) - ref).max() / np.abs(np.diag(ref)).max()
    assert err <= 2e-6, "GRM max|dK|/max diag = %g" % err


@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e5, "mixed"])
def test_grm_dense_h2_range(scale, syrk_variant):
    """SnpData.read_kernel (dense f32 operand, N >= 4096): the fp16x2 split of the block in HBM
    (k_split_h2 + k_syrk_h2<DENSE>) for columns whose max |z| lies in [2^-2, 2^15), the f32-MFMA
    kernel on the device-side flag otherwise (scale 1e-3 / 1e5 / one tiny column) -- vs the f64
    product of the same f32 values, Identity standardizer (values used as given)."""
    rng = np.random.default_rng(11)
    n, m = 4200, 45
    v = rng.standard_normal((n, m)).astype(np.float32)
    if scale == "mixed":
        v[:, 7] *= 1e-4
    else:
        v *= np.float32(scale)
    v[rng.random(v.shape) < 0.01] = 0
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(m)], val=v)
    ref = v.astype(np.float64).dot(v.astype(np.float64).T)
    K = d.read_kernel(Identity(), dtype=np.float32).val
    grm_close(K, ref, 1e-5)
    err = np.abs(K.astype(np.float64) - ref).max() / np.abs(np.diag(ref)).max()
    assert err <= 2e-6, "GRM max|dK|/max diag = %g" % err
    Zs = v.astype(np.float64).copy(order="F")
    O.standardize_native(Zs)
    grm_close(d.read_kernel(Unit(), dtype=np.float32).val, Zs.dot(Zs.T), 1e-5)


@pytest.mark.parametrize("m_per_block,chunk", [(45, 0), (70, 0), (70, 32)])
def test_grm_dense_session_blocks_mixed_range(m_per_block, chunk):
    """The generic block loop at N >= 4096 in f32 (snpmi_grm_add_dense: SnpReader._read_kernel's
    K += Z_b Z_b^T, snpreader.py:651-655, K kept on the device): several blocks accumulate into
    one session, one of them scaled out of fp16 range so that block alone takes the f32-MFMA
    fallback while its neighbours stay on the fp16x2 stage-image kernel; m not a multiple of 32
    and more than two 32-SNP stages per block -- vs the f64 product of the same values."""
    rng = np.random.default_rng(m_per_block)
    n, nblk = 4200, 4
    blocks = [rng.standard_normal((n, m_per_block)).astype(np.float32) for _ in range(nblk)]
    blocks[2] *= np.float32(1e-4)  # outside [2^-2, 2^15): this block runs on k_syrk256d
    ref = np.zeros((n, n))
    N.call("snpmi_set_kernel_variant", b"dense_chunk", chunk)  # 32: stage images in 32-SNP chunks
    try:
        N.call("snpmi_grm_begin", n, N.DT_F32)
        for k, blk in enumerate(blocks):
            order_c = k % 2
            arr = np.ascontiguousarray(blk) if order_c else np.asfortranarray(blk)
            N.call("snpmi_grm_add_dense_f32", N.ptr(arr), n, m_per_block, order_c)
            b64 = blk.astype(np.float64)
            ref += b64.dot(b64.T)
        K = np.empty((n, n), dtype=np.float32)
        factor = ctypes.c_double()
        N.call("snpmi_grm_end", 0, ctypes.byref(factor), N.ptr(K))
    finally:
        N.call("snpmi_set_kernel_variant", b"dense_chunk", 0)
    grm_close(K, ref, 1e-5)
    err = np.abs(K.astype(np.float64) - ref).max() / np.abs(np.diag(ref)).max()
    assert err <= 2e-6, "GRM max|dK|/max diag = %g" % err


@pytest.mark.parametrize("n", [300, 4200])
@pytest.mark.parametrize("codes", [1, 0])
def test_grm_dense_genotype_columns_reencoded(n, codes):
    """A dense f32 operand whose columns take <= 4 distinct values (a standardized SnpData) is
    re-encoded exactly as 2-bit codes + per-SNP LUT and runs on the packed fp16x2 SYRK (codes=1);
    codes=0 forces the dense kernels.  Columns include -0.0 / +0.0 (distinct bit patterns), a
    NaN-free imputed column, a constant column and a 4-valued column -- vs the f64 product of the
    same f32 values."""
    rng = np.random.default_rng(n)
    m = 70
    g = (rng.random((n, m)) < 0.3).astype(np.float64) + (rng.random((n, m)) < 0.3)
    g[rng.random(g.shape) < 0.02] = np.nan
    Z = g.copy(order="F")
    O.standardize_native(Z)
    v = Z.astype(np.float32)
    v[:, 3] = 0.0
    v[::2, 3] = -0.0
    v[:, 5] = 2.5
    v[:, 7] = np.array([1.5, -2.0, 0.25, 7.0], dtype=np.float32)[rng.integers(0, 4, n)]
    ref = v.astype(np.float64).dot(v.astype(np.float64).T)
    N.call("snpmi_set_kernel_variant", b"dense_codes", codes)
    try:
        K = np.empty((n, n), dtype=np.float32)
        st = np.empty((m, 2), dtype=np.float32)
        vf = np.asfortranarray(v)
        N.call("snpmi_grm_dense_f32", N.ptr(vf), n, m, 0, N.STD_NONE, 0.0, 0.0, 0, N.ptr(st), 0, None, N.ptr(K))
    finally:
        N.call("snpmi_set_kernel_variant", b"dense_codes", 1)
    grm_close(K, ref, 1e-5)
    err = np.abs(K.astype(np.float64) - ref).max() / np.abs(np.diag(ref)).max()
    assert err <= 2e-6, "GRM max|dK|/max diag = %g" % err


# ---------------------------------------------------------------------------------- device API
class Dev:
    """Tiny RAII helper over snpmi_dev_alloc/free."""

    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        N.call("snpmi_dev_alloc", ctypes.byref(self.p), int(nbytes))
        self.nbytes = nbytes

    def __del__(self):
        try:
            N.call("snpmi_dev_free", self.p)
        except Exception:
            pass

    def get(self, arr):
        N.call("snpmi_memcpy_d2h", N.ptr(arr), self.p, arr.nbytes)
        return arr

    def put(self, arr):
        N.call("snpmi_memcpy_h2d", self.p, N.ptr(np.ascontiguousarray(arr)), arr.nbytes)


def synth_dev(n, m, seed, miss=0.01, sid0=0):
    pitch = N.lib().snpmi_packed_pitch(n)
    buf = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", buf.p, pitch, n, sid0, m, seed, miss, N.ptr(x), N.ptr(cdf), len(x))
    return buf, pitch


def test_device_synth_matches_oracle():
    for n in (1003, 4096):
        buf, pitch = synth_dev(n, 50, 11, sid0=7)
        got = buf.get(np.empty((50, pitch), dtype=np.uint8))
        exp = O.synth_bed(11, n, 7, 50, 0.01, pitch=pitch)
        assert np.array_equal(got, exp)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_device_decode_standardize_large_properties(dtype):
    """10k x 2k synthetic: sampled columns bit-exact vs oracle; every column mean~0 / var~1."""
    n, m = 10000, 2000
    buf, pitch = synth_dev(n, m, 2)
    host = buf.get(np.empty((m, pitch), dtype=np.uint8))
    sz = np.dtype(dtype).itemsize
    ld = (n + 15) // 16 * 16
    lut, st, out = Dev(m * 4 * sz), Dev(m * 2 * sz), Dev(m * ld * sz)
    dt = N.dt_code(dtype)
    N.call("snpmi_dev_snp_stats", buf.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
    N.call("snpmi_dev_decode", buf.p, pitch, n, m, lut.p, dt, 0, out.p, ld)
    vals = out.get(np.empty((m, ld), dtype=dtype))[:, :n]
    stats = st.get(np.empty((m, 2), dtype=dtype))
    cols = np.random.default_rng(0).choice(m, 64, replace=False)
    packed = host[:, : (n + 3) // 4].reshape(-1)
    exp, est = O.decode_standardize(packed, n, m, sid_index=cols, dtype=dtype)
    assert np.array_equal(vals[cols].T, exp) and np.array_equal(stats[cols], est)
    v64 = vals.astype(np.float64)
    poly = np.isfinite(stats[:, 1])
    assert np.abs(v64.sum(1)[poly]).max() < 1e-2 * n ** 0.5
    assert np.all(v64[~poly] == 0)


@pytest.mark.parametrize("n,world", [(300, 1), (700, 3), (1100, 4), (4100, 2), (4500, 3)])
def test_grm_partitioned_blocks_assemble_k(n, world, syrk_variant):
    """cfg5 mode: every rank's 256x256 blocks (simulated ranks on one GPU) assemble to K."""
    rng = np.random.default_rng(n)
    val = rng.integers(0, 3, size=(n, 45)).astype(np.float64)
    val[rng.random(val.shape) < 0.03] = np.nan
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(45)], val=val)
    Z = val.astype(np.float32).copy(order="F")
    O.standardize_native(Z)
    ref = Z.astype(np.float64).dot(Z.astype(np.float64).T)
    with tempfile.TemporaryDirectory() as tmp:
        Bed.write(os.path.join(tmp, "p.bed"), d, count_A1=False)
        body = O.read_bed_bytes(os.path.join(tmp, "p.bed"))
    pitch = N.lib().snpmi_packed_pitch(n)
    host = np.zeros((45, pitch), dtype=np.uint8)
    bpc = (n + 3) // 4
    host[:, :bpc] = body.reshape(45, bpc)
    packed = Dev(host.nbytes)
    packed.put(host)
    lut, st = Dev(45 * 16), Dev(45 * 8)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, 45, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
    K = np.full((((n + 255) // 256) * 256,) * 2, np.nan)
    r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
    for r in range(world):
        nloc = N.lib().snpmi_grm_part_blocks(n, r, world)
        blocks = Dev(max(nloc, 1) * 256 * 256 * 4)
        N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, 45, lut.p, r, world, blocks.p, 0)
        out = blocks.get(np.empty((max(nloc, 1), 256, 256), dtype=np.float32))
        for b in range(nloc):
            N.call("snpmi_grm_part_coords", n, r, world, b, ctypes.byref(r0), ctypes.byref(c0))
            i, j = r0.value, c0.value
            K[i:i + 256, j:j + 256] = out[b]
            K[j:j + 256, i:i + 256] = out[b].T
    grm_close(K[:n, :n], ref, 1e-5)


# ---------------------------------------------------------------------------------- BED writer (§8f f2)
def _write_bytes(val, count_A1=False):
    from pysnptools_amd.snpreader._write import write_bed_body

    with tempfile.TemporaryDirectory() as tmp:
        p = os.path.join(tmp, "w.bed")
        write_bed_body(p, val, count_A1)
        return O.read_bed_bytes(p)


@pytest.mark.parametrize("name,n_iid", [("gen1", 190), ("gen4", 198), ("n300", 300)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int8])
@pytest.mark.parametrize("order", ["F", "C"])
def test_bed_write_reproduces_reference_files(name, n_iid, dtype, order):
    """The HIP encoder rewrites files the reference itself wrote, byte for byte (pad bits incl.)."""
    v8 = g("generate")[name + "_val_i8"] if name != "n300" else g("n300")["val_i8"]
    val = v8 if dtype == np.int8 else from_i8(v8).astype(dtype)
    val = np.array(val, order=order)
    assert np.array_equal(_write_bytes(val), body(name))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 255, 256, 257, 1023, 1024, 1025, 1030, 4099])
@pytest.mark.parametrize("m", [1, 63, 65, 130])
def test_bed_write_shapes_vs_oracle(n, m):
    rng = np.random.default_rng(n * 1000 + m)
    v = rng.integers(0, 3, size=(n, m)).astype(np.float64)
    v[rng.random((n, m)) < 0.05] = np.nan
    for count_A1 in (False, True):
        exp = O.encode(v, count_A1).reshape(-1)
        for dtype in (np.float32, np.float64):
            for order in ("F", "C"):
                got = _write_bytes(np.array(v, dtype=dtype, order=order), count_A1)
                assert np.array_equal(got, exp), (dtype, order, count_A1)


@pytest.mark.parametrize("bad", [0.5, -1.0, 3.0, np.inf])
def test_bed_write_rejects_bad_values(bad):
    v = np.zeros((10, 4))
    v[7, 2] = bad
    with tempfile.TemporaryDirectory() as tmp:
        p = os.path.join(tmp, "bad.bed")
        from pysnptools_amd.snpreader._write import write_bed_body

        with pytest.raises(ValueError):
            write_bed_body(p, v, False)
        assert not os.path.exists(p)
        v8 = np.zeros((10, 4), dtype=np.int8)
        v8[3, 1] = 5
        with pytest.raises(ValueError):
            write_bed_body(p, v8, False)
        assert not os.path.exists(p)


def test_bed_write_snpdata_round_trip_and_metadata():
    """Bed.write (bed.py:229-316): .bed by the HIP encoder, .fam/.bim text, read back exactly."""
    b = bed("n300")
    d = b[:, ::3].read()
    with tempfile.TemporaryDirectory() as tmp:
        for a1 in (False, True):
            w = Bed.write(os.path.join(tmp, "rt.bed"), d, count_A1=a1)
            back = w.read()
            assert np.array_equal(back.val, d.val, equal_nan=True)
            assert np.array_equal(back.iid, d.iid) and np.array_equal(back.sid, d.sid)
            np.testing.assert_array_equal(back.pos, d.pos)


@pytest.mark.parametrize("order_c", [0, 1])
def test_dev_encode_large(order_c):
    """Grid-stride paths of k_encode_f/c at a size with many waves per CU."""
    n, m = 20011, 700
    pitch = N.lib().snpmi_packed_pitch(n)
    rng = np.random.default_rng(7 + order_c)
    v = rng.integers(0, 3, size=(n, m)).astype(np.float32)
    v[rng.random((n, m)) < 0.01] = np.nan
    if order_c:
        host, ld = np.ascontiguousarray(v), m
    else:
        ld = (n + 15) // 16 * 16
        host = np.zeros((m, ld), dtype=np.float32)
        host[:, :n] = v.T
    dv, dp = ctypes.c_void_p(), ctypes.c_void_p()
    N.call("snpmi_dev_alloc", ctypes.byref(dv), host.nbytes)
    N.call("snpmi_dev_alloc", ctypes.byref(dp), pitch * m)
    try:
        N.call("snpmi_memcpy_h2d", dv, N.ptr(host), host.nbytes)
        bad = ctypes.c_uint64(99)
        N.call("snpmi_dev_encode", dv, N.DT_F32, order_c, ld, n, m, 0, dp, pitch, ctypes.byref(bad))
        out = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(out), dp, out.nbytes)
    finally:
        N.call("snpmi_dev_free", dv)
        N.call("snpmi_dev_free", dp)
    assert bad.value == 0
    bpc = (n + 3) // 4
    assert np.array_equal(out[:, :bpc], O.encode(v))


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1023, 1025, 5000, 700_000])
@pytest.mark.parametrize("kind,use_stats,count_a1", [(N.STD_UNIT, 0, 0), (N.STD_BETA, 0, 1), (N.STD_NONE, 0, 0),
                                                     (N.STD_UNIT, 1, 0)])
def test_fused_decode_standardize_equals_two_kernels(n, kind, use_stats, count_a1):
    """snpmi_dev_decode_standardize (LDS-resident column; > 150 KiB columns fall back to the
    re-reading kernel, as does decode variant 1) == k_snp_stats + k_decode_f, bit for bit."""
    m = 3 if n > 100_000 else 37
    buf, pitch = synth_dev(n, m, 5 + n)
    ld = (n + 15) // 16 * 16
    a, b = (1.0, 25.0) if kind == N.STD_BETA else (0.0, 0.0)
    outs = []
    for fused, variant in ((False, 0), (True, 0), (True, 1)):
        N.call("snpmi_set_kernel_variant", b"decode", variant)
        lut, st, out = Dev(m * 16), Dev(m * 8), Dev(m * ld * 4)
        if use_stats:
            stats_in = np.tile(np.array([[0.9, 0.7]], dtype=np.float32), (m, 1))
            st.put(stats_in)
        if fused:
            N.call("snpmi_dev_decode_standardize", buf.p, pitch, n, m, count_a1, kind, a, b, use_stats, N.DT_F32,
                   st.p, lut.p, out.p, ld)
        else:
            N.call("snpmi_dev_snp_stats", buf.p, pitch, n, m, count_a1, kind, a, b, use_stats, N.DT_F32, st.p, lut.p)
            N.call("snpmi_dev_decode", buf.p, pitch, n, m, lut.p, N.DT_F32, 0, out.p, ld)
        outs.append((out.get(np.empty((m, ld), dtype=np.float32))[:, :n], lut.get(np.empty((m, 4), dtype=np.float32)),
                     st.get(np.empty((m, 2), dtype=np.float32))))
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    for o in outs[1:]:
        for q, (x, y) in enumerate(zip(outs[0], o)):
            if q == 2 and kind == N.STD_NONE:
                continue  # Identity writes no stats
            assert np.array_equal(x, y, equal_nan=True)
    if kind == N.STD_UNIT and not use_stats and n <= 5000:
        host = buf.get(np.empty((m, pitch), dtype=np.uint8))
        exp, est = O.decode_standardize(np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1), n, m,
                                        count_A1=bool(count_a1), dtype=np.float32)
        assert np.array_equal(outs[1][0].T, exp) and np.array_equal(outs[1][2], est)


@pytest.mark.parametrize("n,m", [(20_011, 40), (100_003, 2050), (250_001, 1501), (500_000, 1100), (700_003, 3)])
@pytest.mark.parametrize("kind", ["random", "reversed_stride2", "sorted", "stride7", "stride3_tail"])
def test_dev_repack_random_gather(n, m, kind):
    """snpmi_dev_repack: columns staged in LDS in groups of K = 4 / 2 / 1 (by column size; more
    groups than workgroups, so the register prefetch of the next group runs), > 150 KiB columns
    on the global-gather fallback -- repacked codes decode to the source codes at the gathered
    iids, and every pad bit and pad byte of the destination pitch is zero."""
    buf, pitch = synth_dev(n, m, 17)
    rng = np.random.default_rng(n)
    if kind == "random":
        idx = rng.choice(n, size=n // 3, replace=True).astype(np.uint64)
    elif kind == "reversed_stride2":
        idx = np.arange(n - 1, -1, -2, dtype=np.uint64)
    elif kind == "stride7":  # windows of 2 columns per workgroup (K = 2)
        idx = np.arange(3, n, 7, dtype=np.uint64)
    elif kind == "stride3_tail":  # last 8192-code chunk holds one code
        idx = np.arange(0, n, 3, dtype=np.uint64)
        idx = idx[:max(len(idx) // 8192, 1) * 8192 + 1]
    else:
        idx = np.sort(rng.choice(n, size=n // 2 + 7, replace=False)).astype(np.uint64)
    n_out = len(idx)
    pitch_out = N.lib().snpmi_packed_pitch(n_out)
    didx, dst = Dev(n_out * 8), Dev(pitch_out * m)
    N.call("snpmi_dev_memset", dst.p, 0xA5, pitch_out * m)  # the kernel must write the pad itself
    didx.put(idx)
    N.call("snpmi_dev_repack", buf.p, pitch, n, didx.p, n_out, m, dst.p, pitch_out)
    src = buf.get(np.empty((m, pitch), dtype=np.uint8))
    got = dst.get(np.empty((m, pitch_out), dtype=np.uint8))
    full = O.decode(np.ascontiguousarray(src[:, :(n + 3) // 4]).reshape(-1), n, m, dtype=np.int8)
    sub = O.decode(np.ascontiguousarray(got[:, :(n_out + 3) // 4]).reshape(-1), n_out, m, dtype=np.int8)
    assert np.array_equal(sub, full[idx.astype(np.int64)])
    if n_out % 4:
        assert np.all((got[:, n_out // 4] >> (2 * (n_out % 4))) == 0)
    assert np.all(got[:, (n_out + 3) // 4:] == 0)
    # the dword-per-lane windowed kernel (decode variant 17) writes the same bytes
    N.call("snpmi_set_kernel_variant", b"decode", 17)
    try:
        N.call("snpmi_dev_memset", dst.p, 0x5A, pitch_out * m)
        N.call("snpmi_dev_repack", buf.p, pitch, n, didx.p, n_out, m, dst.p, pitch_out)
    finally:
        N.call("snpmi_set_kernel_variant", b"decode", 0)
    assert np.array_equal(dst.get(np.empty((m, pitch_out), dtype=np.uint8)), got)


def test_diag_k_to_n_snp_side_and_trained():
    """test.py:204-218: DiagKtoN on SNP data gives trace(Z Z^T) = N; the trained factor
    re-applies it; kernel side on a non-contiguous view is staged through a copy."""
    from pysnptools_amd.standardizer import DiagKtoN, DiagKtoNTrained

    np.random.seed(42)
    m = np.random.random((100, 1000))
    ref_factor = 100.0 / m.reshape(-1).dot(m.reshape(-1))
    with pytest.warns(DeprecationWarning):
        _, tr = DiagKtoN()._standardize_snps(m, return_trained=True)
    np.testing.assert_almost_equal(100, np.sum(np.diag(m.dot(m.T))))
    assert abs(tr.factor - ref_factor) < 1e-12 * ref_factor
    for dtype in (np.float32, np.float64):
        d = SnpData(iid=[["a", str(i)] for i in range(100)], sid=["s%d" % j for j in range(1000)],
                    val=np.random.random((100, 1000)).astype(dtype))
        v0 = d.val.copy()
        d.standardize(DiagKtoN())
        assert abs(np.trace(d.val.astype(np.float64).dot(d.val.T.astype(np.float64))) - 100) < 1e-3
        again = SnpData(iid=d.iid, sid=d.sid, val=v0)
        f = 100.0 / float(np.vdot(v0.astype(np.float64), v0.astype(np.float64)))
        DiagKtoNTrained(f).standardize(again)
        np.testing.assert_allclose(again.val, d.val, rtol=1e-6 if dtype == np.float32 else 1e-13)
    K = np.random.random((60, 60))
    K = K.dot(K.T)
    kd = KernelData(iid=[["a", str(i)] for i in range(60)], val=K.copy())
    kd.standardize()
    np.testing.assert_allclose(np.trace(kd.val), 60, rtol=1e-12)


@pytest.mark.parametrize("std,a,b", [(Unit(), 0, 0), (Beta(1, 25), 1, 25)])
@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-5)])
@pytest.mark.parametrize("order", ["F", "C"])
def test_nancnc_and_reversed_subsets_vs_python_path(std, a, b, dtype, tol, order):
    """NaNCNCTestCases (test.py:1201-1358) + load_and_standardize (test.py:642-651, 812-862):
    reversed iid/sid subsets, NaN at [0,0], a constant (SNC) column 1 -> both standardize to 0,
    and the rest matches the reference's Python path (restated by the oracle)."""
    b300 = bed("n300")
    for iids in (None, np.arange(299, 0, -2), np.array([5, 0, 17, 299, 150])):
        for sids in (None, np.arange(1014, 0, -2), np.array([3, 1, 400])):
            r = b300 if iids is None else b300[iids, :]
            r = r if sids is None else r[:, sids]
            d = r.read(order=order, dtype=dtype)
            d.val[0, 0] = np.nan
            d.val[:, 1] = 1.0
            exp = np.array(d.val, dtype=np.float64, order=order)
            O.standardize_python(exp, is_beta=isinstance(std, Beta), a=a, b=b)
            d.standardize(std)
            assert d.val[0, 0] == 0 and np.all(d.val[:, 1] == 0)
            rel_close(d.val, exp, tol)


@pytest.mark.parametrize("block_size", [None, 100, 1015])
@pytest.mark.parametrize("order", ["C", "F"])
def test_generic_block_loop_keeps_k_on_device(block_size, order):
    """snpreader.py:629-668 for a standardizer the fused path does not cover (SNP-side DiagKtoN):
    per-block standardize, Z Z^T accumulated in HBM (snpmi_grm_add_dense_*)."""
    from pysnptools_amd.standardizer import DiagKtoN

    b = bed("n300")
    K = b.read_kernel(DiagKtoN(), block_size=block_size, order=order, dtype=np.float64).val
    full = from_i8(g("n300")["val_i8"])
    full[np.isnan(full)] = 0  # n300 has no missing values; keeps the restatement simple
    bs = 1015 if block_size is None else block_size
    ref = np.zeros((300, 300))
    for s0 in range(0, 1015, bs):
        z = full[:, s0:s0 + bs].copy()
        z *= np.sqrt(300.0 / z.reshape(-1).dot(z.reshape(-1)))
        ref += z.dot(z.T)
    grm_close(K, ref, 1e-10)
    assert K.flags[order + "_CONTIGUOUS"]


def test_grm_count_a1_and_trained(syrk_variant):
    """count_A1=True flips every genotype (x -> 2 - x, test.py:226-232), so z -> -z and K is
    unchanged; the oracle built on the count_A1 decode agrees.  A trained standardizer (stats of
    SNPs 0..599 applied to the same SNPs through use_stats) reproduces the untrained K."""
    for dtype, tol in ((np.float32, 1e-5), (np.float64, 1e-10)):
        for std in (Unit(), Beta(1, 25)):
            k1 = bed("n300", count_A1=True)[:, :600].read_kernel(std, dtype=dtype).val
            k0 = bed("n300")[:, :600].read_kernel(std, dtype=dtype).val
            Z = O.decode(body("n300"), 300, 1015, count_A1=True, sid_index=np.arange(600))
            if isinstance(std, Unit):
                O.standardize_native(Z)
            else:
                O.standardize_native(Z, is_beta=True, a=1.0, b=25.0)
            ref = Z.dot(Z.T)
            grm_close(k1, ref, tol)
            grm_close(k0, ref, tol)
    _, trained = bed("n300")[:, :600].read(dtype=np.float64).standardize(Unit(), return_trained=True)
    kt = SnpKernel(bed("n300")[:, :600], trained).read(dtype=np.float32).val
    grm_close(kt, bed("n300")[:, :600].read_kernel(Unit(), dtype=np.float64).val, 1e-5)


@pytest.mark.parametrize("name,rows,world,std", [("n300", None, 1, "unit"), ("n300", None, 3, "beta"),
                                                  ("toydata", slice(None, None, 2), 2, "unit"),
                                                  ("toydata", slice(None, None, -1), 4, "unit")])
def test_grm_partitioned_from_file(name, rows, world, std):
    """cfg5 from a .bed (snpmi_grm_part_bed_f32 / shard.grm_partitioned): every rank's blocks,
    assembled, == the replicated f32 GRM and the f64 oracle; trained stats == the Bed path's."""
    from pysnptools_amd.shard import assemble_partitioned, grm_partitioned

    b = bed(name)
    r = b if rows is None else b[rows, :]
    stdz = Unit() if std == "unit" else Beta(1, 25)
    parts, trained = [], None
    for rank in range(world):
        blocks, coords, trained = grm_partitioned(r, stdz, rank, world)
        # blocks kept in HBM (accumulated in place, no copy-out) == the host copy, bit for bit
        hb, hcoords, _ = grm_partitioned(r, stdz, rank, world, out="hbm")
        assert np.array_equal(hb.get(), blocks) and np.array_equal(hcoords, coords)
        parts.append((blocks, coords))
    K = assemble_partitioned(parts, r.iid_count)
    n, m = SHAPES[name]
    iid = None if rows is None else np.arange(n)[rows]
    Z = O.decode(body(name), n, m, iid_index=iid)
    if std == "unit":
        O.standardize_native(Z)
    else:
        O.standardize_native(Z, is_beta=True, a=1.0, b=25.0)
    grm_close(K, Z.dot(Z.T), 1e-5)
    Kr, tr = r.read_kernel(stdz, dtype=np.float32), None
    np.testing.assert_allclose(K, Kr.val, rtol=0, atol=1e-5 * np.abs(np.diag(Kr.val)).max())  # summation orders differ
    _, tr = r.read(dtype=np.float32).standardize(stdz, return_trained=True)
    np.testing.assert_array_equal(np.asarray(trained.stats), np.asarray(tr.stats))


@pytest.mark.parametrize("slices", [2, 3, 8])
@pytest.mark.parametrize("n", [300, 600, 4100])
def test_grm_split_k(n, slices):
    """Split-K bf16x3 SYRK (partial tile sets + ordered reduce; auto below ~16k iids): forced
    slice counts, ragged SNP tails, accumulate across .bed chunks -- == the f64 oracle."""
    rng = np.random.default_rng(n + slices)
    m = 1000 + 37 * slices
    val = rng.integers(0, 3, size=(n, m)).astype(np.float64)
    val[rng.random(val.shape) < 0.05] = np.nan
    d = SnpData(iid=[["a", str(i)] for i in range(n)], sid=["s%d" % j for j in range(m)], val=val)
    Z = val.copy(order="F")
    O.standardize_native(Z)
    ref = Z.dot(Z.T)
    N.call("snpmi_set_kernel_variant", b"syrk_split", slices)
    try:
        with tempfile.TemporaryDirectory() as tmp:
            b = Bed.write(os.path.join(tmp, "t.bed"), d, count_A1=False)
            grm_close(b.read_kernel(Unit(), dtype=np.float32).val, ref, 1e-5)
            grm_close(b.read_kernel(Unit(), dtype=np.float32, block_size=333).val, ref, 1e-5)
    finally:
        N.call("snpmi_set_kernel_variant", b"syrk_split", 0)
