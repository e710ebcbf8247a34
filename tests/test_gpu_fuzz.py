"""Seeded random parity sweep of the whole path against the oracle (in addition to the fixture-
and property-based tests): random .bed files (n in 1..2600 iids, m in 1..700 SNPs, per-SNP allele
frequency and missing rate, monomorphic / all-missing / single-iid columns), random iid and SNP
selections (sorted, reversed, shuffled, with repeats, slices), every read dtype and order,
count_A1, Unit / Beta standardization and the GRM in f32 and f64, each case compared with the
oracle's restatement of the reference:

* decode (bed.py:337-343): bit-exact incl. NaN / -127 positions;
* Unit / Beta standardize (standardizer.py:90-133, 136-211): the one-pass f64 stats rounded once
  -- Unit bit-exact, Beta <= 1e-6 (f32) / 1e-12 (f64) relative; stats equal;
* GRM (snpreader.py:623-668): max|dK| / max diag <= 2e-6 (f32) / 1e-10 (f64) vs the f64 oracle.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = 36


def _random_bed(rng, path):
    n = int(rng.choice([1, 2, 3, 5, 63, 64, 65, 127, 128, 129, 255, 257, 300, 511, 1000, 1023, 2600]))
    m = int(rng.choice([1, 2, 7, 16, 31, 33, 100, 257, 700]))
    bpc = (n + 3) // 4
    p = rng.uniform(0, 1, size=m)
    miss = rng.uniform(0, 0.4, size=m) * (rng.random(m) < 0.7)
    kind = rng.random(m)
    p[kind < 0.08] = 0.0     # monomorphic
    miss[(kind >= 0.08) & (kind < 0.12)] = 1.0  # all missing
    x = rng.binomial(2, p[None, :], size=(n, m))
    code = np.where(x == 0, 3, np.where(x == 1, 2, 0)).astype(np.uint8)  # count_A1=False coding
    code[rng.random((n, m)) < miss[None, :]] = 1
    full = np.zeros((m, bpc * 4), dtype=np.uint8)
    full[:, :n] = code.T
    body = (full[:, 0::4] | (full[:, 1::4] << 2) | (full[:, 2::4] << 4) | (full[:, 3::4] << 6)).astype(np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(body.tobytes())
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))
    return n, m, body.reshape(-1)


def _random_index(rng, count):
    k = int(rng.integers(0, 6))
    if k == 0 or count == 1:
        return None
    if k == 1:
        return np.arange(count)[::-1]
    if k == 2:
        return rng.permutation(count)[: max(1, count // 2)]
    if k == 3:
        return np.sort(rng.choice(count, size=max(1, count // 3), replace=False))
    if k == 4:
        return rng.integers(0, count, size=max(1, count // 2))  # repeats allowed
    return np.arange(int(rng.integers(0, count)), count, 2)


def _rel_close(got, exp, tol):
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    assert got.shape == exp.shape
    both = (np.isnan(got) & np.isnan(exp)) | (got == exp)  # NaN pairs and equal values (incl. inf)
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    with np.errstate(invalid="ignore"):
        d = np.abs(np.where(both, 0, got - exp))
    assert np.all(d <= tol * np.maximum(np.abs(np.where(both, 0, exp)), 1e-30) + (0 if tol == 0 else 1e-300))


@pytest.mark.parametrize("case", range(CASES))
def test_random_case_vs_oracle(tmp_path, case):
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Beta, Unit

    rng = np.random.default_rng(1000 + case)
    base = os.path.join(str(tmp_path), "r")
    n, m, body = _random_bed(rng, base)
    count_a1 = bool(rng.random() < 0.3)
    iids, sids = _random_index(rng, n), _random_index(rng, m)
    bed = Bed(base + ".bed", count_A1=count_a1)
    sub = bed if iids is None else bed[iids, :]
    sub = sub if sids is None else sub[:, sids]
    ii = None if iids is None else np.asarray(iids, dtype=np.uint64)
    si = None if sids is None else np.asarray(sids, dtype=np.uint64)
    order = "C" if rng.random() < 0.4 else "F"
    # decode, every dtype
    for dt in (np.float32, np.float64, np.int8):
        # int8 stays int8 only with _require_float32_64=False (pstdata.py:139-147 widens it to f64)
        got = sub.read(order=order, dtype=dt, _require_float32_64=dt != np.int8).val
        exp = O.decode(body, n, m, count_A1=count_a1, iid_index=ii, sid_index=si, order=order, dtype=dt)
        assert got.dtype == exp.dtype
        assert np.array_equal(got, exp, equal_nan=dt != np.int8)
    # standardize
    for dt in (np.float32, np.float64):
        v = O.decode(body, n, m, count_A1=count_a1, iid_index=ii, sid_index=si, order=order, dtype=dt)
        st = O.standardize_native(v)
        d, tr = sub.read(order=order, dtype=dt).standardize(Unit(), return_trained=True)
        assert np.array_equal(d.val, v)
        assert np.array_equal(np.asarray(tr.stats), st, equal_nan=True)
        a, b = (1.0, 25.0) if rng.random() < 0.5 else (float(rng.uniform(0.5, 3)), float(rng.uniform(0.5, 30)))
        vb = O.decode(body, n, m, count_A1=count_a1, iid_index=ii, sid_index=si, order=order, dtype=dt)
        O.standardize_native(vb, True, a, b)
        db = sub.read(order=order, dtype=dt).standardize(Beta(a, b))
        _rel_close(db.val, vb, 1e-6 if dt == np.float32 else 1e-12)
    # GRM from the file (fused path) in both dtypes
    for dt, tol in ((np.float32, 2e-6), (np.float64, 1e-10)):
        K = sub.read_kernel(Unit(), dtype=dt).val
        Z = O.decode(body, n, m, count_A1=count_a1, iid_index=ii, sid_index=si, dtype=np.float64)
        O.standardize_native(Z)
        ref = Z.dot(Z.T)
        scale = max(np.abs(np.diag(ref)).max(), 1e-300)
        assert K.shape == ref.shape
        assert np.abs(K - ref).max() <= tol * scale, (dt, n, m)


DENSE_CASES = 24


@pytest.mark.parametrize("case", range(DENSE_CASES))
def test_random_in_memory_case_vs_oracle(case):
    """In-memory SnpData (host arrays, the reference's SnpData path): random genotype-valued
    matrices with NaN (and, every third case, one column of arbitrary floats) in F or C order,
    f32 / f64:

    * SnpData.standardize(Unit() | Beta(a, b)) (standardizer.py:90-133) vs the oracle's one-pass
      restatement: Unit bit-exact for genotype-valued matrices (<= 1e-6 / 1e-12 relative with a
      float column, whose f64 sums depend on the addition order), Beta <= 1e-6 / 1e-12 relative;
    * SnpData.read_kernel(Unit()) (snpdata.py:190-214 -> snpmi_grm_dense_*: genotype columns
      re-encoded as codes + LUT, other columns on the dense kernels) and SnpKernel(...).read()
      .standardize() with DiagKtoN (snpkernel.py, diag_K_to_N.py:54-64) vs the f64 oracle."""
    from pysnptools_amd.kernelreader import SnpKernel
    from pysnptools_amd.snpreader import SnpData
    from pysnptools_amd.standardizer import Beta, Unit

    rng = np.random.default_rng(5000 + case)
    n = int(rng.choice([2, 3, 17, 64, 129, 300, 1000, 2048]))
    m = int(rng.choice([1, 3, 16, 40, 129, 300]))
    dt = np.float32 if rng.random() < 0.5 else np.float64
    order = "C" if rng.random() < 0.5 else "F"
    p = rng.uniform(0, 1, size=m)
    g = rng.binomial(2, p[None, :], size=(n, m)).astype(np.float64)
    g[rng.random((n, m)) < rng.uniform(0, 0.3)] = np.nan
    genotype_only = not (case % 3 == 0 and m > 1)
    if not genotype_only:
        g[:, m // 2] = rng.normal(0, 3, size=n)  # not genotype-valued
    val = np.array(g, dtype=dt, order=order)
    iid = [["f", str(i)] for i in range(n)]
    sid = [str(j) for j in range(m)]
    # standardize (in place on a copy, as SnpData.standardize does)
    exp = np.array(val, dtype=dt, order=order)
    st = O.standardize_native(exp)
    d, tr = SnpData(iid=iid, sid=sid, val=np.array(val, order=order)).standardize(Unit(), return_trained=True)
    if genotype_only:  # integer sums: every summation order gives the same f64 stats
        assert np.array_equal(d.val, exp, equal_nan=True)
        assert np.array_equal(np.asarray(tr.stats), st, equal_nan=True)
    else:  # a float column's f64 sums depend on the order of the additions (last bits)
        _rel_close(d.val, exp, 1e-6 if dt == np.float32 else 1e-12)
        _rel_close(tr.stats, st, 1e-6 if dt == np.float32 else 1e-12)
    a, b = float(rng.uniform(0.5, 3)), float(rng.uniform(0.5, 30))
    expb = np.array(val, dtype=dt, order=order)
    O.standardize_native(expb, True, a, b)
    db = SnpData(iid=iid, sid=sid, val=np.array(val, order=order)).standardize(Beta(a, b))
    _rel_close(db.val, expb, 1e-6 if dt == np.float32 else 1e-12)
    # GRM of the in-memory values
    Z = np.array(val, dtype=np.float64, order="F")
    O.standardize_native(Z)
    Z = Z.astype(dt).astype(np.float64)  # the dtype's standardized values, as the GRM sees them
    ref = Z.dot(Z.T)
    scale = max(np.abs(np.diag(ref)).max(), 1e-300)
    tol = 2e-6 if dt == np.float32 else 1e-10
    sd = SnpData(iid=iid, sid=sid, val=np.array(val, order=order))
    K = sd.read_kernel(Unit(), dtype=dt).val
    assert np.abs(K - ref).max() <= tol * scale
    kd = SnpKernel(sd, Unit()).read(dtype=dt).standardize()  # DiagKtoN
    tr_ref = np.trace(ref)
    if tr_ref > 0:
        assert np.abs(kd.val - ref * (n / tr_ref)).max() <= tol * scale * (n / tr_ref) + 1e-300
    assert np.array_equal(sd.val, np.array(val, order=order), equal_nan=True)  # input untouched
