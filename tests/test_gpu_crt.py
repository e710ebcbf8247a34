"""float64 GRM on the int8 MFMA (residues modulo the first R of 15 coprime moduli, R chosen per SNP
block on the device from the block's own bound max_i sum_s q_is^2 -- syrk_crt.hip k_crt_bound /
k_crt_r).  The reference computes this K in float64 (snpreader.py:528,623-668); the oracle here is
its one-pass Unit standardize + Z Z^T in f64 (oracle/oracle.py).  One test drives the bound to the
worst case (one iid carries the minor allele of every SNP: K_ii ~ m 2^2F, all 15 moduli needed),
one runs SnpGen-like data whose rare variants set the block exponent (fewer moduli)."""
import ctypes
import os
import tempfile

import numpy as np
import pytest

from oracle import oracle as O
from pysnptools_amd import _native as N
from pysnptools_amd.snpreader import Bed, SnpData
from pysnptools_amd.standardizer import Unit

pytestmark = pytest.mark.gpu


def _grm_f64(v):
    n, m = v.shape
    with tempfile.TemporaryDirectory() as tmp:
        b = Bed.write(os.path.join(tmp, "c.bed"), SnpData(iid=[["f", str(i)] for i in range(n)],
                                                           sid=["s%d" % j for j in range(m)], val=v), count_A1=False)
        s, c = ctypes.c_uint64(), ctypes.c_uint64()
        N.call("snpmi_crt_moduli_stats", ctypes.byref(s), ctypes.byref(c), 1)
        K = b.read_kernel(Unit(), dtype=np.float64).val
        N.call("snpmi_crt_moduli_stats", ctypes.byref(s), ctypes.byref(c), 1)
    Z = v.copy(order="F")
    O.standardize_native(Z)
    Kref = Z.dot(Z.T)
    err = np.abs(K - Kref).max() / np.abs(np.diag(Kref)).max()
    return err, s.value / max(c.value, 1), c.value


def test_crt_worst_case_bound_uses_every_modulus():
    rng = np.random.default_rng(11)
    n, m = 1000, 3000
    v = rng.binomial(2, rng.uniform(0.05, 0.5, m), size=(n, m)).astype(np.float64)
    v[:, : m // 2] = 0.0
    v[0, : m // 2] = 2.0  # iid 0 alone carries these SNPs: a ~ sqrt(n) for all of them, K_00 ~ m 2^2F
    err, R, launches = _grm_f64(v)
    assert launches >= 1 and R == 15, R
    assert err <= 1e-12, err


def test_crt_rare_variant_blocks_use_fewer_moduli():
    import sys

    from conftest import ROOT

    sys.path.insert(0, ROOT)
    import bench

    rng = np.random.default_rng(12)
    n, m = 2000, 8000
    x, cdf = bench.maf_table(n)
    maf = x[np.searchsorted(cdf, rng.random(m))]
    v = rng.binomial(2, maf, size=(n, m)).astype(np.float64)
    v[rng.random(v.shape) < 0.01] = np.nan
    err, R, launches = _grm_f64(v)
    assert launches >= 1 and R <= 14, R
    assert err <= 1e-12, err
