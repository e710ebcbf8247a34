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


def _kernel_f64(v, per_block=1):
    """K through the public reader, with the moduli counts it ran: (K, launch-wide R, launches,
    mean per-block R_b, blocks)."""
    n, m = v.shape
    s, c, sb, cb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    with tempfile.TemporaryDirectory() as tmp:
        b = Bed.write(os.path.join(tmp, "c.bed"), SnpData(iid=[["f", str(i)] for i in range(n)],
                                                           sid=["s%d" % j for j in range(m)], val=v), count_A1=False)
        N.call("snpmi_set_kernel_variant", b"crt_block", per_block)
        try:
            N.call("snpmi_crt_moduli_stats", ctypes.byref(s), ctypes.byref(c), 1)
            N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sb), ctypes.byref(cb), 1)
            K = b.read_kernel(Unit(), dtype=np.float64).val
            N.call("snpmi_crt_moduli_stats", ctypes.byref(s), ctypes.byref(c), 1)
            N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sb), ctypes.byref(cb), 1)
        finally:
            N.call("snpmi_set_kernel_variant", b"crt_block", 1)
    return K, s.value / max(c.value, 1), c.value, sb.value / max(cb.value, 1), cb.value


def _grm_f64(v):
    K, R, launches, Rb, blocks = _kernel_f64(v)
    Z = v.copy(order="F")
    O.standardize_native(Z)
    Kref = Z.dot(Z.T)
    err = np.abs(K - Kref).max() / np.abs(np.diag(Kref)).max()
    nb = (v.shape[0] + 255) // 256
    assert blocks == launches * nb * (nb + 1) // 2, (blocks, launches, nb)
    assert 1.0 <= Rb <= R, (Rb, R)
    return err, R, launches


def test_crt_worst_case_bound_uses_every_modulus():
    rng = np.random.default_rng(11)
    n, m = 1000, 3000
    v = rng.binomial(2, rng.uniform(0.05, 0.5, m), size=(n, m)).astype(np.float64)
    v[:, : m // 2] = 0.0
    v[0, : m // 2] = 2.0  # iid 0 alone carries these SNPs: a ~ sqrt(n) for all of them, K_00 ~ m 2^2F
    err, R, launches = _grm_f64(v)
    assert launches >= 1 and R == 15, R
    assert err <= 1e-12, err


def test_crt_per_block_moduli_same_bits_as_launch_wide():
    """The worst-case data again: the panel of iid 0 needs all 15 moduli, the blocks away from it
    fewer (sqrt(M_bi M_bj) < M_0), and K is the same bits as with the launch-wide R (hook
    "crt_block" = 0): the symmetric mixed-radix digits above R_b are zero either way."""
    rng = np.random.default_rng(11)
    n, m = 1000, 3000
    v = rng.binomial(2, rng.uniform(0.05, 0.5, m), size=(n, m)).astype(np.float64)
    v[:, : m // 2] = 0.0
    v[0, : m // 2] = 2.0
    K1, R1, _, Rb1, _ = _kernel_f64(v, 1)
    K0, R0, _, Rb0, _ = _kernel_f64(v, 0)
    assert R1 == R0 == 15 and Rb0 == 15, (R1, R0, Rb0)
    assert Rb1 < 15, Rb1
    assert np.array_equal(K0, K1)


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


def test_crt_chunks_match_f64_mfma():
    """N = 30000: the 7021 256-blocks need two residue chunks (4 GiB of scratch per chunk).  The
    tiles equal the f64-MFMA path's (variant 71) to 1e-12 of max |K| after a fresh launch and
    after an accumulating second launch, and tile (0, 0) matches the f64 oracle."""
    from test_gpu_parity import Dev, synth_dev

    n, m = 30000, 512
    buf, pitch = synth_dev(n, 2 * m, 23)
    lut, st = Dev(2 * m * 4 * 8), Dev(2 * m * 2 * 8)
    N.call("snpmi_dev_snp_stats", buf.p, pitch, n, 2 * m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F64, st.p, lut.p)
    tb = N.lib().snpmi_grm_tile_bytes(n, N.DT_F64)
    outs = []
    for v in (0, 71):
        tiles = Dev(tb)
        N.call("snpmi_set_kernel_variant", b"syrk", v)
        try:
            N.call("snpmi_dev_syrk_packed", buf.p, pitch, n, m, lut.p, N.DT_F64, tiles.p, 0)
            one = tiles.get(np.empty(tb // 8, dtype=np.float64))
            N.call("snpmi_dev_syrk_packed", ctypes.c_void_p(buf.p.value + m * pitch), pitch, n, m,
                   ctypes.c_void_p(lut.p.value + m * 32), N.DT_F64, tiles.p, 1)
            two = tiles.get(np.empty(tb // 8, dtype=np.float64))
        finally:
            N.call("snpmi_set_kernel_variant", b"syrk", 0)
        outs.append((one, two))
    # compare K entries only: the pad rows/columns (iid >= n) of the last tile row/column are
    # scratch that the extraction never reads, and the two paths leave different values there
    nt = (n + 127) // 128
    tj = np.repeat(np.arange(nt), np.arange(1, nt + 1))
    ti = np.concatenate([np.arange(j + 1) for j in range(nt)])
    vc = n - (nt - 1) * 128
    for a, b in zip(outs[0], outs[1]):
        for x in (a, b):
            T = x.reshape(-1, 128, 128)
            T[tj == nt - 1, :, vc:] = 0
            T[ti == nt - 1, vc:, :] = 0
        assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max()
    # tile (0, 0) = K[0:128, 0:128] over all 2m SNPs vs the oracle
    packed = buf.get(np.empty((2 * m, pitch), dtype=np.uint8))
    Z = O.decode(np.ascontiguousarray(packed[:, :(n + 3) // 4]).reshape(-1), n, 2 * m, dtype=np.float64)
    O.standardize_native(Z)
    Kref = Z[:128].dot(Z[:128].T)
    got = outs[0][1][:128 * 128].reshape(128, 128)
    iu = np.triu_indices(128)
    assert np.abs(got[iu] - Kref[iu]).max() <= 1e-12 * np.abs(np.diag(Kref)).max()


def test_public_f64_switch_selects_the_f64_mfma():
    """pysnptools_amd.set_grm_f64: 'mfma' runs f64 GRMs on the f64 MFMA (no CRT launches), 'crt' back
    to the int8 residues; both within 1e-12 of max diag of the reference's own toydata GRM."""
    import ctypes
    import os

    import numpy as np

    import pysnptools_amd
    from conftest import DATA
    from pysnptools_amd import _native as N
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    gold = np.load(os.path.join(DATA, "toydata.kernel.npz"))["val"]
    bed = Bed(os.path.join(DATA, "toydata.bed"), count_A1=False)
    sr, nl = ctypes.c_uint64(), ctypes.c_uint64()
    out = {}
    try:
        for path in ("mfma", "crt"):
            pysnptools_amd.set_grm_f64(path)
            N.call("snpmi_crt_moduli_stats", ctypes.byref(sr), ctypes.byref(nl), 1)
            out[path] = bed.read_kernel(Unit()).val
            N.call("snpmi_crt_moduli_stats", ctypes.byref(sr), ctypes.byref(nl), 1)
            assert (nl.value == 0) == (path == "mfma"), (path, nl.value)
    finally:
        pysnptools_amd.set_grm_f64("crt")
    scale = np.abs(np.diag(gold)).max()
    for path, K in out.items():
        assert np.abs(K - gold).max() / scale <= 1e-12, path
    import pytest
    with pytest.raises(ValueError):
        pysnptools_amd.set_grm_f64("f32")


@pytest.mark.parametrize("n,m,parts", [(300, 1015, 0), (1000, 129, 0), (4100, 3000, 0), (30000, 300, 0),
                                       (2300, 700, 3)])
def test_warp_specialised_residue_syrk_is_bit_identical(n, m, parts):
    """k_syrk_i8w (hook "crt" = 1: loader waves beside the MFMA waves; 2: without its read order and
    wave priorities) produces the same residues as k_syrk_i8r, hence the same f64 K bit for bit -- replicated tiles (one and several residue
    chunks, stage counts 2..24, n not a multiple of 256) and a cfg5 part (part_tab layout)."""
    _forms_bit_identical(b"crt", n, m, parts, forms=(0, 1, 2))


@pytest.mark.parametrize("n,m,parts", [(4100, 3000, 0), (30000, 300, 0), (2300, 700, 3)])
def test_per_block_moduli_bit_identical_on_device(n, m, parts):
    """hook "crt_block": moduli per 256-block vs the launch-wide R, through the device entry points
    (replicated tiles, residue chunks, a cfg5 part)."""
    _forms_bit_identical(b"crt_block", n, m, parts)


def _forms_bit_identical(hook, n, m, parts, forms=(0, 1)):
    """The forms of `hook` give the same f64 tiles bit for bit."""
    from test_gpu_parity import Dev, synth_dev

    buf, pitch = synth_dev(n, m, 31 + n)
    lut, st = Dev(m * 32), Dev(m * 16)
    N.call("snpmi_dev_snp_stats", buf.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F64, st.p, lut.p)
    outs = []
    for form in forms:
        N.call("snpmi_set_kernel_variant", hook, form)
        try:
            if parts:
                nloc = N.lib().snpmi_grm_part_blocks(n, 1, parts)
                k = Dev(nloc * 65536 * 8)
                N.call("snpmi_dev_syrk_packed_part_f64", buf.p, pitch, n, m, lut.p, 1, parts, k.p, 0)
                outs.append(k.get(np.empty(nloc * 65536, dtype=np.float64)))
            else:
                tb = N.lib().snpmi_grm_tile_bytes(n, N.DT_F64)
                k = Dev(tb)
                N.call("snpmi_dev_syrk_packed", buf.p, pitch, n, m, lut.p, N.DT_F64, k.p, 0)
                outs.append(k.get(np.empty(tb // 8, dtype=np.float64)))
        finally:
            N.call("snpmi_set_kernel_variant", hook, 1)
    assert outs[0].size and all(np.array_equal(outs[0], o) for o in outs[1:])
