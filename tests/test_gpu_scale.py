"""BASELINE configs[1] and configs[2] at full size on the GPU (device-resident synthetic BED).

Checks that do not need a CPU pass over the whole matrix:
  * sampled columns of every 8192-SNP block bit-exact (Unit) / <=1e-6 rel (Beta) vs the oracle
    on the same packed bytes;
  * every column: sum_i z_ij == 0 and (Unit) sum_i z_ij^2 == n_obs for polymorphic SNPs,
    missing -> exactly 0, SNC -> all zeros -- to f32 rounding.
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


class Dev:
    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        N.call("snpmi_dev_alloc", ctypes.byref(self.p), int(nbytes))

    def __del__(self):
        try:
            N.call("snpmi_dev_free", self.p)
        except Exception:
            pass

    def at(self, off):
        return ctypes.c_void_p(self.p.value + off)


def run_config(n, m, seed, miss, std_kind, a, b, block=8192, samples=12):
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", packed.p, pitch, n, 0, m, seed, miss, N.ptr(x), N.ptr(cdf), len(x))
    lut, st, out = Dev(block * 16), Dev(block * 8), Dev(block * ld * 4)
    rng = np.random.default_rng(seed)
    bpc = (n + 3) // 4
    n_poly = 0
    for s0 in range(0, m, block):
        cnt = min(block, m - s0)
        N.call("snpmi_dev_snp_stats", packed.at(s0 * pitch), pitch, n, cnt, 0, std_kind, a, b, 0, N.DT_F32, st.p, lut.p)
        N.call("snpmi_dev_decode", packed.at(s0 * pitch), pitch, n, cnt, lut.p, N.DT_F32, 0, out.p, ld)
        stats = np.empty((cnt, 2), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(stats), st.p, stats.nbytes)
        cols = np.sort(rng.choice(cnt, size=min(samples, cnt), replace=False))
        got = np.empty((len(cols), ld), dtype=np.float32)
        pk = np.empty((len(cols), pitch), dtype=np.uint8)
        for q, c in enumerate(cols):
            N.call("snpmi_memcpy_d2h", N.ptr(got[q]), out.at(int(c) * ld * 4), ld * 4)
            N.call("snpmi_memcpy_d2h", N.ptr(pk[q]), packed.at((s0 + int(c)) * pitch), pitch)
        body = np.ascontiguousarray(pk[:, :bpc]).reshape(-1)
        exp, est = O.decode_standardize(body, n, len(cols), is_beta=std_kind == N.STD_BETA, a=a, b=b,
                                        dtype=np.float32)
        assert np.array_equal(est, stats[cols])
        g = got[:, :n].T
        if std_kind == N.STD_UNIT:
            assert np.array_equal(g, exp)
        else:
            np.testing.assert_allclose(g, exp, rtol=1e-6, atol=1e-7)
        # properties of the sampled columns
        raw = O.decode(body, n, len(cols))
        miss_mask = np.isnan(raw)
        assert np.all(g[miss_mask] == 0)
        g64 = g.astype(np.float64)
        poly = np.isfinite(stats[cols, 1])
        n_poly += int(poly.sum())
        scale = np.abs(g64).max(0) + 1e-30
        assert np.all(np.abs(g64.sum(0))[poly] <= 1e-5 * n * scale[poly])
        if std_kind == N.STD_UNIT:
            nobs = (~miss_mask).sum(0)
            np.testing.assert_allclose((g64 ** 2).sum(0)[poly], nobs[poly], rtol=1e-5)
            assert np.all(g64[:, ~poly] == 0)
    return n_poly


def test_config1_10k_x_100k_unit():
    """BASELINE configs[1]: synthetic BED 10k iid x 100k SNP, Unit, f32."""
    assert run_config(10_000, 100_000, seed=2, miss=0.01, std_kind=N.STD_UNIT, a=0.0, b=0.0) > 0


def test_config2_100k_x_1m_beta():
    """BASELINE configs[2]: 100k iid x 1M SNP, Beta(1,25) + NaN impute (21.8% missing, snpgen.py:166)."""
    assert run_config(100_000, 1_000_000, seed=3, miss=0.218, std_kind=N.STD_BETA, a=1.0, b=25.0, samples=4) > 0


def test_grm_config4_50k_x_500k():
    """BASELINE configs[3] at full size: 50k iids x 500k SNPs, Unit, f32 GRM accumulated on the
    device over 10k-SNP blocks (fp16x2 split on the fp16 MFMA, bf16x3 as its range fallback).  K
    restricted to 96 sampled iids
    (rows AND columns, incl. iids 0 and n-1) against the f64 oracle over all 500k SNPs -- only
    those iids are decoded; stats from the code counts of every iid -- max|dK| <= 1e-5 max diag,
    and the diagonal elementwise within 1e-5."""
    n, m, B = 50_000, 500_000, 10_000
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", packed.p, pitch, n, 0, m, 4, 0.01, N.ptr(x), N.ptr(cdf), len(x))
    tiles = Dev(N.lib().snpmi_grm_tile_bytes(n, N.DT_F32))
    lut, st = Dev(B * 16), Dev(B * 8)
    for s0 in range(0, m, B):
        cnt = min(B, m - s0)
        N.call("snpmi_dev_snp_stats", packed.at(s0 * pitch), pitch, n, cnt, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
               st.p, lut.p)
        N.call("snpmi_dev_syrk_packed", packed.at(s0 * pitch), pitch, n, cnt, lut.p, N.DT_F32, tiles.p, int(s0 > 0))
    rng = np.random.default_rng(4)
    sample = np.unique(np.concatenate([[0, n - 1], rng.choice(n, size=94, replace=False)])).astype(np.uint64)
    ns = len(sample)
    didx, dout = Dev(ns * 8), Dev(ns * ns * 4)
    N.call("snpmi_memcpy_h2d", didx.p, N.ptr(sample), sample.nbytes)
    N.call("snpmi_dev_grm_extract", tiles.p, n, N.DT_F32, didx.p, ns, didx.p, ns, 1, 1.0, dout.p)
    K = np.empty((ns, ns), dtype=np.float32)
    N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
    del tiles
    host = np.empty((m, pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    del packed
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    del host
    stats = O.snp_stats(body, n, m)
    Zs = O.decode(body, n, m, iid_index=sample, dtype=np.float64)
    O.standardize_native(Zs, use_stats=True, stats=stats)
    Kref = Zs.dot(Zs.T)
    scale = np.abs(np.diag(Kref)).max()
    err = float(np.abs(K.astype(np.float64) - Kref).max() / scale)
    assert err <= 1e-5, "cfg4 GRM sample vs f64 oracle: %g" % err
    np.testing.assert_allclose(np.diag(K), np.diag(Kref), rtol=1e-5)
    assert np.array_equal(K, K.T)


@pytest.mark.parametrize("part,dtype,m", [(0, np.float32, 2048), (5, np.float32, 2048), (0, np.float64, 8192)])
def test_config4_partitioned_500k_iids(part, dtype, m):
    """BASELINE configs[4] at its iid count: K of 500,000 iids is 500 GB (f32 upper triangle), so it
    is partitioned as 256x256 blocks over the 8 parts of the 8-GPU plan (snpmi_dev_syrk_packed_part,
    whole 16x16-block supertiles per part); this runs part `part` of 8 over `m` synthetic SNPs (~64
    GB of f32 / ~125 GB of f64 K blocks in HBM) and checks a diagonal and an off-diagonal block and
    the part's last one against the f64 oracle on just those iids, with stats over all 500k iids
    (the reference replicates K, snpreader.py:643-655, which cannot hold this).  float64 -- the
    reference's default GRM dtype (snpreader.py:528,623) -- runs the int8-CRT part kernels
    (snpmi_dev_syrk_packed_part_f64) and must match within 1e-12 of max diag; f32 within 1e-5."""
    n, P = 500_000, 8
    isz = np.dtype(dtype).itemsize
    pitch = N.lib().snpmi_packed_pitch(n)
    nloc = N.lib().snpmi_grm_part_blocks(n, part, P)
    nb = (n + 255) // 256
    assert sum(N.lib().snpmi_grm_part_blocks(n, r, P) for r in range(P)) == nb * (nb + 1) // 2
    packed = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", packed.p, pitch, n, 0, m, 11, 0.01, N.ptr(x), N.ptr(cdf), len(x))
    lut, st = Dev(m * 4 * isz), Dev(m * 2 * isz)
    blocks = Dev(nloc * 256 * 256 * isz)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.dt_code(np.dtype(dtype)), st.p,
           lut.p)
    if dtype == np.float64:
        N.call("snpmi_dev_syrk_packed_part_f64", packed.p, pitch, n, m, lut.p, part, P, blocks.p, 0)
    else:
        N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, part, P, blocks.p, 0)
    N.call("snpmi_stream_sync")
    host = np.empty((m, pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    del packed
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    stats = O.snp_stats(body, n, m)
    # the part's diagonal block nearest the start, an off-diagonal one, and its very last block
    # (which touches the padded iids 499,968..500,223 when it sits in the last block column)
    want = {"diag": None, "off": None, "last": nloc - 1}
    r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
    for b in range(min(nloc, 300)):
        N.call("snpmi_grm_part_coords", n, part, P, b, ctypes.byref(r0), ctypes.byref(c0))
        if r0.value == c0.value and want["diag"] is None:
            want["diag"] = b
        if r0.value != c0.value and want["off"] is None:
            want["off"] = b
    assert want["diag"] is not None and want["off"] is not None
    tol = 1e-12 if dtype == np.float64 else 1e-5
    for what, b in want.items():
        N.call("snpmi_grm_part_coords", n, part, P, b, ctypes.byref(r0), ctypes.byref(c0))
        rows = np.arange(r0.value, min(r0.value + 256, n))
        cols = np.arange(c0.value, min(c0.value + 256, n))
        blk = np.empty((256, 256), dtype=dtype)
        N.call("snpmi_memcpy_d2h", N.ptr(blk), blocks.at(b * 256 * 256 * isz), blk.nbytes)
        Zr = O.decode(body, n, m, iid_index=rows, dtype=np.float64)
        Zc = O.decode(body, n, m, iid_index=cols, dtype=np.float64)
        O.standardize_native(Zr, use_stats=True, stats=stats)
        O.standardize_native(Zc, use_stats=True, stats=stats)
        ref = Zr.dot(Zc.T)
        scale = max(np.abs(np.diag(ref)).max() if r0.value == c0.value else np.abs(ref).max(), 1.0)
        err = np.abs(blk[:len(rows), :len(cols)].astype(np.float64) - ref).max() / scale
        assert err <= tol, "%s block %d (%d, %d): %g" % (what, b, r0.value, c0.value, err)
        if r0.value == c0.value:
            np.testing.assert_allclose(np.diag(blk)[:len(rows)], np.diag(ref), rtol=tol)


class _OneRank:
    rank, world, rccl, n_gpus, local_rank, device, can_reduce = 0, 1, False, 1, 0, 0, False

    def barrier(self):
        pass

    def max(self, x):
        return x


def test_config5_streamed_500k_iids_over_100k_snps():
    """configs[4]'s per-rank job beyond one block: part 0 of the 8-part plan at 500,000 iids over
    106,496 SnpGen-shaped SNPs (21.8% missing) in 4 streamed blocks (8192, then 3 x 32768 SNPs) through
    shard.PartitionedGrm (pinned host slots generated on host threads, uploads under the previous
    block's SYRK, f32 K blocks accumulated in HBM) -- bench.py's grm5 leg at a tenth of its SNPs.
    Sample blocks (first diagonal, first off-diagonal, the last one with the padded iids) vs the
    f64 oracle over all SNPs (stats over every iid), <= 1e-5 of max diag; per-SNP stats bit-exact."""
    import os
    import sys

    from conftest import ROOT

    sys.path.insert(0, ROOT)
    import bench

    args = bench.parse(["--grm5-iid", "500000", "--grm5-sid", "106496", "--steps", "1", "--warmup", "0"])
    assert args.grm5_miss == 0.218 and args.grm5_block == 32768
    r = bench.leg_grm5(N, args, _OneRank())
    assert r["blocks"] == 4 and len(r["block_ms"]) == 4
    picks, stats = r["parity_sample"]
    assert set(picks) == {"diag", "off", "last"}
    p = bench.grm5_parity(args, picks, stats, min(16, os.cpu_count() or 1))
    assert p["stats_bit_exact"], p
    assert p["max_abs_err_over_max_diag"] <= 1e-5, p
