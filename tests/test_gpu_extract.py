"""The tile-blocked K extraction (k_grm_extract_rows, api.hip grm_finish / snpmi_dev_grm_extract):

* the whole K through snpmi_dev_grm_extract(ri = ci = NULL) equals the generic gather kernel
  with explicit identity indices, bit for bit, for n not a multiple of 64 or 128, f32 and f64;
* a host K large enough to go through several 1 GiB row blocks (the second block starts at a row
  that is not a multiple of 64) equals the HBM-resident K of the same call bit for bit, is
  exactly symmetric, and matches the f64 oracle GRM (snpreader.py:623-668) on rows that straddle
  the block boundary.
"""
import ctypes
import os

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


@pytest.mark.parametrize("dt,n", [(np.float32, 1000), (np.float32, 4157), (np.float64, 333), (np.float64, 2050),
                                  (np.float32, 2), (np.float32, 64), (np.float32, 129), (np.float64, 65),
                                  (np.float64, 128)])
def test_identity_extract_matches_gather(dt, n):
    m = 300
    code = N.DT_F32 if dt == np.float32 else N.DT_F64
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", packed.p, pitch, n, 0, m, 11, 0.05, N.ptr(x), N.ptr(cdf), len(x))
    es = np.dtype(dt).itemsize
    lut, st = Dev(m * 4 * es), Dev(m * 2 * es)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, code, st.p, lut.p)
    tiles = Dev(N.lib().snpmi_grm_tile_bytes(n, code))
    N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, code, tiles.p, 0)
    idx = np.arange(n, dtype=np.uint64)
    didx = Dev(n * 8)
    N.call("snpmi_memcpy_h2d", didx.p, N.ptr(idx), idx.nbytes)
    outs = []
    for ri, ci, scale in ((None, None, 1.0), (didx.p, didx.p, 1.0), (None, None, 0.75), (didx.p, didx.p, 0.75)):
        out = Dev(n * n * es)
        N.call("snpmi_dev_grm_extract", tiles.p, n, code, ri, n, ci, n, 1, scale, out.p)
        K = np.empty((n, n), dtype=dt)
        N.call("snpmi_memcpy_d2h", N.ptr(K), out.p, K.nbytes)
        outs.append(K)
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[2], outs[3])
    assert np.array_equal(outs[0], outs[0].T)
    assert np.abs(outs[0]).max() > 0


@pytest.mark.parametrize("dt,n", [(np.float32, 2), (np.float32, 129), (np.float32, 4157), (np.float64, 65),
                                  (np.float64, 2050), (np.float64, 3001)])
def test_every_extract_shape_matches_gather(dt, n):
    """Hook "extract" 1-7 (round 3's row kernel, the read-once kernel's other block shapes, and the
    pipelined kernel in three shapes) give the shipped kernel's K bit for bit, with a scale."""
    m = 200
    code = N.DT_F32 if dt == np.float32 else N.DT_F64
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(pitch * m)
    x, cdf = O.maf_table(n)
    N.call("snpmi_dev_synth_bed", packed.p, pitch, n, 0, m, 13, 0.05, N.ptr(x), N.ptr(cdf), len(x))
    es = np.dtype(dt).itemsize
    lut, st = Dev(m * 4 * es), Dev(m * 2 * es)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, code, st.p, lut.p)
    tiles = Dev(N.lib().snpmi_grm_tile_bytes(n, code))
    N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, code, tiles.p, 0)
    out = Dev(n * n * es)

    def whole(v):
        N.call("snpmi_set_kernel_variant", b"extract", v)
        try:
            N.call("snpmi_dev_memset", out.p, 0xff, n * n * es)
            N.call("snpmi_dev_grm_extract", tiles.p, n, code, None, n, None, n, 1, 0.75, out.p)
        finally:
            N.call("snpmi_set_kernel_variant", b"extract", 0)
        K = np.empty((n, n), dtype=dt)
        N.call("snpmi_memcpy_d2h", N.ptr(K), out.p, K.nbytes)
        return K

    ref = whole(0)
    assert np.array_equal(ref, ref.T) and np.isfinite(ref).all()
    for v in range(1, 8):
        assert np.array_equal(whole(v), ref), v


def _write_bed(path, n, m, seed):
    rng = np.random.default_rng(seed)
    bpc = (n + 3) // 4
    codes = rng.choice(np.array([0, 1, 2, 3], dtype=np.uint8), size=(m, bpc * 4), p=[0.3, 0.05, 0.35, 0.3])
    codes[:, n:] = 0  # pad bits
    body = (codes[:, 0::4] | (codes[:, 1::4] << 2) | (codes[:, 2::4] << 4) | (codes[:, 3::4] << 6)).astype(np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(body.tobytes())
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))
    return body.reshape(-1)


def test_host_k_in_row_blocks_equals_hbm_k(tmp_path, monkeypatch):
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    n, m = 12_000, 257  # f64 K = 1.15 GB: host rows go in blocks of 11184 (2^30 / (8 n)), not a multiple of 64
    base = os.path.join(str(tmp_path), "big")
    body = _write_bed(base, n, m, 5)
    bed = Bed(base + ".bed", count_A1=False)
    Kh = bed.read_kernel(Unit(), dtype=np.float64).val
    monkeypatch.setenv("ARRAY_MODULE", "hbm")
    Kd = bed.read_kernel(Unit(), dtype=np.float64).val.get()
    assert np.array_equal(Kh, Kd)
    assert np.array_equal(Kh, Kh.T)
    del Kd
    rows = np.array([0, 11183, 11184, 11185, n - 1])
    Z = O.decode_standardize(body, n, m, dtype=np.float64)[0]
    ref = Z[rows].dot(Z.T)
    assert np.abs(Kh[rows] - ref).max() <= 1e-10 * np.abs(np.diag(Kh)).max()


@pytest.fixture(scope="module")
def wide_bed(tmp_path_factory):
    """A 200k-iid x 24k-SNP .bed (1.2 GB; random codes, 25% missing): GRM calls on it stream 4
    chunks (2048, 10618, 10618, 716 SNPs at 50 KB per column) through 16 pinned pieces each."""
    n, m = 200_000, 24_000
    base = os.path.join(str(tmp_path_factory.mktemp("wide")), "wide")
    body = np.random.default_rng(9).integers(0, 256, size=m * (n // 4), dtype=np.uint8)
    with open(base + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(body.tobytes())
    with open(base + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(base + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))
    return base, body, n, m


@pytest.mark.parametrize("dt,tol", [(np.float32, 1e-5), (np.float64, 1e-10)])
def test_multi_chunk_file_grm_vs_oracle(wide_bed, dt, tol):
    """Bed[iids, :].read_kernel(Unit()) over several chunks and pinned pieces (api.hip
    stage_chunk / grm_stream_bed: 1/8-size first chunk, device-resident stats) vs the oracle's
    blocked GRM of the same iid subset (snpreader.py:623-668), and the trained stats."""
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    base, body, n, m = wide_bed
    iids = np.arange(0, n, 100)
    bed = Bed(base + ".bed", count_A1=False)
    K, trained = bed[iids, :]._read_kernel(Unit(), dtype=dt, return_trained=True)
    ref, stats = O.grm_from_bed(body, n, m, iid_index=iids.astype(np.uint64), block_size=4096)
    assert np.abs(K - ref).max() <= tol * np.abs(np.diag(ref)).max()
    assert np.allclose(trained.stats, stats, rtol=1e-6 if dt == np.float32 else 1e-12, atol=0)
