"""snpmi_host_synth_bed (the host-side synthetic .bed source of the streamed cfg5 legs) against a
NumPy restatement of its specification, including the pad bits, iid counts that are not
multiples of 16 and the scalar/AVX2 boundary; and the genotype frequencies it produces."""
import ctypes

import numpy as np
import pytest

from pysnptools_amd import _native as N

M64 = (1 << 64) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def _lowbias32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


def _maf_table(n):
    w0, w1 = -0.6482249, -8.49790398
    x = np.logspace(np.log10(0.1 / n), np.log10(0.5), 100, base=10)
    y = np.exp(w0 * np.log(x) + w1)
    cdf = np.cumsum(y / y.sum())
    cdf[-1] = 1.0
    return np.ascontiguousarray(x), np.ascontiguousarray(cdf)


def _spec(n, pitch, sid0, m, seed, miss, x, cdf):
    out = np.zeros((m, pitch), dtype=np.uint8)
    sc = 4294967296.0

    def thr(t):
        return 0xFFFFFFFF if t >= sc else int(t)

    for j in range(m):
        sid = sid0 + j
        h = _splitmix64(((seed * 0xD1B54A32D192ED03) & M64) ^ (((sid + 1) * 0x8CB92BA72F3D8DD7) & M64))
        u = (h >> 11) * (1.0 / 9007199254740992.0)
        lo = min(int(np.searchsorted(cdf, u, side="left")), len(x) - 1)  # first k with u <= cdf[k]
        maf = x[lo]
        keep = 1.0 - miss
        kb = _splitmix64(((seed + 0x632BE59BD9B4E019) & M64) ^ ((sid * 0x9E6C63D0676A9A99) & M64)) >> 32
        thm, t3, t2 = thr(miss * sc), thr(keep * maf * maf * sc), thr(keep * 2.0 * maf * (1.0 - maf) * sc)
        i = np.arange(n, dtype=np.uint64)
        uu = _lowbias32(np.uint64(kb) ^ ((i * np.uint64(0x9E3779B9)) & np.uint64(0xFFFFFFFF)))
        a = (uu - np.uint64(thm)) & np.uint64(0xFFFFFFFF)
        code = np.where(uu < thm, 1, np.where(a < t3, 3, np.where(((a - np.uint64(t3)) & np.uint64(0xFFFFFFFF)) < t2,
                                                                    2, 0))).astype(np.uint8)
        pad = np.zeros(pitch * 4, dtype=np.uint8)
        pad[:n] = code
        q = pad.reshape(-1, 4)
        out[j] = q[:, 0] | (q[:, 1] << 2) | (q[:, 2] << 4) | (q[:, 3] << 6)
    return out


def _host_synth(n, pitch, sid0, m, seed, miss, threads=3):
    x, cdf = _maf_table(n)
    buf = np.full((m, pitch), 0xAB, dtype=np.uint8)  # pad bytes must be overwritten with zeros
    N.call("snpmi_host_synth_bed", N.ptr(buf), pitch, n, sid0, m, seed, miss, N.ptr(x), N.ptr(cdf), len(x), threads)
    return buf, x, cdf


@pytest.mark.parametrize("n", [1, 15, 16, 17, 127, 128, 129, 300, 1000, 4099, 40003])
def test_matches_spec(n):
    pitch = N.lib().snpmi_packed_pitch(n)
    buf, x, cdf = _host_synth(n, pitch, 1234567, 7, 5, 0.218)
    np.testing.assert_array_equal(buf, _spec(n, pitch, 1234567, 7, 5, 0.218, x, cdf))


def test_genotype_frequencies():
    n, m = 20000, 64
    pitch = N.lib().snpmi_packed_pitch(n)
    buf, x, cdf = _host_synth(n, pitch, 0, m, 9, 0.1)
    codes = np.stack([(buf[:, :(n + 3) // 4] >> (2 * k)) & 3 for k in range(4)], axis=2).reshape(m, -1)[:, :n]
    assert abs((codes == 1).mean() - 0.1) < 0.005  # missing rate
    # per SNP: heterozygote share among observed ~ 2p(1-p) of the SNP's drawn MAF
    obs = codes != 1
    het = ((codes == 2) & obs).sum(1) / obs.sum(1)
    hom = ((codes == 3) & obs).sum(1) / obs.sum(1)
    maf_hat = het / 2 + hom
    assert np.all(maf_hat <= 0.6) and np.corrcoef(het, 2 * maf_hat * (1 - maf_hat))[0, 1] > 0.95


def test_threads_do_not_change_the_bytes():
    n, m = 70001, 5
    pitch = N.lib().snpmi_packed_pitch(n)
    a, _, _ = _host_synth(n, pitch, 77, m, 3, 0.01, threads=1)
    b, _, _ = _host_synth(n, pitch, 77, m, 3, 0.01, threads=8)
    np.testing.assert_array_equal(a, b)


def test_bad_arguments():
    x, cdf = _maf_table(100)
    buf = np.zeros((1, 64), dtype=np.uint8)
    with pytest.raises(ValueError):
        N.call("snpmi_host_synth_bed", N.ptr(buf), 63, 100, 0, 1, 1, 0.0, N.ptr(x), N.ptr(cdf), len(x), 1)
    with pytest.raises(ValueError):
        N.call("snpmi_host_synth_bed", N.ptr(buf), 64, 100, 0, 1, 1, 0.0, N.ptr(x), N.ptr(cdf), 0, 1)
    assert ctypes.sizeof(ctypes.c_void_p) == 8
