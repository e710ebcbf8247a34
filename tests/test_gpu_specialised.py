"""The warp-specialised fp16x2 SYRK (k_syrk_h2s, hook "h2" = 1: loader waves beside the MFMA
waves, round 6) against the MODE-4 kernel it replaces (k_syrk_h2, loader in every wave): the same
products in the same order per accumulator and the same SegFlush points, so the tiles must be
equal bit for bit -- whole launches (one and several SegFlush rounds), the column groups of the
overlapped collective, and a cfg5 part (the part layout table)."""
import ctypes

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


def _data(n, m, seed):
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, seed, 0.05)
    lut, st = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
    return packed, pitch, lut


def _get(dev, count):
    out = np.empty(count, dtype=np.float32)
    N.call("snpmi_stream_sync")
    N.call("snpmi_memcpy_d2h", N.ptr(out), dev.p, out.nbytes)
    return out


def _both(fn):
    outs = []
    for form in (0, 1):
        N.call("snpmi_set_kernel_variant", b"h2", form)
        try:
            outs.append(fn())
        finally:
            N.call("snpmi_set_kernel_variant", b"h2", 1)
    return outs


@pytest.mark.parametrize("n,m", [(4100, 1015), (20000, 3000), (30000, 30000), (16384, 40), (8000, 30000)])
def test_h2s_whole_launch_bit_identical(n, m):
    """Whole launches, incl. the split-K grids of n <~ 16k (k_syrk_h2s with gridDim.y slices) and
    several SegFlush rounds (30000 SNPs)."""
    packed, pitch, lut = _data(n, m, 7 + m)
    tb = N.lib().snpmi_grm_tile_bytes(n, N.DT_F32)
    tiles = bench.Dev(N, tb)

    def run():
        N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, N.DT_F32, tiles.p, 0)
        return _get(tiles, tb // 4)

    a, b = _both(run)
    assert np.array_equal(a, b)
    for d in (packed, lut, tiles):
        d.free()


def test_h2s_column_groups_bit_identical():
    """The overlapped collective's grouped last launch (no collective: the tiles only)."""
    from pysnptools_amd.shard import ShardedGrm

    n, m = 30000, 3000
    packed, pitch, lut = _data(n, m, 11)
    stats = bench.Dev(N, m * 8)

    def run():
        g = ShardedGrm(n, np.float32, None, "none")
        N.call("snpmi_grm_add_packed_reduce_f32", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, stats.p, 0, 0, 3,
               None)
        t, count = g.tiles()
        out = np.empty(count, dtype=np.float32)
        N.call("snpmi_stream_sync")
        N.call("snpmi_memcpy_d2h", N.ptr(out), t, out.nbytes)
        g.abort()
        assert N.kernel_variant("overlap_groups") == 3
        return out

    a, b = _both(run)
    assert np.array_equal(a, b)
    for d in (packed, lut, stats):
        d.free()


@pytest.mark.parametrize("n,m,part,parts", [(2300, 30000, 1, 3), (9000, 700, 5, 8)])
def test_h2s_part_bit_identical(n, m, part, parts):
    packed, pitch, lut = _data(n, m, 13)
    nloc = N.lib().snpmi_grm_part_blocks(n, part, parts)
    blocks = bench.Dev(N, nloc * 65536 * 4)

    def run():
        N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, part, parts, blocks.p, 0)
        return _get(blocks, nloc * 65536)

    a, b = _both(run)
    assert a.size and np.array_equal(a, b)
    for d in (packed, lut, blocks):
        d.free()
