"""cfg5 part layout (syrk.hip part_layout, round 5): every LOCAL kernel reads its block from the
part's layout table -- whole 16x16-block supertiles dealt round-robin over the parts, stored
supertile by supertile -- and writes it to the table slot; the exact f64 diagonal finds the part's
diagonal blocks through the diagonal-slot table.  The blocks of every part, with several SegFlush
cuts per launch and a ragged last block, match the f64 oracle at the f32 bar, and the parts of a
plan together cover K once."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from oracle import oracle as O
from pysnptools_amd import _native as N
from pysnptools_amd.shard import part_coords

pytestmark = pytest.mark.gpu


def _part_blocks(packed, pitch, n, m, lut, part, parts):
    nloc = N.lib().snpmi_grm_part_blocks(n, part, parts)
    dev = bench.Dev(N, max(nloc, 1) * 256 * 256 * 4)
    try:
        N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, part, parts, dev.p, 0)
        b = np.empty((nloc, 256, 256), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(b), dev.p, b.nbytes)
    finally:
        dev.free()
    return b


@pytest.mark.parametrize("n,m,parts,seg", [(5000, 3000, 3, 1024), (9000, 1500, 8, 512), (4500, 700, 8, 0),
                                           (300, 500, 1, 256), (40000, 300, 8, 0)])
def test_part_blocks_match_the_oracle(n, m, parts, seg):
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    lut, stats = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    seg_default = N.kernel_variant("seg")
    out = []
    try:
        bench.synth(N, packed.p, pitch, n, 0, m, 23, 0.2)
        N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
        N.call("snpmi_set_kernel_variant", b"seg", seg)
        for part in range(parts):
            out.append(_part_blocks(packed, pitch, n, m, lut, part, parts))
        host = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    finally:
        N.call("snpmi_set_kernel_variant", b"seg", seg_default)
        for d in [packed, lut, stats]:
            d.free()
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    Z, _ = O.decode_standardize(body, n, m, dtype=np.float64)
    K = Z.dot(Z.T)
    scale = np.abs(np.diag(K)).max()
    nb = (n + 255) // 256
    seen = np.zeros((nb, nb), dtype=np.int32)
    for part in range(parts):
        coords = part_coords(n, part, parts)
        assert len(coords) == len(out[part])
        for b in range(len(coords)):
            r, c = int(coords[b, 0]), int(coords[b, 1])
            seen[r // 256, c // 256] += 1
            ref = K[r:min(r + 256, n), c:min(c + 256, n)]
            got = out[part][b, :ref.shape[0], :ref.shape[1]].astype(np.float64)
            assert np.abs(got - ref).max() / scale <= 1e-5, (part, b)
            if r == c:  # the exact diagonal
                np.testing.assert_allclose(np.diag(got), np.diag(ref), rtol=2e-7)
    assert np.array_equal(seen, np.triu(np.ones((nb, nb), dtype=np.int32)))


@pytest.mark.parametrize("n,m,parts,f64_path", [(5000, 3000, 3, 0), (40000, 700, 1, 0), (9000, 1500, 8, 0),
                                                (5000, 600, 3, 1)])
def test_part_blocks_f64_match_the_oracle(n, m, parts, f64_path):
    """float64 parts (the reference's default GRM dtype, snpreader.py:528,623): the int8 residue SYRK
    + CRT reconstruction over the part's layout (n = 40000 as one part: 12,403 blocks, three residue
    chunks of <= 4 GiB), and with hook f64 = 1 every block on the f64 MFMA kernel in part mode (four
    128-quadrants per block) -- each within 1e-12 of max diag of the f64 oracle."""
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    lut, stats = bench.Dev(N, m * 32), bench.Dev(N, m * 16)
    out = []
    try:
        bench.synth(N, packed.p, pitch, n, 0, m, 29, 0.1)
        N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F64, stats.p, lut.p)
        N.call("snpmi_set_kernel_variant", b"f64", f64_path)
        try:
            for part in range(parts):
                nloc = N.lib().snpmi_grm_part_blocks(n, part, parts)
                dev = bench.Dev(N, max(nloc, 1) * 256 * 256 * 8)
                try:
                    N.call("snpmi_dev_syrk_packed_part_f64", packed.p, pitch, n, m, lut.p, part, parts, dev.p, 0)
                    b = np.empty((nloc, 256, 256), dtype=np.float64)
                    N.call("snpmi_memcpy_d2h", N.ptr(b), dev.p, b.nbytes)
                finally:
                    dev.free()
                out.append(b)
        finally:
            N.call("snpmi_set_kernel_variant", b"f64", 0)
        host = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    finally:
        for d in [packed, lut, stats]:
            d.free()
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    Z, _ = O.decode_standardize(body, n, m, dtype=np.float64)
    K = Z.dot(Z.T)
    scale = np.abs(np.diag(K)).max()
    worst = 0.0
    for part in range(parts):
        coords = part_coords(n, part, parts)
        for b in range(len(coords)):
            r, c = int(coords[b, 0]), int(coords[b, 1])
            ref = K[r:min(r + 256, n), c:min(c + 256, n)]
            got = out[part][b, :ref.shape[0], :ref.shape[1]]
            worst = max(worst, np.abs(got - ref).max() / scale)
    assert worst <= 1e-12, worst
