"""cfg5 part kernel block order (syrk.hip part_supertile_order): k_syrk_h2<LOCAL> walks the part's
256x256 blocks in 64-block supertile order by default, in the triangular order under hook
part_order=1 and in 16-block supertiles under part_order=2; each
block's storage slot and SegFlush phase follow the block, not the workgroup, so both orders give
the same K blocks bit for bit (here with several SegFlush cuts per launch and a ragged last block),
and the blocks match the f64 oracle at the f32 bar."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from oracle import oracle as O
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,part,parts,seg", [(5000, 3000, 1, 3, 1024), (9000, 1500, 0, 8, 512),
                                                (4500, 700, 7, 8, 0), (300, 500, 0, 1, 256)])
def test_part_block_orders_agree(n, m, part, parts, seg):
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    lut, stats = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    nloc = N.lib().snpmi_grm_part_blocks(n, part, parts)
    blocks = [bench.Dev(N, nloc * 256 * 256 * 4) for _ in range(3)]
    seg_default = N.kernel_variant("seg")
    out = []
    try:
        bench.synth(N, packed.p, pitch, n, 0, m, 23, 0.2)
        N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
        N.call("snpmi_set_kernel_variant", b"seg", seg)
        for k, v in enumerate((0, 1, 2)):
            N.call("snpmi_set_kernel_variant", b"part_order", v)
            try:
                N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, part, parts, blocks[k].p, 0)
            finally:
                N.call("snpmi_set_kernel_variant", b"part_order", 0)
            b = np.empty((nloc, 256, 256), dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(b), blocks[k].p, b.nbytes)
            out.append(b)
        host = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    finally:
        N.call("snpmi_set_kernel_variant", b"seg", seg_default)
        for d in [packed, lut, stats] + blocks:
            d.free()
    assert np.array_equal(out[0], out[1]) and np.array_equal(out[2], out[1])
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    Z, _ = O.decode_standardize(body, n, m, dtype=np.float64)
    K = Z.dot(Z.T)
    scale = np.abs(np.diag(K)).max()
    from pysnptools_amd.shard import part_coords

    coords = part_coords(n, part, parts)
    for b in range(nloc):
        r, c = int(coords[b, 0]), int(coords[b, 1])
        ref = K[r:min(r + 256, n), c:min(c + 256, n)]
        got = out[0][b, :ref.shape[0], :ref.shape[1]].astype(np.float64)
        assert np.abs(got - ref).max() / scale <= 1e-5, b
