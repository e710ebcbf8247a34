"""f32 GRM accuracy at large M on SnpGen-shaped data (rare-variant heavy MAF curve, 21.8% missing):
the f32 accumulation chains of the SYRK kernels are cut every `seg` SNPs (12288; syrk.hip SegFlush /
for_segments) and the diagonal is accumulated exactly in f64 (k_diag_*), so one launch over tens
of thousands of SNPs stays within the f32 bar (1e-5 of max diag; asserted here at 6e-6, and at
2e-6 over 200k SNPs) against the f64 oracle.  Before the segmentation one 62.5k-SNP launch of the fp16x2 kernel drifted 2e-5 of max
diag at 50k x 100k (bench `file` leg), because the tiny z^2 of rare-variant SNPs were absorbed into
K_ii ~ 1e5.  Checked for the three f32 kernels: fp16x2 (default), bf16x3 (its range fallback,
variant 36) and the f32 MFMA (variant 20: 2 products per MFMA k-step, so twice the chain steps of
the fp16 kernels per segment), and for the partitioned (cfg5) kernel."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from oracle import oracle as O
from pysnptools_amd import _native as N
from pysnptools_amd.shard import ShardedGrm

pytestmark = pytest.mark.gpu

n, m, R = 20_000, 48_000, 8


@pytest.fixture(scope="module")
def data():
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, 305, 0.218)
    host = np.empty((m, pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    ref = np.zeros((R, n))
    for s0 in range(0, m, 4096):
        sid = np.arange(s0, min(m, s0 + 4096), dtype=np.uint64)
        Z, _ = O.decode_standardize(body, n, m, sid_index=sid, dtype=np.float64)
        ref += Z[:R].dot(Z.T)
    yield packed, pitch, body, ref
    packed.free()


def _rows(packed, pitch):
    stats = bench.Dev(N, m * 8)
    g = ShardedGrm(n, np.float32, None, "none")
    g.add_packed(packed.p, pitch, m, N.STD_UNIT, 0.0, 0.0, 0, stats.p)  # one launch of 48k SNPs
    t, _ = g.tiles()
    ri = np.arange(R, dtype=np.uint64)
    dri, dout = bench.Dev(N, R * 8), bench.Dev(N, R * n * 4)
    N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
    N.call("snpmi_dev_grm_extract", t, n, N.DT_F32, dri.p, R, None, n, 1, 1.0, dout.p)
    K = np.empty((R, n), dtype=np.float32)
    N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
    g.abort()
    for d in (stats, dri, dout):
        d.free()
    return K


@pytest.mark.parametrize("variant,tol", [(0, 6e-6), (36, 6e-6), (20, 6e-6)])
def test_long_launch_within_f32_bar(data, variant, tol):
    packed, pitch, _, ref = data
    N.call("snpmi_set_kernel_variant", b"syrk", variant)
    try:
        K = _rows(packed, pitch)
    finally:
        N.call("snpmi_set_kernel_variant", b"syrk", 0)
    scale = np.abs(np.diag(ref[:, :R])).max()
    err = np.abs(K.astype(np.float64) - ref).max() / scale
    assert err <= tol, err
    diag_rel = np.max(np.abs(np.diag(K[:, :R]) - np.diag(ref[:, :R])) / np.diag(ref[:, :R]))
    assert diag_rel <= tol, diag_rel


def test_partitioned_blocks_within_f32_bar(data):
    """cfg5 kernel (k_syrk_h2<LOCAL>): part 0 of 4 -- its first block (rows/cols 0..255) over all SNPs."""
    packed, pitch, body, ref = data
    lut, stats = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    nloc = N.lib().snpmi_grm_part_blocks(n, 0, 4)
    blocks = bench.Dev(N, nloc * 256 * 256 * 4)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, 0, 4, blocks.p, 0)
    blk = np.empty((256, 256), dtype=np.float32)
    N.call("snpmi_memcpy_d2h", N.ptr(blk), blocks.p, blk.nbytes)
    for d in (lut, stats, blocks):
        d.free()
    scale = np.abs(np.diag(ref[:, :R])).max()
    err = np.abs(blk[:R].astype(np.float64) - ref[:, :256]).max() / scale
    assert err <= 6e-6, err


@pytest.mark.parametrize("m_edge", [8191, 8193, 16415])
@pytest.mark.parametrize("seg", [256, 8192])
def test_segment_flush_edges_vs_oracle(m_edge, seg):
    """SegFlush edge cases on the default fp16x2 kernel: SNP counts one short of / one past / 31
    past a segment boundary, and a 256-SNP segment (a flush every 4 trips: the store-then-atomic
    slot path runs dozens of times per workgroup, 78 workgroups share the slot pool); K rows 0..7
    vs the f64 oracle at the f32 bar, and the segmented K within 2e-6 of max diag of the
    unsegmented one."""
    nn = 3000
    seg_default = N.kernel_variant("seg")
    pitch = N.lib().snpmi_packed_pitch(nn)
    packed = bench.Dev(N, pitch * m_edge)
    bench.synth(N, packed.p, pitch, nn, 0, m_edge, 17, 0.05)
    host = np.empty((m_edge, pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    body = np.ascontiguousarray(host[:, :(nn + 3) // 4]).reshape(-1)
    Z, _ = O.decode_standardize(body, nn, m_edge, dtype=np.float64)
    ref = Z[:R].dot(Z.T)

    def rows(s):
        N.call("snpmi_set_kernel_variant", b"seg", s)
        try:
            stats = bench.Dev(N, m_edge * 8)
            g = ShardedGrm(nn, np.float32, None, "none")
            g.add_packed(packed.p, pitch, m_edge, N.STD_UNIT, 0.0, 0.0, 0, stats.p)
            t, _ = g.tiles()
            ri = np.arange(R, dtype=np.uint64)
            dri, dout = bench.Dev(N, R * 8), bench.Dev(N, R * nn * 4)
            N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
            N.call("snpmi_dev_grm_extract", t, nn, N.DT_F32, dri.p, R, None, nn, 1, 1.0, dout.p)
            K = np.empty((R, nn), dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
            g.abort()
            for d in (stats, dri, dout):
                d.free()
            return K.astype(np.float64)
        finally:
            N.call("snpmi_set_kernel_variant", b"seg", seg_default)

    try:
        Ks, K0 = rows(seg), rows(0)
    finally:
        packed.free()
    scale = np.abs(np.diag(ref[:, :R])).max()
    assert np.abs(Ks - ref).max() / scale <= 1e-5
    assert np.abs(Ks - K0).max() / scale <= 2e-6


def test_default_f32_grm_over_200k_snps_within_2e6():
    """the default f32 GRM (fp16x2 SYRK, 12288-SNP chains, exact f64 diagonal)
    at 50,000 iids x 204,800 SnpGen-shaped SNPs (21.8% missing) through ShardedGrm in launches of
    <= 65536 SNPs, as Bed.read_kernel runs it: K rows 0..7 vs the f64 oracle within 2e-6 of max
    diag (round 3: 4.1-4.9e-6), the diagonal within 1e-6 relative."""
    nn, mm, rows = 50_000, 204_800, 8
    pitch = N.lib().snpmi_packed_pitch(nn)
    packed = bench.Dev(N, pitch * mm)
    stats = bench.Dev(N, mm * 8)
    try:
        bench.synth(N, packed.p, pitch, nn, 0, mm, 311, 0.218)
        g = ShardedGrm(nn, np.float32, None, "none")
        g.add_packed(packed.p, pitch, mm, N.STD_UNIT, 0.0, 0.0, 0, stats.p)
        t, _ = g.tiles()
        ri = np.arange(rows, dtype=np.uint64)
        dri, dout = bench.Dev(N, rows * 8), bench.Dev(N, rows * nn * 4)
        N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
        N.call("snpmi_dev_grm_extract", t, nn, N.DT_F32, dri.p, rows, None, nn, 1, 1.0, dout.p)
        K = np.empty((rows, nn), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
        g.abort()
        dri.free()
        dout.free()
        ref = np.zeros((rows, nn))
        chunk = 8192
        host = np.empty((chunk, pitch), dtype=np.uint8)
        for s0 in range(0, mm, chunk):
            c = min(chunk, mm - s0)
            N.call("snpmi_memcpy_d2h", N.ptr(host), packed.at(s0 * pitch), c * pitch)
            body = np.ascontiguousarray(host[:c, :(nn + 3) // 4]).reshape(-1)
            Z, _ = O.decode_standardize(body, nn, c, dtype=np.float64, num_threads=16)
            ref += Z[:rows].dot(Z.T)
    finally:
        packed.free()
        stats.free()
    scale = np.abs(np.diag(ref[:, :rows])).max()
    err = np.abs(K.astype(np.float64) - ref).max() / scale
    assert err <= 2e-6, err
    diag_rel = np.max(np.abs(np.diag(K[:, :rows]) - np.diag(ref[:, :rows])) / np.diag(ref[:, :rows]))
    assert diag_rel <= 1e-6, diag_rel
