"""The cfg4 K-tile collective overlapped with the SYRK (api.hip grm_add_packed_reduce,
snpmi_grm_add_packed_reduce_f32, shard.ShardedGrm.add_packed_combine): the last SNP chunk's SYRK
runs as column groups of the triangle (launch_syrk_packed_h2_cols: each kernel keeps its full-grid
block identity, so storage and SegFlush phases are unchanged) with each group's diagonal written
back before its tiles are summed on the aux stream.

* without a collective, the grouped call leaves exactly the tiles of snpmi_grm_add_packed_f32 (bit
  for bit) -- 1 to 5 groups, one or two SNP chunks, Unit / Beta(1,25) (rare-SNP weights outside
  fp16's range: the bf16x3 fallback runs inside the groups) / count_A1, use_stats;
* under a real RCCL communicator at world 1 (reduce onto 0 and all-reduce: sums over one rank),
  the same tiles again, so the ranged collectives on the aux stream cover every tile exactly once
  and the compute stream sees them finished."""
import ctypes

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from pysnptools_amd import _native as N
from pysnptools_amd import dist as D
from pysnptools_amd.shard import ShardedGrm

pytestmark = pytest.mark.gpu


def _data(n, m, seed):
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, seed, 0.05)
    return packed, pitch


def _tiles(g):
    t, count = g.tiles()
    out = np.empty(count, dtype=g.dtype)
    N.call("snpmi_stream_sync")
    N.call("snpmi_memcpy_d2h", N.ptr(out), t, out.nbytes)
    return out


def _run(n, m, packed, pitch, kind, a, b, count_a1, parts, collective, dist=None, use_stats=False, dtype=np.float32):
    stats = bench.Dev(N, m * 2 * np.dtype(dtype).itemsize)
    try:
        if use_stats:  # trained stats from a first pass
            g = ShardedGrm(n, dtype, None, "none")
            g.add_packed(packed.p, pitch, m, kind, a, b, 0, stats.p, count_a1)
            g.abort()
        g = ShardedGrm(n, dtype, dist, "none" if collective is None else collective)
        if parts is None:
            g.add_packed(packed.p, pitch, m, kind, a, b, int(use_stats), stats.p, count_a1)
        elif collective is None:
            N.call("snpmi_grm_add_packed_reduce_" + N.suffix(np.dtype(dtype)), packed.p, pitch, n, m, int(count_a1),
                   kind, a, b, int(use_stats), stats.p, 0, 0, parts, None)
        else:
            ev = ctypes.c_void_p()
            N.call("snpmi_event_create", ctypes.byref(ev))
            g.add_packed_combine(packed.p, pitch, m, kind, a, b, int(use_stats), stats.p, count_a1, parts=parts,
                                 syrk_done=ev)
            N.call("snpmi_stream_sync")
            N.call("snpmi_event_destroy", ev)
        out = _tiles(g)
        g.abort()
        return out
    finally:
        stats.free()


CASES = [(30000, 3000, "unit", False, False, 4), (30000, 70000, "unit", False, False, 3),
         (40000, 2000, "beta", False, False, 5), (33000, 1500, "unit", True, True, 2),
         (30000, 1000, "unit", False, False, 1)]


@pytest.mark.parametrize("n,m,std,count_a1,use_stats,parts", CASES)
def test_grouped_syrk_equals_whole_launch(n, m, std, count_a1, use_stats, parts):
    kind, a, b = (N.STD_UNIT, 0.0, 0.0) if std == "unit" else (N.STD_BETA, 1.0, 25.0)
    packed, pitch = _data(n, m, 41)
    try:
        ref = _run(n, m, packed, pitch, kind, a, b, count_a1, None, None, use_stats=use_stats)
        got = _run(n, m, packed, pitch, kind, a, b, count_a1, parts, None, use_stats=use_stats)
    finally:
        packed.free()
    groups = N.kernel_variant("overlap_groups")  # the grouped call ran last
    assert groups == (1 if parts == 1 else min(parts, (n + 4095) // 4096)), groups
    assert np.abs(ref).max() > 0
    assert np.array_equal(ref, got)


@pytest.fixture
def rccl1():
    d = D.init_from_env(force_rccl=True, env={"RANK": "0", "WORLD_SIZE": "1"}, timeout=120)
    try:
        yield d
    finally:
        d.close()


@pytest.mark.parametrize("collective", ["reduce", "allreduce"])
def test_overlapped_collective_world1(rccl1, collective):
    n, m = 30000, 4000
    packed, pitch = _data(n, m, 43)
    try:
        ref = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, None, None)
        got = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, 4, collective, dist=rccl1)
    finally:
        packed.free()
    assert N.kernel_variant("overlap_groups") == 4
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("n,m,std", [(30000, 3000, "unit"), (20000, 70000, "beta")])
def test_f64_crt_chunks_equal_whole_launch(n, m, std):
    """f64: the CRT path's residue chunks cut at block-column boundaries (the overlap groups) give
    the tiles of the plain call bit for bit (one or two SNP chunks)."""
    kind, a, b = (N.STD_UNIT, 0.0, 0.0) if std == "unit" else (N.STD_BETA, 1.0, 25.0)
    packed, pitch = _data(n, m, 47)
    try:
        ref = _run(n, m, packed, pitch, kind, a, b, False, None, None, dtype=np.float64)
        got = _run(n, m, packed, pitch, kind, a, b, False, 2, None, dtype=np.float64)
    finally:
        packed.free()
    nb = (n + 255) // 256
    assert N.kernel_variant("overlap_groups") >= (2 if nb * (nb + 1) // 2 * 15 * 65536 > (4 << 30) else 1)
    assert np.abs(ref).max() > 0
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("collective", ["reduce", "allreduce"])
def test_overlapped_collective_world1_f64(rccl1, collective):
    n, m = 30000, 2000
    packed, pitch = _data(n, m, 53)
    try:
        ref = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, None, None, dtype=np.float64)
        got = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, 2, collective, dist=rccl1, dtype=np.float64)
    finally:
        packed.free()
    assert N.kernel_variant("overlap_groups") >= 2
    assert np.array_equal(ref, got)


def _write_bed(path, n, m, seed):
    rng = np.random.default_rng(seed)
    bpc = (n + 3) // 4
    codes = rng.choice(np.array([0, 1, 2, 3], dtype=np.uint8), size=(m, bpc * 4), p=[0.3, 0.05, 0.35, 0.3])
    codes[:, n:] = 0
    body = (codes[:, 0::4] | (codes[:, 1::4] << 2) | (codes[:, 2::4] << 4) | (codes[:, 3::4] << 6)).astype(np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(body.tobytes())
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("collective", ["reduce", "allreduce"])
def test_grm_sharded_bed_overlapped_world1(rccl1, tmp_path, dtype, collective):
    """shard.grm_sharded from a .bed under a real RCCL communicator: the file stream's last chunk
    runs as column groups (f32) / column-aligned CRT chunks (f64) with the tiles summed on the aux
    stream (snpmi_grm_add_bed_reduce_*); K and the trained stats equal the unoverlapped call
    (collective "none" at world 1) bit for bit."""
    from pysnptools_amd import shard
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    path = str(tmp_path / "w")
    _write_bed(path, 30000, 3000, 61)
    bed = Bed(path, count_A1=False)
    K1, t1, _ = shard.grm_sharded(bed, Unit(), dtype=dtype, collective=collective, dist=rccl1)
    groups = N.kernel_variant("overlap_groups")
    K0, t0, _ = shard.grm_sharded(bed, Unit(), dtype=dtype, collective="none", dist=rccl1)
    assert groups >= 2, groups
    assert np.array_equal(K1, K0)
    np.testing.assert_array_equal(t1.stats, t0.stats)


def _calls():
    return N.kernel_variant("overlap_calls"), N.kernel_variant("overlap_sig")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n", [30000, 6144])
def test_collective_calls_do_not_depend_on_the_ranks_snp_count(rccl1, n, dtype):
    """every rank must issue the same RCCL calls.  Ranks' spans differ by one SNP
    and may straddle a split-K threshold (n = 6144: 1500 SNPs fit one 256-block grid round unsplit,
    3000 SNPs would pick a split grid), and a rank may own no SNPs at all -- the ranged sums
    (count and element ranges) are the same in every case, and K is unchanged by how they ran."""
    sigs = {}
    for m in (1, 700, 1500, 3000, 70000):
        packed, pitch = _data(n, m, 67)
        try:
            ref = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, None, None, dtype=dtype)
            got = _run(n, m, packed, pitch, N.STD_UNIT, 0.0, 0.0, False, 2, "allreduce", dist=rccl1, dtype=dtype)
            sigs[m] = _calls()
        finally:
            packed.free()
        assert np.array_equal(ref, got), m
    g = ShardedGrm(n, dtype, rccl1, "allreduce")  # a rank without SNPs: its zero tiles join the sums
    try:
        g.combine(2)
        sigs[0] = _calls()
        assert not np.any(_tiles(g))
    finally:
        g.abort()
    assert len(set(sigs.values())) == 1, sigs
    calls = sigs[0][0]
    nb = (n + 255) // 256
    if dtype == np.float32:
        assert calls == (2 if n == 30000 else 1), calls  # n = 6144 picks split grids: no column groups
    else:
        assert calls >= (2 if nb * (nb + 1) // 2 * 15 * 65536 > (4 << 30) else 1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_bed_rank_without_snps_issues_the_same_calls(rccl1, tmp_path, dtype):
    """The .bed path: a rank whose span is empty (add_bed_combine with no SNPs) issues the calls of a
    rank that streams SNPs."""
    from pysnptools_amd.snpreader import Bed

    path = str(tmp_path / "e")
    _write_bed(path, 30000, 700, 71)
    bed = Bed(path, count_A1=False)
    sigs = []
    for cols in (np.arange(700, dtype=np.uint64), np.arange(3, dtype=np.uint64), np.zeros(0, dtype=np.uint64)):
        g = ShardedGrm(30000, dtype, rccl1, "reduce")
        stats = np.zeros((len(cols), 2), dtype=dtype)
        try:
            g.add_bed_combine(bed, None, cols, N.STD_UNIT, 0.0, 0.0, 0, stats)
            sigs.append(_calls())
        finally:
            g.abort()
    assert sigs[0] == sigs[1] == sigs[2], sigs
