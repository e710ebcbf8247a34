"""Host-side logic of the mirrored PySnpTools API (no GPU): metadata, index algebra,
subset composition, standardizer bookkeeping and the BED writer."""
import os
import shutil
import tempfile

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from oracle import oracle as O
from pysnptools_amd.pstreader import PstReader
from pysnptools_amd.snpreader import Bed, SnpData
from pysnptools_amd.snpreader.snpreader import _resolve
from pysnptools_amd.standardizer import Beta, BetaTrained, Identity, Unit, UnitTrained
from pysnptools_amd.kernelreader import SnpKernel


def bed(name="n300", **kw):
    return Bed(os.path.join(DATA, name + ".bed"), count_A1=False, **kw)


def test_metadata():
    b = bed()
    assert b.iid_count == 300 and b.sid_count == 1015
    assert b.iid.shape == (300, 2) and b.iid.dtype.type is np.str_
    assert b.pos.shape == (1015, 3)
    assert np.isnan(b.pos[0, 2])  # bp 0 -> NaN (bed.py:188-192)
    t = bed("toydata")
    assert t.iid_count == 500 and t.sid_count == 10000
    assert str(b) == "Bed('%s',count_A1=False)" % os.path.join(DATA, "n300.bed")


def test_count_a1_default_warns():
    with pytest.warns(FutureWarning):
        Bed(os.path.join(DATA, "n300.bed"))


def test_chrom_map_and_bad_chrom():
    with tempfile.TemporaryDirectory() as d:
        for ext in ("bed", "fam"):
            shutil.copy(os.path.join(DATA, "dist_x." + ext), os.path.join(d, "x." + ext))
        lines = open(os.path.join(DATA, "dist_x.bim")).read().splitlines()
        fields = [l.split() for l in lines]
        fields[0][0], fields[1][0], fields[2][0] = "X", "MT", "0"
        with open(os.path.join(d, "x.bim"), "w") as f:
            f.write("\n".join("\t".join(x) for x in fields) + "\n")
        b = Bed(os.path.join(d, "x.bed"), count_A1=False)
        assert b.pos[0, 0] == 23 and b.pos[1, 0] == 26 and np.isnan(b.pos[2, 0])
        fields[3][0] = "chrBAD"
        with open(os.path.join(d, "x.bim"), "w") as f:
            f.write("\n".join("\t".join(x) for x in fields) + "\n")
        with pytest.raises(ValueError):
            Bed(os.path.join(d, "x.bed"), count_A1=False).pos  # test.py:268-278


def test_index_algebra():
    mk = PstReader._make_sparray_or_slice
    arr = PstReader._make_sparray_from_sparray_or_slice
    assert mk(None) == slice(None)
    assert np.array_equal(mk(3), [3])
    assert np.array_equal(mk([True, False, True]), [0, 2])
    assert np.array_equal(arr(10, mk(slice(None, None, -3))), [9, 6, 3, 0])
    assert np.array_equal(arr(10, mk([-1, 0])), [9, 0])
    assert arr(10, mk([])).size == 0
    with pytest.raises(AssertionError):
        mk(1.5)


def test_subset_composition_matches_numpy():
    b = bed()
    s = b[:, ::2][:, ::2][:, ::2][:, ::2]  # snpreader.py:160-170 -> ::16
    base, rows, cols = _resolve(s)
    assert base is b and rows is None
    assert np.array_equal(cols, np.arange(0, 1015, 16))
    s2 = b[::-2, [5, 3, 1]][[0, 2], :]
    base, rows, cols = _resolve(s2)
    assert np.array_equal(rows, np.arange(299, -1, -2)[[0, 2]])
    assert np.array_equal(cols, [5, 3, 1])
    assert np.array_equal(s2.iid, b.iid[::-2][[0, 2]])
    assert np.array_equal(s2.sid, b.sid[[5, 3, 1]])


def test_snpdata_construction_and_repr():
    d = SnpData(iid=[["a", "1"], ["b", "2"]], sid=["s1", "s2", "s3"], val=[[0, 1, 2], [2, 1, np.nan]])
    assert d.val.dtype == np.float64 and d.pos.shape == (3, 3)
    assert repr(d) == "SnpData()"
    with pytest.raises(AssertionError):
        SnpData(iid=[["a", "1"]], sid=["s1"], val=[[0, 1]])
    assert d[:, 1:].sid_count == 2


def test_trained_stats_remap():
    tr = UnitTrained(np.array(["a", "b", "c"]), np.array([[0.1, 1.0], [0.2, 2.0], [0.3, 3.0]]))
    assert np.array_equal(tr.stats_for(np.array(["c", "a"])), [[0.3, 3.0], [0.1, 1.0]])
    bt = BetaTrained(1, 25, np.array(["a", "b"]), np.zeros((2, 2)))
    with pytest.raises(AssertionError):
        bt.stats_for(np.array(["b", "a"]))
    merged = Unit()._merge_trained([tr, UnitTrained(np.array(["d"]), np.array([[0.4, 4.0]]))])
    assert merged.stats.shape == (4, 2) and list(merged.sid) == ["a", "b", "c", "d"]
    assert Beta(1, 25)._merge_trained([bt]).a == 1
    assert UnitTrained(["x"], np.zeros((1, 2))).is_constant and not Unit().is_constant
    assert Identity().is_constant


def test_snpkernel_pushdown_rules():
    b = bed()
    k = SnpKernel(b, Unit())
    assert not isinstance(k[::2], SnpKernel)  # non-constant standardizer: subset after the GRM
    tr = UnitTrained(b.sid, np.ones((b.sid_count, 2)))
    k2 = SnpKernel(b, tr)[[1, 2, 3]]
    assert isinstance(k2, SnpKernel) and k2.iid_count == 3  # constant: pushed down (snpkernel.py:98-99)


def test_bed_reader_compat_surface():
    """The shim exposes every bed_reader name PySnpTools imports, with metadata parsing."""
    import inspect

    import pysnptools_amd.bed_reader_compat as br

    for name in ("open_bed", "to_bed", "standardize_f32", "standardize_f64", "subset_f64_f64", "subset_f32_f64",
                 "subset_f32_f32", "get_num_threads"):
        assert hasattr(br, name)
    assert list(inspect.signature(br.standardize_f32).parameters) == [
        "val", "is_beta", "a", "b", "apply_in_place", "use_stats", "stats", "num_threads"]
    with br.open_bed(os.path.join(DATA, "n300.bed"), count_A1=False) as ob:
        assert ob.iid_count == 300 and ob.sid_count == 1015
        assert ob.fid[0] == "POP1" and len(ob.sid) == 1015 and ob.chromosome[0] == "1"
    assert br.get_num_threads(3) == 3


@pytest.mark.parametrize("n,world", [(1, 1), (256, 2), (300, 3), (1000, 4), (5000, 8), (500000, 8)])
def test_grm_partition_covers_upper_triangle_once(n, world):
    """cfg5 block ownership (snpmi_grm_part_*): disjoint, complete, balanced (pure host arithmetic);
    whole supertiles are dealt, so the balance is by supertile (at 500k iids x 8 parts within 1%)."""
    import ctypes

    from pysnptools_amd import _native as N

    nb = (n + 255) // 256
    total = nb * (nb + 1) // 2
    counts = [N.lib().snpmi_grm_part_blocks(n, r, world) for r in range(world)]
    assert sum(counts) == total
    if n == 500000:
        assert max(counts) / min(counts) < 1.01, counts
    if total > 20000:
        return
    seen = set()
    r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
    for r in range(world):
        for b in range(counts[r]):
            N.call("snpmi_grm_part_coords", n, r, world, b, ctypes.byref(r0), ctypes.byref(c0))
            assert r0.value <= c0.value and c0.value < nb * 256
            seen.add((r0.value, c0.value))
    assert len(seen) == total


def test_array_module_seam():
    """util/__init__.py:652-730: numpy default, 'hbm' = the device module, 'cupy' falls back to
    numpy when CuPy is absent (it is, in this image), unknown names raise."""
    import types

    from pysnptools_amd import _native as N
    from pysnptools_amd import hbm
    from pysnptools_amd.util import array_module, asnumpy, get_array_module

    assert array_module() is np and array_module("numpy") is np and array_module(np) is np
    assert array_module("hbm") is hbm and hbm.ndarray is hbm.HbmArray
    assert array_module("cupy") is np
    with pytest.raises(ValueError):
        array_module("tensorflow")
    a = np.arange(6.0).reshape(2, 3)
    assert asnumpy(a) is a and get_array_module(a) is np
    # the ctypes binding passes a device buffer's own address, a NumPy array's data pointer
    fake = types.SimpleNamespace(snpmi_ptr=N.ctypes.c_void_p(0x1234))
    assert N.ptr(fake).value == 0x1234 and N.ptr(a).value == a.ctypes.data


def test_array_module_env(monkeypatch):
    from pysnptools_amd import hbm
    from pysnptools_amd.util import _on_device, array_module

    monkeypatch.setenv("ARRAY_MODULE", "hbm")
    assert array_module() is hbm and _on_device()
    monkeypatch.setenv("ARRAY_MODULE", "numpy")
    assert not _on_device(None, np.zeros(2))


def test_bed_gather_packed_host_only():
    """snpmi_bed_gather_packed (the per-rank share gather of the cfg5 plan) is host code: the
    selected columns' bytes exactly as in the file, zero-padded to the pitch, index errors raised."""
    from pysnptools_amd import _native as N

    path = os.path.join(DATA, "n300.bed")
    n, m = 300, 1015
    body = O.read_bed_bytes(path)
    bpc = (n + 3) // 4
    cols = np.array([1014, 0, 7, 7, 500], dtype=np.uint64)
    pitch = N.lib().snpmi_packed_pitch(n)
    out = np.full((len(cols), pitch), 0xCD, dtype=np.uint8)
    N.call("snpmi_bed_gather_packed", path.encode(), n, m, N.ptr(cols), len(cols), pitch, N.ptr(out), 2)
    ref = np.frombuffer(body, dtype=np.uint8).reshape(m, bpc)[cols.astype(np.int64)]
    np.testing.assert_array_equal(out[:, :bpc], ref)
    assert not out[:, bpc:].any()
    with pytest.raises(IndexError):
        N.call("snpmi_bed_gather_packed", path.encode(), n, m, N.ptr(np.array([m], dtype=np.uint64)), 1, pitch,
               N.ptr(out), 1)
    with pytest.raises(ValueError):
        N.call("snpmi_bed_gather_packed", path.encode(), n, m + 1, None, 1, pitch, N.ptr(out), 1)


@pytest.mark.parametrize("n,parts", [(1, 1), (300, 1), (300, 3), (5000, 8), (70001, 7)])
def test_part_coords_match_the_library(n, parts):
    """shard.part_coords (vectorised) == snpmi_grm_part_coords for every local block of every part,
    and the parts tile the upper triangle of 256-blocks exactly once (host code, no GPU)."""
    import ctypes

    from pysnptools_amd import _native as N
    from pysnptools_amd.shard import part_coords

    nb = (n + 255) // 256
    seen = set()
    r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
    for part in range(parts):
        co = part_coords(n, part, parts)
        for k in range(len(co)):
            N.call("snpmi_grm_part_coords", n, part, parts, k, ctypes.byref(r0), ctypes.byref(c0))
            assert (r0.value, c0.value) == tuple(co[k])
            seen.add(tuple(co[k]))
    assert seen == {(256 * i, 256 * j) for j in range(nb) for i in range(j + 1)}


@pytest.mark.parametrize("n,parts", [(500000, 8), (50000, 8), (5000, 8), (70001, 7), (300, 3)])
def test_parts_own_whole_supertiles(n, parts):
    """The ownership unit: S x S-block supertiles (S = 16 when each part gets >= 4 of them, smaller
    otherwise) dealt round-robin in triangular order; a part's blocks are stored supertile by
    supertile, block column by block column inside, so consecutive workgroups share code panels."""
    from pysnptools_amd.shard import part_coords

    nb = (n + 255) // 256
    S = next((s for s in (16, 8, 4, 2) if -(-nb // s) * (-(-nb // s) + 1) // 2 >= 4 * parts), 1)
    if n >= 50000:
        assert S == 16
    for part in range(parts):
        co = part_coords(n, part, parts) // 256
        if not len(co):
            continue
        I, J = co[:, 0] // S, co[:, 1] // S
        T = J * (J + 1) // 2 + I
        assert np.all(T % parts == part)
        assert np.all(np.diff(T) >= 0)  # supertiles in triangular order, each contiguous
        same = np.diff(T) == 0
        key = co[:, 1] * nb + co[:, 0]  # column by column inside a supertile
        assert np.all(np.diff(key)[same] > 0)


@pytest.mark.parametrize("m,block,first", [(0, 32768, None), (1, 32768, None), (106496, 32768, None),
                                           (1_000_000, 32768, None), (1000, 97, None), (50, 97, 50), (7, 1, None)])
def test_block_spans_cover_the_stream(m, block, first):
    """shard.block_spans (cfg5's stream plan): a quarter-size first block, then full blocks, covering
    [0, m) once in order."""
    from pysnptools_amd.shard import block_spans

    spans = block_spans(m, block, first)
    assert sum(c for _, c in spans) == m
    assert all(s0 == sum(c for _, c in spans[:k]) for k, (s0, _) in enumerate(spans))
    if spans:
        assert spans[0][1] == min(m, first or max(1, block // 4))
        assert all(0 < c <= block for _, c in spans)
        assert all(c == block for _, c in spans[1:-1])
    if (m, block) == (1_000_000, 32768):
        assert len(spans) == 32
