"""SnpMemMap / PstMemMap (reference snpreader/snpmemmap.py, pstreader/pstmemmap.py).

CPU: the reference's TestSnpMemMap.test1 / TestPstMemMap.test1 flows (empty -> fill -> slice ->
flush -> reopen), the reference-shipped fixtures tiny.snp.memmap (format version 1) and
tiny.pst.memmap (version 2) read WITHOUT unpickling their object records, and a header that
would need code execution is refused.  GPU: SnpMemMap.write of a Bed streams decode +
standardize blocks through the HIP path; the file equals the oracle's per-block result."""
import io
import os
import pickle

import numpy as np
import pytest

from conftest import DATA
from oracle import oracle as O
from pysnptools_amd.pstreader import PstMemMap
from pysnptools_amd.pstreader.pstmemmap import _load_record
from pysnptools_amd.snpreader import Bed, SnpData, SnpMemMap
from pysnptools_amd.standardizer import Unit


def test_snpmemmap_empty_fill_reopen(tmp_path):
    """snpmemmap.py:250-275 (TestSnpMemMap.test1, first half)."""
    fn = str(tmp_path / "tiny.snp.memmap")
    s2 = SnpMemMap.empty(iid=[["fam0", "iid0"], ["fam0", "iid1"]], sid=["snp334", "snp349", "snp921"], filename=fn,
                         order="F", dtype=np.float64)
    assert isinstance(s2.val, np.memmap)
    s2.val[:, :] = [[0., 2., 0.], [0., 1., 2.]]
    assert np.array_equal(s2[[1], [1]].read(view_ok=True).val, np.array([[1.]]))
    s2.flush()
    assert isinstance(s2.val, np.memmap)
    assert np.array_equal(s2[[1], [1]].read(view_ok=True).val, np.array([[1.]]))
    s2.flush()
    s3 = SnpMemMap(fn)
    assert np.array_equal(s3[[1], [1]].read(view_ok=True).val, np.array([[1.]]))
    assert isinstance(s3.val, np.memmap)
    assert s3.iid_count == 2 and s3.sid_count == 3
    snpdata = s3.read(view_ok=True)
    assert isinstance(snpdata.val, np.memmap)
    assert np.array_equal(s3.read(order="C", dtype=np.float32).val, np.array([[0., 2., 0.], [0., 1., 2.]], np.float32))
    assert np.array_equal(s3[:, ::2].read().val, np.array([[0., 0.], [0., 2.]]))
    assert repr(s3) == "SnpMemMap('%s')" % fn
    assert list(s3.sid) == ["snp334", "snp349", "snp921"] and s3.iid[1, 1] == "iid1"


def test_pstmemmap_empty_and_write(tmp_path):
    """pstmemmap.py:345-375 (TestPstMemMap.test1) + PstMemMap.write round trip, C order, val_shape."""
    fn = str(tmp_path / "tiny.pst.memmap")
    p2 = PstMemMap.empty(row=["a", "b", "c"], col=["y", "z"], filename=fn, row_property=["A", "B", "C"], order="F",
                         dtype=np.float64)
    p2.val[:, :] = [[1, 2], [3, 4], [np.nan, 6]]
    assert np.array_equal(p2[[0], [0]].read(view_ok=True).val, np.array([[1.]]))
    p2.flush()
    p3 = PstMemMap(fn)
    assert np.array_equal(p3[[0], [0]].read(view_ok=True).val, np.array([[1.]]))
    assert list(p3.row_property) == ["A", "B", "C"]
    from pysnptools_amd.pstreader import PstData
    for order in ("F", "C"):
        v = np.asarray(np.arange(24, dtype=np.float32).reshape(4, 3, 2), order=order)
        pd = PstData(row=list("abcd"), col=list("xyz"), val=v)
        out = PstMemMap.write(str(tmp_path / ("w%s.pst.memmap" % order)), pd)
        back = PstMemMap(out.filename)
        assert back.val.dtype == np.float32 and back.val.shape == (4, 3, 2)
        assert np.array_equal(np.asarray(back.val), v) and back.val.flags[order + "_CONTIGUOUS"]


def test_reference_fixtures_read_without_unpickling():
    """Reference-shipped files (examples/tiny.snp.memmap: version 1; tiny.pst.memmap: version 2):
    values from their doctests (snpmemmap.py:31-35, pstmemmap.py:24-28)."""
    s = SnpMemMap(os.path.join(DATA, "tiny.snp.memmap"))
    assert s.val[0, 1] == 2.0 and s.iid_count == 2 and s.sid_count == 3
    assert s.val.dtype == np.float64 and list(s.sid) == ["snp334", "snp349", "snp921"]
    p = PstMemMap(os.path.join(DATA, "tiny.pst.memmap"))
    assert p.val[0, 1] == 2.0 and p.row_count == 3 and p.col_count == 2


def test_object_record_that_needs_execution_is_refused():
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    buf = io.BytesIO()
    np.save(buf, np.array([Evil()], dtype=object), allow_pickle=True)
    buf.seek(0)
    with pytest.raises(ValueError):
        _load_record(buf)
    # the benign records the format uses are understood
    for val, want in ((np.dtype(np.float32), np.dtype(np.float32)), (None, None), (3, 3)):
        b = io.BytesIO()
        np.save(b, np.array([val], dtype=object), allow_pickle=True)
        b.seek(0)
        assert _load_record(b)[0] == want
    assert pickle is not None


@pytest.mark.gpu
@pytest.mark.parametrize("order,dtype", [("F", np.float32), ("C", np.float64)])
def test_snpmemmap_write_bed_streams_gpu_blocks(tmp_path, order, dtype):
    """SnpMemMap.write(fn, bed, Unit(), block_size=b): each block of SNPs decoded and
    standardized on the GPU (its own stats, as snpmemmap.py:222-226) == oracle per block."""
    b = Bed(os.path.join(DATA, "n300.bed"), count_A1=False)
    out = SnpMemMap.write(str(tmp_path / "n300.snp.memmap"), b[:, 7:407], standardizer=Unit(), order=order,
                          dtype=dtype, block_size=96)
    body = O.read_bed_bytes(os.path.join(DATA, "n300.bed"))
    for s0 in range(0, 400, 96):
        cols = np.arange(7 + s0, 7 + min(s0 + 96, 400))
        ref = O.decode(body, 300, 1015, sid_index=cols, dtype=dtype)
        O.standardize_native(ref)
        got = np.asarray(out.val[:, s0:s0 + len(cols)])
        np.testing.assert_array_equal(got, ref)
    assert out.val.flags[order + "_CONTIGUOUS"] and out.val.dtype == dtype
    assert list(out.sid[:2]) == list(b.sid[7:9]) and np.array_equal(out.pos, b.pos[7:407], equal_nan=True)
    # the memmap is a SnpReader: its GRM through the dense path == Z Z^T of the file
    K = out.read_kernel(Unit(), dtype=np.float64).val
    Z = np.array(out.val, dtype=np.float64)
    O.standardize_native(Z)
    np.testing.assert_allclose(K, Z.dot(Z.T), rtol=1e-9, atol=1e-6 * np.abs(np.diag(K)).max())


@pytest.mark.gpu
def test_snpmemmap_write_snpdata_whole(tmp_path):
    """In-memory input: standardized whole, then copied (snpmemmap.py:216-218)."""
    rng = np.random.default_rng(3)
    v = rng.integers(0, 3, size=(50, 30)).astype(np.float64)
    v[rng.random(v.shape) < 0.1] = np.nan
    d = SnpData(iid=[["f", str(i)] for i in range(50)], sid=["s%d" % j for j in range(30)], val=v.copy())
    out = SnpMemMap.write(str(tmp_path / "d.snp.memmap"), d, standardizer=Unit())
    ref = v.copy(order="F")
    O.standardize_native(ref)
    np.testing.assert_array_equal(np.asarray(out.val), ref)
