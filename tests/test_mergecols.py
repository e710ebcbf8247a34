"""Generic column merge (reference pstreader/_mergecols.py:8-159).  CPU: metadata, checks and
the no-pickle cache; GPU: reads across pieces (2-D and 3-D values, subsets, F/C) against NumPy."""
import numpy as np
import pytest

from pysnptools_amd.pstreader import PstData, _MergeCols


def _pieces(k=None, seed=0):
    rng = np.random.default_rng(seed)
    rows = [["f", "i%d" % i] for i in range(7)]
    out, vals = [], []
    start = 0
    for w in (3, 1, 4):
        v = rng.standard_normal((7, w) if k is None else (7, w, k))
        cols = [["c", str(start + j)] for j in range(w)]
        out.append(PstData(row=rows, col=cols, val=v, col_property=np.arange(start, start + w, dtype=float)))
        vals.append(v)
        start += w
    return out, np.concatenate(vals, axis=1)


def test_mergecols_metadata_and_checks(tmp_path):
    pieces, _ = _pieces()
    m = _MergeCols(pieces)
    assert m.row_count == 7 and m.col_count == 8 and list(m.col_count_list) == [3, 1, 4]
    assert np.array_equal(m.col[:, 1], [str(j) for j in range(8)])
    assert np.array_equal(m.col_property, np.arange(8.0))
    assert repr(m).startswith("_MergeCols(")
    with pytest.raises(AssertionError):  # duplicate columns
        _MergeCols([pieces[0], pieces[0]]).col
    other = PstData(row=[["g", str(i)] for i in range(7)], col=[["x", "y"]], val=np.zeros((7, 1)))
    with pytest.raises(AssertionError):  # rows differ
        _MergeCols([pieces[0], other]).row
    assert _MergeCols([pieces[0], pieces[0]], skip_check=True).col_count == 6
    cache = str(tmp_path / "m.npz")
    a = _MergeCols(pieces, cache_file=cache)
    b = _MergeCols(pieces, cache_file=cache)  # loaded from the cache, allow_pickle=False
    assert np.array_equal(a.col, b.col) and np.array_equal(a.row, b.row)
    assert np.array_equal(a.col_count_list, b.col_count_list)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [None, 2])
@pytest.mark.parametrize("order", ["F", "C", "A"])
def test_mergecols_reads_across_pieces(k, order):
    pieces, full = _pieces(k, seed=3)
    m = _MergeCols(pieces)
    got = m.read(order=order, dtype=np.float64).val
    assert np.array_equal(got, full)
    for ri, ci in ((slice(None, None, -2), [7, 0, 3, 4]), ([5, 1], slice(2, 5)), (slice(None), [6])):
        sub = m[ri, ci].read(order=order, dtype=np.float32).val
        rows, cols = np.arange(7)[ri], np.arange(8)[ci]
        assert np.array_equal(sub, full[np.ix_(rows, cols)].astype(np.float32))
