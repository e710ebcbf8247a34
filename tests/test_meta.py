""".fam/.bim parsing in C against a plain-Python restatement of the
whitespace-split PLINK format and the reference fixtures.  Host-only: runs without a GPU."""
import os
import tempfile

import numpy as np
import pytest

from conftest import DATA
from pysnptools_amd.snpreader import Bed
from pysnptools_amd.snpreader.bed import _text_f64, _text_scan, _text_strings


def py_columns(path):
    with open(path, encoding="utf-8") as f:
        return [line.split() for line in f if line.strip()]


@pytest.mark.parametrize("name", ["n300", "snpgen", "dist_x", "toydata", "gen1", "gen4"])
def test_fixture_metadata_matches_python_split(name):
    b = Bed(os.path.join(DATA, name + ".bed"), count_A1=False)
    fam = py_columns(os.path.join(DATA, name + ".fam"))
    bim = py_columns(os.path.join(DATA, name + ".bim"))
    assert np.array_equal(b.iid, np.array([[r[0], r[1]] for r in fam], dtype=str))
    assert np.array_equal(b.sid, np.array([r[1] for r in bim], dtype=str))
    cm = np.array([float(r[2]) for r in bim])
    bp = np.array([float(r[3]) for r in bim])
    cm[cm == 0] = np.nan
    bp[bp == 0] = np.nan
    np.testing.assert_array_equal(b.pos[:, 1], cm)
    np.testing.assert_array_equal(b.pos[:, 2], bp)


def test_whitespace_blank_lines_crlf_unicode_and_no_final_newline():
    text = "  a1\tb1 0 0 1 -9\r\n\n\nfam2   été 0 0 2 1\n\t\n x y 0 0 0 0"
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "t.fam")
        with open(p, "w", encoding="utf-8", newline="") as f:
            f.write(text)
        rows, w = _text_scan(p, 2, 2)
        assert rows == 3
        assert list(_text_strings(p, 0, rows, w[0])) == ["a1", "fam2", "x"]
        assert list(_text_strings(p, 1, rows, w[1])) == ["b1", "été", "y"]
        np.testing.assert_array_equal(_text_f64(p, 5, rows), [-9, 1, 0])


def test_errors_map_to_value_error():
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "t.bim")
        with open(p, "w") as f:
            f.write("1 s1 0 10 A C\n1 s2 0.5\n")
        with pytest.raises(ValueError):
            _text_scan(p, 4, 2)
        with open(p, "w") as f:
            f.write("1 s1 0 10 A C\n1 s2 zero 11 A C\n")
        rows, _ = _text_scan(p, 4, 2)
        with pytest.raises(ValueError):
            _text_f64(p, 2, rows)
        with pytest.raises(IOError):
            _text_scan(os.path.join(d, "missing.bim"), 4, 2)
        open(p, "w").close()
        assert _text_scan(p, 4, 2)[0] == 0


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_large_file_threaded_split(threads):
    """Line ranges cut per thread must neither drop nor duplicate lines (200k-line .bim)."""
    rng = np.random.default_rng(threads)
    n = 200_000
    chrom = rng.integers(1, 27, n)
    bp = rng.integers(1, 10**9, n)
    cm = np.round(rng.random(n) * 100, 4)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "big.bim")
        with open(p, "w") as f:
            for i in range(n):
                f.write("%d\trs%d\t%r\t%d\tA\tG\n" % (chrom[i], i, float(cm[i]), bp[i]))
        rows, w = _text_scan(p, 4, 2, threads)
        assert rows == n
        sid = _text_strings(p, 1, rows, w[1], threads)
        assert sid[0] == "rs0" and sid[-1] == "rs%d" % (n - 1)
        assert np.array_equal(sid, np.array(["rs%d" % i for i in range(n)]))
        np.testing.assert_array_equal(_text_f64(p, 3, rows, threads), bp.astype(np.float64))
        np.testing.assert_array_equal(_text_f64(p, 2, rows, threads), cm)
