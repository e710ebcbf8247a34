"""A ``bed_reader``-compatible module over libsnpmi -- the reference-side binding.

PySnpTools imports five things from the Rust/PyO3 package ``bed_reader``:
``open_bed`` (bed.py:137-145, 337-343; snpreader.py:720,735), ``to_bed`` (bed.py:300-314),
``standardize_f32/f64`` (standardizer.py:114,120), ``subset_f64_f64/f32_f64/f32_f32``
(util/__init__.py:341-375) and ``get_num_threads`` (util/__init__.py:335).  This module
provides exactly those names with the same call signatures, backed by the HIP C ABI, so
an unmodified PySnpTools can run its hot path on MI355X::

    import sys, pysnptools_amd.bed_reader_compat as br
    sys.modules["bed_reader"] = br          # before `import pysnptools`

(see INTEGRATION.md).  Only the features PySnpTools uses are provided.
"""
import os

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.util import get_num_threads as _policy

__all__ = ["open_bed", "to_bed", "standardize_f32", "standardize_f64", "subset_f64_f64", "subset_f32_f64",
           "subset_f32_f32", "get_num_threads"]


def get_num_threads(num_threads=None):
    return _policy(num_threads)


def _columns(path, ncols=6):
    """The 6 whitespace-delimited PLINK columns of a .fam/.bim as str arrays (C parser)."""
    from pysnptools_amd.snpreader.bed import _text_scan, _text_strings

    rows, w = _text_scan(path, ncols, ncols)
    if rows == 0:
        return []
    return [_text_strings(path, c, rows, w[c]) for c in range(ncols)]


class open_bed(object):
    """Subset of bed-reader's ``open_bed``: metadata properties + ``read``."""

    def __init__(self, filepath, iid_count=None, sid_count=None, properties={}, count_A1=True, num_threads=None,
                 skip_format_check=False, fam_filepath=None, bim_filepath=None):
        self.filepath = str(filepath)
        base = self.filepath[:-4] if self.filepath.lower().endswith(".bed") else self.filepath
        self._fam = str(fam_filepath) if fam_filepath else base + ".fam"
        self._bim = str(bim_filepath) if bim_filepath else base + ".bim"
        self.count_A1 = count_A1
        self._num_threads = num_threads
        self._props = dict(properties)
        self._fam_cols = None
        self._bim_cols = None
        self._iid_count = iid_count
        self._sid_count = sid_count
        self._checked = skip_format_check

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def _famc(self):
        if self._fam_cols is None:
            self._fam_cols = _columns(self._fam)
        return self._fam_cols

    def _bimc(self):
        if self._bim_cols is None:
            self._bim_cols = _columns(self._bim)
        return self._bim_cols

    def _prop(self, name, fam, col, conv=None):
        # given properties are converted to bed-reader's dtypes too (str / float32 / int32)
        if self._props.get(name) is not None:
            v = np.asarray(self._props[name])
            return conv(v) if conv else v.astype(str)
        cols = self._famc() if fam else self._bimc()
        v = cols[col] if cols else np.empty(0, dtype=str)
        return conv(v) if conv else v

    @property
    def fid(self):
        return self._prop("fid", True, 0)

    @property
    def iid(self):
        return self._prop("iid", True, 1)

    @property
    def sid(self):
        return self._prop("sid", False, 1)

    @property
    def chromosome(self):
        return self._prop("chromosome", False, 0)

    @property
    def cm_position(self):
        return self._prop("cm_position", False, 2, lambda v: v.astype(np.float32))

    @property
    def bp_position(self):
        return self._prop("bp_position", False, 3, lambda v: v.astype(np.float64).astype(np.int32))

    @property
    def iid_count(self):
        return self._iid_count if self._iid_count is not None else len(self.iid)

    @property
    def sid_count(self):
        return self._sid_count if self._sid_count is not None else len(self.sid)

    def read(self, index=None, dtype="float32", order="F", force_python_only=False, num_threads=None):
        dtype = np.dtype(dtype)
        if not self._checked:
            N.call("snpmi_bed_check", self.filepath.encode(), self.iid_count, self.sid_count)
            self._checked = True
        iid_index, sid_index = (None, None) if index is None else index
        ri = None if iid_index is None else N.index_array(np.arange(self.iid_count)[iid_index])
        ci = None if sid_index is None else N.index_array(np.arange(self.sid_count)[sid_index])
        n = self.iid_count if ri is None else len(ri)
        m = self.sid_count if ci is None else len(ci)
        out = np.empty((n, m), dtype=dtype, order=order)
        N.call("snpmi_bed_read_" + N.suffix(dtype), self.filepath.encode(), self.iid_count, self.sid_count,
               int(bool(self.count_A1)), N.ptr(ri), n, N.ptr(ci), m, 1 if order == "C" else 0, N.ptr(out),
               get_num_threads(num_threads if num_threads is not None else self._num_threads))
        return out


def to_bed(filepath, val, properties={}, count_A1=True, fam_filepath=None, bim_filepath=None,
           force_python_only=False, num_threads=None):
    """Write a .bed/.fam/.bim triple (SNP-major)."""
    from pysnptools_amd.snpreader import SnpData
    from pysnptools_amd.snpreader._write import write_bed

    val = np.asarray(val)
    n, m = val.shape
    fid = properties.get("fid", ["0"] * n)
    iid = properties.get("iid", [str(i + 1) for i in range(n)])
    sid = properties.get("sid", ["sid%d" % (j + 1) for j in range(m)])
    pos = np.column_stack([np.asarray(properties.get(k, np.zeros(m)), dtype=float)
                           for k in ("chromosome", "cm_position", "bp_position")]) if m else np.empty((0, 3))
    sd = SnpData(iid=np.column_stack([fid, iid]).astype(str), sid=np.asarray(sid, dtype=str), val=val, pos=pos,
                 _require_float32_64=False)
    write_bed(str(filepath), sd, count_A1, {})


def _standardize(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads):
    assert val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]
    order_c = 1 if val.flags["C_CONTIGUOUS"] else 0
    cols = val.shape[1]
    st = np.ascontiguousarray(stats, dtype=val.dtype)
    N.call("snpmi_standardize_" + N.suffix(val.dtype), N.ptr(val), val.shape[0], cols, order_c, int(bool(is_beta)),
           float(a), float(b), int(bool(apply_in_place)), int(bool(use_stats)), N.ptr(st), get_num_threads(num_threads))
    if not use_stats:
        stats[...] = st


def standardize_f64(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads):
    _standardize(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads)


def standardize_f32(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads):
    _standardize(val, is_beta, a, b, apply_in_place, use_stats, stats, num_threads)


def _subset(fn, val_in, iid_index, sid_index, val_out, num_threads):
    assert val_in.ndim == 3 and val_out.ndim == 3
    in_c = 1 if val_in.flags["C_CONTIGUOUS"] else 0
    out_c = 1 if val_out.flags["C_CONTIGUOUS"] else 0
    ri, ci = N.index_array(iid_index), N.index_array(sid_index)
    N.call(fn, N.ptr(val_in), val_in.shape[0], val_in.shape[1], val_in.shape[2], in_c, N.ptr(ri), len(ri), N.ptr(ci),
           len(ci), out_c, N.ptr(val_out), get_num_threads(num_threads))


def subset_f64_f64(val_in, iid_index, sid_index, val_out, num_threads):
    _subset("snpmi_subset_f64_f64", val_in, iid_index, sid_index, val_out, num_threads)


def subset_f32_f64(val_in, iid_index, sid_index, val_out, num_threads):
    _subset("snpmi_subset_f32_f64", val_in, iid_index, sid_index, val_out, num_threads)


def subset_f32_f32(val_in, iid_index, sid_index, val_out, num_threads):
    _subset("snpmi_subset_f32_f32", val_in, iid_index, sid_index, val_out, num_threads)
