"""PLINK .bed/.bim/.fam reader (reference snpreader/bed.py).

Where the reference hands ``open_bed(...).read(index=(iid_idx, sid_idx), order, dtype)``
to the Rust crate bed-reader (bed.py:337-343), this reader calls
``snpmi_bed_read_{f32,f64,i8}``: the selected packed columns are uploaded to HBM and
decoded by a HIP kernel.  Metadata (.fam/.bim) is parsed on the host.
"""
import os
import warnings

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.snpreader.snpreader import SnpReader
from pysnptools_amd.util import get_num_threads

plink_chrom_map = {"X": 23, "Y": 24, "XY": 25, "MT": 26}
reverse_plink_chrom_map = {23: "X", 24: "Y", 25: "XY", 26: "MT"}


def _text_scan(path, min_fields, n_cols, num_threads=None):
    import ctypes

    rows = ctypes.c_uint64()
    widths = np.zeros(max(n_cols, 1), dtype=np.uint64)
    N.call("snpmi_text_scan", path.encode(), min_fields, n_cols, ctypes.byref(rows), N.ptr(widths),
           get_num_threads(num_threads))
    return rows.value, widths


def _text_bytes(path, col, rows, width, num_threads=None):
    """Column ``col`` of a whitespace-delimited file as fixed-width bytes (C parser, f1)."""
    width = max(int(width), 1)
    raw = np.empty(rows, dtype="S%d" % width)
    N.call("snpmi_text_strings", path.encode(), col, rows, width, N.ptr(raw), get_num_threads(num_threads))
    return raw


def _to_str(raw):
    try:
        return raw.astype(str)
    except UnicodeDecodeError:
        return np.char.decode(raw, "utf-8")


def _text_strings(path, col, rows, width, num_threads=None):
    """Column ``col`` of a whitespace-delimited file as a NumPy str array."""
    return _to_str(_text_bytes(path, col, rows, width, num_threads))


def _text_f64(path, col, rows, num_threads=None):
    out = np.empty(rows, dtype=np.float64)
    N.call("snpmi_text_f64", path.encode(), col, rows, N.ptr(out), get_num_threads(num_threads))
    return out


class Bed(SnpReader):
    """Random-access reads of a PLINK .bed/.bim/.fam triple (SNP-major .bed only)."""

    def __init__(self, filename, count_A1=None, iid=None, sid=None, pos=None, num_threads=None,
                 skip_format_check=False, fam_filename=None, bim_filename=None, chrom_map=plink_chrom_map):
        super(Bed, self).__init__()
        self._ran_once = False
        self.filename = SnpReader._name_of_other_file(filename, remove_suffix="bed", add_suffix="bed")
        self.fam_filename = fam_filename or SnpReader._name_of_other_file(self.filename, "bed", "fam")
        self.bim_filename = bim_filename or SnpReader._name_of_other_file(self.filename, "bed", "bim")
        if count_A1 is None:
            warnings.warn("'count_A1' was not set. For now it will default to 'False', but in the future it will "
                          "default to 'True'", FutureWarning)
            count_A1 = False
        self.count_A1 = count_A1
        self._skip_format_check = skip_format_check
        self._original_iid = iid
        self._original_sid = sid
        self._original_pos = pos
        self._num_threads = num_threads
        self.chrom_map = chrom_map

    def __repr__(self):
        return "{0}('{1}',count_A1={2})".format(self.__class__.__name__, self.filename, self.count_A1)

    @property
    def row(self):
        if not hasattr(self, "_row"):
            if self._original_iid is not None:
                self._row = np.array(self._original_iid, dtype="str").reshape(-1, 2)
            else:
                rows, w = _text_scan(self.fam_filename, 2, 2, self._num_threads)
                fid = _text_strings(self.fam_filename, 0, rows, w[0], self._num_threads)
                iid = _text_strings(self.fam_filename, 1, rows, w[1], self._num_threads)
                self._row = np.array([fid, iid], dtype="str").T.reshape(-1, 2)
        return self._row

    def _bim_scan(self):
        if not hasattr(self, "_bim_shape"):
            self._bim_shape = _text_scan(self.bim_filename, 4, 2, self._num_threads)
        return self._bim_shape

    @property
    def col(self):
        if not hasattr(self, "_col"):
            if self._original_sid is not None:
                self._col = np.array(self._original_sid, dtype="str")
            else:
                rows, w = self._bim_scan()
                self._col = _text_strings(self.bim_filename, 1, rows, w[1], self._num_threads)
        return self._col

    @property
    def col_property(self):
        if not hasattr(self, "_col_property"):
            if self._original_pos is not None:
                pos = np.array(self._original_pos, dtype=float).reshape(-1, 3)
            else:
                rows, w = self._bim_scan()
                pos = np.empty((rows, 3), dtype=np.float64)
                pos[:, 0] = self._chromosomes(_text_bytes(self.bim_filename, 0, rows, w[0], self._num_threads))
                pos[:, 1] = _text_f64(self.bim_filename, 2, rows, self._num_threads)
                pos[:, 2] = _text_f64(self.bim_filename, 3, rows, self._num_threads)
            pos[pos == 0] = np.nan  # PLINK's missing chromosome/position
            self._col_property = pos
        return self._col_property

    def _chromosomes(self, chrom):
        """chrom_map then float(), per distinct value (bed.py:180-186; ValueError for e.g. 'chrBAD')."""
        uniq, inv = np.unique(chrom, return_inverse=True)
        names = _to_str(uniq)
        vals = np.array([float(self.chrom_map.get(u, u)) for u in names], dtype=np.float64)
        return vals[inv.reshape(-1)] if len(uniq) else np.empty(0)

    def _run_once(self):
        if self._ran_once:
            return
        self.row
        self.col
        self.col_property
        if not self._skip_format_check:
            N.call("snpmi_bed_check", self.filename.encode(), len(self._row), len(self._col))
        self._ran_once = True

    def copyinputs(self, copier):
        for suffix in ("bed", "bim", "fam"):
            copier.input(SnpReader._name_of_other_file(self.filename, remove_suffix="bed", add_suffix=suffix))

    def _read(self, iid_index_or_none, sid_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        dtype = np.dtype(dtype)
        if order == "A":
            order = "F"
        if dtype not in (np.float32, np.float64, np.int8):
            raise ValueError("dtype '{0}' not supported; use float32, float64 or int8".format(dtype))
        ri = N.index_array(iid_index_or_none)
        ci = N.index_array(sid_index_or_none)
        n = self.iid_count if ri is None else len(ri)
        m = self.sid_count if ci is None else len(ci)
        out = np.empty((n, m), dtype=dtype, order=order)
        threads = get_num_threads(num_threads if num_threads is not None else self._num_threads)
        N.call("snpmi_bed_read_" + N.suffix(dtype), self.filename.encode(), self.iid_count, self.sid_count,
               int(bool(self.count_A1)), N.ptr(ri), n, N.ptr(ci), m, 1 if order == "C" else 0, N.ptr(out), threads)
        return out

    @staticmethod
    def write(filename, snpdata, count_A1=False, force_python_only=False, _require_float32_64=True, num_threads=None,
              reverse_chrom_map={}):
        """Write ``snpdata`` as a .bed/.bim/.fam triple (bed.py:229-316); returns a :class:`Bed`.
        Values must be 0, 1, 2 or missing (NaN / -127)."""
        from pysnptools_amd.snpreader._write import write_bed

        if count_A1 is None:
            warnings.warn("'count_A1' was not set. For now it will default to 'False', but in the future it will "
                          "default to 'True'", FutureWarning)
            count_A1 = False
        filename = SnpReader._name_of_other_file(filename, remove_suffix="bed", add_suffix="bed")
        write_bed(filename, snpdata, count_A1, reverse_chrom_map)
        return Bed(filename, count_A1=count_A1)
