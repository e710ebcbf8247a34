"""PstData kept in a memory-mapped file (reference pstreader/pstmemmap.py).

File format (the reference's, version 2, pstmemmap.py:150-165): a run of ``np.save`` records --
magic 22891, "pstmemmap", 2, row, col, row_property, col_property, [dtype], [order],
[val_shape] -- followed by the raw values at ``offset``.  Version 1 (no magic; row first, no
val_shape) is read too.

The reference stores ``[dtype]`` and ``[val_shape]`` as numpy object arrays, i.e. pickles.
Files are written the same way (so the reference can read them), but NOTHING is unpickled
when reading: plain records go through ``np.load(allow_pickle=False)``, and object records are
disassembled with ``pickletools.genops`` (an opcode parser that constructs no objects), from
which only a numpy float dtype code, an int or None is accepted.
"""
import logging
import os
import pickletools
import shutil
import warnings

import numpy as np

from pysnptools_amd.pstreader.pstdata import PstData
from pysnptools_amd.pstreader.pstreader import PstReader

_magic_number = 22891
_DTYPE_CODES = {"f8": np.float64, "<f8": np.float64, "float64": np.float64, "d": np.float64,
                "f4": np.float32, "<f4": np.float32, "float32": np.float32, "f": np.float32}
_DTYPE_GLOBALS = {"numpy float64": np.float64, "numpy float32": np.float32}
_STRING_OPS = ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "SHORT_BINSTRING", "BINSTRING", "UNICODE",
               "STRING")
_INT_OPS = ("BININT", "BININT1", "BININT2", "LONG1", "INT", "LONG")
_MEMO_OPS = ("BINPUT", "LONG_BINPUT", "MEMOIZE", "BINGET", "LONG_BINGET", "GET", "PUT")


def _object_record_value(fp):
    """The single element of a pickled 1-element object array, read without executing it."""
    ops = []
    for op, arg, _ in pickletools.genops(fp):
        ops.append((op.name, arg))
        if op.name == "STOP":
            break
    starts = [i for i, (name, _) in enumerate(ops) if name == "EMPTY_LIST"]
    if not starts:
        raise ValueError("unrecognised object record in memmap header")
    tail = [(n, a) for n, a in ops[starts[-1] + 1:] if n not in _MEMO_OPS]
    for k, (name, arg) in enumerate(tail):
        if name == "NONE":
            return None
        if name in _INT_OPS:
            return int(arg)
        if name == "GLOBAL":
            if arg in _DTYPE_GLOBALS:
                return np.dtype(_DTYPE_GLOBALS[arg])
            if arg == "numpy dtype":
                for n2, a2 in tail[k + 1:]:
                    if n2 in _STRING_OPS:
                        return np.dtype(_DTYPE_CODES[a2 if isinstance(a2, str) else a2.decode()])
            raise ValueError("memmap header: unsupported object %r" % (arg,))
        if name in _STRING_OPS:
            code = arg if isinstance(arg, str) else arg.decode()
            if code in _DTYPE_CODES:
                return np.dtype(_DTYPE_CODES[code])
            raise ValueError("memmap header: unsupported dtype code %r" % (code,))
    raise ValueError("memmap header: empty object record")


def _load_record(fp):
    """One ``np.save`` record: plain arrays via allow_pickle=False; object arrays -> [value]."""
    pos = fp.tell()
    version = np.lib.format.read_magic(fp)
    reader = np.lib.format.read_array_header_1_0 if version == (1, 0) else np.lib.format.read_array_header_2_0
    with warnings.catch_warnings():  # headers of Python-2-written files (reference examples)
        warnings.simplefilter("ignore", UserWarning)
        _, _, dtype = reader(fp)
        if dtype.hasobject:
            return np.array([_object_record_value(fp)], dtype=object)
        fp.seek(pos)
        return np.load(fp, allow_pickle=False)


def _as_str(a):
    """Header string arrays: byte strings (Python-2-written files) -> str."""
    if a.dtype.kind == "S":
        return a.astype("str")
    return a


class PstMemMap(PstData):
    """A PstData whose ``val`` is an ``np.memmap`` (data larger than memory).

    ``PstMemMap(filename)`` opens an existing ``*.pst.memmap``; see :meth:`empty` and :meth:`write`.
    """

    def __init__(self, filename):
        PstReader.__init__(self)
        self._ran_once = False
        self._filename = filename

    def __repr__(self):
        return "{0}('{1}')".format(self.__class__.__name__, self._filename)

    def __getstate__(self):
        return self.filename

    def __setstate__(self, state):
        self.__init__(state)

    @property
    def val(self):
        self._run_once()
        return self._val

    @val.setter
    def val(self, new_value):
        self._run_once()
        if self._val is new_value:
            return
        raise Exception("PstMemMap val's cannot be set to a different array")

    @property
    def row(self):
        self._run_once()
        return self._row

    @property
    def col(self):
        self._run_once()
        return self._col

    @property
    def row_property(self):
        self._run_once()
        return self._row_property

    @property
    def col_property(self):
        self._run_once()
        return self._col_property

    @property
    def offset(self):
        """Byte position in the file where the memory-mapped values start."""
        self._run_once()
        return self._offset

    @property
    def filename(self):
        return self._filename

    @staticmethod
    def empty(row, col, filename, row_property=None, col_property=None, order="F", dtype=np.float64, val_shape=None):
        """Create an empty PstMemMap on disk (pstmemmap.py:104-141)."""
        self = PstMemMap(filename)
        self._empty_inner(row, col, filename, row_property, col_property, order, np.dtype(dtype), val_shape)
        return self

    def _empty_inner(self, row, col, filename, row_property, col_property, order, dtype, val_shape):
        self._ran_once = True
        self._dtype = np.dtype(dtype)
        self._order = order
        row = PstData._fixup_input(row)
        col = PstData._fixup_input(col)
        row_property = PstData._fixup_input(row_property, count=len(row))
        col_property = PstData._fixup_input(col_property, count=len(col))
        with open(filename, "wb") as fp:
            np.save(fp, np.array([_magic_number]))
            np.save(fp, np.array(["pstmemmap"]))
            np.save(fp, np.array([2]))
            np.save(fp, row)
            np.save(fp, col)
            np.save(fp, row_property)
            np.save(fp, col_property)
            np.save(fp, np.array([self._dtype]))  # object record, as the reference writes it
            np.save(fp, np.array([self._order]))
            np.save(fp, np.array([val_shape]))
            self._offset = fp.tell()
        shape = (len(row), len(col)) if val_shape is None else (len(row), len(col), val_shape)
        val = np.memmap(filename, offset=self._offset, dtype=self._dtype, mode="r+", order=order, shape=shape)
        PstData.__init__(self, row, col, val, row_property, col_property, name="np.memmap('{0}')".format(filename))

    def _run_once(self):
        if self._ran_once:
            return
        row, col, val, row_property, col_property = self._run_once_inner()
        PstData.__init__(self, row, col, val, row_property, col_property, name="np.memmap('{0}')".format(self._filename))

    def _run_once_inner(self):
        self._ran_once = True
        with open(self._filename, "rb") as fp:
            first = _load_record(fp)
            if len(first) == 1 and first.dtype.kind in "iu" and first[0] == _magic_number:
                fmt = str(_as_str(_load_record(fp))[0])
                version = int(_load_record(fp)[0])
                assert fmt == "pstmemmap", "Expect format of 'pstmemmap'"
                assert version == 2, "Expect version of 2"
                row = _as_str(_load_record(fp))
                col = _as_str(_load_record(fp))
                row_property = _as_str(_load_record(fp))
                col_property = _as_str(_load_record(fp))
                self._dtype = np.dtype(_load_record(fp)[0])
                self._order = str(_as_str(_load_record(fp))[0])
                vs = _load_record(fp)[0]
                val_shape = None if vs is None else int(vs)
            else:  # version 1
                row = _as_str(first)
                col = _as_str(_load_record(fp))
                row_property = _as_str(_load_record(fp))
                col_property = _as_str(_load_record(fp))
                self._dtype = np.dtype(_load_record(fp)[0])
                self._order = str(_as_str(_load_record(fp))[0])
                val_shape = None
            self._offset = fp.tell()
        shape = (len(row), len(col)) if val_shape is None else (len(row), len(col), val_shape)
        val = np.memmap(self._filename, offset=self._offset, dtype=self._dtype, mode="r", order=self._order, shape=shape)
        return row, col, val, row_property, col_property

    def copyinputs(self, copier):
        copier.input(self._filename)

    _read_accepts_slices = True

    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        # the reference reads memmaps through NumPy (pstmemmap.py:276-282): slices stay views of
        # the file; a selection is gathered on the host, only the selected bytes are touched
        dtype = np.dtype(dtype)
        val = self.val
        ri = slice(None) if row_index_or_none is None else row_index_or_none
        ci = slice(None) if col_index_or_none is None else col_index_or_none
        if isinstance(ri, slice) and isinstance(ci, slice):
            sub = val[ri, ci]
            shares = True
        else:
            rows = self._make_sparray_from_sparray_or_slice(self.row_count, self._make_sparray_or_slice(ri))
            cols = self._make_sparray_from_sparray_or_slice(self.col_count, self._make_sparray_or_slice(ci))
            sub = val[np.ix_(rows, cols)] if val.ndim == 2 else val[np.ix_(rows, cols, np.arange(val.shape[2]))]
            shares = False
        want = "K" if order == "A" else order
        if not self._array_properties_are_ok(sub, order, dtype):
            sub = np.array(sub, dtype=dtype, order=want)
            shares = False
        if shares and not view_ok:
            sub = sub.copy(order="K")
        return sub

    @staticmethod
    def _order(pstdata):
        if pstdata.val.flags["F_CONTIGUOUS"]:
            return "F"
        if pstdata.val.flags["C_CONTIGUOUS"]:
            return "C"
        raise Exception("Don't know order of PstData's value")

    def flush(self):
        """Flush ``val`` to disk and close the file (it is reopened on the next access)."""
        if self._ran_once:
            self._val.flush()
            del self._val
            self._val = None
            self._ran_once = False

    @staticmethod
    def write(filename, pstdata):
        """Write a PstData to PstMemMap format; returns the PstMemMap (pstmemmap.py:300-320)."""
        self = PstMemMap.empty(pstdata.row, pstdata.col, filename + ".temp", row_property=pstdata.row_property,
                               col_property=pstdata.col_property, order=PstMemMap._order(pstdata),
                               dtype=pstdata.val.dtype, val_shape=pstdata.val_shape)
        if pstdata.val_shape is None:
            self.val[:, :] = pstdata.val
        else:
            self.val[:, :, :] = pstdata.val
        self.flush()
        if os.path.exists(filename):
            os.remove(filename)
        shutil.move(filename + ".temp", filename)
        logging.debug("Done writing " + filename)
        return PstMemMap(filename)
