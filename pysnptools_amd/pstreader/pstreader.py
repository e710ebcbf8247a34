"""Lazy 2-D matrix reader: row/col ids, properties and the index algebra of the "slice" step.

Behaviour follows the reference's ``PstReader`` (pstreader/pstreader.py): indexers may be
slices, integer or boolean arrays, lists or scalars (pstreader.py:618-645); they are
materialised as ``uintp`` arrays (:648-654) and composed through nested subsets
(pstreader/_subset.py:114-142).  Gathers of in-memory values go through
``util.sub_matrix`` (HIP).
"""
import numbers

import numpy as np

from pysnptools_amd import util as pstutil


class PstReader(object):
    """Base class of every matrix reader (SnpReader, KernelReader)."""

    def __init__(self, *args, **kwargs):
        super(PstReader, self).__init__()

    # ------------------------------------------------------------------ ids
    @property
    def row(self):
        raise NotImplementedError

    @property
    def col(self):
        raise NotImplementedError

    @property
    def row_count(self):
        return len(self.row)

    @property
    def col_count(self):
        return len(self.col)

    @property
    def shape(self):
        return (self.row_count, self.col_count)

    @property
    def row_property(self):
        raise NotImplementedError

    @property
    def col_property(self):
        raise NotImplementedError

    # ------------------------------------------------------------------ reading
    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        raise NotImplementedError

    def read(self, order="F", dtype=np.float64, force_python_only=False, view_ok=False, num_threads=None):
        from pysnptools_amd.pstreader.pstdata import PstData

        val = self._read(None, None, order, np.dtype(dtype), force_python_only, view_ok, num_threads)
        return PstData(self.row, self.col, val, row_property=self.row_property, col_property=self.col_property,
                       name=str(self))

    def __getitem__(self, row_indexer_and_col_indexer):
        from pysnptools_amd.pstreader._subset import _PstSubset

        row_indexer, col_indexer = row_indexer_and_col_indexer
        return _PstSubset(self, row_indexer, col_indexer)

    # ------------------------------------------------------------------ id -> index
    @staticmethod
    def _makekey(item):
        if isinstance(item, (str, numbers.Integral, float)):
            return item
        try:
            hash(item)
            return item
        except TypeError:
            return tuple(PstReader._makekey(x) for x in item)

    def row_to_index(self, list):
        if not hasattr(self, "_row_to_index"):
            lookup = {}
            for i, item in enumerate(self.row):
                key = self._makekey(item)
                if key in lookup:
                    raise Exception("Expect row to appear in data only once. ({0})".format(key))
                lookup[key] = i
            self._row_to_index = lookup
        return np.fromiter((self._row_to_index[self._makekey(x)] for x in list), np.int_)

    def col_to_index(self, list):
        if not hasattr(self, "_col_to_index"):
            keys = [self._makekey(x) for x in self.col]
            lookup = {k: i for i, k in enumerate(keys)}
            assert len(lookup) == self.col_count, "Expect col to appear in data only once."
            self._col_to_index = lookup
        return np.fromiter((self._col_to_index[self._makekey(x)] for x in list), np.int_)

    def copyinputs(self, copier):
        raise NotImplementedError

    # ------------------------------------------------------------------ index algebra
    @staticmethod
    def _is_all_slice(index_or_none):
        return index_or_none is None or (isinstance(index_or_none, slice) and index_or_none == slice(None))

    @staticmethod
    def _make_sparray_or_slice(indexer):
        """slice -> slice; None -> slice(None); scalar -> [i]; bools -> positions; else int array."""
        if indexer is None:
            return slice(None)
        if isinstance(indexer, slice):
            return indexer
        if isinstance(indexer, np.ndarray):
            return PstReader._process_ndarray(indexer)
        if np.isscalar(indexer):
            assert isinstance(indexer, numbers.Integral), "Expect scalar indexes to be integers"
            return np.array([indexer])
        return PstReader._process_ndarray(np.array(indexer))

    @staticmethod
    def _process_ndarray(indexer):
        if len(indexer) == 0:
            return np.zeros(0, dtype=np.intp)
        if indexer.dtype == bool:
            return np.flatnonzero(indexer)
        assert np.issubdtype(indexer.dtype, np.integer), "Indexer of unknown type"
        return indexer

    @staticmethod
    def _make_sparray_from_sparray_or_slice(count, indexer):
        """Absolute ``uintp`` positions (negatives wrap, as NumPy indexing does)."""
        if isinstance(indexer, slice):
            return np.arange(*indexer.indices(count), dtype=np.uintp)
        positions = np.arange(count, dtype=np.uintp)[indexer]
        return np.ascontiguousarray(positions.reshape(-1), dtype=np.uintp)

    @staticmethod
    def _array_properties_are_ok(val, order, dtype):
        if val.dtype != np.dtype(dtype):
            return False
        if order == "F":
            return val.flags["F_CONTIGUOUS"]
        if order == "C":
            return val.flags["C_CONTIGUOUS"]
        return True

    def _apply_sparray_or_slice_to_val(self, val, row_indexer_or_none, col_indexer_or_none, order, dtype,
                                       force_python_only, num_threads):
        """Sub-matrix of an in-memory ``val`` as (array, shares_memory) (pstreader.py:669-738)."""
        dtype = np.dtype(dtype)
        whole = self._is_all_slice(row_indexer_or_none) and self._is_all_slice(col_indexer_or_none)
        if whole and (order == "A" or (order == "F" and val.flags["F_CONTIGUOUS"])
                      or (order == "C" and val.flags["C_CONTIGUOUS"])) and val.dtype == dtype:
            return val, True
        rows = self._make_sparray_from_sparray_or_slice(self.row_count, self._make_sparray_or_slice(row_indexer_or_none))
        cols = self._make_sparray_from_sparray_or_slice(self.col_count, self._make_sparray_or_slice(col_indexer_or_none))
        if val.dtype in (np.float32, np.float64) and dtype in (np.float32, np.float64):
            return pstutil.sub_matrix(val, rows, cols, order=order, dtype=dtype, num_threads=num_threads), False
        # non-float payloads (e.g. int8 genotypes): plain NumPy gather of a copy
        sub = val[np.ix_(rows, cols)] if val.ndim == 2 else val[np.ix_(rows, cols, np.arange(val.shape[2]))]
        sub = np.array(sub, dtype=dtype, order="K" if order == "A" else order)
        return sub, False
