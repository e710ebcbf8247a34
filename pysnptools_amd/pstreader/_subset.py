"""Lazy row/column subset of a PstReader (reference pstreader/_subset.py).

Indexers compose: ``r[:, ::2][:, ::2]`` reads the inner reader once with ``::4``
(composed as index arrays, _subset.py:114-142)."""
import numpy as np

from pysnptools_amd.pstreader.pstreader import PstReader


class _PstSubset(PstReader):
    def __init__(self, internal, row_indexer, col_indexer):
        super(_PstSubset, self).__init__()
        self._ran_once = False
        self._internal = internal
        self._row_indexer = PstReader._make_sparray_or_slice(row_indexer)
        self._col_indexer = PstReader._make_sparray_or_slice(col_indexer)

    def __repr__(self):
        return "{0}[{1},{2}]".format(self._internal, _nice(self._row_indexer), _nice(self._col_indexer))

    def copyinputs(self, copier):
        self._internal.copyinputs(copier)

    def _run_once(self):
        if self._ran_once:
            return
        self._ran_once = True
        self._row = self._internal.row[self._row_indexer]
        self._col = self._internal.col[self._col_indexer]
        if self._row.dtype == self._col.dtype and np.array_equal(self._row, self._col):
            self._col = self._row
        self._row_property = self._internal.row_property[self._row_indexer]
        self._col_property = self._internal.col_property[self._col_indexer]

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

    _read_accepts_slices = True

    def _composed_indices(self, row_indexer, col_indexer):
        """Absolute index arrays (or None for 'all') into the innermost reader."""
        rows = _compose(self._internal.row_count, self._row_indexer, self.row_count, row_indexer)
        cols = _compose(self._internal.col_count, self._col_indexer, self.col_count, col_indexer)
        return rows, cols

    def _read(self, row_indexer, col_indexer, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        rows, cols = self._composed_indices(row_indexer, col_indexer)
        return self._internal._read(rows, cols, order, np.dtype(dtype), force_python_only, view_ok, num_threads)

    @staticmethod
    def compose_indexer_with_indexer(countA, indexerA, countB, indexerB):
        return _compose(countA, indexerA, countB, indexerB)


def _compose(count_a, indexer_a, count_b, indexer_b):
    if PstReader._is_all_slice(indexer_a):
        if PstReader._is_all_slice(indexer_b):
            return None
        return PstReader._make_sparray_from_sparray_or_slice(count_b, PstReader._make_sparray_or_slice(indexer_b))
    index_a = PstReader._make_sparray_from_sparray_or_slice(count_a, indexer_a)
    if PstReader._is_all_slice(indexer_b):
        return index_a
    index_b = PstReader._make_sparray_from_sparray_or_slice(count_b, PstReader._make_sparray_or_slice(indexer_b))
    return index_a[index_b]


def _nice(ix):
    if isinstance(ix, slice):
        parts = ["" if v is None else str(v) for v in (ix.start, ix.stop)]
        s = ":".join(parts)
        return s + ("" if ix.step is None else ":" + str(ix.step)) if s != ":" or ix.step else ":"
    if len(ix) == 1:
        return str(ix[0])
    head = ",".join(str(i) for i in ix[:10])
    return "[{0}]".format(head) if len(ix) < 10 else "[{0},...]".format(head)
