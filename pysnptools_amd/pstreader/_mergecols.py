"""Column-wise concatenation of readers that share their rows (reference
pstreader/_mergecols.py:8-159): the generic merge behind ``_MergeSIDs`` (SNP shards, DistributedBed)
and any other PstReader pieces (e.g. 3-D PstData / PstMemMap pieces).

Reads dispatch each requested column range to the piece that holds it; a read that spans several
pieces is assembled into one array ('A' -> F order, NaN-initialised as the reference does).
"""
import logging

import numpy as np

from pysnptools_amd.pstreader.pstreader import PstReader


class _MergeCols(PstReader):
    def __init__(self, reader_list, cache_file=None, skip_check=False):
        super(_MergeCols, self).__init__()
        assert len(reader_list) > 0, "Expect at least one reader"
        self.skip_check = skip_check
        self.reader_list = list(reader_list)
        self._repr_string = "{0}({1})".format(type(self).__name__, ",".join(str(s) for s in self.reader_list))
        if cache_file is not None:
            import os

            if not os.path.exists(cache_file):
                self._run_once()
                self._savez(cache_file)
            else:
                self._load(cache_file)

    def __repr__(self):
        return self._repr_string

    # metadata cache (_mergecols.py:24-38); written and read without pickle
    _count_key = "col_count_list"

    def _savez(self, cache_file):
        np.savez(cache_file, _row=np.array(self._row, dtype="S"), _row_property=self._row_property,
                 _col=np.array(self._col, dtype="S"), _col_property=self._col_property,
                 **{self._count_key: self.col_count_list})

    def _load(self, cache_file):
        with np.load(cache_file, allow_pickle=False) as data:
            self._col = np.array(data["_col"], dtype="str")
            self._col_property = data["_col_property"]
            self.col_count_list = np.array(data[self._count_key])
            assert ("_row" in data) == ("_row_property" in data)
            self._row = np.array(data["_row"], dtype="str")
            self._row_property = data["_row_property"]
        self._has_run_once = True

    def _run_once(self):
        """Rows (and row properties) must agree across pieces and columns must be distinct
        unless ``skip_check`` (_mergecols.py:40-77)."""
        if getattr(self, "_has_run_once", False):
            return
        self._has_run_once = True
        first = self.reader_list[0]
        self._row = first.row
        self._row_property = first.row_property
        cols, props, counts, seen = [], [], [], set()
        for k, reader in enumerate(self.reader_list):
            if k % 10 == 0:
                logging.info("%s looking at reader #%d: %s", type(self).__name__, k, reader)
            if not self.skip_check:
                assert np.array_equal(self._row, reader.row), "Expect rows to be the same across all files"
                np.testing.assert_equal(self._row_property, reader.row_property)
                before = len(seen)
                seen.update(tuple(c) if np.ndim(c) else c for c in reader.col.tolist())
                assert len(seen) == before + reader.col_count, "Expect cols to be distinct in all files"
            cols.append(reader.col)
            props.append(reader.col_property)
            counts.append(reader.col_count)
        self._col = np.concatenate(cols)
        self._col_property = np.concatenate(props)
        self.col_count_list = np.array(counts)

    @property
    def row(self):
        self._run_once()
        return self._row

    @property
    def col(self):
        self._run_once()
        return self._col

    @property
    def col_property(self):
        self._run_once()
        return self._col_property

    @property
    def row_property(self):
        self._run_once()
        return self._row_property

    @property
    def val_shape(self):
        return self.reader_list[0].val_shape

    def copyinputs(self, copier):
        self._run_once()
        for reader in self.reader_list:
            copier.input(reader)

    def _pieces(self, col_index):
        """[(reader_index, mask into col_index, relative index)] (_mergecols.py:104-115)."""
        self._run_once()
        out = []
        start = 0
        for k, count in enumerate(self.col_count_list):
            stop = start + int(count)
            here = (col_index >= start) & (col_index < stop)
            if here.any():
                out.append((k, here, col_index[here] - start))
            start = stop
        return out

    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        dtype = np.dtype(dtype)
        col_index = np.arange(self.col_count) if col_index_or_none is None else np.asarray(col_index_or_none)
        n = self.row_count if row_index_or_none is None else len(row_index_or_none)
        pieces = self._pieces(col_index)
        if len(pieces) == 0:
            return self.reader_list[0]._read(row_index_or_none, col_index, order, dtype, force_python_only, view_ok,
                                             num_threads)
        if len(pieces) == 1:
            k, _, rel = pieces[0]
            return self.reader_list[k]._read(row_index_or_none, rel, order, dtype, force_python_only, view_ok,
                                             num_threads)
        order = "F" if order in ("A", None) else order
        val = None
        for k, here, rel in pieces:
            logging.debug("reading %d columns from piece %d", len(rel), k)
            piece = self.reader_list[k]._read(row_index_or_none, rel, order, dtype, force_python_only, True,
                                              num_threads)
            if val is None:
                shape = (n, len(col_index)) + tuple(piece.shape[2:])
                val = np.empty(shape, dtype=dtype, order=order)
                if dtype.kind == "f":
                    val.fill(np.nan)
            val[:, here] = piece
        return val
