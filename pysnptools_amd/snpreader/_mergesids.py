"""SNP-wise concatenation of readers that share their iids (reference
pstreader/_mergecols.py:8-159 + snpreader/_mergesids.py:5-25) -- the in-memory face of
DistributedBed and of per-chromosome / per-GPU SNP shards.

Reads dispatch each requested SNP range to its piece (every piece a native BED read).  The
GRM of a merged set of Beds runs as one GPU session (``snpmi_grm_begin`` / ``add_bed`` per
piece / ``end``): K accumulates in HBM across pieces; see ``SnpReader._read_kernel``.
"""
import logging

import numpy as np

from pysnptools_amd.snpreader.snpreader import SnpReader


class _MergeSIDs(SnpReader):
    def __init__(self, reader_list, cache_file=None, skip_check=False):
        super(_MergeSIDs, self).__init__()
        assert len(reader_list) > 0, "Expect at least one reader"
        self.skip_check = skip_check
        self.reader_list = list(reader_list)
        self._repr_string = "_MergeSIDs({0})".format(",".join(str(s) for s in self.reader_list))
        if cache_file is not None:
            import os

            if not os.path.exists(cache_file):
                self._run_once()
                self._savez(cache_file)
            else:
                self._load(cache_file)

    def __repr__(self):
        return self._repr_string

    # metadata cache (_mergesids.py:9-25); loaded without pickle
    def _savez(self, cache_file):
        np.savez(cache_file, _row=np.array(self._row, dtype="S"), _row_property=self._row_property,
                 _col=np.array(self._col, dtype="S"), _col_property=self._col_property,
                 sid_count_list=self.col_count_list)

    def _load(self, cache_file):
        with np.load(cache_file, allow_pickle=False) as data:
            self._col = np.array(data["_col"], dtype="str")
            self._col_property = np.array(data["_col_property"], dtype=np.float64)
            self.col_count_list = np.array(data["sid_count_list"])
            assert ("_row" in data) == ("_row_property" in data)
            self._row = np.array(data["_row"], dtype="str")
            self._row_property = data["_row_property"]
        self._has_run_once = True

    def _run_once(self):
        if getattr(self, "_has_run_once", False):
            return
        self._has_run_once = True
        first = self.reader_list[0]
        self._row = first.row
        self._row_property = first.row_property
        cols, props, counts, seen = [], [], [], set()
        for reader in self.reader_list:
            if not self.skip_check:
                assert np.array_equal(self._row, reader.row), "Expect rows to be the same across all files"
                before = len(seen)
                seen.update(reader.col.tolist())
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

    def _pieces(self, col_index):
        """[(reader_index, mask into col_index, relative index)] (_mergecols.py:104-115)."""
        out = []
        start = 0
        for k, count in enumerate(self.col_count_list):
            stop = start + int(count)
            here = (col_index >= start) & (col_index < stop)
            if here.any():
                out.append((k, here, col_index[here] - start))
            start = stop
        return out

    def _read(self, iid_index_or_none, sid_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        dtype = np.dtype(dtype)
        col_index = np.arange(self.col_count) if sid_index_or_none is None else np.asarray(sid_index_or_none)
        n = self.row_count if iid_index_or_none is None else len(iid_index_or_none)
        pieces = self._pieces(col_index)
        if len(pieces) == 0:
            return self.reader_list[0]._read(iid_index_or_none, col_index, order, dtype, force_python_only, view_ok,
                                             num_threads)
        if len(pieces) == 1:
            k, _, rel = pieces[0]
            return self.reader_list[k]._read(iid_index_or_none, rel, order, dtype, force_python_only, view_ok,
                                             num_threads)
        order = "F" if order in ("A", None) else order
        val = np.empty((n, len(col_index)), dtype=dtype, order=order)
        for k, here, rel in pieces:
            logging.debug("reading %d SNPs from piece %d", len(rel), k)
            val[:, here] = self.reader_list[k]._read(iid_index_or_none, rel, order, dtype, force_python_only, True,
                                                     num_threads)
        return val
