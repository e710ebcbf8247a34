"""KernelNpz: a GRM on disk as .npz (reference kernelreader/kernelnpz.py + pstreader/pstnpz.py).

Keys ``row``, ``col``, ``row_property``, ``col_property``, ``val`` (pstnpz.py:114-131); the
legacy two-array form (``arr_0`` = iids, ``arr_1`` = val) is read too.  Files are loaded with
``allow_pickle=False``: string ids must be stored as NumPy string arrays, as the reference
writes them.  ``write`` is how a K computed on the GPU is persisted.
"""
import numpy as np

from pysnptools_amd.kernelreader.kernelreader import KernelReader


class KernelNpz(KernelReader):
    def __init__(self, filename):
        super(KernelNpz, self).__init__()
        self._ran_once = False
        self._filename = filename

    def __repr__(self):
        return "{0}('{1}')".format(self.__class__.__name__, self._filename)

    def _run_once(self):
        if self._ran_once:
            return
        self._ran_once = True
        with np.load(self._filename, allow_pickle=False) as data:
            if len(data.keys()) == 2 and "arr_0" in data.keys():
                self._row = np.array(data["arr_0"], dtype="str")
                self._col = self._row
                self._row_property = np.empty((len(self._row), 0))
                self._col_property = np.empty((len(self._col), 0))
            else:
                self._row = np.array(data["row"], dtype="str")
                self._col = np.array(data["col"], dtype="str")
                if np.array_equal(self._row, self._col):
                    self._col = self._row  # square: iid0 is iid1 (pstnpz.py:83-84)
                self._row_property = data["row_property"]
                self._col_property = data["col_property"]

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

    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        with np.load(self._filename, allow_pickle=False) as data:
            val = data["arr_1"] if (len(data.keys()) == 2 and "arr_1" in data.keys()) else data["val"]
        val, _ = self._apply_sparray_or_slice_to_val(val, row_index_or_none, col_index_or_none, order, np.dtype(dtype),
                                                     force_python_only, num_threads)
        return val

    @staticmethod
    def write(filename, kerneldata):
        """Write a KernelData (row/col ids as string arrays) and return the KernelNpz."""
        np.savez(filename, row=np.array(kerneldata.row, dtype="S"), col=np.array(kerneldata.col, dtype="S"),
                 row_property=kerneldata.row_property, col_property=kerneldata.col_property, val=kerneldata.val)
        return KernelNpz(filename)
