"""iid x iid kernel readers (reference kernelreader/kernelreader.py)."""
import numpy as np

from pysnptools_amd.kernelstandardizer import DiagKtoN
from pysnptools_amd.pstreader import PstReader


class KernelReader(PstReader):
    def __init__(self, *args, **kwargs):
        super(KernelReader, self).__init__(*args, **kwargs)

    @property
    def iid(self):
        assert self.iid0 is self.iid1, "When 'iid' is used, iid0 must be the same as iid1"
        return self.iid0

    @property
    def iid0(self):
        return self.row

    @property
    def iid1(self):
        return self.col

    @property
    def iid_count(self):
        assert self.iid0 is self.iid1, "When 'iid_count' is used, iid0 must be the same as iid1"
        return self.iid0_count

    @property
    def iid0_count(self):
        return self.row_count

    @property
    def iid1_count(self):
        return self.col_count

    @property
    def row_property(self):
        if not hasattr(self, "_row_property"):
            self._row_property = np.empty((self.row_count, 0))
        return self._row_property

    @property
    def col_property(self):
        if not hasattr(self, "_col_property"):
            self._col_property = np.empty((self.col_count, 0))
        return self._col_property

    def read(self, order="F", dtype=np.float64, force_python_only=False, view_ok=False, num_threads=None):
        from pysnptools_amd.kernelreader.kerneldata import KernelData

        val = self._read(None, None, order, np.dtype(dtype), force_python_only, view_ok, num_threads)
        return KernelData(iid0=self.iid0, iid1=self.iid1, val=val, name=str(self))

    def iid_to_index(self, list):
        assert self.iid0 is self.iid1, "When 'iid_to_index' is used, iid0 must be the same as iid1"
        return self.iid0_to_index(list)

    def iid0_to_index(self, list):
        return self.row_to_index(list)

    def iid1_to_index(self, list):
        return self.col_to_index(list)

    @staticmethod
    def _makekey(item):
        return tuple(str(i) for i in item)

    def __getitem__(self, iid_indexer_and_snp_indexer):
        from pysnptools_amd.kernelreader._subset import _KernelSubset

        if isinstance(iid_indexer_and_snp_indexer, tuple):
            iid0_indexer, iid1_indexer = iid_indexer_and_snp_indexer
        else:
            iid0_indexer = iid1_indexer = iid_indexer_and_snp_indexer
        return _KernelSubset(self, iid0_indexer, iid1_indexer)

    def _assert_iid0_iid1(self, check_val):
        if check_val:
            assert self._val.ndim == 2, "val should have two dimensions"
            assert self._val.shape == (len(self._row), len(self._col)), \
                "val shape should match that of iid0_count x iid1_count"
        assert self._row.dtype.type is np.str_ and self._row.ndim == 2 and self._row.shape[1] == 2, \
            "iid0 should be dtype str, have two dimensions, and the second dimension should be size 2"
        assert self._col.dtype.type is np.str_ and self._col.ndim == 2 and self._col.shape[1] == 2, \
            "iid1 should be dtype str have two dimensions, and the second dimension should be size 2"

    def _read_with_standardizing(self, to_kerneldata, snp_standardizer=None, kernel_standardizer=DiagKtoN(),
                                 return_trained=False):
        assert to_kerneldata, "When working with non-SnpKernels, to_kerneldata must be 'True'"
        kernel, kernel_trained = self.read().standardize(kernel_standardizer, return_trained=True)
        return (kernel, None, kernel_trained) if return_trained else kernel

    @property
    def val_shape(self):
        return None
