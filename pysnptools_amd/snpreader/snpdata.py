"""In-memory SNP matrix (reference snpreader/snpdata.py)."""
import numpy as np

from pysnptools_amd.pstreader import PstData
from pysnptools_amd.snpreader.snpreader import SnpReader
from pysnptools_amd.standardizer import Identity, Unit


class SnpData(PstData, SnpReader):
    """iid x sid values in memory (``val``), with ``iid`` (N x 2 str), ``sid`` and ``pos`` (M x 3)."""

    def __init__(self, iid, sid, val, pos=None, name=None, parent_string=None, copyinputs_function=None, xp=None,
                 _require_float32_64=True):
        self._val = None
        self._row = PstData._fixup_input(iid, empty_creator=lambda ignore: np.empty([0, 2], dtype="str"), dtype="str")
        self._col = PstData._fixup_input(sid, empty_creator=lambda ignore: np.empty([0], dtype="str"), dtype="str")
        self._row_property = PstData._fixup_input(None, count=len(self._row),
                                                  empty_creator=lambda count: np.empty([count, 0], dtype="str"),
                                                  dtype="str")
        self._col_property = PstData._fixup_input(pos, count=len(self._col),
                                                  empty_creator=lambda count: np.full([count, 3], np.nan))
        self._val = PstData._fixup_input_val(val, row_count=len(self._row), col_count=len(self._col),
                                             _require_float32_64=_require_float32_64, xp=xp)
        self._xp = xp
        self._assert_iid_sid_pos()
        self._name = name or parent_string or ""
        self._std_string_list = []

    def _assert_iid_sid_pos(self):
        assert self._val.shape[:2] == (len(self._row), len(self._col)), "val shape should match that of iid_row x sid_row"
        assert self._row.dtype.type is np.str_ and self._row.ndim == 2 and self._row.shape[1] == 2, \
            "iid should be dtype str, have two dimensions, and the second dimension should be size 2"
        assert self._col.dtype.type is np.str_ and self._col.ndim == 1, "sid should be of dtype of str and one dimensional"

    @property
    def val(self):
        return self._val

    @val.setter
    def val(self, new_value):
        self._val = PstData._fixup_input_val(new_value, row_count=len(self._row), col_count=len(self._col),
                                             xp=self._xp)
        self._assert_iid_sid_pos()

    def allclose(self, value, equal_nan=True):
        return PstData.allclose(self, value, equal_nan=equal_nan)

    def standardize(self, standardizer=Unit(), block_size=None, return_trained=False, force_python_only=False,
                    num_threads=None):
        """Standardize ``val`` in place (on the GPU); returns self (and the trained standardizer)."""
        self._std_string_list.append(str(standardizer))
        _, trained = standardizer.standardize(self, return_trained=True, force_python_only=force_python_only,
                                              num_threads=num_threads)
        return (self, trained) if return_trained else self

    def _read_kernel(train, standardizer, block_size=None, order="A", dtype=np.float64, force_python_only=False,
                     view_ok=False, return_trained=False, num_threads=None, _diag_k_to_n=False):
        """K = val val^T (snpdata.py:190-214) when already standardized, else the general path."""
        return SnpReader._read_kernel(train, standardizer, block_size=block_size, order=order, dtype=dtype,
                                      force_python_only=force_python_only, view_ok=view_ok,
                                      return_trained=return_trained, num_threads=num_threads,
                                      _diag_k_to_n=_diag_k_to_n)

    def __repr__(self):
        stds = ",".join(self._std_string_list)
        if self._name == "":
            return "{0}({1})".format(self.__class__.__name__, stds)
        return "{0}({1}{2})".format(self.__class__.__name__, self._name, "," + stds if stds else "")
