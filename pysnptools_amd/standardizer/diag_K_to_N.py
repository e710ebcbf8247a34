"""DiagKtoN: scale so that trace(K) = N (reference standardizer/diag_K_to_N.py).

Every form runs on the GPU: on a kernel the trace and the scale (``snpmi_diag_k_to_n_*``;
the fused GRM path applies it before K leaves the device), on SNP data the sum of squares and
the sqrt(factor) scale (``snpmi_diag_k_to_n_snps_*``), and a trained factor through
``snpmi_scale_*``.  Non-contiguous or non-float inputs are staged through a contiguous copy.
"""
import warnings

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.standardizer.standardizer import Standardizer


def _float_work(val):
    """(contiguous float32/float64 array to operate on, whether it is a copy)."""
    if val.dtype in (np.float32, np.float64) and (val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]):
        return val, False
    return np.ascontiguousarray(val, dtype=val.dtype if val.dtype in (np.float32, np.float64) else np.float64), True


def _factor_ptr(f):
    return f.ctypes.data_as(N.ctypes.POINTER(N.ctypes.c_double))


def _scale_kernel_inplace(kerneldata):
    """factor = N / trace(K); K *= factor when |factor - 1| > 1e-15 (diag_K_to_N.py:54-64)."""
    val = kerneldata._val
    n = val.shape[0]
    assert val.shape == (n, n), "DiagKtoN expects a square kernel"
    work, copied = _float_work(val)
    f = np.zeros(1, dtype=np.float64)
    # trace and scale are layout independent for a square matrix held contiguously
    N.call("snpmi_diag_k_to_n_" + N.suffix(work.dtype), N.ptr(work), n, _factor_ptr(f))
    if copied:
        val[...] = work
    return float(f[0])


def _scale_inplace(val, scale):
    work, copied = _float_work(val)
    N.call("snpmi_scale_" + N.suffix(work.dtype), N.ptr(work), work.size, float(scale))
    if copied:
        val[...] = work


class DiagKtoN(Standardizer):
    """diag(K)=N standardization of the data"""

    def __init__(self, deprecated_iid_count=None):
        super(DiagKtoN, self).__init__()
        if deprecated_iid_count is not None:
            warnings.warn("'iid_count' is deprecated (and not needed, since can get iid_count from SNPs val's first dimension",
                          DeprecationWarning)

    def __repr__(self):
        return "{0}()".format(self.__class__.__name__)

    def standardize(self, input, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        from pysnptools_amd.kernelreader import KernelReader

        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        if isinstance(input, KernelReader) and hasattr(input, "val"):
            factor = _scale_kernel_inplace(input)
            return (input, DiagKtoNTrained(factor)) if return_trained else input
        return self._standardize_snps(input, return_trained=return_trained)

    def _standardize_snps(self, snps, return_trained=False, force_python_only=False, num_threads=None):
        """factor = rows / sum(val^2); val *= sqrt(factor) (diag_K_to_N.py:75-95), on the GPU."""
        if hasattr(snps, "val"):
            val = snps.val
        else:
            warnings.warn("standardizing an nparray instead of a SnpData is deprecated", DeprecationWarning)
            val = snps
        work, copied = _float_work(val)
        f = np.zeros(1, dtype=np.float64)
        N.call("snpmi_diag_k_to_n_snps_" + N.suffix(work.dtype), N.ptr(work), work.shape[0],
               int(np.prod(work.shape[1:])), _factor_ptr(f))
        if copied:
            val[...] = work
        factor = float(f[0])
        return (snps, DiagKtoNTrained(factor)) if return_trained else snps


class DiagKtoNTrained(Standardizer):
    def __init__(self, factor):
        super(DiagKtoNTrained, self).__init__()
        self.factor = factor

    @property
    def is_constant(self):
        return abs(self.factor - 1.0) < 1e-15

    def __repr__(self):
        return "{0}({1})".format(self.__class__.__name__, self.factor)

    def standardize(self, input, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        from pysnptools_amd.kernelreader import KernelReader

        if isinstance(input, KernelReader) and hasattr(input, "val"):
            if not self.is_constant:
                _scale_inplace(input._val, self.factor)
        else:
            val = input.val if hasattr(input, "val") else input
            if not self.is_constant:
                _scale_inplace(val, np.sqrt(self.factor))
        return (input, self) if return_trained else input
