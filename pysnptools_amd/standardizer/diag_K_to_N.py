"""DiagKtoN: scale so that trace(K) = N (reference standardizer/diag_K_to_N.py).

On a kernel the trace and the scale run on the GPU (``snpmi_diag_k_to_n_*``); the fused
GRM path applies it before K leaves the device (``snpmi_grm_*(..., diag_k_to_n=1)``).
"""
import warnings

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.standardizer.standardizer import Standardizer


def _scale_kernel_inplace(kerneldata):
    """factor = N / trace(K); K *= factor when |factor - 1| > 1e-15 (diag_K_to_N.py:54-64)."""
    val = kerneldata._val
    n = val.shape[0]
    if val.dtype in (np.float32, np.float64) and val.shape == (n, n) and (val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]):
        f = np.zeros(1, dtype=np.float64)
        fn = "snpmi_diag_k_to_n_" + N.suffix(val.dtype)
        # trace and scale are layout independent for a square matrix held contiguously
        N.call(fn, N.ptr(val), n, f.ctypes.data_as(N.ctypes.POINTER(N.ctypes.c_double)))
        return float(f[0])
    factor = float(kerneldata.iid_count) / np.diag(val).sum()
    if abs(factor - 1.0) > 1e-15:
        kerneldata._val *= factor
    return factor


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
        val = snps.val if hasattr(snps, "val") else snps
        squared_sum = float(np.vdot(val.reshape(-1, order="A"), val.reshape(-1, order="A")))
        factor = float(val.shape[0]) / squared_sum
        if abs(factor - 1.0) > 1e-15:
            val *= np.sqrt(factor)
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
                input._val *= self.factor
        else:
            val = input.val if hasattr(input, "val") else input
            if not self.is_constant:
                val *= np.sqrt(self.factor)
        return (input, self) if return_trained else input
