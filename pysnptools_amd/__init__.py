"""pysnptools_amd -- MI355X-native (gfx950/HIP) BED decode -> slice -> standardize -> GRM.

A drop-in for PySnpTools' hot path (``Bed``, ``SnpData``, ``Unit``/``Beta`` standardizers,
``SnpKernel``/``read_kernel``, ``DiagKtoN``) whose arithmetic runs in libsnpmi.so
(include/snpmi.h).  There is no CPU fallback: compute calls raise if the HIP library or a
GPU is missing.
"""
__version__ = "0.1.0"

from pysnptools_amd import _native  # noqa: F401
