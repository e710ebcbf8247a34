"""pysnptools_amd -- MI355X-native (gfx950/HIP) BED decode -> slice -> standardize -> GRM.

A drop-in for PySnpTools' hot path (``Bed``, ``SnpData``, ``Unit``/``Beta`` standardizers,
``SnpKernel``/``read_kernel``, ``DiagKtoN``) whose arithmetic runs in libsnpmi.so
(include/snpmi.h).  There is no CPU fallback: compute calls raise if the HIP library or a
GPU is missing.
"""
__version__ = "0.1.0"

import os as _os

from pysnptools_amd import _native  # noqa: F401

_F64_GRM = {"crt": 0, "mfma": 1}


def set_grm_f64(path):
    """How float64 GRMs (the reference's default dtype) are computed on this process's GPU:

    * ``"crt"`` (default): exact integer products on the int8 MFMA.  Each SNP block's LUT values
      are quantised to integers at the block's exponent with F = 51-52 fraction bits (|error| <=
      2^-(F+1) of the block's largest |standardized value|); K_int is exact (residues modulo
      coprime moduli + Chinese remainder theorem) and converted to f64.  A block with a rare
      variant (|value| ~ sqrt(n)) costs typical values ~8 of their 52 bits: ~1e-13 relative per
      value (measured 1.9e-14 of max diag(K) vs the f64 oracle at 50k x 500k).  2.8x the f64 MFMA.
    * ``"mfma"``: the f64 MFMA (v_mfma_f64_16x16x4) on f64 standardized values -- every product
      rounded as NumPy's float64 dot does, for callers that need K accurate per element at the
      f64 rounding level.  ~3x slower.

    The environment variable ``PST_F64_GRM`` sets the default for new processes."""
    if path not in _F64_GRM:
        raise ValueError("set_grm_f64: path must be 'crt' or 'mfma'")
    _native.call("snpmi_set_kernel_variant", b"f64", _F64_GRM[path])


if _os.environ.get("PST_F64_GRM"):
    try:
        set_grm_f64(_os.environ["PST_F64_GRM"])
    except ImportError:  # no HIP library: every compute call raises anyway
        pass
    except ValueError as _e:  # a bad value must not break CPU-only imports
        import warnings as _warnings

        _warnings.warn("PST_F64_GRM=%r ignored: %s" % (_os.environ["PST_F64_GRM"], _e))
