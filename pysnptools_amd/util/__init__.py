"""Utilities of the hot path: thread-count policy, the array-module seam and sub_matrix.

Mirrors ``pysnptools.util`` (reference util/__init__.py) for the functions the BED -> GRM
path uses.  ``sub_matrix`` runs as a HIP gather kernel (libsnpmi ``snpmi_subset_*``,
replacing bed-reader's ``subset_*``, util/__init__.py:341-375).
"""
import os
from types import ModuleType

import numpy as np

from pysnptools_amd import _native as N


def get_num_threads(num_threads=None):
    """bed-reader's thread policy (bed.py:34-36): argument, else PST_NUM_THREADS, NUM_THREADS,
    MKL_NUM_THREADS, else the CPU count."""
    if num_threads is not None:
        return int(num_threads)
    for key in ("PST_NUM_THREADS", "NUM_THREADS", "MKL_NUM_THREADS"):
        if key in os.environ:
            return int(os.environ[key])
    return os.cpu_count() or 1


def array_module(xp=None):
    """The array module of the host API.  Values handed to and from the API are NumPy
    arrays; device residency is managed inside libsnpmi (the reference's optional CuPy
    seam, util/__init__.py:652-695, has no counterpart: the GPU path is always on)."""
    xp = xp or os.environ.get("ARRAY_MODULE", "numpy")
    if isinstance(xp, ModuleType):
        return xp
    if xp in ("numpy", "cupy"):
        return np
    raise ValueError("Don't know ARRAY_MODULE '%s'" % xp)


def asnumpy(a):
    return np.asarray(a)


def get_array_module(a):
    return np


def sub_matrix(val, row_index_list, col_index_list, order="A", dtype=np.float64, num_threads=None):
    """Gather ``val[row_index_list][:, col_index_list]`` (2-D or 3-D) into a new array of
    ``dtype`` and ``order`` ('A' = F if val is F-contiguous else C), util/__init__.py:271-393."""
    eff = ("F" if val.flags["F_CONTIGUOUS"] else "C") if order == "A" else order
    dtype = np.dtype(dtype)
    if val.ndim == 2:
        rows, cols = val.shape
        k = 1
    elif val.ndim == 3:
        rows, cols, k = val.shape
    else:
        raise ValueError("Expect val dimensions of 2 or 3")
    if not (val.flags["F_CONTIGUOUS"] or val.flags["C_CONTIGUOUS"]):
        raise Exception("input order must be 'F' or 'C'")
    ri = N.index_array(row_index_list)
    ci = N.index_array(col_index_list)
    shape = (len(ri), len(ci)) if val.ndim == 2 else (len(ri), len(ci), k)
    if val.dtype == np.float64:
        fn, work = "snpmi_subset_f64_f64", np.float64
    elif val.dtype == np.float32:
        fn, work = ("snpmi_subset_f32_f32", np.float32) if dtype == np.float32 else ("snpmi_subset_f32_f64", np.float64)
    else:
        raise Exception("input dtype '%s' not known, only float64 and float32" % val.dtype)
    if dtype not in (np.float32, np.float64):
        raise Exception("dtype '%s' not known, only float64 and float32" % dtype)
    out = np.empty(shape, dtype=work, order=eff)
    if out.size:
        in_c = 1 if val.flags["C_CONTIGUOUS"] else 0
        N.call(fn, N.ptr(val), rows, cols, k, in_c, N.ptr(ri), len(ri), N.ptr(ci), len(ci),
               0 if eff == "F" else 1, N.ptr(out), get_num_threads(num_threads))
    if out.dtype != dtype:
        out = out.astype(dtype, order=eff)
    return out
