"""Utilities of the hot path: thread-count policy, the array-module seam and sub_matrix.

Mirrors ``pysnptools.util`` (reference util/__init__.py) for the functions the BED -> GRM
path uses.  ``sub_matrix`` runs as a HIP gather kernel (libsnpmi ``snpmi_subset_*``,
replacing bed-reader's ``subset_*``, util/__init__.py:341-375).
"""
import logging
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


_warn_array_module_once = False


def array_module(xp=None):
    """The array module that holds ``val`` of SnpData / KernelData (util/__init__.py:652-695):
    the argument, else the ARRAY_MODULE environment variable, else numpy.  ``'hbm'`` selects
    :mod:`pysnptools_amd.hbm` (values resident in the GPU's HBM; the compute is on the GPU either
    way).  ``'cupy'`` imports CuPy if it is installed, else falls back to numpy with one warning,
    as the reference does."""
    xp = xp or os.environ.get("ARRAY_MODULE", "numpy")
    if isinstance(xp, ModuleType):
        return xp
    if xp == "numpy":
        return np
    if xp == "hbm":
        from pysnptools_amd import hbm

        return hbm
    if xp == "cupy":
        try:
            import cupy as cp

            return cp
        except ModuleNotFoundError as e:
            global _warn_array_module_once
            if not _warn_array_module_once:
                logging.warning("Using numpy. (%s)" % e)
                _warn_array_module_once = True
            return np
    raise ValueError("Don't know ARRAY_MODULE '%s'" % xp)


def asnumpy(a):
    """A NumPy array of ``a`` (device arrays are copied to the host; util/__init__.py:698-713)."""
    if isinstance(a, np.ndarray):
        return a
    return a.get()


def get_array_module(a):
    """The array module of ``a`` (util/__init__.py:716-730)."""
    from pysnptools_amd import hbm

    if isinstance(a, hbm.HbmArray):
        return hbm
    return np


def _on_device(*arrays):
    """True when values should live in HBM: any of ``arrays`` already does, or ARRAY_MODULE=hbm."""
    from pysnptools_amd import hbm

    return any(isinstance(a, hbm.HbmArray) for a in arrays) or array_module() is hbm


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
    from pysnptools_amd import hbm

    dev = isinstance(val, hbm.HbmArray)  # a device input gives a device output (no host copy)
    if val.dtype == np.float64:
        fn, work = "snpmi_subset_f64_f64", np.float64
    elif val.dtype == np.float32:
        fn, work = ("snpmi_subset_f32_f32", np.float32) if dtype == np.float32 else ("snpmi_subset_f32_f64", np.float64)
    else:
        raise Exception("input dtype '%s' not known, only float64 and float32" % val.dtype)
    if dtype not in (np.float32, np.float64):
        raise Exception("dtype '%s' not known, only float64 and float32" % dtype)
    out = hbm.empty(shape, dtype=work, order=eff) if dev else np.empty(shape, dtype=work, order=eff)
    if out.size:
        in_c = 1 if val.flags["C_CONTIGUOUS"] else 0
        N.call(fn, N.ptr(val), rows, cols, k, in_c, N.ptr(ri), len(ri), N.ptr(ci), len(ci),
               0 if eff == "F" else 1, N.ptr(out), get_num_threads(num_threads))
    if out.dtype != dtype:
        out = out.astype(dtype, order=eff)
    return out


# ---------------------------------------------------------------------- iid intersection (util/__init__.py:18-265)
def _all_same(iids_list):
    for a, b in zip(iids_list[:-1], iids_list[1:]):
        if not np.array_equal(a, b):
            return False
    return True


def intersect_ids(idslist):
    """(deprecated in the reference) N x L int array: for each iid present in every non-None
    list, its index in each list (-1 for None lists); rows ordered by the first non-None
    list's index, then sorted on column 0 as the reference does (util/__init__.py:221-265).
    A repeated id takes the index of its last occurrence."""
    L = len(idslist)
    observed = np.array([ids is not None for ids in idslist], dtype=bool)
    order = []
    index = {}
    first = True
    for k, ids in enumerate(idslist):
        if ids is None:
            continue
        ids = np.asarray(ids)
        keys = list(zip(ids[:, 0].tolist(), ids[:, 1].tolist()))
        if first:
            first = False
            for i, key in enumerate(keys):
                if key not in index:
                    order.append(key)
                entry = np.full(L, np.nan)
                entry[k] = i
                index[key] = entry
        else:
            for i, key in enumerate(keys):
                e = index.get(key)
                if e is not None:
                    e[k] = i
    indarr = np.array([index[key] for key in order], dtype=float).reshape(len(order), L)
    indarr[:, ~observed] = -1
    indarr = indarr[~np.isnan(indarr).any(1)]
    indarr = np.array(indarr, dtype=int)
    return indarr[indarr[:, 0].argsort()]


def _reindex_snpkernel(snpkernel, iididx, is_test=False):
    """Intersect BEFORE standardizing: the SNP reader is iid-subset, so the GRM decodes only
    those iids (the iid-gather path of snpmi_grm_bed_*, k_repack)."""
    from pysnptools_amd.kernelreader import SnpKernel

    assert not is_test, "test kernels (iid1 != iid0) are not on the GRM path"
    return SnpKernel(snpkernel.snpreader[iididx, :], snpkernel.standardizer, block_size=snpkernel.block_size)


def _reindex_phen_dict(phen_dict, iididx):
    vals = phen_dict["vals"]
    phen_dict["vals"] = vals[iididx] if vals.ndim == 1 else vals[iididx, :]
    phen_dict["iid"] = phen_dict["iid"][iididx]
    return phen_dict


def intersect_apply(data_list, sort_by_dataset=True, intersect_before_standardize=True, is_test=False):
    """Restrict every dataset to the iids they all share, in one consistent order
    (util/__init__.py:18-173).  Accepts None, SnpReader, KernelReader (SnpKernel: subset
    before standardization when ``intersect_before_standardize``), phenotype dicts
    {'iid','vals'} and (val, iid) tuples; returns the list unchanged if the iids already agree."""
    from pysnptools_amd.kernelreader import SnpKernel

    iid_list, reindex_list = [], []
    for data in data_list:
        if data is None:
            iid, reindex = None, (lambda data, idx: None)
        elif intersect_before_standardize and isinstance(data, SnpKernel):
            iid = data.iid1 if is_test else data.iid0
            reindex = (lambda data, idx, t=is_test: _reindex_snpkernel(data, idx, t))
        elif isinstance(data, dict):
            iid, reindex = data["iid"], _reindex_phen_dict
        elif isinstance(data, tuple):
            iid = data[1]
            reindex = (lambda data, idx: (data[0][idx], data[1][idx]))
        elif hasattr(data, "iid1") and is_test:
            iid, reindex = data.iid1, (lambda data, idx: data[:, idx])
        else:
            iid = data.iid
            square = hasattr(data, "col") and iid is data.col
            reindex = (lambda data, idx: data[idx]) if square else (lambda data, idx: data[idx, :])
        iid_list.append(iid)
        reindex_list.append(reindex)
    if len(iid_list) == 0:
        raise Exception("Expect a least one input item")
    if _all_same(iid_list):
        return data_list
    indarr = intersect_ids(iid_list)
    assert indarr.shape[0] > 0, "no individuals remain after intersection, check that ids match in files"
    if sort_by_dataset:
        for k, iid in enumerate(iid_list):
            if iid is not None:
                indarr = indarr[np.argsort(indarr[:, k])]
                break
    return [reindex_list[k](data_list[k], indarr[:, k]) for k in range(indarr.shape[1])]
