"""Standardizer base + the native dispatcher (reference standardizer/standardizer.py).

``_standardize_unit_and_beta`` is the drop-in point of bed-reader's ``standardize_f32/f64``
(standardizer.py:90-133): it runs ``snpmi_standardize_{f32,f64}`` (HIP) in place.  The
reference's NumPy fallback for non-contiguous or non-float arrays is replaced by a
contiguous staging copy -- there is no CPU arithmetic path.
"""
import warnings

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.util import get_num_threads


def _std_args(standardizer):
    """(kind, a, b, use_stats, stats, sid) the native GRM/read paths understand, or None."""
    from pysnptools_amd.standardizer import Beta, BetaTrained, Identity, Unit, UnitTrained

    if isinstance(standardizer, Unit):
        return (N.STD_UNIT, np.nan, np.nan, False, None, None)
    if isinstance(standardizer, Beta):
        return (N.STD_BETA, float(standardizer.a), float(standardizer.b), False, None, None)
    if isinstance(standardizer, UnitTrained):
        return (N.STD_UNIT, np.nan, np.nan, True, standardizer.stats, standardizer.sid)
    if isinstance(standardizer, BetaTrained):
        return (N.STD_BETA, float(standardizer.a), float(standardizer.b), True, standardizer.stats, standardizer.sid)
    if isinstance(standardizer, Identity):
        return (N.STD_NONE, np.nan, np.nan, False, None, None)
    return None


class Standardizer(object):
    """Base class of SNP standardizers (``Unit``, ``Beta``, trained forms, ``Identity``)."""

    def __init__(self):
        super(Standardizer, self).__init__()

    def standardize(self, snps, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        raise NotImplementedError("subclass {0} needs to implement method '.standardize'".format(
            self.__class__.__name__))

    @property
    def is_constant(self):
        return False

    def _merge_trained(self, trained_list):
        raise Exception("Not defined")

    @staticmethod
    def _standardize_unit_and_beta(snps, is_beta, a, b, apply_in_place, use_stats, stats, num_threads,
                                   force_python_only=False):
        """In-place Unit/Beta standardization of ``snps`` (iid x sid) on the GPU; returns stats
        [sid_count, 2] (mean, std) in snps' dtype and order.  ``force_python_only`` is accepted
        for API compatibility; the HIP path is the only implementation."""
        assert snps.flags["C_CONTIGUOUS"] or snps.flags["F_CONTIGUOUS"], "Expect snps to be order 'C' or order 'F'"
        assert snps.dtype in (np.float64, np.float32), "snps must be a float in order to standardize in place."
        order_c = 1 if snps.flags["C_CONTIGUOUS"] else 0
        rows, cols = snps.shape
        stats_c = np.empty((cols, 2), dtype=snps.dtype)
        if use_stats:
            given = np.asarray(stats, dtype=snps.dtype)
            assert given.shape == (cols, 2), "stats must have size [sid_count,2]"
            stats_c[...] = given
        fn = "snpmi_standardize_" + N.suffix(snps.dtype)
        N.call(fn, N.ptr(snps), rows, cols, order_c, int(bool(is_beta)), float(a), float(b), int(bool(apply_in_place)),
               int(bool(use_stats)), N.ptr(stats_c), get_num_threads(num_threads))
        order = "F" if (snps.flags["F_CONTIGUOUS"] and not snps.flags["C_CONTIGUOUS"]) else "C"
        if use_stats:
            return stats if isinstance(stats, np.ndarray) else stats_c
        return np.array(stats_c, order=order)


class _CannotBeTrained(Standardizer):
    def __init__(self, name):
        super(_CannotBeTrained, self).__init__()
        self.name = name

    def __repr__(self):
        return "{0}({1})".format(self.__class__.__name__, self.name)

    def standardize(self, snps, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        raise Exception("Standardizer '{0}' cannot be trained".format(self))
