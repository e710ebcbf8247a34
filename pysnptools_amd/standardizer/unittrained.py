"""Unit standardizer with fixed (trained) stats (reference standardizer/unittrained.py)."""
import warnings

import numpy as np

from pysnptools_amd.standardizer.standardizer import Standardizer


class UnitTrained(Standardizer):
    def __init__(self, sid, stats):
        super(UnitTrained, self).__init__()
        self.sid = sid
        self.stats = stats
        self.sid_to_index = None

    def __repr__(self):
        return "{0}(stats={1},sid={2})".format(self.__class__.__name__, self.stats, self.sid)

    @property
    def is_constant(self):
        return True

    def stats_for(self, sid):
        """Stats rows for ``sid`` (re-mapped by name when the order differs, unittrained.py:53-58)."""
        if len(self.sid) == len(sid) and np.array_equal(self.sid, sid):
            return self.stats
        if self.sid_to_index is None:
            self.sid_to_index = {s: i for i, s in enumerate(self.sid)}
        return np.array([self.stats[self.sid_to_index[s]] for s in sid]).reshape(-1, 2)

    def standardize(self, snps, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        if hasattr(snps, "val"):
            val, stats = snps.val, self.stats_for(snps.sid)
        else:
            warnings.warn("standardizing an nparray instead of a SnpData is deprecated", DeprecationWarning)
            val, stats = snps, self.stats
        self._standardize_unit_and_beta(val, is_beta=False, a=np.nan, b=np.nan, apply_in_place=True, use_stats=True,
                                        stats=stats, num_threads=num_threads, force_python_only=force_python_only)
        return (snps, self) if return_trained else snps
