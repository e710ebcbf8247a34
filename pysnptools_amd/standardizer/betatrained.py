"""Beta standardizer with fixed (trained) stats (reference standardizer/betatrained.py)."""
import warnings

import numpy as np

from pysnptools_amd.standardizer.standardizer import Standardizer


class BetaTrained(Standardizer):
    def __init__(self, a, b, sid, stats):
        super(BetaTrained, self).__init__()
        self.a = a
        self.b = b
        self.sid = sid
        self.stats = stats

    def __repr__(self):
        return "{0}(a={1},b={2},stats={3},sid={4})".format(self.__class__.__name__, self.a, self.b, self.stats,
                                                          self.sid)

    @property
    def is_constant(self):
        return True

    def stats_for(self, sid):
        assert np.array_equal(self.sid, sid), "sid in training and use must be the same and in the same order"
        return self.stats

    def standardize(self, snps, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        if hasattr(snps, "val"):
            val, stats = snps.val, self.stats_for(snps.sid)
        else:
            warnings.warn("standardizing an nparray instead of a SnpData is deprecated", DeprecationWarning)
            val, stats = snps, self.stats
        self._standardize_unit_and_beta(val, is_beta=True, a=self.a, b=self.b, apply_in_place=True, use_stats=True,
                                        stats=stats, num_threads=num_threads, force_python_only=force_python_only)
        return (snps, self) if return_trained else snps
