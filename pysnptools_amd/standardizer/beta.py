"""Beta(a, b) standardizer: (x - mean) * BetaPDF(maf; a, b), missing -> 0
(reference standardizer/beta.py, weights standardizer.py:199-205)."""
import warnings

import numpy as np

from pysnptools_amd.standardizer.standardizer import Standardizer


class Beta(Standardizer):
    def __init__(self, a, b):
        super(Beta, self).__init__()
        self.a = a
        self.b = b

    def __repr__(self):
        return "{0}(a={1},b={2})".format(self.__class__.__name__, self.a, self.b)

    def standardize(self, snpdata, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        from pysnptools_amd.standardizer.betatrained import BetaTrained

        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        if hasattr(snpdata, "val"):
            val = snpdata.val
        else:
            warnings.warn("standardizing an nparray instead of a SnpData is deprecated", DeprecationWarning)
            val = snpdata
        stats = self._standardize_unit_and_beta(val, is_beta=True, a=self.a, b=self.b, apply_in_place=True,
                                                use_stats=False, stats=None, num_threads=num_threads,
                                                force_python_only=force_python_only)
        if return_trained:
            assert hasattr(snpdata, "val"), "return_trained=True must be used with SnpData"
            return snpdata, BetaTrained(self.a, self.b, snpdata.sid, stats)
        return snpdata

    def _merge_trained(self, trained_list):
        from pysnptools_amd.standardizer.betatrained import BetaTrained

        sid = np.concatenate([t.sid for t in trained_list])
        stats = np.concatenate([t.stats for t in trained_list])
        a_set = {t.a for t in trained_list}
        b_set = {t.b for t in trained_list}
        assert len(a_set) <= 1, "Expect all BetaTrained's to have the same 'a'"
        assert len(b_set) <= 1, "Expect all BetaTrained's to have the same 'b'"
        return BetaTrained(next(iter(a_set), None), next(iter(b_set), None), sid, stats)
