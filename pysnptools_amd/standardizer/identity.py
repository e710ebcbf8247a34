"""No-op standardizer (reference standardizer/identity.py)."""
import warnings

from pysnptools_amd.standardizer.standardizer import Standardizer


class Identity(Standardizer):
    def __init__(self):
        super(Identity, self).__init__()

    def standardize(self, snps, block_size=None, return_trained=False, force_python_only=False, num_threads=None):
        if block_size is not None:
            warnings.warn("block_size is deprecated (and not needed, since standardization is in-place",
                          DeprecationWarning)
        return (snps, self) if return_trained else snps

    @property
    def is_constant(self):
        return True

    def __repr__(self):
        return "{0}()".format(self.__class__.__name__)

    def _merge_trained(self, trained_list):
        return self
