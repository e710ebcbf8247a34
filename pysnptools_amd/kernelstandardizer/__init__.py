"""Kernel standardizers (reference kernelstandardizer/__init__.py)."""


class KernelStandardizer(object):
    def standardize(self, kerneldata, return_trained=False, force_python_only=False, num_threads=None):
        raise NotImplementedError("subclass {0} needs to implement method '.standardize'".format(
            self.__class__.__name__))


class Identity(KernelStandardizer):
    def __init__(self):
        super(Identity, self).__init__()

    def standardize(self, kerneldata, return_trained=False, force_python_only=False, num_threads=None):
        return (kerneldata, self) if return_trained else kerneldata

    def __repr__(self):
        return "{0}()".format(self.__class__.__name__)


from pysnptools_amd.standardizer import DiagKtoN, DiagKtoNTrained  # noqa: E402
