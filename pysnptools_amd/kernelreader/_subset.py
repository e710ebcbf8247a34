from pysnptools_amd.kernelreader.kernelreader import KernelReader
from pysnptools_amd.pstreader._subset import _PstSubset


class _KernelSubset(KernelReader, _PstSubset):
    def __init__(self, *args, **kwargs):
        super(_KernelSubset, self).__init__(*args, **kwargs)
