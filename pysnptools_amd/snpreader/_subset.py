from pysnptools_amd.pstreader._subset import _PstSubset
from pysnptools_amd.snpreader.snpreader import SnpReader


class _SnpSubset(_PstSubset, SnpReader):
    def __init__(self, *args, **kwargs):
        super(_SnpSubset, self).__init__(*args, **kwargs)
