"""SNP-wise concatenation of readers that share their iids (reference
pstreader/_mergecols.py:8-159 + snpreader/_mergesids.py:5-25) -- the in-memory face of
DistributedBed and of per-chromosome / per-GPU SNP shards.

Reads dispatch each requested SNP range to its piece (every piece a native BED read).  The
GRM of a merged set of Beds runs as one GPU session (``snpmi_grm_begin`` / ``add_bed`` per
piece / ``end``): K accumulates in HBM across pieces; see ``SnpReader._read_kernel``.
"""
import numpy as np

from pysnptools_amd.pstreader._mergecols import _MergeCols
from pysnptools_amd.snpreader.snpreader import SnpReader


class _MergeSIDs(_MergeCols, SnpReader):
    """SNP shards sharing their iids (snpreader/_mergesids.py:5-25): the generic column merge with
    the SnpReader API; the .bed-only case feeds the GRM session (SnpReader._read_kernel)."""

    _count_key = "sid_count_list"

    def __init__(self, reader_list, cache_file=None, skip_check=False):
        super(_MergeSIDs, self).__init__(reader_list, cache_file=cache_file, skip_check=skip_check)

    def _load(self, cache_file):
        _MergeCols._load(self, cache_file)
        self._col_property = np.array(self._col_property, dtype=np.float64)
