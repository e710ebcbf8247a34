from pysnptools_amd.snpreader.snpreader import SnpReader
from pysnptools_amd.snpreader.snpdata import SnpData
from pysnptools_amd.snpreader.bed import Bed
from pysnptools_amd.snpreader._mergesids import _MergeSIDs
from pysnptools_amd.snpreader.distributedbed import DistributedBed
from pysnptools_amd.snpreader.snpmemmap import SnpMemMap
