from pysnptools_amd.pstreader.pstreader import PstReader
from pysnptools_amd.pstreader.pstdata import PstData
from pysnptools_amd.pstreader._subset import _PstSubset
from pysnptools_amd.pstreader.pstmemmap import PstMemMap
from pysnptools_amd.pstreader._mergecols import _MergeCols
