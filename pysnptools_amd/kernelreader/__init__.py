from pysnptools_amd.kernelreader.kernelreader import KernelReader
from pysnptools_amd.kernelreader.kerneldata import KernelData
from pysnptools_amd.kernelreader.snpkernel import SnpKernel
from pysnptools_amd.kernelreader.kernelnpz import KernelNpz
from pysnptools_amd.kernelreader.partitionedkernel import PartitionedKernel, set_grm_partition  # noqa: E402
