"""SnpKernel: the lazy GRM of a SnpReader + standardizer (reference kernelreader/snpkernel.py).

Reading it runs the fused GPU GRM (SnpReader._read_kernel); for constant (trained)
standardizers an iid subset is pushed down to the SNP reader so only the requested
individuals are decoded (snpkernel.py:81-82, 98-99).
"""
import logging

import numpy as np

from pysnptools_amd.kernelreader.kerneldata import KernelData
from pysnptools_amd.kernelreader.kernelreader import KernelReader
from pysnptools_amd.kernelstandardizer import DiagKtoN
from pysnptools_amd.standardizer import Identity as SS_Identity


class SnpKernel(KernelReader):
    def __init__(self, snpreader, standardizer=None, block_size=None):
        super(SnpKernel, self).__init__()
        assert standardizer is not None, "'standardizer' must be provided"
        self.snpreader = snpreader
        self.standardizer = standardizer
        self.block_size = block_size

    @property
    def row(self):
        return self.snpreader.iid

    @property
    def col(self):
        return self._col if hasattr(self, "_col") else self.snpreader.iid

    def __repr__(self):
        return self._internal_repr(self.standardizer)

    def _internal_repr(self, standardizer):
        s = "SnpKernel({0},standardizer={1}".format(self.snpreader, standardizer)
        if self.block_size is not None:
            s += ",block_size={0}".format(self.block_size)
        return s + ")"

    def copyinputs(self, copier):
        copier.input(self.snpreader)
        copier.input(self.standardizer)

    def _partitioned(self, dtype, num_threads=None):
        """The K of this SnpKernel computed partitioned over the process group (cfg5,
        ``shard.grm_partitioned``: each rank keeps its 256x256 blocks in HBM) when
        ``partitionedkernel.use_partitioned`` says the replicated K does not fit (or the mode is
        "always"), as a ``PartitionedKernel``.  The answer -- the blocks, or None: the replicated path
        applies -- is cached per (dtype, partition mode, group), so later sub-matrix reads of this
        SnpKernel reuse the blocks and an "auto" decision runs its group collective once; the cache
        holds HBM (cfg5: tens of GB per rank) until ``release_partitioned()`` and is never pickled."""
        from pysnptools_amd import dist as dist_mod
        from pysnptools_amd.kernelreader.partitionedkernel import (PartitionedKernel, grm_partition_mode,
                                                                   use_partitioned)
        from pysnptools_amd.snpreader.bed import Bed
        from pysnptools_amd.snpreader.snpreader import _resolve
        from pysnptools_amd.standardizer.standardizer import _std_args

        dtype = np.dtype(dtype)
        group = dist_mod.current()
        key = (dtype.str, grm_partition_mode(), id(group), group.world if group is not None else 1)
        cache = self.__dict__.setdefault("_pk", {})
        if key in cache:
            return cache[key]
        if dtype not in (np.float32, np.float64) or _std_args(self.standardizer) is None:
            return None
        if not isinstance(_resolve(self.snpreader)[0], Bed) or not use_partitioned(self.snpreader.iid_count, dtype,
                                                                                   group):
            cache[key] = None
            return None
        from pysnptools_amd import shard

        kw = {} if self.block_size is None else {"block_size": int(self.block_size)}
        blocks, _, trained = shard.grm_partitioned(self.snpreader, self.standardizer, out="hbm", dtype=dtype,
                                                   num_threads=num_threads, dist=group, **kw)
        pk = PartitionedKernel(self.snpreader.iid, blocks, dist=group, name=str(self))
        pk.snp_trained = trained
        cache[key] = pk
        return pk

    def release_partitioned(self):
        """Drop the cached partitioned K (frees its HBM blocks) and the cached routing decisions."""
        self.__dict__.pop("_pk", None)

    def __getstate__(self):
        state = dict(self.__dict__)
        state.pop("_pk", None)  # device memory and group-bound decisions do not travel
        return state

    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        dtype = np.dtype(dtype)
        if (self.standardizer.is_constant and row_index_or_none is not None and col_index_or_none is not None
                and np.array_equal(row_index_or_none, col_index_or_none)):
            sub = SnpKernel(self.snpreader[row_index_or_none, :], self.standardizer, block_size=self.block_size)
            pk = sub._partitioned(dtype, num_threads)
            if pk is not None:
                return pk._read(None, None, order, dtype, force_python_only, view_ok, num_threads)
            return sub.snpreader._read_kernel(self.standardizer, self.block_size, order, dtype, force_python_only,
                                              view_ok, num_threads=num_threads)
        pk = self._partitioned(dtype, num_threads)
        if pk is not None:
            return pk._read(row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok,
                            num_threads)
        whole = self.snpreader._read_kernel(self.standardizer, self.block_size, order, dtype, force_python_only,
                                            view_ok, num_threads=num_threads)
        val, _ = self._apply_sparray_or_slice_to_val(whole, row_index_or_none, col_index_or_none, order, dtype,
                                                     force_python_only, num_threads)
        return val

    def __getitem__(self, iid_indexer_and_snp_indexer):
        if isinstance(iid_indexer_and_snp_indexer, tuple):
            row_index_or_none, col_index_or_none = iid_indexer_and_snp_indexer
        else:
            row_index_or_none = col_index_or_none = iid_indexer_and_snp_indexer
        if (self.standardizer.is_constant and row_index_or_none is not None and col_index_or_none is not None
                and np.array_equal(row_index_or_none, col_index_or_none)):
            return SnpKernel(self.snpreader[row_index_or_none, :], self.standardizer, block_size=self.block_size)
        return KernelReader.__getitem__(self, iid_indexer_and_snp_indexer)

    def _read_with_standardizing(self, to_kerneldata, kernel_standardizer=DiagKtoN(), return_trained=False,
                                 num_threads=None):
        """(K, snp_trained, kernel_trained) as FaST-LMM uses it (snpkernel.py:104-132).  With the
        default DiagKtoN, the trace and scale run on the GPU before K is copied out."""
        logging.info("Starting '_read_with_standardizing'")
        from pysnptools_amd.kernelreader.partitionedkernel import PartitionedKernel

        pk = (self._partitioned(np.float64, num_threads)
              if to_kerneldata and PartitionedKernel.supports(kernel_standardizer) else None)
        if pk is not None:  # K partitioned over the group: DiagKtoN from the trace summed over the parts
            kernel, _, kernel_trained = pk._read_with_standardizing(to_kerneldata, None, kernel_standardizer,
                                                                    return_trained=True, num_threads=num_threads)
            return (kernel, pk.snp_trained, kernel_trained) if return_trained else kernel
        if to_kerneldata:
            from pysnptools_amd.standardizer import DiagKtoNTrained
            from pysnptools_amd.standardizer.diag_K_to_N import DiagKtoN as _DiagKtoN

            fused = type(kernel_standardizer) is _DiagKtoN
            res = self.snpreader._read_kernel(self.standardizer, block_size=self.block_size, return_trained=True,
                                              num_threads=num_threads, _diag_k_to_n=fused)
            val, snp_trained = res[0], res[1]
            kernel = KernelData(iid=self.snpreader.iid, val=val, name=str(self))
            if fused and res[2] is not None:
                kernel_trained = DiagKtoNTrained(res[2])
            else:
                kernel, kernel_trained = kernel.standardize(kernel_standardizer, return_trained=True,
                                                            num_threads=num_threads)
        else:
            from pysnptools_amd.snpreader.snpreader import _read_and_standardize

            snpdata, snp_trained = _read_and_standardize(self.snpreader, self.standardizer, num_threads=num_threads)
            snpdata, kernel_trained = snpdata.standardize(kernel_standardizer, return_trained=True,
                                                          num_threads=num_threads)
            kernel = SnpKernel(snpdata, SS_Identity())
        logging.info("Ending '_read_with_standardizing'")
        return (kernel, snp_trained, kernel_trained) if return_trained else kernel

    @property
    def sid(self):
        return self.snpreader.sid

    @property
    def sid_count(self):
        return self.snpreader.sid_count

    @property
    def pos(self):
        return self.snpreader.pos

    def read_snps(self, order="F", dtype=np.float64, force_python_only=False, view_ok=False, num_threads=None):
        from pysnptools_amd.snpreader.snpreader import _read_and_standardize

        return _read_and_standardize(self.snpreader, self.standardizer, order, dtype, force_python_only,
                                     num_threads)[0]
