"""PartitionedKernel: a GRM too large to replicate, served through the KernelReader API.

The reference holds K as one n x n array on one process (snpreader.py:623-668 builds it; the
KernelReader API -- ``read`` kernelreader.py:245-302, ``__getitem__`` :342-350, SnpKernel's
``_read`` snpkernel.py:78-101 -- hands out K or any K[iid0, iid1]).  At configs[4]'s 500k iids K is
1 TB (f32: 500 GB in its upper triangle), so the cfg5 plan (``shard.grm_partitioned``)
keeps it partitioned: each rank of the process group holds its own 256x256 blocks of the upper
triangle in HBM -- whole 16x16-block supertiles dealt round-robin (include/snpmi.h,
``snpmi_grm_part_coords``).

``PartitionedKernel`` is the KernelReader over those blocks.  ``_read(iid0_index, iid1_index)``
extracts the requested sub-matrix ON THE DEVICE from this rank's blocks (entries of blocks other
ranks own are 0; ``snpmi_grm_part_extract_*``) and sums the ranks' outputs over the group (an
all-reduce of the sub-matrix, exact: one owner per entry), so every rank returns K[iid0, iid1] --
the same SPMD contract as ``Bed.read_kernel`` under a group.  ``__getitem__`` composes subsets as
every KernelReader does (kernelreader.py:342-350).  ``_read_with_standardizing`` applies DiagKtoN
(diag_K_to_N.py:54-59) from the trace summed over the parts, lazily (a scale on extraction).
``write`` / ``load`` persist each rank's blocks beside a metadata file (the KernelNpz role for a K
that no single file or process holds).

``SnpKernel(reader, std).read()``, ``SnpKernel(...)[iid0, iid1].read()`` and
``SnpKernel._read_with_standardizing`` (FaST-LMM's entry point) route here under an open process group
when the replicated K would not fit one GPU's HBM (``set_grm_partition``; forced with "always").
``Bed.read_kernel`` / ``SnpReader._read_kernel`` keep the replicated path: they return a KernelData
holding the whole K on every rank, which a K that needs partitioning cannot be.
"""
import json
import os

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.kernelreader.kernelreader import KernelReader
from pysnptools_amd.kernelstandardizer import DiagKtoN

_MODES = ("auto", "always", "never")
_mode = [os.environ.get("PST_GRM_PARTITION", "auto")]


def set_grm_partition(mode):
    """When ``SnpKernel.read`` / ``SnpKernel._read_with_standardizing`` compute K partitioned (cfg5) instead of
    replicated on every rank: ``"auto"`` (default) -- under a process group of > 1 rank when the
    replicated upper-triangle tiles would take more than 80% of the device's free HBM;
    ``"always"`` -- whenever the fused GPU path applies (a Bed and Unit/Beta/trained/Identity),
    also at world 1 (one part); ``"never"`` -- the replicated path.  ``PST_GRM_PARTITION`` sets the
    default for new processes."""
    if mode not in _MODES:
        raise ValueError("set_grm_partition: mode must be one of %s" % (_MODES,))
    _mode[0] = mode


def grm_partition_mode():
    return _mode[0] if _mode[0] in _MODES else "auto"


def use_partitioned(n, dtype, group):
    """Whether a GRM of ``n`` iids in ``dtype`` is computed partitioned (see ``set_grm_partition``)."""
    mode = grm_partition_mode()
    if mode == "never":
        return False
    if mode == "always":
        return True
    if group is None or group.world <= 1:
        return False
    import ctypes

    free, total = ctypes.c_uint64(), ctypes.c_uint64()
    N.call("snpmi_device_memory", ctypes.byref(free), ctypes.byref(total))
    tiles = int(N.lib().snpmi_grm_tile_bytes(int(n), N.dt_code(np.dtype(dtype))))
    need = tiles + int(n) * int(n) * np.dtype(dtype).itemsize // 8  # + the extraction row blocks
    # one decision for the whole group (free memory differs between ranks; ranks that decided
    # differently would run different collectives)
    return bool(group.max(1.0 if need > 0.8 * free.value else 0.0) > 0.5)


class PartitionedKernel(KernelReader):
    """K[iid0, iid1] of a GRM whose K is partitioned over the ranks of a process group.

    ``iid``: the n iids (the K's rows and columns); ``blocks``: this rank's [n_local, 256, 256]
    blocks (an ``hbm.HbmArray``, or host memory that is uploaded once); ``part`` / ``parts``: its
    part of the plan (default: the group's rank / world); ``dist``: the group (default
    ``pysnptools_amd.dist.current()``; None or world 1: the blocks are the whole K when parts is
    1); ``scale``: a factor applied on extraction (DiagKtoN).

    Without a group, a part of a plan of several (``parts`` > 1, e.g. one part of a job whose parts
    run one after another) serves only the entries of the blocks it owns: a read that needs any
    other block raises ValueError instead of returning its zeros."""

    def __init__(self, iid, blocks, part=None, parts=None, dist=None, scale=1.0, name=None):
        super(PartitionedKernel, self).__init__()
        from pysnptools_amd import dist as dist_mod
        from pysnptools_amd import hbm
        from pysnptools_amd.pstreader import PstData

        self._row = PstData._fixup_input(iid, empty_creator=lambda ignore: np.empty([0, 2], dtype="str"), dtype="str")
        self._col = self._row
        self.n = len(self._row)
        self.dist = dist if dist is not None else dist_mod.current()
        world = self.dist.world if self.dist is not None else 1
        rank = self.dist.rank if self.dist is not None else 0
        self.part = rank if part is None else int(part)
        self.parts = world if parts is None else int(parts)
        if self.parts != world and world > 1:
            raise ValueError("a partitioned K over a group of %d ranks must have %d parts, not %d"
                             % (world, world, self.parts))
        nloc = N.lib().snpmi_grm_part_blocks(self.n, self.part, self.parts)
        assert tuple(blocks.shape) == (nloc, 256, 256), "blocks must be [%d, 256, 256]" % nloc
        self.dtype = np.dtype(blocks.dtype)
        assert self.dtype in (np.float32, np.float64), "blocks must be float32 or float64"
        if getattr(blocks, "snpmi_ptr", None) is None:  # host blocks (e.g. a memory map): uploaded in 1 GiB pieces
            import ctypes

            dev = hbm.empty((nloc, 256, 256), dtype=self.dtype, order="C")
            bb = 256 * 256 * self.dtype.itemsize
            per = max(1, (1 << 30) // bb)
            for b0 in range(0, nloc, per):
                piece = np.ascontiguousarray(blocks[b0:b0 + per])
                N.call("snpmi_memcpy_h2d", ctypes.c_void_p(dev.snpmi_ptr.value + b0 * bb), N.ptr(piece), piece.nbytes)
            blocks = dev
        self.blocks = blocks
        self.scale = float(scale)
        self._name = name or "PartitionedKernel(n=%d, part %d of %d)" % (self.n, self.part, self.parts)

    def __repr__(self):
        return self._name

    @property
    def row(self):
        return self._row

    @property
    def col(self):
        return self._col

    def _grouped(self):
        return self.parts > 1 and self.dist is not None and self.dist.world > 1

    def coords(self):
        """[n_local, 2] (row0, col0) of this rank's blocks."""
        from pysnptools_amd.shard import part_coords

        return part_coords(self.n, self.part, self.parts)

    # ------------------------------------------------------------------ reading
    def _read(self, row_index_or_none, col_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        from pysnptools_amd import hbm
        from pysnptools_amd.util import array_module

        dtype = np.dtype(dtype)
        order = "F" if order == "A" else order
        ri, ci = N.index_array(row_index_or_none), N.index_array(col_index_or_none)
        nr = self.n if ri is None else len(ri)
        nc = self.n if ci is None else len(ci)
        if self.parts > 1 and not self._grouped():
            self._check_owned(ri, ci)
        out = hbm.empty((nr, nc), dtype=self.dtype, order=order)
        N.call("snpmi_grm_part_extract_" + N.suffix(self.dtype), self.blocks.snpmi_ptr, self.n, self.part, self.parts,
               N.ptr(ri), nr, N.ptr(ci), nc, 1 if order == "C" else 0, self.scale, out.snpmi_ptr)
        if self._grouped() and nr * nc:  # every rank holds its blocks' entries, 0 elsewhere: sum them
            self.dist.sum_dev(out.snpmi_ptr, nr * nc, self.dtype, None)
            N.call("snpmi_stream_sync")
        if array_module(None) is hbm and dtype == self.dtype:
            return out
        val = out.get()
        return val if val.dtype == dtype else val.astype(dtype, order=order)

    def _check_owned(self, ri, ci):
        """A part read without its group: every block the sub-matrix touches must be this part's."""
        nb = (self.n + 255) // 256
        bi = np.unique(np.arange(self.n) // 256 if ri is None else ri // 256)
        bj = np.unique(np.arange(self.n) // 256 if ci is None else ci // 256)
        if len(bi) == 0 or len(bj) == 0:
            return
        co = self.coords() // 256
        owned = np.zeros(nb * (nb + 1) // 2, dtype=bool)
        owned[co[:, 1] * (co[:, 1] + 1) // 2 + co[:, 0]] = True
        lo, hi = np.minimum.outer(bi, bj), np.maximum.outer(bi, bj)
        if not owned[hi * (hi + 1) // 2 + lo].all():
            raise ValueError("K[iid0, iid1] needs blocks outside part %d of %d; read it under the process group of "
                             "all %d parts" % (self.part, self.parts, self.parts))

    def _check_whole(self, what):
        """A part of a plan of several, read without its group, holds only its share of the diagonal:
        ``what`` needs every part (the contract ``_check_owned`` enforces for sub-matrix reads)."""
        if self.parts > 1 and not self._grouped():
            raise ValueError("%s of a K partitioned into %d parts needs all of them: part %d alone holds only its share "
                             "of the diagonal; run it under the process group of all %d parts"
                             % (what, self.parts, self.part, self.parts))

    def trace(self):
        """trace(K) (before ``scale``): each part's diagonal entries, summed over the group."""
        import ctypes

        self._check_whole("trace(K)")
        t = ctypes.c_double(0.0)
        N.call("snpmi_grm_part_trace_" + N.suffix(self.dtype), self.blocks.snpmi_ptr, self.n, self.part, self.parts,
               ctypes.byref(t))
        tr = np.array([t.value], dtype=np.float64)
        if self._grouped():
            tr = np.asarray(self.dist.sum_host(tr), dtype=np.float64)
        return float(tr[0])

    @staticmethod
    def supports(kernel_standardizer):
        """Kernel standardizers a partitioned K applies as a scale on extraction: DiagKtoN (factor from
        the trace summed over the parts), DiagKtoNTrained (its own factor) and Identity (none)."""
        from pysnptools_amd.kernelstandardizer import DiagKtoNTrained
        from pysnptools_amd.kernelstandardizer import Identity as KernelIdentity

        return isinstance(kernel_standardizer, (DiagKtoN, DiagKtoNTrained, KernelIdentity))

    def _read_with_standardizing(self, to_kerneldata, snp_standardizer=None, kernel_standardizer=DiagKtoN(),
                                 return_trained=False, num_threads=None):
        """The kernel standardizer over the partitioned K as a scale on every later extraction
        (``to_kerneldata``: the whole scaled K as a KernelData, else the scaled reader):

        * DiagKtoN (diag_K_to_N.py:54-59): factor = n / trace, trace summed over the parts, applied
          when |factor - 1| > 1e-15; returns DiagKtoNTrained(factor);
        * DiagKtoNTrained (diag_K_to_N.py:115-127, a factor trained on another K, as FaST-LMM passes
          for test kernels): its own factor, applied unless it is constant;
        * Identity (kernelstandardizer/__init__.py): no scale.

        Any other kernel standardizer raises ValueError (SnpKernel falls back to the replicated K)."""
        from pysnptools_amd.kernelstandardizer import DiagKtoNTrained
        from pysnptools_amd.kernelstandardizer import Identity as KernelIdentity

        if isinstance(kernel_standardizer, DiagKtoN):
            factor = float(self.n) / self.trace()
            scale, trained = (factor if abs(factor - 1.0) > 1e-15 else 1.0), DiagKtoNTrained(factor)
        elif isinstance(kernel_standardizer, DiagKtoNTrained):
            f = float(kernel_standardizer.factor)
            scale, trained = (1.0 if kernel_standardizer.is_constant else f), kernel_standardizer
        elif isinstance(kernel_standardizer, KernelIdentity):
            scale, trained = 1.0, kernel_standardizer
        else:
            raise ValueError("a partitioned K supports the DiagKtoN, DiagKtoNTrained and Identity kernel "
                             "standardizers, not %r" % (kernel_standardizer,))
        if to_kerneldata:
            self._check_whole("reading the whole K")
        scaled = PartitionedKernel(self._row, self.blocks, self.part, self.parts, self.dist, scale=self.scale * scale,
                                   name=self._name + ".standardize(%r)" % (kernel_standardizer,))
        kernel = scaled.read(num_threads=num_threads) if to_kerneldata else scaled
        return (kernel, None, trained) if return_trained else kernel

    # ------------------------------------------------------------------ persistence
    @staticmethod
    def _paths(path, part, parts):
        return path + ".meta.json", path + ".iid.npy", "%s.part%dof%d.npy" % (path, part, parts)

    def write(self, path):
        """Persist this rank's blocks (``path.part<p>of<P>.npy``, written through a memory map in
        1 GiB pieces) and, on part 0, the iids and layout (``path.iid.npy``, ``path.meta.json``)."""
        meta, iidp, bp = self._paths(path, self.part, self.parts)
        nloc = self.blocks.shape[0]
        mm = np.lib.format.open_memmap(bp + ".tmp", mode="w+", dtype=self.dtype, shape=(nloc, 256, 256))
        per = max(1, (1 << 30) // (256 * 256 * self.dtype.itemsize))
        import ctypes

        for b0 in range(0, nloc, per):
            b1 = min(nloc, b0 + per)
            N.call("snpmi_memcpy_d2h", N.ptr(mm[b0:b1]),
                   ctypes.c_void_p(self.blocks.snpmi_ptr.value + b0 * 256 * 256 * self.dtype.itemsize),
                   (b1 - b0) * 256 * 256 * self.dtype.itemsize)
        mm.flush()
        del mm
        os.replace(bp + ".tmp", bp)
        if self.part == 0:
            np.save(iidp, np.array(self._row, dtype="U"), allow_pickle=False)
            with open(meta + ".tmp", "w") as f:
                json.dump({"format": "pysnptools_amd.PartitionedKernel/1", "n": self.n, "parts": self.parts,
                           "dtype": self.dtype.str, "scale": self.scale,
                           "layout": "256x256 upper-triangle blocks, supertiles dealt round-robin "
                                     "(snpmi_grm_part_coords)"}, f)
            os.replace(meta + ".tmp", meta)
        if self._grouped():
            self.dist.barrier()
        return self

    @staticmethod
    def load(path, part=None, parts=None, dist=None):
        """A PartitionedKernel from ``write``'s files: this rank's blocks (memory-mapped, uploaded to
        HBM once) under ``dist`` (default: the current group)."""
        from pysnptools_amd import dist as dist_mod

        d = dist if dist is not None else dist_mod.current()
        meta, iidp, _ = PartitionedKernel._paths(path, 0, 1)
        with open(meta) as f:
            m = json.load(f)
        world = d.world if d is not None else 1
        part = (d.rank if d is not None else 0) if part is None else int(part)
        parts = int(m["parts"]) if parts is None else int(parts)
        if parts != int(m["parts"]):
            raise ValueError("'%s' holds %d parts, not %d" % (path, m["parts"], parts))
        if world > 1 and world != parts:
            raise ValueError("'%s' holds %d parts: load it under a group of %d ranks (or one part alone)"
                             % (path, parts, parts))
        iid = np.load(iidp, allow_pickle=False)
        blocks = np.load(PartitionedKernel._paths(path, part, parts)[2], mmap_mode="r", allow_pickle=False)
        assert blocks.dtype == np.dtype(m["dtype"]) and len(iid) == int(m["n"])
        return PartitionedKernel(iid, blocks, part, parts, d, scale=float(m.get("scale", 1.0)),
                                 name="PartitionedKernel('%s')" % path)
