"""SnpReader: iid x sid genotype readers and the GRM entry point (reference snpreader/snpreader.py).

``_read_kernel`` (snpreader.py:623-668) is where the hot path is dispatched:

* a ``Bed`` (optionally sliced) with Unit/Beta/trained/Identity standardization runs as ONE
  native call, ``snpmi_grm_bed_{f32,f64}``: packed codes are uploaded once, standardized
  through per-SNP LUTs inside the MFMA SYRK staging, and K accumulates in HBM;
* an in-memory ``SnpData`` runs ``snpmi_grm_dense_{f32,f64}`` (standardize + SYRK on the GPU);
* anything else (custom readers or standardizers) follows the reference's block loop,
  each block's Z Z^T still computed on the GPU.

``block_size`` keeps its meaning for the generic loop; the native paths chunk SNPs
internally (the result differs only by floating-point summation order).
"""
import logging
import warnings

import numpy as np

from pysnptools_amd import _native as N
from pysnptools_amd.pstreader import PstReader
from pysnptools_amd.util import get_num_threads


class SnpReader(PstReader):
    """Reader of a matrix of SNP values: rows are individuals (iid), columns SNPs (sid)."""

    def __init__(self, *args, **kwargs):
        super(SnpReader, self).__init__(*args, **kwargs)

    @property
    def iid(self):
        return self.row

    @property
    def iid_count(self):
        return self.row_count

    @property
    def sid(self):
        return self.col

    @property
    def sid_count(self):
        return self.col_count

    @property
    def pos(self):
        return self.col_property

    @property
    def row_property(self):
        if not hasattr(self, "_row_property"):
            self._row_property = np.empty((self.row_count, 0))
        return self._row_property

    def _read(self, iid_index_or_none, sid_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        raise NotImplementedError

    def read(self, order="F", dtype=np.float64, force_python_only=False, view_ok=False, num_threads=None,
             _require_float32_64=True, xp=None):
        """Values as a :class:`SnpData` (order 'F' | 'C' | 'A', dtype float64 | float32 [| int8 for Bed]).

        ``xp`` (or ARRAY_MODULE) = 'hbm' keeps ``val`` in the GPU's HBM (:mod:`pysnptools_amd.hbm`);
        a Bed (or a subset of one) is then decoded straight into HBM."""
        from pysnptools_amd import hbm
        from pysnptools_amd.snpreader.snpdata import SnpData
        from pysnptools_amd.util import array_module

        dtype = np.dtype(dtype)
        xp = array_module(xp)
        val = _read_bed_into_hbm(self, order, dtype, num_threads) if xp is hbm else None
        if val is None:
            val = self._read(None, None, order, dtype, force_python_only, view_ok, num_threads)
        return SnpData(self.iid, self.sid, val, pos=self.pos, name=str(self), _require_float32_64=_require_float32_64,
                       xp=xp)

    def iid_to_index(self, list):
        return self.row_to_index(list)

    def sid_to_index(self, list):
        return self.col_to_index(list)

    def __getitem__(self, iid_indexer_and_snp_indexer):
        from pysnptools_amd.snpreader._subset import _SnpSubset

        iid_indexer, snp_indexer = iid_indexer_and_snp_indexer
        return _SnpSubset(self, iid_indexer, snp_indexer)

    def read_kernel(self, standardizer=None, block_size=None, order="A", dtype=np.float64, force_python_only=False,
                    view_ok=False, num_threads=None):
        """The iid x iid kernel (GRM) of the standardized SNPs, as a KernelData (snpreader.py:528-561).

        Numerics: ``dtype=float32`` runs as the fp16x2 split on the fp16 MFMA (22 of f32's 24
        bits per value, exact products, f32 accumulation restarted every 12288 SNPs, the diagonal
        accumulated exactly in f64): within ~1e-6
        of max diag(K) of the exact GRM.  ``dtype=float64`` (default) runs as exact integer products
        of 51-52-bit quantised values on the int8 MFMA (~1e-13 relative per value when a rare
        variant sets the block's scale); ``pysnptools_amd.set_grm_f64("mfma")`` selects the f64 MFMA
        instead (f64 rounding of every product).  Under an open ``pysnptools_amd.dist`` process
        group of more than one rank, each rank computes its SNP shard and RCCL all-reduces K."""
        assert standardizer is not None, "'standardizer' must be provided"
        from pysnptools_amd.kernelreader import SnpKernel

        snpkernel = SnpKernel(self, standardizer=standardizer, block_size=block_size)
        return snpkernel.read(order, np.dtype(dtype), force_python_only, view_ok, num_threads)

    def kernel(self, standardizer, allowlowrank=False, block_size=10000, blocksize=None, num_threads=None):
        warnings.warn(".kernel(...) is deprecated. Use '.read_kernel(...).val", DeprecationWarning)
        if blocksize is not None:
            block_size = blocksize
        return self._read_kernel(standardizer, block_size=block_size, num_threads=num_threads)

    # ------------------------------------------------------------------ GRM
    @staticmethod
    def _as_snpdata(snpreader, standardizer, force_python_only, order, dtype, num_threads):
        """(standardized SnpData, trained standardizer), reusing in-memory data when possible
        (snpreader.py:606-621)."""
        from pysnptools_amd import standardizer as stdizer

        dtype = np.dtype(dtype)
        if (hasattr(snpreader, "val") and snpreader.val.dtype == dtype and isinstance(standardizer, stdizer.Identity)
                and (order == "A" or (order == "C" and snpreader.val.flags["C_CONTIGUOUS"])
                     or (order == "F" and snpreader.val.flags["F_CONTIGUOUS"]))):
            return snpreader, stdizer.Identity()
        return _read_and_standardize(snpreader, standardizer, order, dtype, force_python_only, num_threads)

    def _read_kernel(self, standardizer, block_size=None, order="A", dtype=np.float64, force_python_only=False,
                     view_ok=False, return_trained=False, num_threads=None, _diag_k_to_n=False):
        dtype = np.dtype(dtype)
        fast = _native_grm(self, standardizer, dtype, num_threads, _diag_k_to_n)
        if fast is not None:
            K, trained, factor = fast
            K = K.T if order == "F" else K  # K is exactly symmetric: .T is its F-contiguous form
            if _diag_k_to_n:
                return K, trained, factor
            return (K, trained) if return_trained else K
        K, trained = self._read_kernel_blocks(standardizer, block_size, order, dtype, force_python_only, num_threads)
        if isinstance(trained, _LazyMerge) and (return_trained or _diag_k_to_n):
            trained = trained.merge()
        if _diag_k_to_n:
            return K, trained, None
        return (K, trained) if return_trained else K

    def _read_kernel_blocks(self, standardizer, block_size, order, dtype, force_python_only, num_threads):
        """The reference's generic loop (snpreader.py:629-668) for readers/standardizers the
        fused path does not cover: each block is read + standardized, then its Z Z^T is added to
        a K held in HBM (snpmi_grm_begin / add_dense / end) -- no host-side K +=."""
        from pysnptools_amd import hbm
        from pysnptools_amd.util import _on_device

        n = self.iid_count
        if dtype not in (np.float32, np.float64):
            raise ValueError("GRM dtype must be float32 or float64")
        sfx = N.suffix(dtype)
        # all at once unless the SNPs outnumber both the block and the iids (snpreader.py:629)
        whole = block_size is None or self.sid_count <= block_size or self.sid_count <= self.iid_count
        bs = self.sid_count if whole else block_size
        # K on xp (snpreader.py:638-643): in HBM when the values are or ARRAY_MODULE=hbm
        K = (hbm.empty if _on_device(getattr(self, "val", None)) else np.empty)((n, n), dtype=dtype)
        trained_list = []
        N.call("snpmi_grm_begin", n, N.dt_code(dtype))
        try:
            for start in range(0, self.sid_count, max(bs, 1)):
                reader = self if (start == 0 and bs >= self.sid_count) else self[:, start:start + bs]
                data, trained = SnpReader._as_snpdata(reader, standardizer, force_python_only, "A", dtype,
                                                      num_threads)
                trained_list.append(trained)
                val = data.val
                if not (val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]):  # (never an HbmArray)
                    val = np.asfortranarray(val)
                order_c = 1 if val.flags["C_CONTIGUOUS"] and not val.flags["F_CONTIGUOUS"] else 0
                N.call("snpmi_grm_add_dense_" + sfx, N.ptr(val), val.shape[0], val.shape[1], order_c)
        finally:
            N.call("snpmi_grm_end", 0, None, N.ptr(K))
        if whole:
            return (K.T if order == "F" else K), trained_list[0]
        # merged lazily: the reference merges only when the trained standardizer is asked for
        # (snpreader.py:666), and e.g. DiagKtoN cannot merge
        return (K.T if order == "F" else K), _LazyMerge(standardizer, trained_list)

    def copyinputs(self, copier):
        raise NotImplementedError

    @staticmethod
    def _name_of_other_file(filename, remove_suffix, add_suffix):
        if filename.lower().endswith(remove_suffix.lower()):
            filename = filename[0:-1 - len(remove_suffix)]
        return filename + "." + add_suffix

    @property
    def val_shape(self):
        return None


class _LazyMerge(object):
    def __init__(self, standardizer, trained_list):
        self.standardizer, self.trained_list = standardizer, trained_list

    def merge(self):
        return self.standardizer._merge_trained(self.trained_list)


# ---------------------------------------------------------------------- native dispatch
def _read_bed_into_hbm(reader, order, dtype, num_threads):
    """Decode a Bed (or a subset of one) straight into an HbmArray; None for other readers."""
    from pysnptools_amd import hbm
    from pysnptools_amd.snpreader.bed import Bed

    base, rows, cols = _resolve(reader)
    if not isinstance(base, Bed):
        return None
    base._run_once()
    if dtype not in (np.float32, np.float64, np.int8):
        raise ValueError("dtype '{0}' not supported; use float32, float64 or int8".format(dtype))
    order = "F" if order == "A" else order
    ri, ci = N.index_array(rows), N.index_array(cols)
    n = base.iid_count if ri is None else len(ri)
    m = base.sid_count if ci is None else len(ci)
    out = hbm.empty((n, m), dtype=dtype, order=order)
    threads = get_num_threads(num_threads if num_threads is not None else base._num_threads)
    N.call("snpmi_bed_read_" + N.suffix(dtype), base.filename.encode(), base.iid_count, base.sid_count,
           int(bool(base.count_A1)), N.ptr(ri), n, N.ptr(ci), m, 1 if order == "C" else 0, N.ptr(out), threads)
    return out


def _read_and_standardize(reader, standardizer, order="F", dtype=np.float64, force_python_only=False,
                          num_threads=None):
    """``reader.read(order, dtype).standardize(standardizer, return_trained=True)`` -- the reference's
    two calls (snpreader.py:606-621, snpkernel.py:104-132) -- as ONE native call when ``reader`` is a
    Bed (or a subset of one) and the standardizer Unit / Beta / their trained forms:
    ``snpmi_bed_read_standardize_*`` computes each SNP's stats from its code counts and decodes
    straight to standardized values through a per-SNP table (the same f64 formula, so the values and
    stats are bit-identical to the two calls), writing the values once instead of decoding them and
    then reading + rewriting them.  Other readers / standardizers, and ``force_python_only=True``
    (the caller asked for the reference's separate read + standardize steps), take the two calls."""
    from pysnptools_amd import hbm
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.snpreader.snpdata import SnpData
    from pysnptools_amd.standardizer.standardizer import _std_args
    from pysnptools_amd.util import array_module

    dtype = np.dtype(dtype)
    args = _std_args(standardizer) if dtype in (np.float32, np.float64) else None
    base, rows, cols = _resolve(reader) if args is not None and args[0] != N.STD_NONE else (None, None, None)
    if force_python_only or not isinstance(base, Bed):
        return reader.read(order=order, dtype=dtype).standardize(standardizer, return_trained=True,
                                                                 force_python_only=force_python_only,
                                                                 num_threads=num_threads)
    kind, a, b, use_stats, _, _ = args
    base._run_once()
    sid = reader.sid
    order = "F" if order == "A" else order
    ri, ci = N.index_array(rows), N.index_array(cols)
    n = base.iid_count if ri is None else len(ri)
    m = base.sid_count if ci is None else len(ci)
    stats = (np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype) if use_stats
             else np.empty((m, 2), dtype=dtype))
    xp = array_module(None)
    out = (hbm.empty if xp is hbm else np.empty)((n, m), dtype=dtype, order=order)
    threads = get_num_threads(num_threads if num_threads is not None else base._num_threads)
    N.call("snpmi_bed_read_standardize_" + N.suffix(dtype), base.filename.encode(), base.iid_count, base.sid_count,
           int(bool(base.count_A1)), N.ptr(ri), n, N.ptr(ci), m, 1 if order == "C" else 0, kind, a, b,
           int(use_stats), N.ptr(stats), N.ptr(out), threads)
    data = SnpData(reader.iid, sid, out, pos=reader.pos, name=str(reader), xp=xp)
    data._std_string_list.append(str(standardizer))
    return data, _trained_from(standardizer, kind, a, b, sid, stats)


def _resolve(reader):
    """(innermost reader, absolute iid index or None, absolute sid index or None)."""
    from pysnptools_amd.pstreader._subset import _PstSubset

    if isinstance(reader, _PstSubset):
        base, r0, c0 = _resolve(reader._internal)
        reader._run_once()
        rows, cols = reader._composed_indices(None, None)
        rows = rows if r0 is None else (r0 if rows is None else r0[rows])
        cols = cols if c0 is None else (c0 if cols is None else c0[cols])
        return base, rows, cols
    return reader, None, None


def _trained_from(standardizer, kind, a, b, sid, stats):
    from pysnptools_amd import standardizer as stdizer

    if kind == N.STD_NONE:
        return stdizer.Identity()
    if isinstance(standardizer, (stdizer.UnitTrained, stdizer.BetaTrained)):
        return standardizer
    if kind == N.STD_UNIT:
        return stdizer.UnitTrained(sid, stats)
    return stdizer.BetaTrained(standardizer.a, standardizer.b, sid, stats)


def _bed_pieces(base):
    """The _MergeSIDs behind a DistributedBed / _MergeSIDs whose pieces are all Beds, else None."""
    from pysnptools_amd.snpreader._mergesids import _MergeSIDs
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.snpreader.distributedbed import DistributedBed

    if isinstance(base, DistributedBed):
        base._run_once()
        base = base._merge
    if isinstance(base, _MergeSIDs) and all(isinstance(r, Bed) for r in base.reader_list):
        base._run_once()
        return base
    return None


def _add_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, dtype, num_threads, only=None):
    """snpmi_grm_add_bed_* for every piece holding requested SNPs (``only``: piece subset)."""
    sfx = N.suffix(dtype)
    col_index = np.arange(merged.col_count) if cols is None else np.asarray(cols)
    ri = N.index_array(rows)
    for k, here, rel in merged._pieces(col_index):
        if only is not None and k not in only:
            continue
        piece = merged.reader_list[k]
        pst = np.ascontiguousarray(stats[here])
        N.call("snpmi_grm_add_bed_" + sfx, piece.filename.encode(), merged.row_count,
               int(merged.col_count_list[k]), int(bool(piece.count_A1)), N.ptr(ri), n, N.ptr(N.index_array(rel)),
               len(rel), kind, a, b, int(use_stats), N.ptr(pst), get_num_threads(num_threads))
        if not use_stats:
            stats[here] = pst


def _grm_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, diag_k_to_n, fptr, K, dtype, num_threads):
    """One GPU session over the pieces: K accumulates in HBM across files (snpmi_grm_begin/add/end)."""
    N.call("snpmi_grm_begin", n, N.dt_code(dtype))
    try:
        _add_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, dtype, num_threads)
    finally:
        N.call("snpmi_grm_end", int(bool(diag_k_to_n)), fptr, N.ptr(K))


def _native_grm(reader, standardizer, dtype, num_threads, diag_k_to_n):
    """Fused GPU GRM for Bed / SnpData sources; None when not applicable."""
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.standardizer.standardizer import _std_args

    if dtype not in (np.float32, np.float64):
        return None
    args = _std_args(standardizer)
    if args is None:
        return None
    kind, a, b, use_stats, given, _ = args
    base, rows, cols = _resolve(reader)
    sid = reader.sid
    if use_stats:
        stats = np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype)
    else:
        stats = np.empty((len(sid), 2), dtype=dtype)
    n = reader.iid_count
    from pysnptools_amd import hbm
    from pysnptools_amd.util import _on_device

    # K stays in HBM when the source values do or ARRAY_MODULE=hbm (snpreader.py:638-643)
    K = (hbm.empty if _on_device(getattr(base, "val", None)) else np.empty)((n, n), dtype=dtype)
    factor = np.full(1, np.nan, dtype=np.float64)
    fptr = factor.ctypes.data_as(N.ctypes.POINTER(N.ctypes.c_double))
    sfx = N.suffix(dtype)
    merged = _bed_pieces(base)
    from pysnptools_amd import dist as dist_mod

    group = dist_mod.current()
    if group is not None and group.world > 1 and (merged is not None or isinstance(base, Bed)):
        # one process per GPU (pysnptools_amd.dist.init_from_env): every rank calls read_kernel,
        # streams its SNP shard / pieces, and the RCCL all-reduce gives every rank the same K
        from pysnptools_amd import shard

        run = shard.grm_pieces if merged is not None else shard.grm_sharded
        return run(reader, standardizer, dtype=dtype, collective="allreduce", diag_k_to_n=diag_k_to_n, out=K,
                   num_threads=num_threads, dist=group)
    if merged is not None:
        _grm_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, diag_k_to_n, fptr, K, dtype, num_threads)
    elif isinstance(base, Bed):
        base._run_once()
        ri, ci = N.index_array(rows), N.index_array(cols)
        N.call("snpmi_grm_bed_" + sfx, base.filename.encode(), base.iid_count, base.sid_count, int(bool(base.count_A1)),
               N.ptr(ri), n, N.ptr(ci), len(sid), kind, a, b, int(use_stats), N.ptr(stats), int(bool(diag_k_to_n)),
               fptr, N.ptr(K), get_num_threads(num_threads))
    elif hasattr(base, "val") and base.val.ndim == 2:
        if rows is None and cols is None:
            val = base.val
        else:
            val = base._read(rows, cols, "A", base.val.dtype, False, True, num_threads)
        val = val if val.dtype == dtype else val.astype(dtype, order="K")
        if not (val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]):
            val = np.ascontiguousarray(val)
        order_c = 1 if val.flags["C_CONTIGUOUS"] else 0
        N.call("snpmi_grm_dense_" + sfx, N.ptr(val), val.shape[0], val.shape[1], order_c, kind, a, b, int(use_stats),
               N.ptr(stats), int(bool(diag_k_to_n)), fptr, N.ptr(K))
    else:
        return None
    trained = _trained_from(standardizer, kind, a, b, sid, stats)
    return K, trained, float(factor[0])
