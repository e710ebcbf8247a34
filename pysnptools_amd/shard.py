"""The GRM across the GPUs of one node, one process per GPU.

K = sum_b Z_b Z_b^T over SNP blocks b (snpreader.py:651-655), so the SNPs can be summed in any
grouping.  Two plans:

* **SNP-sharded (cfg4)** -- ``grm_sharded`` (a Bed or a subset of one), ``grm_pieces``
  (DistributedBed pieces) and bench.py's cfg4 leg: rank r owns the contiguous SNP range
  [r*M/p, (r+1)*M/p) (``rank_span_blocks``; ranks differ by at most one SNP), streams it through
  the fused decode -> standardize -> MFMA SYRK into a partial K held as upper-triangle tiles in
  HBM (``ShardedGrm``), then ONE collective over xGMI combines the partials: ``ncclReduce(sum)``
  onto the rank that returns K (``collective="reduce"``, half the bytes of an all-reduce) or
  ``ncclAllReduce(sum)`` when every rank needs K (``"allreduce"``; what ``Bed.read_kernel`` uses
  under an open process group, so every rank's call returns K).  The f32 tiles run on the fp16
  MFMA pipe as three products of each value's fp16x2 split, the f64 tiles on the int8 MFMA as
  exact residue products.  Per-SNP stats are computed only by the rank that owns
  the SNP and summed over ranks (zeros elsewhere -- exact), which is ``Unit._merge_trained``'s
  concatenation (unit.py:53-56) in SNP order.
* **K-partitioned (cfg5)** -- ``grm_partitioned``: K (1 TB at 500k iids) is too large to
  replicate, so each rank keeps only its 256x256 blocks and reads every SNP; no collective.
"""
import ctypes

import numpy as np

COLLECTIVES = ("reduce", "allreduce", "none")


def snp_blocks(n_sid, block_size):
    """[(start, count)] covering range(n_sid) in blocks of ``block_size``."""
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, n_sid - s0)) for s0 in range(0, n_sid, block_size)]


def rank_blocks(n_sid, block_size, rank, world):
    """The blocks rank ``rank`` of ``world`` owns in a round-robin plan (used by the gloo
    rehearsal of the reduction, tests/test_distributed.py)."""
    assert 0 <= rank < world
    return snp_blocks(n_sid, block_size)[rank::world]


def rank_span(n_sid, rank, world):
    """[lo, hi): the contiguous SNP range rank ``rank`` of ``world`` owns."""
    assert 0 <= rank < world
    return n_sid * rank // world, n_sid * (rank + 1) // world


def rank_span_blocks(n_sid, block_size, rank, world):
    """Rank ``rank``'s span ``rank_span`` in blocks of at most ``block_size`` -- ranks differ by at
    most one SNP, where round-robin whole blocks leave them a block apart (50 blocks over 8 ranks:
    7 vs 6.25 on average)."""
    lo, hi = rank_span(n_sid, rank, world)
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, hi - s0)) for s0 in range(lo, hi, block_size)]


def merge_order(n_sid, block_size, world):
    """For each global block (in SNP order): (owner rank, index within that rank's round-robin list)."""
    out = []
    for b, _ in enumerate(snp_blocks(n_sid, block_size)):
        out.append((b % world, b // world))
    return out


def rank_pieces(piece_sizes, rank, world):
    """Piece indices rank ``rank`` of ``world`` owns when a DistributedBed's pieces (SNP shards
    of unequal size) are spread over GPUs: largest piece first onto the least-loaded rank
    (ties -> lowest rank), a deterministic plan every rank computes identically."""
    assert 0 <= rank < world
    order = sorted(range(len(piece_sizes)), key=lambda k: (-int(piece_sizes[k]), k))
    load = [0] * world
    owner = {}
    for k in order:
        r = min(range(world), key=lambda q: (load[q], q))
        owner[k] = r
        load[r] += int(piece_sizes[k])
    return sorted(k for k, r in owner.items() if r == rank)


def _layout(dist, rank, world):
    from pysnptools_amd import dist as dist_mod

    d = dist if dist is not None else dist_mod.current()
    if rank is None:
        rank = d.rank if d is not None else 0
    if world is None:
        world = d.world if d is not None else 1
    assert 0 <= rank < world, "rank %d of world %d" % (rank, world)
    return d, int(rank), int(world)


class ShardedGrm(object):
    """One rank's part of a SNP-sharded GRM: a GRM session (``snpmi_grm_begin``) whose upper-
    triangle tiles accumulate this rank's SNPs, one collective over the ranks, then K.

    ``collective``: "reduce" (K on ``root`` only; the other ranks' ``finish`` returns None),
    "allreduce" (K on every rank) or "none" (no collective: ``finish`` returns this rank's
    partial K -- the caller combines, e.g. tests that simulate the ranks on one GPU)."""

    def __init__(self, n, dtype, dist=None, collective="reduce", root=0, rank=None, world=None):
        from pysnptools_amd import _native as N

        if collective not in COLLECTIVES:
            raise ValueError("collective must be one of %s" % (COLLECTIVES,))
        self.N, self.n, self.dtype = N, int(n), np.dtype(dtype)
        if self.dtype not in (np.float32, np.float64):
            raise ValueError("GRM dtype must be float32 or float64")
        self.dist, self.collective, self.root = dist, collective, int(root)
        self.world = int(world) if world is not None else (dist.world if dist is not None else 1)
        self.rank = int(rank) if rank is not None else (dist.rank if dist is not None else 0)
        if collective != "none" and self.world > 1 and not (dist is not None and dist.rccl):
            raise RuntimeError("a %s over %d ranks needs an RCCL communicator (dist.init_from_env)"
                               % (collective, self.world))
        if not 0 <= self.root < self.world:
            raise ValueError("root %d out of range" % self.root)
        self._open = True
        N.call("snpmi_grm_begin", self.n, N.dt_code(self.dtype))

    # ------------------------------------------------------------------ accumulate
    def add_bed(self, bed, iid_index, sid_index, kind, a, b, use_stats, stats, num_threads=None):
        """Stream SNPs ``sid_index`` (absolute, of ``bed``) of iids ``iid_index`` (None = all)
        through the fused decode -> standardize -> SYRK; ``stats`` [len(sid_index), 2] in/out."""
        from pysnptools_amd.util import get_num_threads

        N = self.N
        ri, ci = N.index_array(iid_index), N.index_array(sid_index)
        if len(ci) == 0:
            return
        N.call("snpmi_grm_add_bed_" + N.suffix(self.dtype), bed.filename.encode(), bed.iid_count, bed.sid_count,
               int(bool(bed.count_A1)), N.ptr(ri), self.n, N.ptr(ci), len(ci), kind, a, b, int(use_stats),
               N.ptr(stats), get_num_threads(num_threads))

    def add_packed(self, packed, pitch, n_sid, kind, a, b, use_stats, stats, count_a1=False):
        """Packed SNP columns already in HBM (device pointer, [n_sid][pitch] bytes of all the
        session's iids); ``stats`` host or device [n_sid, 2]."""
        N = self.N
        N.call("snpmi_grm_add_packed_" + N.suffix(self.dtype), packed, pitch, self.n, n_sid, int(bool(count_a1)),
               kind, a, b, int(use_stats), stats if isinstance(stats, ctypes.c_void_p) else N.ptr(stats))

    def tiles(self):
        """(device pointer, element count) of this rank's tiles."""
        t, count = ctypes.c_void_p(), ctypes.c_uint64()
        self.N.call("snpmi_grm_session_tiles", ctypes.byref(t), ctypes.byref(count))
        return t, count.value

    # ------------------------------------------------------------------ combine + finish
    def combine(self):
        """The collective over xGMI (enqueued on the library stream): in-place ncclReduce onto
        ``root`` or ncclAllReduce of the tile buffer.  No-op for "none"; at world size 1 it runs
        only when a communicator exists (bench.py --force-rccl exercises the real calls)."""
        N = self.N
        if self.collective == "none" or self.dist is None or not self.dist.rccl:
            return
        t, count = self.tiles()
        if self.collective == "reduce":
            N.call("snpmi_rccl_reduce_sum", t, count, N.dt_code(self.dtype), self.root)
        else:
            N.call("snpmi_rccl_allreduce_sum", t, count, N.dt_code(self.dtype))

    def holds_k(self):
        return self.collective != "reduce" or self.rank == self.root

    def finish(self, out=None, diag_k_to_n=False):
        """(K or None, DiagKtoN factor or NaN).  K is ``out`` (n x n, host or HbmArray) or a new
        NumPy array on ranks that hold it; the session ends on every rank."""
        N = self.N
        factor = np.full(1, np.nan, dtype=np.float64)
        K = None
        if self.holds_k():
            K = out if out is not None else np.empty((self.n, self.n), dtype=self.dtype)
        self._open = False
        N.call("snpmi_grm_end", int(bool(diag_k_to_n)) if K is not None else 0,
               factor.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), N.ptr(K))
        return K, float(factor[0])

    def abort(self):
        if self._open:
            self._open = False
            self.N.call("snpmi_grm_end", 0, None, None)


def _sum_stats(d, stats, collective, world):
    """Per-SNP stats computed by their owner ranks (zeros elsewhere), summed over the ranks."""
    if collective == "none" or world == 1:
        return stats
    return d.sum_host(stats)


def grm_sharded(reader, standardizer, rank=None, world=None, dtype=np.float32, collective="reduce", root=0,
                diag_k_to_n=False, out=None, num_threads=None, dist=None):
    """SNP-sharded GRM of a Bed (or a subset of one) with one process per GPU -- the multi-GPU
    form of ``SnpReader._read_kernel`` (snpreader.py:623-668).

    Rank ``rank`` of ``world`` (default: from ``dist`` or ``pysnptools_amd.dist.current()``)
    streams only its contiguous SNP span (``rank_span``) from the .bed through the fused GPU GRM,
    then the partial K tiles are combined by ``collective`` (see ``ShardedGrm``).  Returns
    (K, trained standardizer, DiagKtoN factor or NaN): K is None on non-root ranks of a "reduce";
    with "none" K is this rank's partial sum and the stats cover only its SNPs (zeros elsewhere)."""
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.snpreader.snpreader import _resolve, _trained_from
    from pysnptools_amd.standardizer.standardizer import _std_args

    d, rank, world = _layout(dist, rank, world)
    dtype = np.dtype(dtype)
    args = _std_args(standardizer)
    if args is None:
        raise ValueError("grm_sharded supports Unit/Beta/UnitTrained/BetaTrained/Identity")
    if collective == "none" and diag_k_to_n:
        raise ValueError("DiagKtoN needs the combined K (collective 'reduce' or 'allreduce')")
    kind, a, b, use_stats, _, _ = args
    base, rows, cols = _resolve(reader)
    if not isinstance(base, Bed):
        raise ValueError("grm_sharded streams a Bed (or a subset of one); DistributedBed: grm_pieces")
    base._run_once()
    sid = reader.sid
    n, m = reader.iid_count, len(sid)
    lo, hi = rank_span(m, rank, world)
    col_index = np.arange(base.sid_count, dtype=np.uint64) if cols is None else np.asarray(cols, dtype=np.uint64)
    if use_stats:
        stats = np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype)
        mine = np.ascontiguousarray(stats[lo:hi])
    else:
        stats = np.zeros((m, 2), dtype=dtype)
        mine = np.zeros((hi - lo, 2), dtype=dtype)
    g = ShardedGrm(n, dtype, d, collective, root, rank, world)
    try:
        g.add_bed(base, rows, col_index[lo:hi], kind, a, b, use_stats, mine,
                  num_threads if num_threads is not None else base._num_threads)
        g.combine()
        if kind != 0 and not use_stats:
            stats[lo:hi] = mine
            stats = _sum_stats(d, stats, collective, world)
        K, factor = g.finish(out, diag_k_to_n)
    except BaseException:
        g.abort()
        raise
    return K, _trained_from(standardizer, kind, a, b, sid, stats), factor


def grm_pieces(reader, standardizer, rank=None, world=None, dtype="float32", diag_k_to_n=False, num_threads=None,
               collective="allreduce", root=0, out=None, dist=None):
    """GRM of a DistributedBed / _MergeSIDs of Beds with one process per GPU: rank ``rank``
    streams only its pieces (``rank_pieces``) into its partial K, then ``collective`` combines
    the ranks (default all-reduce: every rank extracts K, with DiagKtoN if asked).  The per-SNP
    stats are summed the same way (zeros for SNPs a rank did not own).
    Returns (K, trained standardizer, DiagKtoN factor or NaN)."""
    from pysnptools_amd.snpreader.snpreader import _add_pieces, _bed_pieces, _resolve, _trained_from
    from pysnptools_amd.standardizer.standardizer import _std_args

    d, rank, world = _layout(dist, rank, world)
    dtype = np.dtype(dtype)
    args = _std_args(standardizer)
    assert args is not None, "grm_pieces supports Unit/Beta/UnitTrained/BetaTrained/Identity"
    kind, a, b, use_stats, _, _ = args
    base, rows, cols = _resolve(reader)
    merged = _bed_pieces(base)
    assert merged is not None, "grm_pieces needs a DistributedBed or a _MergeSIDs of Beds"
    sid = reader.sid
    n = reader.iid_count
    stats = (np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype) if use_stats
             else np.zeros((len(sid), 2), dtype=dtype))
    mine = set(rank_pieces(merged.col_count_list, rank, world))
    g = ShardedGrm(n, dtype, d, collective, root, rank, world)
    try:
        _add_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, dtype, num_threads, only=mine)
        g.combine()
        if kind != 0 and not use_stats:
            stats = _sum_stats(d, stats, collective, world)
        K, factor = g.finish(out, diag_k_to_n)
    except BaseException:
        g.abort()
        raise
    return K, _trained_from(standardizer, kind, a, b, sid, stats), factor


def grm_partitioned(reader, standardizer, rank, world, out=None, num_threads=None):
    """cfg5 GRM of a Bed (or a subset of one) too large to replicate: K is
    partitioned over ``world`` ranks as the 256x256 blocks of its upper triangle
    (``snpmi_grm_part_coords``); this rank streams every selected SNP through the fused
    decode -> standardize -> fp16x2 MFMA SYRK (bf16x3 when a LUT is outside fp16's range) and
    keeps only its own blocks -- no collective.  Stats are computed per rank from all iids
    (identical on every rank).

    Returns (blocks [n_local, 256, 256] float32 -- ``out`` if given, e.g. an ``np.memmap`` of a
    file, or ``"hbm"`` / an ``hbm.HbmArray`` to keep the blocks in device memory (accumulated in
    place, no copy-out) --, coords [n_local, 2] int64 = (row0, col0) of each block, trained
    standardizer).  Entries of a block beyond iid n-1 are padding."""
    from pysnptools_amd import _native as N
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.snpreader.snpreader import _resolve, _trained_from
    from pysnptools_amd.standardizer.standardizer import _std_args
    from pysnptools_amd.util import get_num_threads

    args = _std_args(standardizer)
    assert args is not None, "grm_partitioned supports Unit/Beta/UnitTrained/BetaTrained/Identity"
    kind, a, b, use_stats, _, _ = args
    base, rows, cols = _resolve(reader)
    assert isinstance(base, Bed), "grm_partitioned streams a Bed file"
    base._run_once()
    sid = reader.sid
    n = reader.iid_count
    stats = (np.ascontiguousarray(standardizer.stats_for(sid), dtype=np.float32) if use_stats
             else np.empty((len(sid), 2), dtype=np.float32))
    nloc = N.lib().snpmi_grm_part_blocks(n, rank, world)
    if isinstance(out, str) and out == "hbm":
        from pysnptools_amd import hbm

        out = hbm.empty((nloc, 256, 256), dtype=np.float32, order="C")
    elif out is None:
        out = np.empty((nloc, 256, 256), dtype=np.float32)
    assert tuple(out.shape) == (nloc, 256, 256) and np.dtype(out.dtype) == np.float32
    assert getattr(out, "order", None) == "C" if hasattr(out, "snpmi_ptr") else out.flags["C_CONTIGUOUS"]
    ri, ci = N.index_array(rows), N.index_array(cols)
    N.call("snpmi_grm_part_bed_f32", base.filename.encode(), base.iid_count, base.sid_count,
           int(bool(base.count_A1)), N.ptr(ri), n, N.ptr(ci), len(sid), kind, a, b, int(use_stats), N.ptr(stats),
           rank, world, N.ptr(out), get_num_threads(num_threads))
    coords = np.empty((nloc, 2), dtype=np.int64)
    r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
    for k in range(nloc):
        N.call("snpmi_grm_part_coords", n, rank, world, k, ctypes.byref(r0), ctypes.byref(c0))
        coords[k] = (r0.value, c0.value)
    return out, coords, _trained_from(standardizer, kind, a, b, sid, stats)


def assemble_partitioned(parts, n):
    """Full symmetric n x n K (float32) from every rank's (blocks, coords) -- for sizes that fit."""
    nb = (n + 255) // 256
    K = np.zeros((nb * 256, nb * 256), dtype=np.float32)
    for blocks, coords in parts:
        for blk, (i, j) in zip(blocks, coords):
            K[i:i + 256, j:j + 256] = blk
            K[j:j + 256, i:i + 256] = blk.T
    return K[:n, :n]
