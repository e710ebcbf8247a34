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
* **K-partitioned (cfg5)** -- ``PartitionedGrm`` / ``grm_partitioned``: K (1 TB at 500k iids) is
  too large to replicate, so each rank keeps only its 256x256 blocks of K.  Every rank needs every
  SNP, so per SNP block each rank uploads only its 1/p share of the packed columns and one
  ``ncclAllGather`` rebuilds the block on every rank (packed codes are 16x smaller than f32
  values); no reduction.
"""
import ctypes

import numpy as np

COLLECTIVES = ("reduce", "allreduce", "none")


def snp_blocks(n_sid, block_size):
    """[(start, count)] covering range(n_sid) in blocks of ``block_size``."""
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, n_sid - s0)) for s0 in range(0, n_sid, block_size)]


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
        if collective != "none" and self.world > 1 and not (dist is not None and dist.can_reduce):
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

    def add_bed_combine(self, bed, iid_index, sid_index, kind, a, b, use_stats, stats, num_threads=None, parts=2):
        """``add_bed`` of this rank's LAST SNPs + ``combine``, overlapped under a real RCCL
        communicator (``snpmi_grm_add_bed_reduce_*``: the file stream's last chunk runs as column
        groups / CRT chunks whose tiles are summed on the aux stream under the rest of that chunk's
        SYRK; the same K bit for bit).  Otherwise the two calls run one after the other."""
        if not (self.collective != "none" and self.dist is not None and self.dist.rccl):
            self.add_bed(bed, iid_index, sid_index, kind, a, b, use_stats, stats, num_threads)
            self.combine(parts)
            return
        from pysnptools_amd.util import get_num_threads

        N = self.N
        ri, ci = N.index_array(iid_index), N.index_array(sid_index)
        if len(ci) == 0:  # no SNPs on this rank: its zero tiles join the others' ranged sums
            self.combine(parts)
            return
        N.call("snpmi_grm_add_bed_reduce_" + N.suffix(self.dtype), bed.filename.encode(), bed.iid_count,
               bed.sid_count, int(bool(bed.count_A1)), N.ptr(ri), self.n, N.ptr(ci), len(ci), kind, a, b,
               int(use_stats), N.ptr(stats), get_num_threads(num_threads),
               1 if self.collective == "reduce" else 2, self.root, int(parts))

    def add_packed(self, packed, pitch, n_sid, kind, a, b, use_stats, stats, count_a1=False):
        """Packed SNP columns already in HBM (device pointer, [n_sid][pitch] bytes of all the
        session's iids); ``stats`` host or device [n_sid, 2]."""
        N = self.N
        N.call("snpmi_grm_add_packed_" + N.suffix(self.dtype), packed, pitch, self.n, n_sid, int(bool(count_a1)),
               kind, a, b, int(use_stats), stats if isinstance(stats, ctypes.c_void_p) else N.ptr(stats))

    def add_packed_combine(self, packed, pitch, n_sid, kind, a, b, use_stats, stats, count_a1=False, parts=2,
                           syrk_done=None):
        """``add_packed`` of this rank's LAST SNPs + ``combine``, overlapped under a real RCCL
        communicator (``snpmi_grm_add_packed_reduce_f32/f64``: f32 runs the last SYRK launch as
        ``parts`` column groups of the triangle, f64 uses the CRT path's residue chunks; each
        finished group's tiles are summed over the ranks on the aux stream under the next group's
        work; the same K bit for bit).  ``stats`` must then be device memory.  Otherwise the two
        calls run one after the other (the host rehearsal group, no collective).  ``syrk_done``: optional event
        (``snpmi_event_create``) recorded after the last SYRK, for timing."""
        N = self.N
        dev_stats = isinstance(stats, ctypes.c_void_p)
        if self.collective != "none" and self.dist is not None and self.dist.rccl and dev_stats:
            N.call("snpmi_grm_add_packed_reduce_" + N.suffix(self.dtype), packed, pitch, self.n, n_sid,
                   int(bool(count_a1)), kind, a, b, int(use_stats), stats, 1 if self.collective == "reduce" else 2,
                   self.root, int(parts), syrk_done)
            return
        self.add_packed(packed, pitch, n_sid, kind, a, b, use_stats, stats, count_a1)
        if syrk_done is not None:
            N.call("snpmi_event_record", syrk_done)
        self.combine(parts)

    def tiles(self):
        """(device pointer, element count) of this rank's tiles."""
        t, count = ctypes.c_void_p(), ctypes.c_uint64()
        self.N.call("snpmi_grm_session_tiles", ctypes.byref(t), ctypes.byref(count))
        return t, count.value

    # ------------------------------------------------------------------ combine + finish
    def combine(self, parts=2):
        """The collective over xGMI: under RCCL, ``snpmi_grm_session_sum`` -- in-place ncclReduce
        onto ``root`` or ncclAllReduce of the tile buffer as the same ranged calls the overlapped
        ``add_*_combine(parts=parts)`` issue (a function of n, dtype and ``parts`` only), so a rank
        that owns no SNPs, or adds them unoverlapped, pairs its calls with every other rank's.  The
        host rehearsal group stages one sum of the whole buffer through host memory
        (``Dist.sum_dev``).  No-op for "none"; at world size 1 it runs only when a communicator
        exists (bench.py --force-rccl exercises the real calls)."""
        if self.collective == "none" or self.dist is None or not self.dist.can_reduce:
            return
        if not self.dist.rccl and self.dist.world == 1:
            return
        if self.dist.rccl:
            self.N.call("snpmi_grm_session_sum", 1 if self.collective == "reduce" else 2, self.root, int(parts))
            return
        t, count = self.tiles()
        self.dist.sum_dev(t, count, self.dtype, self.root if self.collective == "reduce" else None)

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
        g.add_bed_combine(base, rows, col_index[lo:hi], kind, a, b, use_stats, mine,
                          num_threads if num_threads is not None else base._num_threads)
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


def part_coords(n, part, parts):
    """[nloc, 2] int64 (row0, col0) of the 256x256 upper-triangle blocks part ``part`` of ``parts``
    owns, in its storage order (``snpmi_grm_part_coords_all``: whole supertiles dealt round-robin,
    include/snpmi.h)."""
    from pysnptools_amd import _native as N

    nloc = N.lib().snpmi_grm_part_blocks(n, part, parts)
    coords = np.empty((nloc, 2), dtype=np.uint64)
    N.call("snpmi_grm_part_coords_all", n, part, parts, N.ptr(coords))
    return coords.astype(np.int64)


class _DevBuf(object):
    def __init__(self, N, nbytes, host=False):
        self.N, self.host, self.p = N, host, ctypes.c_void_p()
        N.call("snpmi_host_alloc" if host else "snpmi_dev_alloc", ctypes.byref(self.p), max(int(nbytes), 1))

    def at(self, off):
        return ctypes.c_void_p(self.p.value + int(off))

    def free(self):
        if self.p:
            self.N.call("snpmi_host_free" if self.host else "snpmi_dev_free", self.p)
            self.p = None


def block_spans(m, block, first_block=None):
    """[(s0, count)] covering SNPs [0, m): ``first_block`` SNPs (default block/4, at least 1), then
    blocks of ``block`` -- PartitionedGrm's stream plan."""
    block = max(1, int(block))
    first = max(1, min(block, int(first_block) if first_block else block // 4))
    out, s0 = [], 0
    while s0 < m:
        cnt = min(first if s0 == 0 else block, m - s0)
        out.append((s0, cnt))
        s0 += cnt
    return out


class PartitionedGrm(object):
    """cfg5: the GRM of a SNP stream whose K is too large to replicate, as one
    process per GPU.  K is partitioned into the 256x256 blocks of its upper triangle, grouped into
    16x16-block supertiles dealt round-robin over the parts (``part_coords``); this process
    accumulates part ``part``.

    Per SNP block of ``block`` SNPs (the reference's block loop, snpreader.py:643-655; the first
    block is ``first_block`` = block/4 SNPs, so less host work precedes the first kernel; 32768-SNP
    blocks amortise the read-modify-write of the part's K blocks that ends every SYRK launch, which
    at 8192 cost ~5% of the launch -- the kernel holds one workgroup per CU, so that epilogue does
    not overlap its MFMAs):

    1. ``fill(host_ptr, s0, count)`` writes this rank's share -- packed columns [s0, s0+count) of the
       stream, all ``n_src`` iids, ``pitch_src`` bytes each -- into a pinned host slot (a .bed gather,
       ``snpmi_bed_gather_packed``; bench.py: a synthetic generator).  Rank r of the ``world`` ranks
       of ``dist`` owns columns [r*ms, (r+1)*ms) of each block, ms = ceil(block/world).
    2. The copy stream uploads the share into its slot of a device block buffer.
    3. ``dist.allgather_dev`` (ncclAllGather over xGMI, on the library's aux stream) rebuilds the
       whole block on every rank.
    4. iid selection (``k_repack*``), per-SNP stats + LUT (``k_snp_stats``; every rank sees every
       iid of the SNP, so the stats are identical on every rank without an exchange), then the fp16x2
       MFMA SYRK adds the block into this part's K blocks (``snpmi_dev_syrk_packed_part``).

    Two slots: block k+1's fill (host threads), upload (copy stream) and all-gather (aux stream) run
    under block k's kernels; the compute stream waits on events only.  At world 1 the all-gather is
    a no-op and the one rank fills whole blocks -- a single-GPU run of any part (``parts`` may exceed
    ``world``: bench.py computes part 0 of the 8-GPU plan on one GPU)."""

    def __init__(self, n_src, m, kind, a=0.0, b=0.0, use_stats=False, stats=None, iid_index=None, count_a1=False,
                 dist=None, part=None, parts=None, block=32768, out=None, timing=False, first_block=None,
                 dtype=np.float32):
        from pysnptools_amd import _native as N

        self.N = N
        self.dtype = np.dtype(dtype)
        if self.dtype not in (np.float32, np.float64):
            raise ValueError("GRM dtype must be float32 or float64")
        self.dist = dist
        self.world = dist.world if dist is not None else 1
        self.rank = dist.rank if dist is not None else 0
        self.part = self.rank if part is None else int(part)
        self.parts = self.world if parts is None else int(parts)
        if not 0 <= self.part < self.parts:
            raise ValueError("part %d of %d" % (self.part, self.parts))
        if self.world > 1 and not (dist.rccl or hasattr(dist, "allgather_bytes")):
            raise RuntimeError("the cfg5 all-gather over %d ranks needs a process group" % self.world)
        self.n_src, self.m = int(n_src), int(m)
        self.iid = N.index_array(iid_index)
        self.n = self.n_src if self.iid is None else len(self.iid)
        self.kind, self.a, self.b, self.use_stats, self.count_a1 = int(kind), float(a), float(b), bool(use_stats), count_a1
        self.block = max(1, int(block))
        # a smaller first block: its fill and upload are the only exposed host work of the stream
        self.first_block = max(1, min(self.block, int(first_block) if first_block else self.block // 4))
        self.ms = (self.block + self.world - 1) // self.world
        self.pitch_src = N.lib().snpmi_packed_pitch(self.n_src)
        self.pitch = N.lib().snpmi_packed_pitch(self.n)
        self.nloc = N.lib().snpmi_grm_part_blocks(self.n, self.part, self.parts)
        self.timing = timing
        self._bufs = []
        try:
            self._alloc(stats, out)
        except BaseException:
            self.close()
            raise

    def _alloc(self, stats, out):
        N = self.N
        blk = self.world * self.ms * self.pitch_src
        self.dev = [_DevBuf(N, blk), _DevBuf(N, blk)]
        self.host = [_DevBuf(N, self.ms * self.pitch_src, host=True), _DevBuf(N, self.ms * self.pitch_src, host=True)]
        self._bufs += self.dev + self.host
        self.rep = None
        if self.iid is not None:
            self.rep = _DevBuf(N, self.block * self.pitch)
            self.idx = _DevBuf(N, max(1, len(self.iid)) * 8)
            if len(self.iid):
                N.call("snpmi_memcpy_h2d", self.idx.p, N.ptr(self.iid), self.iid.nbytes)
            self._bufs += [self.rep, self.idx]
        isz = self.dtype.itemsize
        self.lut = _DevBuf(N, self.block * 4 * isz)
        self.stats_dev = _DevBuf(N, max(1, self.m) * 2 * isz)
        self._bufs += [self.lut, self.stats_dev]
        if self.use_stats:
            st = np.ascontiguousarray(stats, dtype=self.dtype)
            assert st.shape == (self.m, 2), "stats must be [m, 2]"
            N.call("snpmi_memcpy_h2d", self.stats_dev.p, N.ptr(st), st.nbytes)
        # the part's K blocks: in HBM (out="hbm" / an HbmArray: accumulated in place) or host
        if isinstance(out, str) and out == "hbm":
            from pysnptools_amd import hbm

            out = hbm.empty((self.nloc, 256, 256), dtype=self.dtype, order="C")
        if out is None:
            out = np.empty((self.nloc, 256, 256), dtype=self.dtype)
        assert tuple(out.shape) == (self.nloc, 256, 256) and np.dtype(out.dtype) == self.dtype
        assert getattr(out, "order", None) == "C" if hasattr(out, "snpmi_ptr") else out.flags["C_CONTIGUOUS"]
        self.out = out
        dev_out = getattr(out, "snpmi_ptr", None)
        if dev_out is not None:
            self.blocks = dev_out
        else:
            self._kbuf = _DevBuf(N, self.nloc * 256 * 256 * isz)
            self._bufs.append(self._kbuf)
            self.blocks = self._kbuf.p
        self._ev = []

    def _event(self):
        e = ctypes.c_void_p()
        self.N.call("snpmi_event_create", ctypes.byref(e))
        self._ev.append(e)
        return e

    def run(self, fill, progress=None):
        """Stream the ``m`` SNPs through steps 1-4 (see the class doc).  Returns per-block timings
        (ms, HIP events on the compute stream) when ``timing`` was set, else None.  ``progress(k,
        nblk)`` (optional) is called on the host after block k is enqueued."""
        N = self.N
        spans = self.spans()
        nblk = len(spans)
        up = [self._event(), self._event()]  # copy stream: share of the slot uploaded (host slot free)
        done = [self._event(), self._event()]  # compute stream: the slot's kernels are done
        gathered = [self._event(), self._event()]  # aux stream: the slot's block is all-gathered
        used = [False, False]
        marks = [(self._event(), self._event()) for _ in range(nblk)] if self.timing else None
        if self.m == 0 or self.n == 0:
            N.call("snpmi_dev_memset", self.blocks, 0, self.nloc * 256 * 256 * self.dtype.itemsize)
        for k in range(nblk if self.n else 0):
            s0, cnt = spans[k]
            ms = (cnt + self.world - 1) // self.world
            mine0 = min(cnt, self.rank * ms)
            mine = max(0, min(ms, cnt - mine0))
            slot = k & 1
            if used[slot]:
                N.call("snpmi_event_sync", up[slot])  # the host slot's previous upload has finished
            if mine:
                fill(self.host[slot].p, s0 + mine0, mine)
            dst = self.dev[slot].at(self.rank * ms * self.pitch_src)
            if used[slot]:
                N.call("snpmi_stream_wait_event", done[slot], 1)  # the device slot's readers are done
            N.call("snpmi_memcpy_async", dst, self.host[slot].p, ms * self.pitch_src, 0, 1)
            N.call("snpmi_event_record_on", up[slot], 1)
            if self.world > 1 or (self.dist is not None and self.dist.rccl):  # in place at world 1
                # the all-gather runs on the aux stream, so block k+1's exchange over xGMI overlaps
                # block k's SYRK on the compute stream; the compute stream waits on its event
                N.call("snpmi_stream_wait_event", up[slot], 2)
                N.call("snpmi_set_stream", 2)
                try:
                    self.dist.allgather_dev(dst, self.dev[slot].p, ms * self.pitch_src)
                finally:
                    N.call("snpmi_set_stream", 0)
                N.call("snpmi_event_record_on", gathered[slot], 2)
                N.call("snpmi_stream_wait_event", gathered[slot], 0)
            else:
                N.call("snpmi_stream_wait_event", up[slot], 0)
            used[slot] = True
            if marks:
                N.call("snpmi_event_record", marks[k][0])
            packed, pitch = self.dev[slot].p, self.pitch_src
            if self.rep is not None:
                N.call("snpmi_dev_repack", packed, pitch, self.n_src, self.idx.p, self.n, cnt, self.rep.p, self.pitch)
                packed, pitch = self.rep.p, self.pitch
            st = ctypes.c_void_p(self.stats_dev.p.value + s0 * 2 * self.dtype.itemsize)
            N.call("snpmi_dev_snp_stats", packed, pitch, self.n, cnt, int(bool(self.count_a1)), self.kind, self.a,
                   self.b, int(self.use_stats), N.dt_code(self.dtype), st, self.lut.p)
            N.call("snpmi_dev_syrk_packed_part" + ("_f64" if self.dtype == np.float64 else ""), packed, pitch, self.n,
                   cnt, self.lut.p, self.part, self.parts, self.blocks, int(k > 0))
            if marks:
                N.call("snpmi_event_record", marks[k][1])
            N.call("snpmi_event_record", done[slot])
            if progress is not None:
                progress(k, nblk)
        N.call("snpmi_stream_sync")
        if not marks:
            return None
        out = ctypes.c_float()
        res = []
        for a, b in marks:
            N.call("snpmi_event_elapsed_ms", a, b, ctypes.byref(out))
            res.append(float(out.value))
        return res

    def spans(self):
        """[(s0, count)] of the SNP blocks (``block_spans``)."""
        return block_spans(self.m, self.block, self.first_block)

    def stats(self):
        """[m, 2] per-SNP (mean, std) of the stream (or the given stats), in the GRM dtype."""
        st = np.empty((self.m, 2), dtype=self.dtype)
        if self.m:
            self.N.call("snpmi_memcpy_d2h", self.N.ptr(st), self.stats_dev.p, st.nbytes)
        return st

    def coords(self):
        """[nloc, 2] int64: (row0, col0) of each local block."""
        return part_coords(self.n, self.part, self.parts)

    def finish(self):
        """The part's blocks (``out``: copied from HBM when it is host memory)."""
        if getattr(self.out, "snpmi_ptr", None) is None and self.nloc:
            self.N.call("snpmi_memcpy_d2h", self.N.ptr(self.out), self.blocks, self.out.nbytes)
        return self.out

    def close(self):
        for e in self._ev if hasattr(self, "_ev") else []:
            self.N.call("snpmi_event_destroy", e)
        self._ev = []
        for bf in self._bufs:
            bf.free()
        self._bufs = []


def _partitioned_bed(base, rows, cols, kind, a, b, use_stats, stats, dist, part, parts, block_size, out, threads,
                     dtype=np.float32):
    """``PartitionedGrm`` over a .bed: each rank's share of a block gathered from the file's mmap
    (``snpmi_bed_gather_packed``).  Returns (blocks, coords, stats)."""
    from pysnptools_amd import _native as N

    m = base.sid_count if cols is None else len(cols)
    col_index = np.arange(base.sid_count, dtype=np.uint64) if cols is None else np.ascontiguousarray(cols, dtype=np.uint64)
    path = base.filename.encode()
    g = PartitionedGrm(base.iid_count, m, kind, a, b, use_stats, stats, iid_index=rows, count_a1=base.count_A1,
                       dist=dist, part=part, parts=parts, block=block_size, out=out, dtype=dtype)

    def fill(host, s0, cnt):
        N.call("snpmi_bed_gather_packed", path, base.iid_count, base.sid_count, N.ptr(col_index[s0:s0 + cnt]), cnt,
               g.pitch_src, host, threads)

    try:
        g.run(fill)
        blocks = g.finish()
        coords = g.coords()
        if not use_stats:
            stats = g.stats()
    finally:
        g.close()
    return blocks, coords, stats


def grm_partitioned(reader, standardizer, rank=None, world=None, out=None, num_threads=None, dist=None,
                    block_size=32768, dtype=np.float32):
    """cfg5 GRM of a Bed (or a subset of one) too large to replicate: K is
    partitioned over the ranks as the 256x256 blocks of its upper triangle
    (``snpmi_grm_part_coords``) and this rank keeps only its own blocks.

    * Under a process group (``dist``, or ``pysnptools_amd.dist.current()``, world > 1): the §8e
      plan, ``PartitionedGrm`` -- each rank reads only its 1/world share of every SNP block from the
      .bed, the RCCL all-gather rebuilds the block, every rank runs stats + the fp16x2 SYRK for its
      part.  ``rank`` / ``world`` must be None or the group's.
    * Without one: part ``rank`` of ``world`` (default 0 of 1) on this GPU alone, streaming every
      SNP of the .bed itself (``snpmi_grm_part_bed_f32``) -- e.g. the parts of a job run one by one.

    ``dtype``: float32 (fp16x2 MFMA, exact diagonal) or float64 -- the reference's default GRM
    dtype (snpreader.py:528,623) -- on the int8 MFMA as exact residue products.

    Returns (blocks [n_local, 256, 256] of ``dtype`` -- ``out`` if given, e.g. an ``np.memmap`` of a
    file, or ``"hbm"`` / an ``hbm.HbmArray`` to keep the blocks in device memory (accumulated in
    place, no copy-out) --, coords [n_local, 2] int64 = (row0, col0) of each block, trained
    standardizer).  Entries of a block beyond iid n-1 are padding."""
    from pysnptools_amd import _native as N
    from pysnptools_amd import dist as dist_mod
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
    dtype = np.dtype(dtype)
    if dtype not in (np.float32, np.float64):
        raise ValueError("GRM dtype must be float32 or float64")
    stats = (np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype) if use_stats
             else np.empty((len(sid), 2), dtype=dtype))
    d = dist if dist is not None else dist_mod.current()
    threads = get_num_threads(num_threads if num_threads is not None else base._num_threads)
    if d is not None and d.world > 1:
        if (rank is not None and rank != d.rank) or (world is not None and world != d.world):
            raise ValueError("rank/world %s/%s differ from the process group's %d/%d" % (rank, world, d.rank, d.world))
        blocks, coords, stats = _partitioned_bed(base, rows, cols, kind, a, b, use_stats, stats, d, d.rank, d.world,
                                                 block_size, out, threads, dtype)
        return blocks, coords, _trained_from(standardizer, kind, a, b, sid, stats)
    rank = 0 if rank is None else int(rank)
    world = 1 if world is None else int(world)
    nloc = N.lib().snpmi_grm_part_blocks(n, rank, world)
    if isinstance(out, str) and out == "hbm":
        from pysnptools_amd import hbm

        out = hbm.empty((nloc, 256, 256), dtype=dtype, order="C")
    elif out is None:
        out = np.empty((nloc, 256, 256), dtype=dtype)
    assert tuple(out.shape) == (nloc, 256, 256) and np.dtype(out.dtype) == dtype
    assert getattr(out, "order", None) == "C" if hasattr(out, "snpmi_ptr") else out.flags["C_CONTIGUOUS"]
    ri, ci = N.index_array(rows), N.index_array(cols)
    N.call("snpmi_grm_part_bed_" + N.suffix(dtype), base.filename.encode(), base.iid_count, base.sid_count,
           int(bool(base.count_A1)), N.ptr(ri), n, N.ptr(ci), len(sid), kind, a, b, int(use_stats), N.ptr(stats),
           rank, world, N.ptr(out), threads)
    return out, part_coords(n, rank, world), _trained_from(standardizer, kind, a, b, sid, stats)


def assemble_partitioned(parts, n):
    """Full symmetric n x n K (the blocks' dtype) from every rank's (blocks, coords) -- for sizes
    that fit."""
    nb = (n + 255) // 256
    dt = next((np.dtype(b.dtype) for b, _ in parts if len(b)), np.dtype(np.float32))
    K = np.zeros((nb * 256, nb * 256), dtype=dt)
    for blocks, coords in parts:
        for blk, (i, j) in zip(blocks, coords):
            K[i:i + 256, j:j + 256] = blk
            K[j:j + 256, i:i + 256] = blk.T
    return K[:n, :n]
