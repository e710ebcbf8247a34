"""SNP-block sharding of the GRM across ranks.

K = sum_b Z_b Z_b^T over SNP blocks b (snpreader.py:651-655), so blocks can be summed in
any grouping: rank r takes blocks r, r+p, r+2p, ... (round-robin keeps the ranks within
one block of each other), accumulates a partial K in HBM, and one all-reduce(sum) of the
upper-triangle K tiles over xGMI (RCCL) yields K on every rank.  Stats per block are local
and are gathered in block order (Unit._merge_trained, unit.py:53-56).
"""


def snp_blocks(n_sid, block_size):
    """[(start, count)] covering range(n_sid) in blocks of ``block_size``."""
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, n_sid - s0)) for s0 in range(0, n_sid, block_size)]


def rank_blocks(n_sid, block_size, rank, world):
    """The blocks rank ``rank`` of ``world`` owns (round-robin)."""
    assert 0 <= rank < world
    return snp_blocks(n_sid, block_size)[rank::world]


def rank_span_blocks(n_sid, block_size, rank, world):
    """Balanced plan: rank ``rank`` owns the contiguous SNP range [r*M/p, (r+1)*M/p), streamed
    in blocks of at most ``block_size`` -- ranks differ by at most one SNP, where round-robin
    whole blocks leave them a block apart (50 blocks over 8 ranks: 7 vs 6.25 on average)."""
    assert 0 <= rank < world
    lo, hi = n_sid * rank // world, n_sid * (rank + 1) // world
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, hi - s0)) for s0 in range(lo, hi, block_size)]


def merge_order(n_sid, block_size, world):
    """For each global block (in SNP order): (owner rank, index within that rank's list)."""
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


def grm_pieces(reader, standardizer, rank, world, dtype="float32", diag_k_to_n=False, num_threads=None):
    """GRM of a DistributedBed / _MergeSIDs of Beds with one process per GPU.

    Rank ``rank`` streams only its pieces (``rank_pieces``) through the fused
    decode->standardize->MFMA SYRK into a device-resident K; one RCCL all-reduce of the
    upper-triangle tiles (``snpmi_rccl_allreduce_sum``) sums the ranks; every rank then
    extracts the full K (with DiagKtoN if asked).  The per-SNP stats each rank computed are
    summed the same way (zeros for SNPs a rank did not own).  The RCCL communicator must be
    initialised (``snpmi_rccl_init``) when world > 1.
    Returns (K, trained standardizer, DiagKtoN factor or NaN)."""
    import ctypes

    import numpy as np

    from pysnptools_amd import _native as N
    from pysnptools_amd.snpreader.snpreader import _add_pieces, _bed_pieces, _resolve, _trained_from
    from pysnptools_amd.standardizer.standardizer import _std_args

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
    K = np.empty((n, n), dtype=dtype)
    factor = np.full(1, np.nan, dtype=np.float64)
    N.call("snpmi_grm_begin", n, N.dt_code(dtype))
    try:
        _add_pieces(merged, rows, cols, n, kind, a, b, use_stats, stats, dtype, num_threads, only=mine)
        if world > 1:
            tiles, count = ctypes.c_void_p(), ctypes.c_uint64()
            N.call("snpmi_grm_session_tiles", ctypes.byref(tiles), ctypes.byref(count))
            N.call("snpmi_rccl_allreduce_sum", tiles, count.value, N.dt_code(dtype))
            N.call("snpmi_stream_sync")
            if kind != N.STD_NONE and not use_stats:
                stats = _allreduce_host(N, stats)
    finally:
        N.call("snpmi_grm_end", int(bool(diag_k_to_n)), factor.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
               N.ptr(K))
    return K, _trained_from(standardizer, kind, a, b, sid, stats), float(factor[0])


def _allreduce_host(N, arr):
    """Sum a host array over ranks through a device buffer + RCCL (stats of owned SNPs)."""
    import ctypes

    import numpy as np

    buf = np.ascontiguousarray(arr, dtype=np.float64)
    dev = ctypes.c_void_p()
    N.call("snpmi_dev_alloc", ctypes.byref(dev), buf.nbytes)
    try:
        N.call("snpmi_memcpy_h2d", dev, N.ptr(buf), buf.nbytes)
        N.call("snpmi_rccl_allreduce_sum", dev, buf.size, N.DT_F64)
        N.call("snpmi_memcpy_d2h", N.ptr(buf), dev, buf.nbytes)
    finally:
        N.call("snpmi_dev_free", dev)
    return buf.astype(arr.dtype)


def grm_partitioned(reader, standardizer, rank, world, out=None, num_threads=None):
    """cfg5 GRM of a Bed (or a subset of one) too large to replicate: K is
    partitioned over ``world`` ranks as the 256x256 blocks of its upper triangle
    (``snpmi_grm_part_coords``); this rank streams every selected SNP through the fused
    decode -> standardize -> bf16x3 MFMA SYRK and keeps only its own blocks -- no collective.
    Stats are computed per rank from all iids (identical on every rank).

    Returns (blocks [n_local, 256, 256] float32 -- ``out`` if given, e.g. an ``np.memmap`` of a
    file, or ``"hbm"`` / an ``hbm.HbmArray`` to keep the blocks in device memory (accumulated in
    place, no copy-out) --, coords [n_local, 2] int64 = (row0, col0) of each block, trained
    standardizer).  Entries of a block beyond iid n-1 are padding."""
    import ctypes

    import numpy as np

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
    import numpy as np

    nb = (n + 255) // 256
    K = np.zeros((nb * 256, nb * 256), dtype=np.float32)
    for blocks, coords in parts:
        for blk, (i, j) in zip(blocks, coords):
            K[i:i + 256, j:j + 256] = blk
            K[j:j + 256, i:i + 256] = blk.T
    return K[:n, :n]
