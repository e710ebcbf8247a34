"""Checkpoint / resume for long GRMs ("Checkpoint / resume": the reference
accumulates K in host RAM block by block and loses it on a crash, snpreader.py:643-655).

``read_kernel_checkpointed`` computes the same K as ``Bed.read_kernel`` (snpreader.py:623-668)
as one GPU GRM session over SNP blocks (``snpmi_grm_begin`` / ``snpmi_grm_add_bed_*`` /
``snpmi_grm_end``) and, every ``every`` blocks, persists (the device K tiles, the next block,
the per-SNP stats so far) next to ``path``.  A later call with the same reader, standardizer,
block size and dtype restores the tiles into a new session and continues at the next block, so
an interrupted run resumes instead of starting over; the resumed K is bit-identical to an
uninterrupted checkpointed run (same blocks, same accumulation order).

Commit protocol: each save is a new GENERATION (``path.g<next_block>.tiles.npy`` / ``.stats.npy``)
written beside the previous one, never over it; the JSON names the generation's files and holds
their SHA-1s, and renaming the JSON into place is the commit.  Only then is the previous
generation deleted.  A crash at any point leaves a JSON that names a complete, hash-checked
generation (the previous one until the JSON rename, the new one after), so no block can be
counted twice.  ``_restore`` refuses files whose hash does not match.  Everything is removed
when the GRM completes.
"""
import glob
import hashlib
import json
import os

import numpy as np

from pysnptools_amd import _native as N


class _Interrupted(RuntimeError):
    """Raised by the ``_stop_after`` test hook (a simulated crash after that many blocks)."""


def _digest(idx):
    return None if idx is None else hashlib.sha1(np.ascontiguousarray(idx, dtype=np.uint64).tobytes()).hexdigest()


def _fingerprint(bed_path, n, m, dtype, block_size, kind, a, b, use_stats, rows, cols, count_a1, stats_in):
    st = os.stat(bed_path)
    # the accumulation settings of this process: partial sums of another f64 path (CRT vs f64
    # MFMA), another f32 chain length, exact diagonal on/off or another f32 SYRK kernel would not
    # resume bit-identically
    settings = ({"f64_path": N.kernel_variant("f64")} if np.dtype(dtype) == np.float64
                else {"f32_seg": N.kernel_variant("seg"), "f32_diag": N.kernel_variant("diag"),
                      "f32_syrk": N.kernel_variant("syrk")})
    return {"settings": settings, "bed": os.path.abspath(bed_path), "size": st.st_size, "mtime_ns": st.st_mtime_ns, "n": int(n),
            "m": int(m), "dtype": np.dtype(dtype).str, "block_size": int(block_size), "kind": int(kind),
            "a": None if np.isnan(a) else float(a), "b": None if np.isnan(b) else float(b),
            "use_stats": bool(use_stats), "count_A1": bool(count_a1), "rows": _digest(rows), "cols": _digest(cols),
            "stats_in": None if stats_in is None else hashlib.sha1(np.ascontiguousarray(stats_in).tobytes()).hexdigest()}


def _json_path(path):
    return path + ".json"


def _gen_paths(path, gen):
    return "%s.g%d.tiles.npy" % (path, gen), "%s.g%d.stats.npy" % (path, gen)


class _HashingWriter(object):
    """File wrapper that SHA-1s every byte written through it (np.save writes the header and then
    the data in chunks through ``write`` for a non-file object), so the hash comes from memory
    instead of re-reading a multi-GB file."""

    def __init__(self, f):
        self.f, self.h = f, hashlib.sha1()

    def write(self, b):
        self.h.update(b)
        return self.f.write(b)


class _HashingReader(object):
    """The read-side twin: ``np.lib.format.read_array`` reads a non-file object sequentially
    through ``read``, so the hash of a checkpoint file comes from the one pass that loads it."""

    def __init__(self, f):
        self.f, self.h = f, hashlib.sha1()

    def read(self, n=-1):
        b = self.f.read(n)
        self.h.update(b)
        return b


def _load_npy(p):
    """(array, SHA-1 of the file, bytes after the array) in one read of ``p``."""
    with open(p, "rb") as f:
        r = _HashingReader(f)
        arr = np.lib.format.read_array(r, allow_pickle=False)
        rest = r.read()  # read_array stops at the data's end; a longer file must not pass
    return arr, r.h.hexdigest(), len(rest)


def _write_npy(p, arr):
    """Write ``arr`` as .npy at ``p`` (temp file + fsync + rename); returns the file's SHA-1."""
    with open(p + ".tmp", "wb") as f:
        w = _HashingWriter(f)
        np.save(w, arr, allow_pickle=False)
        f.flush()
        os.fsync(f.fileno())
    os.replace(p + ".tmp", p)
    return w.h.hexdigest()


def _session_tiles():
    import ctypes

    tiles, count = ctypes.c_void_p(), ctypes.c_uint64()
    N.call("snpmi_grm_session_tiles", ctypes.byref(tiles), ctypes.byref(count))
    return tiles, count.value


def _save(path, meta, next_block, stats, dtype):
    """Write generation ``next_block`` (tiles, stats), then commit it by renaming the JSON that
    names it and holds its hashes; then drop the previous generation."""
    jpath = _json_path(path)
    prev = None
    if os.path.exists(jpath):
        with open(jpath) as f:
            prev = json.load(f).get("files")
    tiles, count = _session_tiles()
    host = np.empty(count, dtype=dtype)
    N.call("snpmi_stream_sync")
    N.call("snpmi_memcpy_d2h", N.ptr(host), tiles, host.nbytes)
    tpath, spath = _gen_paths(path, next_block)
    tsha = _write_npy(tpath, host)
    ssha = _write_npy(spath, np.ascontiguousarray(stats))
    files = {"tiles": os.path.basename(tpath), "stats": os.path.basename(spath),
             "tiles_sha1": tsha, "stats_sha1": ssha}
    with open(jpath + ".tmp", "w") as f:
        json.dump(dict(meta, next_block=int(next_block), files=files), f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(jpath + ".tmp", jpath)  # the commit
    if prev:
        for k in ("tiles", "stats"):
            old = os.path.join(os.path.dirname(os.path.abspath(path)), prev[k])
            if old not in (tpath, spath) and os.path.exists(old):
                os.remove(old)


def _restore(path, meta, dtype):
    """next block and stats of a matching checkpoint (tiles copied into the open session), or None."""
    jpath = _json_path(path)
    if not os.path.exists(jpath):
        return None
    with open(jpath) as f:
        saved = json.load(f)
    nb = saved.pop("next_block")
    files = saved.pop("files", None)
    if saved.get("settings") != meta["settings"] and \
            {k: v for k, v in saved.items() if k != "settings"} == {k: v for k, v in meta.items() if k != "settings"}:
        raise ValueError("checkpoint '%s' was written with other GRM kernel settings (%s) than this process's (%s); "
                         "restore them (snpmi_set_kernel_variant) or remove the checkpoint"
                         % (path, saved.get("settings", "none recorded"), meta["settings"]))
    if saved != meta:
        raise ValueError("checkpoint '%s' belongs to another GRM (reader, standardizer, block size or dtype "
                         "differ); remove it or choose another path" % path)
    d = os.path.dirname(os.path.abspath(path))
    if not files:
        raise ValueError("checkpoint '%s' names no tile files" % path)
    tpath, spath = os.path.join(d, files["tiles"]), os.path.join(d, files["stats"])
    loaded = []
    for p, key in ((tpath, "tiles_sha1"), (spath, "stats_sha1")):
        try:
            arr, sha, extra = _load_npy(p)
        except (OSError, ValueError):
            arr, sha, extra = None, None, 0
        if arr is None or extra or sha != files[key]:
            raise ValueError("checkpoint '%s': %s is missing or does not match its recorded hash" % (path, p))
        loaded.append(arr)
    host, stats_saved = loaded
    tiles, count = _session_tiles()
    if host.dtype != np.dtype(dtype) or host.size != count:
        raise ValueError("checkpoint '%s' tiles do not match this GRM" % path)
    N.call("snpmi_memcpy_h2d", tiles, N.ptr(host), host.nbytes)
    N.call("snpmi_stream_sync")
    return nb, stats_saved


def _remove_all(path):
    for p in [_json_path(path), _json_path(path) + ".tmp"] + glob.glob(glob.escape(path) + ".g*.npy*"):
        if os.path.exists(p):
            os.remove(p)


def read_kernel_checkpointed(reader, standardizer, path, block_size=10000, every=10, dtype=np.float64,
                             num_threads=None, _stop_after=None):
    """``reader.read_kernel(standardizer, block_size, dtype=dtype)`` with K checkpointed to
    ``path`` every ``every`` SNP blocks and resumed from it.  ``reader`` is a Bed or a subset of
    one; ``standardizer`` Unit / Beta / their trained forms / Identity.  Returns
    (KernelData, trained standardizer)."""
    from pysnptools_amd.kernelreader import KernelData
    from pysnptools_amd.snpreader.bed import Bed
    from pysnptools_amd.snpreader.snpreader import _resolve, _trained_from
    from pysnptools_amd.standardizer.standardizer import _std_args
    from pysnptools_amd.util import get_num_threads

    dtype = np.dtype(dtype)
    if dtype not in (np.float32, np.float64):
        raise ValueError("GRM dtype must be float32 or float64")
    args = _std_args(standardizer)
    if args is None:
        raise ValueError("read_kernel_checkpointed supports Unit/Beta/UnitTrained/BetaTrained/Identity")
    kind, a, b, use_stats, _, _ = args
    assert block_size >= 1 and every >= 1
    base, rows, cols = _resolve(reader)
    if not isinstance(base, Bed):
        raise ValueError("read_kernel_checkpointed reads a Bed (or a subset of one)")
    base._run_once()
    n, m = reader.iid_count, reader.sid_count
    sid = reader.sid
    stats_in = np.ascontiguousarray(standardizer.stats_for(sid), dtype=dtype) if use_stats else None
    meta = _fingerprint(base.filename, n, m, dtype, block_size, kind, a, b, use_stats, rows, cols, base.count_A1,
                        stats_in)
    col_index = np.arange(base.sid_count, dtype=np.uint64) if cols is None else np.asarray(cols, dtype=np.uint64)
    ri = N.index_array(rows)
    sfx = N.suffix(dtype)
    threads = get_num_threads(num_threads if num_threads is not None else base._num_threads)
    nblocks = (m + block_size - 1) // block_size
    K = np.empty((n, n), dtype=dtype)
    N.call("snpmi_grm_begin", n, N.dt_code(dtype))
    done = False
    try:
        stats = stats_in.copy() if use_stats else np.zeros((m, 2), dtype=dtype)
        got = _restore(path, meta, dtype)
        start = 0
        if got is not None:
            start, stats = got
        for k in range(start, nblocks):
            s0 = k * block_size
            ci = np.ascontiguousarray(col_index[s0:s0 + block_size])
            pst = np.ascontiguousarray(stats[s0:s0 + len(ci)])
            N.call("snpmi_grm_add_bed_" + sfx, base.filename.encode(), base.iid_count, base.sid_count,
                   int(bool(base.count_A1)), N.ptr(ri), n, N.ptr(ci), len(ci), kind, a, b, int(use_stats),
                   N.ptr(pst), threads)
            if not use_stats:
                stats[s0:s0 + len(ci)] = pst
            if (k + 1) % every == 0 and k + 1 < nblocks:
                _save(path, meta, k + 1, stats, dtype)
            if _stop_after is not None and k + 1 >= _stop_after:
                raise _Interrupted("stopped after %d blocks (test hook)" % (k + 1))
        done = True
    finally:
        N.call("snpmi_grm_end", 0, None, N.ptr(K))
    if done:
        _remove_all(path)
    return KernelData(iid=reader.iid, val=K), _trained_from(standardizer, kind, a, b, sid, stats)
