"""Process-group bootstrap for one process per GPU: the control plane of the
SNP-sharded GRM (``shard.grm_sharded``), the DistributedBed GRM (``shard.grm_pieces``) and
bench.py.  The reference has no multi-GPU code; its GRM loop (snpreader.py:643-668) is the
single-process form of what the ranks split.

    d = dist.init_from_env()      # RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE
    K = Bed(path).read_kernel(Unit(), dtype=np.float32)   # SNP shards per rank + RCCL all-reduce
    d.close()

Torch-free on purpose: importing torch beside libsnpmi would load a second libamdhip64 (torch
ships ROCm 7.0, the image 7.2).  The ncclUniqueId goes rank 0 -> other ranks through an O_EXCL
node-local file; barriers and max-over-ranks are RCCL all-reduces.

* Device: ``LOCAL_RANK`` when it is below the visible device count, else device 0 -- so a
  launcher that narrows each rank to one GPU (per-rank ``HIP_VISIBLE_DEVICES``) works.
* Single node: the id file is node-local, so ``WORLD_SIZE != LOCAL_WORLD_SIZE`` is refused at
  once unless ``SNPMI_RCCL_ID_FILE`` names a path on storage every node shares.
* Time limits: the id wait and ``ncclCommInitRank`` (which blocks until every rank joins) are
  bounded by ``timeout`` seconds; past it ``init_from_env`` raises ``TimeoutError`` (a stuck
  communicator init cannot be cancelled, so a caller should exit the process -- bench.py does,
  with a non-zero status).
"""
import contextlib
import ctypes
import json
import os
import socket
import struct
import sys
import tempfile
import threading
import time

_CURRENT = None


@contextlib.contextmanager
def stdout_to_stderr():
    """RCCL prints a version banner on the C stdout (fd 1) around communicator setup; callers
    whose stdout is a protocol (bench.py's one JSON line) keep it clean."""
    import sys

    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def env_layout(env=None):
    """(rank, world, local_rank, local_world) from the launcher's environment."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local_rank = int(env.get("LOCAL_RANK", str(rank)))
    local_world = int(env.get("LOCAL_WORLD_SIZE", str(world)))
    if not (0 <= rank < world) or not (0 <= local_rank < max(local_world, 1)):
        raise ValueError("bad rank layout: RANK=%d WORLD_SIZE=%d LOCAL_RANK=%d LOCAL_WORLD_SIZE=%d"
                         % (rank, world, local_rank, local_world))
    return rank, world, local_rank, local_world


def pick_device(local_rank, n_visible):
    """The device this rank drives: LOCAL_RANK if visible, else 0 (one GPU made visible per rank)."""
    if n_visible < 1:
        raise RuntimeError("no HIP device visible to this rank")
    return local_rank if local_rank < n_visible else 0


def id_file(env=None):
    """Node-local path for the ncclUniqueId: SNPMI_RCCL_ID_FILE if set (bench.py's spawner sets
    it), else derived from the launcher (parent pid + its start time + MASTER_PORT, so no stale
    file of an earlier launcher can match)."""
    env = os.environ if env is None else env
    path = env.get("SNPMI_RCCL_ID_FILE")
    if path:
        return path
    ppid = os.getppid()
    try:
        with open("/proc/%d/stat" % ppid) as f:
            start = f.read().rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        start = "0"
    key = "snpmi_rccl_%d_%s_%s.id" % (ppid, start, env.get("MASTER_PORT", "0"))
    return os.path.join(tempfile.gettempdir(), key)


def publish_id(path, uid):
    """Rank 0: write the id atomically and never over an existing file (O_EXCL + link)."""
    tmp = "%s.%d.tmp" % (path, os.getpid())
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
    with os.fdopen(fd, "wb") as f:
        f.write(bytes(uid))
    try:
        os.link(tmp, path)  # fails if a file of that name exists
    finally:
        os.remove(tmp)


def wait_id(path, timeout, nbytes=128, poll=0.05):
    """Ranks > 0: the id rank 0 published, or TimeoutError after ``timeout`` seconds."""
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as f:
                data = f.read(nbytes)
            if len(data) == nbytes:
                return data
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout:
            raise TimeoutError("no RCCL id from rank 0 at %s after %.0f s" % (path, timeout))
        time.sleep(poll)


def _run_bounded(fn, timeout, what):
    """fn() on a helper thread (ctypes releases the GIL), TimeoutError if it has not returned."""
    box = {}

    def target():
        try:
            box["ok"] = fn()
        except BaseException as e:  # re-raised on the caller's thread
            box["err"] = e

    t = threading.Thread(target=target, daemon=True)
    t.start()
    t.join(timeout)
    if t.is_alive():
        raise TimeoutError("%s did not finish within %.0f s" % (what, timeout))
    if "err" in box:
        raise box["err"]
    return box.get("ok")


class Dist(object):
    """One rank of a single-node process group.  ``rccl`` is False at world size 1 (unless
    forced): then barrier/max/sums are local no-ops and nothing touches RCCL."""

    def __init__(self, rank, world, local_rank, device, rccl, n_gpus):
        self.rank, self.world, self.local_rank, self.device = rank, world, local_rank, device
        self.rccl, self.n_gpus = rccl, n_gpus
        self._closed = False
        # group calls made through this object (the watchdog's dump): count and the last one
        self.ops, self.last_op = 0, None
        self.watchdog_path = None  # set by init_from_env: the job's shared abort-file name

    def _op(self, name):
        self.ops += 1
        self.last_op = name

    def barrier(self):
        self._op("barrier")
        if self.rccl:
            from pysnptools_amd import _native as N

            N.call("snpmi_rccl_barrier")

    def max(self, x):
        self._op("max")
        if not self.rccl:
            return x
        from pysnptools_amd import _native as N

        v = (ctypes.c_double * 1)(float(x))
        N.call("snpmi_rccl_host_allreduce_f64", v, 1, 1)
        return float(v[0])

    def sum_host(self, arr):
        """Elementwise sum over ranks of a host float array (any size, through a device buffer)."""
        import numpy as np

        self._op("sum_host")
        if not self.rccl:
            return np.array(arr, copy=True)
        from pysnptools_amd import _native as N

        buf = np.ascontiguousarray(arr, dtype=np.float64)
        if buf.size == 0:
            return buf.astype(np.asarray(arr).dtype)
        dev = ctypes.c_void_p()
        N.call("snpmi_dev_alloc", ctypes.byref(dev), buf.nbytes)
        try:
            N.call("snpmi_memcpy_h2d", dev, N.ptr(buf), buf.nbytes)
            N.call("snpmi_rccl_allreduce_sum", dev, buf.size, N.DT_F64)
            N.call("snpmi_memcpy_d2h", N.ptr(buf), dev, buf.nbytes)
        finally:
            N.call("snpmi_dev_free", dev)
        return buf.astype(np.asarray(arr).dtype)

    @property
    def can_reduce(self):
        """Whether ``sum_dev`` can combine device buffers over the ranks."""
        return self.rccl

    def sum_dev(self, buf, count, dtype, root=None):
        """In-place elementwise sum over ranks of a device float buffer (``count`` elements of
        ``dtype`` f32/f64): ncclReduce onto ``root`` (the other ranks' buffers are unspecified
        afterwards) or, with ``root=None``, ncclAllReduce.  Enqueued on the library stream."""
        from pysnptools_amd import _native as N

        self._op("sum_dev")
        if not self.rccl:
            if self.world > 1:
                raise RuntimeError("a device sum over %d ranks needs an RCCL communicator" % self.world)
            return
        code = N.dt_code(dtype)
        if root is None:
            N.call("snpmi_rccl_allreduce_sum", buf, int(count), code)
        else:
            N.call("snpmi_rccl_reduce_sum", buf, int(count), code, int(root))

    def allgather_dev(self, send, recv, nbytes):
        """Device all-gather of ``nbytes`` per rank: rank r's ``send`` lands at ``recv + r*nbytes``
        on every rank (ncclAllGather; in place when ``send`` is that slot of ``recv``)."""
        self._op("allgather_dev")
        if not self.rccl:
            if self.world > 1:
                raise RuntimeError("an all-gather over %d ranks needs an RCCL communicator" % self.world)
            return
        from pysnptools_amd import _native as N

        N.call("snpmi_rccl_allgather", send, recv, int(nbytes))

    def close(self):
        global _CURRENT
        if self._closed:
            return
        self._closed = True
        if _CURRENT is self:
            _CURRENT = None
        if self.rccl:
            from pysnptools_amd import _native as N

            with stdout_to_stderr():
                N.call("snpmi_rccl_destroy")
        self._close_host()

    def _close_host(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _send_frame(sock, payload):
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("rehearsal group: a rank closed its connection")
        buf += chunk
    return bytes(buf)


def _recv_frame(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class HostDist(Dist):
    """Rehearsal process group (``SNPMI_DIST_HOST=1``): the rank layout, barriers, max-over-ranks,
    host sums and device all-gathers of a world > 1 job, staged through host memory over local TCP
    sockets (rank 0 relays; its ephemeral port is handed over through the node-local id file, as
    the RCCL id is), with every rank free to share ONE GPU.  No RCCL: the device sums of GRM
    tiles (``sum_dev``, what ``ShardedGrm.combine`` calls) are staged through the host too, so
    ``grm_sharded`` / ``Bed.read_kernel`` run their "reduce" / "allreduce" at world 2-3 on one GPU.  Test infrastructure for the N > 1 control flow on a one-GPU box, where
    RCCL refuses two ranks per device -- never a production path.  (Not torch.distributed: torch's
    ROCm build carries its own HIP runtime, and loading it next to libsnpmi's corrupts the heap.)"""

    def __init__(self, rank, world, local_rank, device, timeout=300.0, env=None):
        Dist.__init__(self, rank, world, local_rank, device, False, world)
        path = id_file(env)
        self._peers, self._sock = [], None
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(world)
            srv.settimeout(timeout)
            publish_id(path, struct.pack("<Q", srv.getsockname()[1]).ljust(128, b"\0"))
            peers = {}
            try:
                while len(peers) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    (r,) = struct.unpack("<I", _recv_exact(conn, 4))
                    peers[r] = conn
            finally:
                srv.close()
                with contextlib.suppress(OSError):
                    os.remove(path)
            self._peers = [peers[r] for r in range(1, world)]
        else:
            (port,) = struct.unpack("<Q", wait_id(path, timeout)[:8])
            sock = socket.create_connection(("127.0.0.1", port), timeout=timeout)
            sock.sendall(struct.pack("<I", rank))
            self._sock = sock

    def allgather_bytes(self, payload):
        """Every rank's ``payload`` (bytes), in rank order, on every rank."""
        self.hub_calls = getattr(self, "hub_calls", 0) + 1
        payload = bytes(payload)
        if self.rank == 0:
            parts = [payload] + [_recv_frame(c) for c in self._peers]
            blob = struct.pack("<I", len(parts)) + b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for c in self._peers:
                _send_frame(c, blob)
        else:
            _send_frame(self._sock, payload)
            blob = _recv_frame(self._sock)
        (cnt,) = struct.unpack_from("<I", blob, 0)
        off, parts = 4, []
        for _ in range(cnt):
            (n,) = struct.unpack_from("<Q", blob, off)
            parts.append(blob[off + 8:off + 8 + n])
            off += 8 + n
        return parts

    def barrier(self):
        self._op("barrier")
        self.allgather_bytes(b"")

    def max(self, x):
        self._op("max")
        return max(struct.unpack("<d", p)[0] for p in self.allgather_bytes(struct.pack("<d", float(x))))

    def _reduce_f64(self, a, root=None):
        """Sum over ranks of the float64 array ``a`` (in rank order, at rank 0), returned on every
        rank (``root=None``) or on ``root`` only (None elsewhere)."""
        import numpy as np

        a = np.ascontiguousarray(a, dtype=np.float64)
        if self.rank == 0:
            tot = a.copy()
            for c in self._peers:
                tot += np.frombuffer(_recv_frame(c), dtype=np.float64).reshape(a.shape)
            for r, c in enumerate(self._peers, start=1):  # 1-byte tag: does the sum follow
                _send_frame(c, b"\x01" + tot.tobytes() if root is None or r == root else b"\x00")
            return tot if root is None or root == 0 else None
        _send_frame(self._sock, a.tobytes())
        back = _recv_frame(self._sock)
        if back[:1] != b"\x01":
            return None
        return np.frombuffer(back[1:], dtype=np.float64).reshape(a.shape).copy()

    def sum_host(self, arr):
        import numpy as np

        self._op("sum_host")
        a = np.asarray(arr)
        return self._reduce_f64(a).astype(a.dtype)

    @property
    def can_reduce(self):
        return True

    def sum_dev(self, buf, count, dtype, root=None):
        """Host-staged form of ``Dist.sum_dev``: the device buffer goes to the host, the ranks' copies
        are summed in float64 at rank 0 and the sum is written back (on every rank, or on ``root``)."""
        import numpy as np

        from pysnptools_amd import _native as N

        self._op("sum_dev")
        host = np.empty(int(count), dtype=dtype)
        N.call("snpmi_stream_sync")
        N.call("snpmi_memcpy_d2h", N.ptr(host), buf, host.nbytes)
        tot = self._reduce_f64(host, root)
        if tot is not None:
            host[:] = tot
            N.call("snpmi_memcpy_h2d", buf, N.ptr(host), host.nbytes)

    def allgather_dev(self, send, recv, nbytes):
        import numpy as np

        from pysnptools_amd import _native as N

        self._op("allgather_dev")
        nbytes = int(nbytes)
        mine = np.empty(nbytes, dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(mine), send, nbytes)
        host = np.frombuffer(b"".join(self.allgather_bytes(mine.tobytes())), dtype=np.uint8)
        N.call("snpmi_memcpy_h2d", recv, N.ptr(host), host.nbytes)

    def _close_host(self):
        for c in self._peers + ([self._sock] if self._sock else []):
            with contextlib.suppress(OSError):
                c.close()
        self._peers, self._sock = [], None


def init_from_env(force_rccl=False, timeout=300.0, env=None, set_current=True):
    """Bind this process to its GPU and, at WORLD_SIZE > 1 (or ``force_rccl``), build the RCCL
    communicator.  Returns the :class:`Dist`; it also becomes :func:`current`, which routes
    ``read_kernel`` of a Bed through the SNP-sharded GRM while it is open."""
    global _CURRENT
    from pysnptools_amd import _native as N

    env = os.environ if env is None else env
    rank, world, local_rank, local_world = env_layout(env)
    if world > 1 and local_world != world and not env.get("SNPMI_RCCL_ID_FILE"):
        raise RuntimeError("pysnptools_amd.dist is single-node: WORLD_SIZE=%d but LOCAL_WORLD_SIZE=%d (set "
                           "SNPMI_RCCL_ID_FILE to a path every node shares to run across nodes)" % (world, local_world))
    device = pick_device(local_rank, N.device_count())
    N.call("snpmi_set_device", device)
    wd_path = id_file(env) + ".watchdog" if world > 1 else None
    if world > 1 and env.get("SNPMI_DIST_HOST"):
        d = HostDist(rank, world, local_rank, device, timeout, env)
        d.watchdog_path = wd_path
        d.barrier()
        if set_current:
            _CURRENT = d
        return d
    rccl, n_gpus = False, 1
    if world > 1 or force_rccl:
        path = id_file(env)
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            with stdout_to_stderr():
                N.call("snpmi_rccl_unique_id", uid, 128)
            publish_id(path, uid)
        else:
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(wait_id(path, timeout))
        def comm_init():
            # the library's current device is per thread: bind the helper thread to this rank's
            # GPU before ncclCommInitRank, or every rank's communicator lands on device 0
            N.call("snpmi_set_device", device)
            N.call("snpmi_rccl_init", world, rank, uid, 128)

        try:
            with stdout_to_stderr():
                _run_bounded(comm_init, timeout, "ncclCommInitRank (rank %d of %d)" % (rank, world))
        finally:
            if rank == 0:
                # every rank has read the id once the communicator exists (or we give up)
                with contextlib.suppress(OSError):
                    os.remove(path)
        rccl = True
        cnt = ctypes.c_int()
        N.call("snpmi_rccl_comm_count", ctypes.byref(cnt))
        n_gpus = cnt.value
    d = Dist(rank, world, local_rank, device, rccl, n_gpus)
    d.watchdog_path = wd_path
    d.barrier()
    if set_current:
        _CURRENT = d
    return d


def current():
    """The open process group of this process, or None."""
    return _CURRENT


class Watchdog(object):
    """Per-rank stall detector for one process-group job (bench.py's N > 1 legs).

    A collective that one rank never joins blocks every other rank inside RCCL forever, and no
    Python exception ever surfaces.  The watchdog thread turns that into a bounded, diagnosed
    failure: the main thread calls :meth:`mark` at every leg and block boundary; when no mark has
    arrived for ``limit`` seconds (``mark(..., limit=)`` widens it for one phase, e.g. the final
    barrier while rank 0 runs its rank-only legs), or when another rank of the job has fired (its
    abort file ``<id file>.watchdog`` exists), it

    * writes ONE line ``[watchdog] rank R {json}`` to stderr: rank, world, leg, detail (e.g. the last
      shard block index), seconds since the mark, the group's own call count and last call, and the
      library's collective trace (``snpmi_rccl_trace``: calls per kind, bytes, the call-sequence
      signature -- equal on ranks that issued the same collectives -- and whether the rank sits in a
      blocking host all-reduce);
    * creates the abort file, so every other rank dumps its line within ``poll`` seconds;
    * calls ``on_fire(diag)`` (bench.py rank 0: a partial JSON line on stdout);
    * ends the process with ``os._exit(exit_code)`` -- no re-exec, no cleanup that could block on the
      GPU; the launcher (bench.py's spawner, torch.distributed.run) then reaps the other ranks.

    :meth:`fail` does the same at once, from an exception handler: a rank that raises outside a
    collective would otherwise leave its peers waiting in one."""

    def __init__(self, dist, limit=300.0, on_fire=None, poll=0.5, exit_code=4, stream=None, path=None):
        self.dist, self.limit, self.on_fire, self.poll = dist, float(limit), on_fire, float(poll)
        # after telling the peers, stay up long enough for them to see the abort file and fire on
        # their own, before this process's exit closes sockets they may be blocked on
        self.grace = max(1.0, 3.0 * self.poll)
        self.exit_code = exit_code
        self.stream = stream if stream is not None else sys.stderr
        self.path = path if path is not None else getattr(dist, "watchdog_path", None)
        self.leg, self.detail, self._limit = "start", None, self.limit
        self._t = time.time()
        self._lock = threading.Lock()
        self._fired = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="snpmi-watchdog", daemon=True)
        self._thread.start()

    def mark(self, leg=None, detail=None, limit=None):
        """Progress: the current leg (None keeps it), a detail (block index...), this phase's limit."""
        with self._lock:
            if leg is not None:
                self.leg = leg
            self.detail = detail
            self._limit = self.limit if limit is None else float(limit)
            self._t = time.time()

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=5)

    def diagnostics(self, reason):
        with self._lock:
            leg, detail, since, lim = self.leg, self.detail, time.time() - self._t, self._limit
        d = self.dist
        diag = {"reason": reason, "rank": getattr(d, "rank", 0), "world": getattr(d, "world", 1), "leg": leg,
                "detail": detail, "seconds_since_mark": round(since, 1), "limit_s": lim,
                "group_ops": getattr(d, "ops", None), "group_last_op": getattr(d, "last_op", None),
                "group": "rccl" if getattr(d, "rccl", False) else ("host" if getattr(d, "world", 1) > 1 else "none")}
        try:
            from pysnptools_amd import _native as N

            diag["rccl_trace"] = N.rccl_trace()
        except Exception as e:  # the library may be absent (CPU tests) or predate the trace
            diag["rccl_trace"] = "unavailable: %s" % e
        return diag

    def fail(self, reason):
        """Fire now (an exception on this rank): dump, tell the peers, exit."""
        self._fire(reason, tell_peers=True)

    def _peer_fired(self):
        return bool(self.path) and os.path.exists(self.path)

    def _fire(self, reason, tell_peers):
        with self._lock:
            fired, self._fired = self._fired, True
        if fired:  # another thread is already dumping and will end the process: wait for it
            while True:
                time.sleep(60)
        diag = self.diagnostics(reason)
        if tell_peers and self.path:
            with contextlib.suppress(OSError):
                fd = os.open(self.path, os.O_WRONLY | os.O_CREAT, 0o600)
                os.write(fd, ("rank %d: %s\n" % (diag["rank"], reason)).encode())
                os.close(fd)
        try:
            self.stream.write("[watchdog] rank %d %s\n" % (diag["rank"], json.dumps(diag, sort_keys=True)))
            self.stream.flush()
            if self.on_fire is not None:
                self.on_fire(diag)
            if tell_peers and self.path:
                time.sleep(self.grace)
        finally:
            with contextlib.suppress(Exception):
                sys.stdout.flush()
            os._exit(self.exit_code)

    def _run(self):
        while not self._stop.wait(self.poll):
            if self._peer_fired():
                self._fire("another rank of the job fired its watchdog (%s)" % self.path, tell_peers=False)
            with self._lock:
                late = time.time() - self._t > self._limit
                lim = self._limit
            if late:
                self._fire("no progress mark for %.0f s" % lim, tell_peers=True)

    def clear(self):
        """Remove the job's abort file (rank 0, after a clean run)."""
        if self.path:
            with contextlib.suppress(OSError):
                os.remove(self.path)
