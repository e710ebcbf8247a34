"""Benchmark of the BED decode -> standardize -> GRM hot path on MI355X.

Metric (BASELINE.json): "SNPs/sec standardized (500k x 1M) + GRM GF/s at 1/2/4/8 GPUs".

  value      = SNPs/s standardized over the metric's fixed 500k-iid x 1M-SNP BED matrix (the UKBB
               shape of configs[4]), resident in HBM as packed 2-bit codes: rank r of N owns SNPs
               [r*1M/N, (r+1)*1M/N) and streams them through stats + decode + Unit in blocks of
               2048 SNPs into an f32 F-order block buffer; no collective on the data path.  STRONG
               scaling (total work fixed); a step = one pass over the 1M SNPs by all ranks.
               `weak` (N > 1) = the same ranks each streaming 1M SNPs per step (their shard N times).
  roofline   = the decode kernel (k_decode_f<float>), HBM bound: algorithmic bytes per launch =
               block * (ceil(N/4) + 4N) / its mean HIP-event duration, vs 8.0 TB/s.
  decode_c   = the C-order form (k_decode_c_reg<float>), same bytes, 500k iids.
  e2e        = packed columns in pinned HOST memory -> H2D on the copy stream -> stats + decode on
               the compute stream (3-slot ring, events only) -> f32 in HBM: the PCIe-inclusive rate,
               with the measured H2D peak of the same buffer beside it.  Never `value`.
  grm        = SnpKernel GRM of configs[3] (50k iid x 500k SNP, Unit, f32): rank r of N owns the
               contiguous SNP span [r*M/N, (r+1)*M/N) and accumulates it through
               pysnptools_amd.shard.ShardedGrm (the same code as shard.grm_sharded, which
               Bed.read_kernel uses under an open process group) into upper-triangle K tiles in
               HBM, <= 65536 SNPs per SYRK launch; then one ncclReduce(sum) of the tiles onto rank 0
               (--grm-collective allreduce: ncclAllReduce).  The f32
               products run on the fp16 MFMA pipe as 3 fp16 products of each value's fp16x2 split
               (f32-level accuracy, f32 accumulate; bf16x3 = 6 bf16 products when a SNP's LUT is
               outside fp16's range).  gflops uses N(N+1)M (SYRK work); roofline
               vs 2.5 PF fp16 dense / 3 = 833.3 TF (the f32-MFMA peak is 157.3).
  grm_f64    = the same GRM in float64 (the reference's default dtype, snpreader.py:528,623) on
               the int8 MFMA: each block's LUT quantised to 51-52-bit integers, K_int computed
               exactly modulo the first R of 15 coprime moduli <= 256 (one int8 SYRK each; R per
               block from the block's bound max_i sum_s q_is^2, on the device), rebuilt by CRT and
               added to the f64 K (syrk_crt.hip).  roofline vs the int8 dense peak (2 x bf16 =
               5.0 POP/s) on the executed ops; f64_equiv_tflops = N(N+1)M / time, beside the f64
               MFMA's 78.6 TF dense peak.
  grm5       = configs[4]: 500k iids x 1M SNPs, K (500 GB f32 upper triangle) partitioned over the
               8 parts of the 8-GPU plan as 256x256 blocks owned by whole 16x16-block supertiles;
               this process computes part `rank` of max(N, 8) over ALL the job's SNPs, streamed in
               32768-SNP blocks (the first a quarter) from pinned host memory inside the timed
               region (each rank's 1/N share + RCCL all-gather at N > 1) -- the whole per-part job
               measured, no projection; parity of sample blocks vs the f64 oracle over all SNPs.
               At N < 8 the rate fields are `part_*` (one part of 8); `single_gpu_job_*_projected`
               = 8 parts one after another on this GPU, labelled as the projection it is.
  beta       = configs[2]: 100k iid x 1M SNP, Beta(1,25) + NaN impute (21.8% missing, SnpGen's
               rate), packed resident in HBM, stats + decode in 2048-SNP blocks (f32, F order).
  file       = the reference's own call path on a synthetic 50k x 100k .bed written to local disk
               (untimed; read from the page cache): Bed.read_kernel(Unit(), float32) with K left in
               HBM and copied out, Bed[:, :10000].read(float32, xp='hbm'), and the cfg3 workload
               Bed.read(float32, xp='hbm').standardize(Beta(1,25)) -- PCIe-inclusive, never `value`.
  cpu_baseline = the oracle's C/OpenMP decode + one-pass Unit standardize (the CPU restatement
               of bed-reader's read + standardize_f32) on a sample of the same packed columns,
               rank 0 at N = 1 only, at the largest usable thread count (affinity / cgroup quota)
               and at 1 thread; grm.cpu_baseline = the reference's block step (NumPy/OpenBLAS
               Z.dot(Z.T), snpdata.py:203-206, + the single-threaded K += of snpreader.py:655) on a
               50k-iid slice, extrapolated to configs[3].

Run: python bench.py [--gpus N --steps K --warmup W].  N > 1 either under torch.distributed.run
(RANK / WORLD_SIZE / LOCAL_RANK from the environment) or as a plain `python bench.py --gpus N`, which
spawns the N rank processes itself before anything touches the GPU and relays rank 0's line.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SNPs/sec standardized (500k×1M) + GRM GF/s at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0
MFMA_F32_PEAK_TFLOPS = 157.3
MFMA_F64_PEAK_TFLOPS = 78.6
MFMA_BF16_PEAK_TFLOPS = 2500.0
# f32 GRM on the fp16 MFMA pipe (same dense rate as bf16): each f32 product = 3 fp16 MFMA
# products of the fp16x2 split (k_syrk_h2; Unit LUTs always fit fp16's range)
SPLIT_PRODUCTS = 3
SPLIT_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
# f64 GRM on the int8 MFMA pipe (i8 = 2x the bf16 rate): one int8 SYRK per modulus
MFMA_I8_PEAK_TOPS = 2 * MFMA_BF16_PEAK_TFLOPS
CRT_MODULI = 15  # kR, pysnptools_amd/csrc/syrk_crt.hip: the most a block can need (R per block, on the device)
GRM5_PLAN_WORLD = 8  # configs[4] is an 8-GPU plan


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n-iid", type=int, default=500_000)
    p.add_argument("--n-sid", type=int, default=1_000_000)
    p.add_argument("--block", type=int, default=2048)
    p.add_argument("--grm-iid", type=int, default=50_000)
    p.add_argument("--grm-sid", type=int, default=500_000)
    p.add_argument("--grm-block", type=int, default=10_000)
    p.add_argument("--skip-grm", action="store_true")
    p.add_argument("--grm-collective", choices=["auto", "reduce", "allreduce"], default="auto",
                   help="cfg4 at N > 1: the timed K-tile collective; auto = allreduce, the RCCL all-reduce configs[3] "
                        "names (every rank gets K, as Bed.read_kernel under a group); reduce = ncclReduce onto rank 0 "
                        "(timed unoverlapped beside it either way: grm.reduce_ms)")
    p.add_argument("--grm-f64", choices=["on", "off"], default="on", help="cfg4 GRM in float64 (reference default)")
    p.add_argument("--grm-overlap-parts", type=int, default=2,
                   help="cfg4 f32 at N > 1: column groups of the last SYRK launch whose K-tile collective "
                        "overlaps the next group's SYRK (1 = SYRK, then one collective)")
    p.add_argument("--grm5", choices=["on", "off"], default="on", help="cfg5 partitioned-K GRM leg")
    p.add_argument("--grm5-iid", type=int, default=500_000)
    p.add_argument("--grm5-sid", type=int, default=1_000_000, help="cfg5: SNPs of the whole job (all timed)")
    p.add_argument("--grm5-block", type=int, default=32768, help="cfg5: SNPs per all-gathered block (the first: 1/4)")
    p.add_argument("--grm5-miss", type=float, default=0.218, help="cfg5: missing rate (SnpGen's 21.8%%)")
    p.add_argument("--grm5-dtype", choices=["f32", "f64"], default="f32",
                   help="cfg5 K dtype: f32 (fp16x2 MFMA) or f64 (the reference's default; int8 MFMA residues + CRT, "
                        "125 GB of blocks per part at 500k iids)")
    p.add_argument("--grm5-parity-max-sid", type=int, default=65536,
                   help="cfg5 at N > 1: the oracle check runs only up to this many SNPs (N = 1: always)")
    p.add_argument("--out-ld", type=int, default=0,
                   help="decode legs: leading dimension (floats) of the timed f32 F-order block buffer; 0 = "
                        "round_up(n, 16), the tight columns the library's reads write")
    p.add_argument("--spread-ld", type=int, default=8_000_000,
                   help="decode legs: column pitch (floats) of the side measurement (frac_spread): a 32 MB pitch "
                        "spreads a 4 GB block over 64 GB of HBM pages (DESIGN 3.1); 0 = no side measurement")
    p.add_argument("--out-ld-c", type=int, default=0,
                   help="C-order decode leg: row pitch (floats) of the output: 0 = the block width (tight rows, "
                        "as the library writes); 32768 = 128 KB rows spread over 64 GB of HBM pages (DESIGN 3.1)")
    p.add_argument("--e2e", choices=["on", "off"], default="on", help="pinned-host -> HBM streaming leg")
    p.add_argument("--e2e-sid", type=int, default=8192, help="SNPs held in pinned host memory")
    p.add_argument("--e2e-passes", type=int, default=4)
    p.add_argument("--skip-cpu", action="store_true")
    p.add_argument("--decode-variant", type=int, default=0, help="snpmi_set_kernel_variant('decode', v) (A/B runs)")
    p.add_argument("--hook", action="append", default=[], metavar="NAME=V",
                   help="snpmi_set_kernel_variant(NAME, V) before the legs (A/B runs; repeatable)")
    p.add_argument("--cpu-seconds", type=float, default=6.0)
    p.add_argument("--seed", type=int, default=5)
    p.add_argument("--force-rccl", action="store_true", help="build the RCCL communicator even at world size 1")
    p.add_argument("--dist-timeout", type=float, default=300.0, help="seconds for the RCCL id wait and init")
    p.add_argument("--watchdog", type=float, default=300.0,
                   help="N > 1: seconds without a progress mark before a rank dumps its diagnostics (leg, block, "
                        "collective trace) to stderr, rank 0 prints a partial JSON line, and the job exits 4")
    p.add_argument("--watchdog-final", type=float, default=1800.0,
                   help="the watchdog's limit while ranks > 0 wait at the final barrier for rank 0's rank-only legs")
    p.add_argument("--selfcheck", choices=["on", "off"], default="on",
                   help="early group self-check leg: communicator size, a small K-tile all-reduce vs the oracle, "
                        "one cfg5 all-gather bit-exact")
    p.add_argument("--side-reps", type=int, default=8,
                   help="decode legs: launches timed on the other column layout beside the timed steps (tight "
                        "if --out-ld spreads the block, else --spread-ld)")
    p.add_argument("--beta", choices=["on", "off"], default="on", help="configs[2] leg: Beta(1,25) at 100k x 1M")
    p.add_argument("--beta-iid", type=int, default=100_000)
    p.add_argument("--beta-sid", type=int, default=1_000_000)
    p.add_argument("--file", choices=["on", "off"], default="on", help="file-backed leg through the mirrored API")
    p.add_argument("--file-iid", type=int, default=50_000)
    p.add_argument("--file-sid", type=int, default=100_000)
    p.add_argument("--file-dir", default=None, help="directory for the synthetic .bed (default: $TMPDIR)")
    p.add_argument("--cpu-grm-iid", type=int, default=50_000, help="GRM CPU baseline: iids of the timed slice")
    p.add_argument("--cpu-grm-sid", type=int, default=256, help="GRM CPU baseline: SNPs of the timed syrk")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------- the box
def _sysfs_card(pci):
    """/sys/class/drm/cardN/device of the GPU at PCI domain:bus:device (None if not found)."""
    import glob

    want = "%04x:%02x:%02x" % tuple(pci)
    for dev in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        try:
            if os.path.basename(os.path.realpath(dev)).startswith(want):
                return dev
        except OSError:
            continue
    return None


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def read_sclk_mhz(card):
    """The GPU's current shader clock from sysfs: hwmon freq1_input (Hz), else the starred level of
    pp_dpm_sclk; None if neither is readable."""
    import glob

    if card is None:
        return None
    for f in glob.glob(os.path.join(card, "hwmon", "hwmon*", "freq1_input")):
        v = _read(f)
        if v and v.isdigit():
            return int(v) / 1e6
    t = _read(os.path.join(card, "pp_dpm_sclk"))
    if t:
        for ln in t.splitlines():
            if ln.strip().endswith("*"):
                try:
                    return float(ln.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
                except (IndexError, ValueError):
                    return None
    return None


def box_info(N, dist):
    """Device ids of the GPU this rank measures on: name, CUs, HBM, UUID, PCI
    address, max SCLK, the sysfs unique_id / serial when readable, the host name."""
    name = ctypes.create_string_buffer(64)
    mem, cus = ctypes.c_uint64(), ctypes.c_int()
    uuid = (ctypes.c_uint8 * 16)()
    pci = (ctypes.c_int * 3)()
    clk = ctypes.c_int()
    N.call("snpmi_device_info", dist.device, name, 64, ctypes.byref(mem), ctypes.byref(cus))
    N.call("snpmi_device_ids", dist.device, uuid, pci, ctypes.byref(clk))
    card = _sysfs_card(list(pci))
    return {"gpu": name.value.decode(errors="replace"), "cus": cus.value, "hbm_bytes": mem.value,
            "uuid": bytes(uuid).hex(), "pci": "%04x:%02x:%02x" % tuple(pci), "sclk_max_mhz": clk.value / 1e3,
            "unique_id": _read(os.path.join(card, "unique_id")) if card else None,
            "serial": _read(os.path.join(card, "serial_number")) if card else None,
            "sysfs": card, "host": socket.gethostname(), "sclk_idle_mhz": read_sclk_mhz(card)}


class ClockSampler(object):
    """Samples the GPU's SCLK from sysfs every 50 ms on a thread while a leg runs (the loaded clock
    the leg's rate depends on; MI355X_MICROARCH.md: devices differ by ~12%)."""

    def __init__(self, box, period=0.05):
        import threading

        self.card, self.period, self.v = box.get("sysfs"), period, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.wait(self.period):
            c = read_sclk_mhz(self.card)
            if c is not None:
                self.v.append(c)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join(timeout=2)

    def summary(self):
        if not self.v:
            return {"samples": 0, "note": "no readable sysfs clock on this box (%s)" % self.card}
        v = np.asarray(self.v)
        return {"samples": int(v.size), "mean": float(v.mean()), "median": float(np.median(v)), "min": float(v.min()),
                "max": float(v.max()), "source": "sysfs (%s), every 50 ms during the leg" % self.card}


# ---------------------------------------------------------------------------- leg 0: group self-check
SELF_N, SELF_M = 600, 3000


def leg_selfcheck(N, args, dist):
    """Before the long legs: does the group work?  (1) the communicator holds
    WORLD_SIZE ranks; (2) a small K-tile all-reduce through the cfg4 code path (ShardedGrm.
    add_packed_combine: each rank its SNP span of a 600-iid x 3000-SNP matrix, Unit, f32, the
    overlapped column groups) -- every rank's K identical (checksums over the group) and rank 0's K vs
    the oracle (f64); (3) one cfg5 block through PartitionedGrm's all-gather, rebuilt bit-exactly;
    (4) every rank issued the same RCCL calls (count and call-sequence signature)."""
    from pysnptools_amd.shard import ShardedGrm, rank_span

    t0 = time.perf_counter()
    res = {"world": dist.world, "n_gpus": dist.n_gpus, "group_size_ok": dist.n_gpus == dist.world}
    n, m = SELF_N, SELF_M
    pitch = N.lib().snpmi_packed_pitch(n)
    full = Dev(N, pitch * m)
    synth(N, full.p, pitch, n, 0, m, args.seed + 900, 0.05)
    lo, hi = rank_span(m, dist.rank, dist.world)
    stats = Dev(N, max(1, hi - lo) * 8)
    coll = "allreduce" if dist.can_reduce and (dist.world > 1 or dist.rccl) else "none"
    g = ShardedGrm(n, np.float32, dist if dist.can_reduce else None, coll, 0, dist.rank, dist.world)
    K = np.empty((n, n), dtype=np.float32)
    try:
        g.add_packed_combine(full.at(lo * pitch), pitch, hi - lo, N.STD_UNIT, 0.0, 0.0, 0, stats.p,
                             parts=args.grm_overlap_parts)
        N.call("snpmi_stream_sync")
        t, _ = g.tiles()
        ri = np.arange(n, dtype=np.uint64)
        dri, dout = Dev(N, n * 8), Dev(N, n * n * 4)
        N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
        N.call("snpmi_dev_grm_extract", t, n, N.DT_F32, dri.p, n, None, n, 1, 1.0, dout.p)
        N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
        dri.free()
        dout.free()
    finally:
        g.abort()
    k64 = K.astype(np.float64)
    sums = (float(k64.sum()), float((k64 * np.arange(1, n + 1)).sum()))
    same = all(dist.max(x) == -dist.max(-x) for x in sums)
    res["allreduce"] = {"collective": coll, "workload": "%d iids x %d SNPs, f32, each rank its SNP span" % (n, m),
                        "every_rank_same_K": bool(same)}
    if dist.rank == 0:
        from oracle import oracle as O

        bpc = (n + 3) // 4
        host = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(host), full.p, host.nbytes)
        Z = O.decode(np.ascontiguousarray(host[:, :bpc]).reshape(-1), n, m, dtype=np.float64)
        O.standardize_native(Z)
        ref = Z.dot(Z.T)
        err = float(np.abs(k64 - ref).max() / np.abs(np.diag(ref)).max())
        res["allreduce"].update(max_abs_err_over_max_diag=err, tolerance=2e-6)
    full.free()
    stats.free()
    if dist.world > 1 or dist.rccl:
        mark(None, "selfcheck all-gather")
        x, cdf = maf_table(4096)

        def fill(host, s0, cnt):
            N.call("snpmi_host_synth_bed", host, N.lib().snpmi_packed_pitch(4096), 4096, s0, cnt, args.seed + 901, 0.05,
                   N.ptr(x), N.ptr(cdf), len(x), 1)

        res["allgather_bit_exact"] = gather_check(N, dist, max(dist.world, GRM5_PLAN_WORLD), fill, 4096, 1024, 1024)
    tr = N.rccl_trace()
    calls, sig48 = float(tr["calls"]), float(int(tr["sig"], 16) & ((1 << 48) - 1))
    res["rccl_calls"] = tr["calls"]
    res["rccl_same_calls_every_rank"] = bool(all(dist.max(v) == -dist.max(-v) for v in (calls, sig48)))
    res["seconds"] = time.perf_counter() - t0
    ok = res["group_size_ok"] and same and res["rccl_same_calls_every_rank"]
    if dist.rank == 0:
        ok = ok and res["allreduce"]["max_abs_err_over_max_diag"] <= 2e-6
    if res.get("allgather_bit_exact") is False:
        ok = False
    res["pass"] = bool(ok) if dist.rank == 0 else None
    return res


# ---------------------------------------------------------------------------- process launch
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


SPAWN_GRACE_S = 15.0


def spawn_ranks(args, argv):
    """`python bench.py --gpus N` without a launcher: start N rank processes (one per GPU) before
    this process touches HIP, relay rank 0's stdout, and exit with the worst rank status."""
    tmp = tempfile.mkdtemp(prefix="snpmi_bench_")
    port = str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, SNPMI_RCCL_ID_FILE=os.path.join(tmp, "rccl.id"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc, deadline = 0, None
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and not rc:
                    # one rank failed: its watchdog left the job's abort file, so the others dump their
                    # diagnostics and exit within a second; whoever is still running after the grace
                    # period would wait in a collective forever
                    rc = code
                    deadline = time.time() + SPAWN_GRACE_S
            if deadline is not None and time.time() > deadline:
                for q in procs:
                    q.kill()
            time.sleep(0.2)
    finally:
        for q in procs:
            q.kill()
        for f in os.listdir(tmp):
            os.remove(os.path.join(tmp, f))
        os.rmdir(tmp)
    return rc


class Dev:
    def __init__(self, N, nbytes):
        self.N = N
        self.p = ctypes.c_void_p()
        N.call("snpmi_dev_alloc", ctypes.byref(self.p), int(nbytes))

    def at(self, off):
        return ctypes.c_void_p(self.p.value + int(off))

    def free(self):
        if self.p:
            self.N.call("snpmi_dev_free", self.p)
            self.p = None


class Events:
    def __init__(self, N, count):
        self.N = N
        self.ev = []
        for _ in range(count):
            e = ctypes.c_void_p()
            N.call("snpmi_event_create", ctypes.byref(e))
            self.ev.append(e)

    def record(self, i, on_copy=0):
        """on_copy: 0 = the calling thread's current stream, 1 = copy stream, 2 = aux stream"""
        if on_copy:
            self.N.call("snpmi_event_record_on", self.ev[i], on_copy)
        else:
            self.N.call("snpmi_event_record", self.ev[i])

    def ms(self, a, b):
        out = ctypes.c_float()
        self.N.call("snpmi_event_elapsed_ms", self.ev[a], self.ev[b], ctypes.byref(out))
        return float(out.value)

    def destroy(self):
        for e in self.ev:
            self.N.call("snpmi_event_destroy", e)


_T0 = time.time()


WD = None  # this rank's pysnptools_amd.dist.Watchdog (N > 1)
RANK = 0
# rank 0: the line's fields measured so far -- what the watchdog prints as a partial JSON line
PARTIAL = {}
RCCL_FALLBACK = {}  # the RCCL init error when the job fell back to the host group


def mark(leg=None, detail=None, limit=None):
    """Watchdog progress mark (no output)."""
    if WD is not None:
        WD.mark(leg, detail, limit)


def progress(msg, limit=None):
    """One line on stderr per leg (a long default run is never silent for minutes) and a watchdog
    mark.  SNPMI_BENCH_STALL="R:PREFIX" (tests) makes rank R hang here at the first leg whose label
    starts with PREFIX, as a rank stuck inside a leg would."""
    sys.stderr.write("[bench %7.1fs] %s\n" % (time.time() - _T0, msg))
    sys.stderr.flush()
    mark(msg, None, limit)
    stall = os.environ.get("SNPMI_BENCH_STALL", "")
    if stall:
        r, _, prefix = stall.partition(":")
        if int(r) == RANK and msg.startswith(prefix):
            sys.stderr.write("[bench] rank %d: SNPMI_BENCH_STALL -- hanging in leg %r\n" % (RANK, msg))
            sys.stderr.flush()
            while True:
                time.sleep(3600)


def partial_line(diag):
    """The watchdog's partial JSON line (rank 0): what was measured before the stall, marked as such."""
    if PARTIAL.get("_printed"):  # the full line is out already (a stall at the final barrier)
        return
    line = {"metric": METRIC, "value": None, "unit": "SNPs/s", "higher_is_better": True, "partial": True,
            "error": "watchdog: %s (rank %d, leg %r)" % (diag["reason"], diag["rank"], diag["leg"])}
    line.update(PARTIAL)
    line["watchdog"] = diag
    print(json.dumps(line, default=str), flush=True)


def maf_table(n_iid):
    # SnpGen's MAF curve (snpreader/snpgen.py:140-151); restated here so the product never
    # imports the oracle
    w0, w1 = -0.6482249, -8.49790398
    x = np.logspace(np.log10(0.1 / n_iid), np.log10(0.5), 100, base=10)
    y = np.exp(w0 * np.log(x) + w1)
    cdf = np.cumsum(y / y.sum())
    cdf[-1] = 1.0
    return np.ascontiguousarray(x), np.ascontiguousarray(cdf)


def synth(N, buf, pitch, n, sid0, m, seed, miss):
    x, cdf = maf_table(n)
    N.call("snpmi_dev_synth_bed", buf, pitch, n, sid0, m, seed, miss, N.ptr(x), N.ptr(cdf), len(x))


def cgroup_cpu_quota():
    """CPUs the cgroup grants (cpu.max on cgroup v2, cfs quota/period on v1), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        return None if quota <= 0 else quota / period
    except (OSError, ValueError):
        return None


def cpu_counts():
    """Every CPU count that bounds this process: the affinity mask, the cgroup quota, the
    machine (os.cpu_count(): on the GPU box the whole host, not this job's share) and
    OMP_NUM_THREADS (the box's per-GPU CPU share).  ``usable`` = the smallest bound."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    usable = aff
    if quota:
        usable = min(usable, max(1, int(quota)))
    if omp:
        usable = min(usable, omp)
    return {"affinity": aff, "cgroup_quota": quota, "os_cpu_count": os.cpu_count(), "omp_num_threads": omp,
            "usable": usable}


def cpu_threads():
    return cpu_counts()["usable"]


def _counts_text(c):
    return ("affinity %d CPUs, cgroup quota %s, os.cpu_count() %d, OMP_NUM_THREADS %s -> %d threads"
            % (c["affinity"], "none" if c["cgroup_quota"] is None else "%.1f" % c["cgroup_quota"],
               c["os_cpu_count"] or 0, c["omp_num_threads"], c["usable"]))


def shard(m, rank, world):
    return m * rank // world, m * (rank + 1) // world


# ---------------------------------------------------------------------------- leg 1: decode + standardize
WIDE_MIN_BYTES = 512 << 20  # block buffers of >= 512 MB take the wide column pitch


def leg_standardize(N, args, dist, n=None, n_sid=None, std=None, a=0.0, b=0.0, miss=0.01, seed=None):
    """Stats + decode of this rank's SNP shard of the n x n_sid packed matrix (resident in HBM) in
    blocks of args.block SNPs into an f32 F-order block buffer; Unit by default, Beta(a, b) with
    std=N.STD_BETA.  Beside the timed steps (untimed): the same kernel on a tight-column buffer
    (frac_tight) and the measured copy / fill ceilings."""
    n = args.n_iid if n is None else n
    n_sid = args.n_sid if n_sid is None else n_sid
    std = N.STD_UNIT if std is None else std
    seed = args.seed if seed is None else seed
    B = args.block
    lo, hi = shard(n_sid, dist.rank, dist.world)
    m = hi - lo
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = Dev(N, pitch * max(m, 1))
    synth(N, packed.p, pitch, n, lo, m, seed, miss)
    nblk = (m + B - 1) // B
    lut, stats = Dev(N, B * 16), Dev(N, B * 8)
    tight = ld
    out = None
    if args.out_ld > ld and B * ld * 4 >= WIDE_MIN_BYTES:
        try:
            out = Dev(N, B * (args.out_ld // 16 * 16) * 4)
            ld = args.out_ld // 16 * 16
        except Exception:  # not enough HBM for the spread layout: tight columns
            out = None
    if out is None:
        out = Dev(N, B * ld * 4)
    ev = Events(N, 2 + 2 * max(nblk, args.side_reps))
    N.call("snpmi_set_kernel_variant", b"decode", args.decode_variant)
    for h in args.hook:
        name, v = h.split("=")
        N.call("snpmi_set_kernel_variant", name.encode(), int(v))

    def run_block(src, cnt, timed, k, dst=None, dld=None):
        N.call("snpmi_dev_snp_stats", src, pitch, n, cnt, 0, std, a, b, 0, N.DT_F32, stats.p, lut.p)
        if timed:
            ev.record(2 + 2 * k)
        N.call("snpmi_dev_decode", src, pitch, n, cnt, lut.p, N.DT_F32, 0, (dst or out).p, dld or ld)
        if timed:
            ev.record(3 + 2 * k)

    def step(timed):
        if timed:
            ev.record(0)
        for k in range(nblk):
            s0 = k * B
            run_block(packed.at(s0 * pitch), min(B, m - s0), timed, k)
        if timed:
            ev.record(1)
        N.call("snpmi_stream_sync")
        return sum(ev.ms(2 + 2 * k, 3 + 2 * k) for k in range(nblk)) if timed else 0.0

    for _ in range(args.warmup):
        step(False)
    dist.barrier()
    N.call("snpmi_stream_sync")
    t0 = time.perf_counter()
    dec_ms_total = 0.0
    for _ in range(args.steps):
        dec_ms_total += step(True)
    N.call("snpmi_stream_sync")
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    weak_wall = None
    if dist.world > 1:
        # weak figure: every rank streams the whole n_sid per step (its shard `world` times)
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps * dist.world):
            step(False)
        N.call("snpmi_stream_sync")
        dist.barrier()
        weak_wall = dist.max(time.perf_counter() - t1)
    launches = args.steps * nblk
    dec_mean_ms = dec_ms_total / max(launches, 1)
    # achieved = bytes of all launches / their summed time (the last block of a shard is partial)
    bytes_per_step = m * ((n + 3) // 4 + 4 * n)
    achieved_gbs = bytes_per_step * args.steps / (dec_ms_total * 1e-3) / 1e9 if dec_ms_total else 0.0
    # side measurement: the same kernel on the other column layout (full blocks only) -- tight columns
    # (what Bed.read(xp='hbm') writes) when the timed buffer is spread, else the spread pitch
    side_ld = tight if ld != tight else args.spread_ld // 16 * 16
    side_gbs = side_ms = None
    full = [k for k in range(nblk) if (k + 1) * B <= m][:args.side_reps]
    if side_ld > 0 and full and (side_ld == tight or (side_ld > ld and B * tight * 4 >= WIDE_MIN_BYTES)):
        side = None
        try:
            side = Dev(N, B * side_ld * 4)
        except Exception:  # the spread layout does not fit beside the matrix: no side figure
            side = None
        if side is not None:
            for k in full[:2]:
                run_block(packed.at(k * B * pitch), B, False, k, side, side_ld)
            for i, k in enumerate(full):
                run_block(packed.at(k * B * pitch), B, True, i, side, side_ld)
            N.call("snpmi_stream_sync")
            side_ms = float(np.mean([ev.ms(2 + 2 * i, 3 + 2 * i) for i in range(len(full))]))
            side_gbs = B * ((n + 3) // 4 + 4 * n) / (side_ms * 1e-3) / 1e9
            side.free()
    # measured stream ceilings (untimed): device-to-device copy and write-only fill, tight bytes
    cbytes = min(B * tight * 4, pitch * m)
    N.call("snpmi_dev_memcpy_d2d", out.p, packed.p, cbytes)
    N.call("snpmi_stream_sync")
    ev.record(0)
    for _ in range(5):
        N.call("snpmi_dev_memcpy_d2d", out.p, packed.p, cbytes)
    ev.record(1)
    N.call("snpmi_stream_sync")
    copy_gbs = 2 * 5 * cbytes / (ev.ms(0, 1) * 1e-3) / 1e9
    ev.record(0)
    for _ in range(5):
        N.call("snpmi_dev_memset", out.p, 0, B * tight * 4)
    ev.record(1)
    N.call("snpmi_stream_sync")
    fill_gbs = 5 * B * tight * 4 / (ev.ms(0, 1) * 1e-3) / 1e9
    cur_ld = ld  # the parity sample is decoded into the timed buffer layout
    sample = gpu_cols = None
    if dist.rank == 0 and not args.skip_cpu:
        # parity sample: the first 512 columns, re-decoded by the same kernels (untimed)
        ncols = min(512, m)
        sample = np.empty((ncols, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
        run_block(packed.p, ncols, False, 0, out, cur_ld)
        gpu_cols = np.empty((ncols, tight), dtype=np.float32)
        if cur_ld == tight:
            N.call("snpmi_memcpy_d2h", N.ptr(gpu_cols), out.p, gpu_cols.nbytes)
        else:
            for j in range(ncols):
                N.call("snpmi_memcpy_d2h", N.ptr(gpu_cols[j]), out.at(j * cur_ld * 4), tight * 4)
    res = dict(wall=wall, weak_wall=weak_wall, dec_mean_ms=dec_mean_ms, achieved_gbs=achieved_gbs,
               side_ld=side_ld, side_gbs=side_gbs, side_ms=side_ms, side_launches=len(full), tight=tight,
               copy_gbs=copy_gbs, fill_gbs=fill_gbs, full_block_bytes=B * ((n + 3) // 4 + 4 * n), launches=launches,
               nblk=nblk, pitch=pitch, sample=sample, gpu_cols=gpu_cols, m=m, out_ld=ld, n=n, n_sid=n_sid,
               steps=args.steps,
               # whole step: k_snp_stats reads every column once, the decode reads it again and writes it
               step_bytes=m * (2 * ((n + 3) // 4) + 4 * n))
    N.call("snpmi_stream_sync")
    ev.destroy()
    for d in (packed, lut, stats, out):
        d.free()
    return res


def leg_decode_c(N, args):
    """C-order decode (k_decode_c_reg<float>): rows of 2048 SNPs at 500k iids, 16-B row pitch."""
    n, B, reps = args.n_iid, args.block, 8
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * B)
    synth(N, packed.p, pitch, n, 0, B, args.seed, 0.01)
    lut, stats = Dev(N, B * 16), Dev(N, B * 8)
    rld, out = B, None
    if args.out_ld_c > B and B * n * 4 >= (1 << 30):
        try:
            out = Dev(N, n * (args.out_ld_c // 4 * 4) * 4)
            rld = args.out_ld_c // 4 * 4
        except Exception:  # not enough HBM for the spread rows: tight rows
            out = None
    if out is None:
        out = Dev(N, B * n * 4)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 1, out.p, rld)
    ev = Events(N, 2 * reps)
    N.call("snpmi_stream_sync")
    for r in range(reps):
        ev.record(2 * r)
        N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 1, out.p, rld)
        ev.record(2 * r + 1)
    N.call("snpmi_stream_sync")
    ms = float(np.mean([ev.ms(2 * r, 2 * r + 1) for r in range(reps)]))
    nbytes = B * ((n + 3) // 4 + 4 * n)
    # parity: C-order rows equal the F-order decode transposed (first 64 iids x all SNPs)
    rows = np.empty((64, B), dtype=np.float32)
    for i in range(64):
        N.call("snpmi_memcpy_d2h", N.ptr(rows[i]), out.at(i * rld * 4), B * 4)
    ld = (n + 15) // 16 * 16
    fout = Dev(N, B * ld * 4)
    N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, fout.p, ld)
    cols = np.empty((B, ld), dtype=np.float32)
    N.call("snpmi_memcpy_d2h", N.ptr(cols), fout.p, cols.nbytes)
    same = bool(np.array_equal(rows, cols[:, :64].T))
    ev.destroy()
    for d in (packed, lut, stats, out, fout):
        d.free()
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"workload": "C-order decode of %d SNPs x %d iids (f32, rows of %d SNPs, row pitch %d floats)"
                        % (B, n, B, rld), "row_ld": rld,
            "kernel": "k_decode_c_reg<float>", "mean_launch_ms": ms, "per_launch_bytes": nbytes,
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "parity": {"check": "rows 0..63 == F-order decode transposed", "bit_exact": same}}


def leg_e2e(N, args):
    """Pinned host -> HBM streaming: packed columns of --e2e-sid SNPs sit in page-locked host memory;
    each 2048-SNP chunk goes H2D on the copy stream into a 3-slot device ring, the compute stream
    waits on its event and runs stats + decode (f32, F order, into HBM), and the copy stream waits
    on the compute event of the chunk that last used a slot before overwriting it."""
    n, B = args.n_iid, args.block
    m = args.e2e_sid // B * B
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    host = ctypes.c_void_p()
    N.call("snpmi_host_alloc", ctypes.byref(host), m * pitch)
    src = Dev(N, m * pitch)
    synth(N, src.p, pitch, n, 0, m, args.seed + 7, 0.01)
    N.call("snpmi_memcpy_d2h", host, src.p, m * pitch)
    ring = [Dev(N, B * pitch) for _ in range(3)]
    lut, stats, out = Dev(N, B * 16), Dev(N, B * 8), Dev(N, B * ld * 4)
    nch = m // B
    total = nch * args.e2e_passes
    ev = Events(N, 4 + 2 * 3)  # 0..3 timing; 4+s = H2D done (slot s); 7+s = compute done (slot s)
    h2d_ev = lambda s: 4 + s  # noqa: E731
    use_ev = lambda s: 7 + s  # noqa: E731

    def stream(timed):
        if timed:
            ev.record(0)
        for c in range(total):
            s = c % 3
            hsrc = ctypes.c_void_p(host.value + (c % nch) * B * pitch)
            if c >= 3:
                N.call("snpmi_stream_wait_event", ev.ev[use_ev(s)], 1)
            N.call("snpmi_memcpy_async", ring[s].p, hsrc, B * pitch, 0, 1)
            ev.record(h2d_ev(s), on_copy=1)
            N.call("snpmi_stream_wait_event", ev.ev[h2d_ev(s)], 0)
            N.call("snpmi_dev_snp_stats", ring[s].p, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
            N.call("snpmi_dev_decode", ring[s].p, pitch, n, B, lut.p, N.DT_F32, 0, out.p, ld)
            ev.record(use_ev(s))
        if timed:
            ev.record(1)
        N.call("snpmi_stream_sync")

    stream(False)
    t0 = time.perf_counter()
    stream(True)
    wall = time.perf_counter() - t0
    ev_ms = ev.ms(0, 1)
    # parity: the last chunk's values == decode of the same columns from HBM
    last = np.empty((B, ld), dtype=np.float32)
    N.call("snpmi_memcpy_d2h", N.ptr(last), out.p, last.nbytes)
    c_last = (total - 1) % nch
    N.call("snpmi_dev_snp_stats", src.at(c_last * B * pitch), pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
           stats.p, lut.p)
    N.call("snpmi_dev_decode", src.at(c_last * B * pitch), pitch, n, B, lut.p, N.DT_F32, 0, out.p, ld)
    ref = np.empty_like(last)
    N.call("snpmi_memcpy_d2h", N.ptr(ref), out.p, ref.nbytes)
    same = bool(np.array_equal(last[:, :n], ref[:, :n]))
    # H2D peak of the same pinned buffer on the copy stream (no kernels)
    ev.record(2, on_copy=1)
    for p in range(args.e2e_passes):
        for c in range(nch):
            N.call("snpmi_memcpy_async", ring[c % 3].p, ctypes.c_void_p(host.value + c * B * pitch), B * pitch, 0, 1)
    ev.record(3, on_copy=1)
    N.call("snpmi_stream_sync")
    peak_gbs = args.e2e_passes * m * pitch / (ev.ms(2, 3) * 1e-3) / 1e9
    ev.destroy()
    N.call("snpmi_host_free", host)
    for d in ring + [src, lut, stats, out]:
        d.free()
    snps = total * B
    pcie_gbs = snps * pitch / (ev_ms * 1e-3) / 1e9
    return {"workload": "%d SNPs x %d iids streamed %d times from pinned host (packed, %d B/SNP) -> stats + "
                        "decode + Unit -> f32 F-order in HBM, 2048-SNP chunks, 3-slot ring, copy stream + "
                        "compute stream" % (m, n, args.e2e_passes, pitch),
            "snps_per_s": snps / (ev_ms * 1e-3), "seconds": ev_ms * 1e-3, "host_wall_s": wall,
            "pcie_GBps": pcie_gbs, "h2d_peak_GBps": peak_gbs, "frac_of_h2d_peak": pcie_gbs / peak_gbs,
            "parity": {"check": "last chunk == decode of the same columns resident in HBM", "bit_exact": same}}


def cpu_baseline_standardize(args, sample, timed=True, n=None, is_beta=False, a=np.nan, b=np.nan):
    """Oracle C/OpenMP decode + one-pass standardize on a bounded sample (rank 0), at the largest
    usable thread count and at 1 thread; with timed=False (N > 1) one untimed pass for parity."""
    from oracle import oracle as O

    n = args.n_iid if n is None else n
    counts = cpu_counts()
    threads = counts["usable"]
    bpc = (n + 3) // 4
    body = np.ascontiguousarray(sample[:, :bpc]).reshape(-1)
    ncols = sample.shape[0]
    ref, _ = O.decode_standardize(body, n, ncols, is_beta=is_beta, a=a, b=b, dtype=np.float32, num_threads=threads)
    if not timed:
        return ref, None

    def rate(th, budget, max_reps):
        done, t0 = 0, time.perf_counter()
        while True:
            O.decode_standardize(body, n, ncols, is_beta=is_beta, a=a, b=b, dtype=np.float32, num_threads=th)
            done += ncols
            el = time.perf_counter() - t0
            if el >= budget or done >= max_reps * ncols:
                return done / el, done // ncols, el

    v_all, reps_all, el_all = rate(threads, args.cpu_seconds, 64)
    v_one, reps_one, el_one = rate(1, args.cpu_seconds / 2, 4)
    return ref, {"value": v_all, "unit": "SNPs/s", "cores": threads, "kind": "port",
                 "single_thread_value": v_one, "cpu_counts": counts,
                 "sample": "%d reps x %d SNP columns x %d iids (first packed columns of the same synthetic matrix), "
                           "f32 %s, oracle/bed_oracle.c oracle_decode_standardize_f32 at %d threads (%s), %.1f s; "
                           "1 thread: %d reps, %.1f s"
                           % (reps_all, ncols, n, "Beta(%g,%g)" % (a, b) if is_beta else "Unit", threads,
                              _counts_text(counts), el_all, reps_one, el_one)}


# ---------------------------------------------------------------------------- leg 2: GRM (cfg4)
def leg_grm(N, args, dist, dtype, keep_tiles=False):
    """cfg4 through pysnptools_amd.shard.ShardedGrm: this rank's contiguous SNP span (packed codes
    generated in HBM by global SNP id, so the shards of any world tile the same matrix) added to
    a GRM session in one call (<= 65536 SNPs per SYRK launch), then the RCCL collective of the
    tiles.  ``keep_tiles`` (tests): a host copy of this rank's tiles after the collective."""
    from pysnptools_amd.shard import ShardedGrm, rank_span

    n, m = args.grm_iid, args.grm_sid
    npdt = np.float32 if dtype == "f32" else np.float64
    dt, esz = (N.DT_F32, 4) if dtype == "f32" else (N.DT_F64, 8)
    pitch = N.lib().snpmi_packed_pitch(n)
    lo, hi = rank_span(m, dist.rank, dist.world)
    my_m = hi - lo
    packed = Dev(N, max(1, my_m) * pitch)
    if my_m:
        synth(N, packed.p, pitch, n, lo, my_m, args.seed + 100, 0.01)
    stats = Dev(N, max(1, my_m) * 2 * esz)
    want = "allreduce" if args.grm_collective == "auto" else args.grm_collective
    collective = want if dist.can_reduce else "none"
    ev = Events(N, 4)
    chunks = (my_m + 65535) // 65536 if my_m else 0

    def session():
        return ShardedGrm(n, npdt, dist if dist.can_reduce else None, collective, 0, dist.rank, dist.world)

    # warm-up: one 10k-SNP piece (scratch allocations, the session tiles, code objects)
    g = session()
    g.add_packed(packed.p, pitch, min(my_m, args.grm_block), N.STD_UNIT, 0.0, 0.0, 0, stats.p)
    N.call("snpmi_stream_sync")
    g.abort()
    sum_r, nlaunch = ctypes.c_uint64(), ctypes.c_uint64()
    if dtype == "f64":
        N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
        N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
    g = session()
    dist.barrier()
    t0 = time.perf_counter()
    ev.record(0)
    # the SYRK of this rank's shard + the K-tile collective, overlapped under a real RCCL
    # communicator (f32: the last launch in column groups, each group's tiles summed on the aux
    # stream under the next group's SYRK); ev 1 = the last SYRK done, ev 2 = K combined
    g.add_packed_combine(packed.p, pitch, my_m, N.STD_UNIT, 0.0, 0.0, 0, stats.p, parts=args.grm_overlap_parts,
                         syrk_done=ev.ev[1])
    ev.record(2)
    N.call("snpmi_stream_sync")
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    crt_moduli = crt_block_moduli = None
    if dtype == "f64":  # moduli the timed launches / blocks ran with (chosen on the device)
        N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
        crt_moduli = sum_r.value / max(nlaunch.value, 1)
        N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
        crt_block_moduli = sum_r.value / max(nlaunch.value, 1) if nlaunch.value else None
    syrk_ms = ev.ms(0, 1) if my_m else 0.0
    coll_ms = ev.ms(1, 2) if collective != "none" else 0.0
    tiles, count = g.tiles()
    trace = None
    if g.holds_k():  # the other ranks' tiles are unspecified after an ncclReduce
        tr = ctypes.c_double()
        N.call("snpmi_dev_grm_trace", tiles, n, dt, ctypes.byref(tr))
        trace = tr.value
    host_tiles = None
    if keep_tiles:
        host_tiles = np.empty(count, dtype=npdt)
        N.call("snpmi_memcpy_d2h", N.ptr(host_tiles), tiles, host_tiles.nbytes)
    unoverlapped = {}
    if collective != "none" and dist.world > 1:
        # beside the timed line (untimed; the tiles are overwritten): each collective alone over the
        # whole tile buffer, unoverlapped -- ncclReduce onto rank 0 (half the bytes: K for one caller)
        # and ncclAllReduce (K on every rank, the configs[3] exchange)
        for name, root in (("reduce", 0), ("allreduce", None)):
            mark(None, "grm %s unoverlapped %s" % (dtype, name))
            dist.barrier()
            ev.record(0)
            dist.sum_dev(tiles, count, npdt, root)
            ev.record(3)
            N.call("snpmi_stream_sync")
            unoverlapped[name + "_ms"] = dist.max(ev.ms(0, 3))
        unoverlapped["bytes"] = count * esz
    g.abort()  # K stays as tiles in HBM; the session ends without the n x n extraction
    nb = (n + 255) // 256
    exec_ratio = SPLIT_PRODUCTS * 2 * 256 * 256 * (nb * (nb + 1) // 2) / (n * (n + 1))  # executed fp16 / algorithmic
    res = dict(wall=wall, syrk_ms=syrk_ms, allreduce_ms=coll_ms, trace=trace, exec_ratio=exec_ratio,
               mean_tflops=(n * (n + 1) * my_m / (syrk_ms * 1e-3) / 1e12) if syrk_ms else 0.0,
               launches=chunks, snps_per_launch=(my_m + chunks - 1) // chunks if chunks else 0,
               my_m=my_m, crt_moduli=crt_moduli, crt_block_moduli=crt_block_moduli, collective=collective,
               tiles=host_tiles, unoverlapped=unoverlapped)
    if dist.rank == 0 and not args.skip_cpu and my_m > 0:
        # parity sample (untimed): K rows 0..63 of the GRM of this rank's first 512 SNPs
        cm, rows = min(512, my_m), 64
        g = ShardedGrm(n, npdt, None, "none")
        g.add_packed(packed.p, pitch, cm, N.STD_UNIT, 0.0, 0.0, 0, stats.p)
        t, _ = g.tiles()
        ri = np.arange(rows, dtype=np.uint64)
        dri, dout = Dev(N, rows * 8), Dev(N, rows * n * esz)
        N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
        N.call("snpmi_dev_grm_extract", t, n, dt, dri.p, rows, None, n, 1, 1.0, dout.p)
        krows = np.empty((rows, n), dtype=npdt)
        N.call("snpmi_memcpy_d2h", N.ptr(krows), dout.p, krows.nbytes)
        g.abort()
        sample = np.empty((cm, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
        res["parity_sample"] = (krows, sample, cm)
        dri.free()
        dout.free()
    ev.destroy()
    for d in (packed, stats):
        d.free()
    return res


def grm_parity(args, krows, sample, cm, tol):
    """Oracle (f64, reference one-pass Unit + NumPy Z Z^T) vs the GPU's K rows."""
    from oracle import oracle as O

    n = args.grm_iid
    bpc = (n + 3) // 4
    Z = O.decode(np.ascontiguousarray(sample[:, :bpc]).reshape(-1), n, cm, dtype=np.float64)
    O.standardize_native(Z)
    rows = krows.shape[0]
    ref = Z[:rows].dot(Z.T)
    scale = np.abs(np.diag(ref[:, :rows])).max()
    err = float(np.abs(krows.astype(np.float64) - ref).max() / scale)
    return {"check": "K rows 0..%d over %d SNPs (first of this rank's blocks), %d iids: GPU %s vs oracle f64"
                     % (rows - 1, cm, n, krows.dtype), "max_abs_err_over_max_diag": err, "pass": err <= tol}


def cpu_baseline_grm(args, dtype):
    """The reference's GRM block step on the host (snpreader.py:651-655): NumPy Z.dot(Z.T)
    (OpenBLAS syrk, snpdata.py:203-206) on a --cpu-grm-iid x --cpu-grm-sid slice, plus the
    single-threaded K += of the n x n result, with the BLAS pool pinned to the usable CPU count;
    extrapolated to configs[3]: 50 blocks of 10k SNPs = 50 x (syrk time x 10k / b + one K +=)."""
    from threadpoolctl import threadpool_info, threadpool_limits

    n, b = args.cpu_grm_iid, args.cpu_grm_sid
    npdt = np.float32 if dtype == "f32" else np.float64
    rng = np.random.default_rng(0)
    Z = rng.standard_normal((n, b)).astype(npdt)
    counts = cpu_counts()
    want = counts["usable"]
    K = np.zeros((n, n), dtype=npdt)  # snpreader.py:643
    K.fill(0)  # touch the pages once: later blocks of the reference's loop add into a resident K
    with threadpool_limits(limits=want, user_api="blas"):
        used = [p.get("num_threads") for p in threadpool_info() if p.get("user_api") == "blas"]
        Z[:2048].dot(Z[:2048].T)  # warm the BLAS pool
        t0 = time.perf_counter()
        Kb = Z.dot(Z.T)
        t_syrk = time.perf_counter() - t0
    t0 = time.perf_counter()
    K += Kb
    t_add = time.perf_counter() - t0
    del Kb, K
    cores = used[0] if used else want
    M, B = args.grm_sid, args.grm_block
    nblocks = (M + B - 1) // B
    per_block = t_syrk * B / b + t_add
    total = nblocks * per_block
    return {"value": n * (n + 1) * M / total / 1e9, "unit": "GF/s", "cores": cores,
            "kind": "port", "cpu_counts": counts, "syrk_s": t_syrk, "k_add_s": t_add,
            "projected_seconds": total,
            "sample": "Z.dot(Z.T) of a %d x %d %s slice (NumPy/OpenBLAS syrk, BLAS pool pinned to %d threads; %s) "
                      "%.2f s + one single-threaded K += of %d x %d %.2f s; projected to %d blocks of %d SNPs as "
                      "%d x (syrk x %d/%d + K +=) = %.0f s" % (n, b, dtype, cores, _counts_text(counts), t_syrk, n, n,
                                                               t_add, nblocks, B, nblocks, B, b, total)}


# ---------------------------------------------------------------------------- leg 3: cfg5 partitioned GRM
def grm5_source(N, n, pitch, seed, miss, threads):
    """This rank's share of a SNP block, generated on host threads straight into the pinned slot
    (snpmi_host_synth_bed: SnpGen's MAF curve, `miss` missing) -- the stand-in for gathering the
    columns of a 125 GB .bed from the page cache, which cannot be written to the box's disk."""
    x, cdf = maf_table(n)

    def fill(host, s0, cnt):
        N.call("snpmi_host_synth_bed", host, pitch, n, s0, cnt, seed, miss, N.ptr(x), N.ptr(cdf), len(x), threads)

    return fill


def grm5_picks(N, n, part, P, nloc):
    """Sample blocks of the part for the parity check: its first diagonal block, its first
    off-diagonal block and its last block (the padded iids past n-1 when it ends the matrix)."""
    want, r0, c0 = {}, ctypes.c_uint64(), ctypes.c_uint64()
    for b in list(range(min(nloc, 256))) + [nloc - 1]:
        N.call("snpmi_grm_part_coords", n, part, P, b, ctypes.byref(r0), ctypes.byref(c0))
        key = "last" if b == nloc - 1 else ("diag" if r0.value == c0.value else "off")
        if key not in want:
            want[key] = (b, r0.value, c0.value)
    return want


def leg_grm5(N, args, dist):
    """configs[4]: 500k iids x 1M SNPs, K (500 GB f32 upper triangle) partitioned
    as 256x256 blocks over the P = max(N, 8) parts of the 8-GPU plan; this process computes part
    `rank` over ALL --grm5-sid SNPs through shard.PartitionedGrm (the package's cfg5 session): per
    block of --grm5-block SNPs each rank generates ITS 1/N share on host threads into a pinned slot,
    the copy stream uploads it under the previous block's kernels, the RCCL all-gather rebuilds the
    block at N > 1, then stats + the fp16x2 SYRK add it into this part's K blocks -- no reduction.
    The timed region is the whole job of this part (at N = 8: the 8-GPU job)."""
    from pysnptools_amd import hbm
    from pysnptools_amd.shard import PartitionedGrm

    n, m, world, rank = args.grm5_iid, args.grm5_sid, dist.world, dist.rank
    dt = np.dtype(np.float64 if args.grm5_dtype == "f64" else np.float32)
    P = max(world, GRM5_PLAN_WORLD)
    threads = cpu_threads()
    pitch = N.lib().snpmi_packed_pitch(n)
    fill = grm5_source(N, n, pitch, args.seed + 200, args.grm5_miss, threads)
    grp = dist if (world > 1 or dist.rccl) else None  # --force-rccl at N = 1: the real all-gather call, in place
    # warm-up (untimed): one block through a session of the same shape (code objects, scratch)
    g = PartitionedGrm(n, min(m, args.grm5_block), N.STD_UNIT, dist=grp, part=rank, parts=P, block=args.grm5_block,
                       out="hbm", dtype=dt)
    try:
        g.run(fill)
    finally:
        g.close()
        del g
    out = hbm.empty((N.lib().snpmi_grm_part_blocks(n, rank, P), 256, 256), dtype=dt, order="C")
    sum_r, nlaunch = ctypes.c_uint64(), ctypes.c_uint64()
    if dt == np.float64:
        N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
        N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
    g = PartitionedGrm(n, m, N.STD_UNIT, dist=grp, part=rank, parts=P, block=args.grm5_block, out=out, timing=True,
                       dtype=dt)
    try:
        N.call("snpmi_stream_sync")
        dist.barrier()
        t0 = time.perf_counter()
        block_ms = g.run(fill, progress=lambda k, nb: progress("grm5 block %d/%d" % (k + 1, nb))
                         if (k + 1) % 4 == 0 else mark(None, "grm5 block %d/%d" % (k + 1, nb)))
        dist.barrier()
        wall = dist.max(time.perf_counter() - t0)
        res = {"wall": wall, "block_ms": block_ms, "n_local_blocks": g.nloc, "m": m, "ms": g.ms, "P": P,
               "pitch": pitch, "blocks": len(block_ms), "threads": threads, "dtype": dt}
        if dt == np.float64:  # moduli per launch the timed blocks ran with (chosen on the device)
            N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
            res["crt_moduli"] = sum_r.value / max(nlaunch.value, 1)
            N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nlaunch), 1)
            res["crt_block_moduli"] = sum_r.value / nlaunch.value if nlaunch.value else None
        if rank == 0 and not args.skip_cpu and (world == 1 or m <= args.grm5_parity_max_sid):
            picks = grm5_picks(N, n, rank, P, g.nloc)
            got = {}
            for key, (b, r0, c0) in picks.items():
                blk = np.empty((256, 256), dtype=dt)
                N.call("snpmi_memcpy_d2h", N.ptr(blk), ctypes.c_void_p(out.snpmi_ptr.value + b * blk.nbytes),
                       blk.nbytes)
                got[key] = (blk, r0, c0)
            res["parity_sample"] = (got, g.stats())
    finally:
        g.close()
        del out
    if world > 1:  # every rank: the all-gather is collective
        res["gather_exact"] = grm5_gather_check(N, args, dist, P, fill)
    return res


def grm5_part_spread(n, P):
    """(largest - smallest) / smallest block count over the P parts of the plan."""
    from pysnptools_amd import _native as N

    c = [N.lib().snpmi_grm_part_blocks(n, r, P) for r in range(P)]
    return (max(c) - min(c)) / max(min(c), 1)


def grm5_gather_check(N, args, dist, P, fill):
    """N > 1: one more block through the same plan (each rank's share + all-gather, untimed); rank 0
    compares the rebuilt block with the block generated whole on its host."""
    return gather_check(N, dist, P, fill, args.grm5_iid, min(args.grm5_sid, args.grm5_block), args.grm5_block)


def gather_check(N, dist, P, fill, n, m, block):
    """One block of m SNPs x n iids through PartitionedGrm's share + all-gather plan; rank 0 returns
    whether the rebuilt block equals the block generated whole on its host (other ranks: None)."""
    from pysnptools_amd.shard import PartitionedGrm

    g = PartitionedGrm(n, m, N.STD_UNIT, dist=dist, part=dist.rank, parts=P, block=block, out="hbm",
                       first_block=m)  # one block: dev[0] holds all of it
    try:
        g.run(fill)
        if dist.rank != 0:
            return None
        whole = np.empty((m, g.pitch_src), dtype=np.uint8)
        fill(ctypes.c_void_p(whole.ctypes.data), 0, m)
        got = np.empty((m, g.pitch_src), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(got), g.dev[0].p, got.nbytes)
        return bool(np.array_equal(got, whole))
    finally:
        g.close()


def grm5_parity(args, picks, gpu_stats, threads):
    """Oracle (f64) for sample 256x256 blocks of the partitioned K over ALL the job's SNPs: each
    block of SNPs is regenerated on the host (the same generator the timed run used), its stats
    computed over every iid by the oracle (oracle_snp_stats, one-pass from code counts), only the
    sample blocks' iids decoded + standardized with those stats, and their products accumulated in
    f64.  Also: the GPU's per-SNP stats (f32) vs the oracle's, bit for bit."""
    from oracle import oracle as O
    from pysnptools_amd import _native as N

    n, m, B = args.grm5_iid, args.grm5_sid, args.grm5_block
    bpc = (n + 3) // 4
    pitch = bpc if bpc % 4 == 0 else N.lib().snpmi_packed_pitch(n)
    fill = grm5_source(N, n, pitch, args.seed + 200, args.grm5_miss, threads)
    sets = {}
    for key, (_, r0, c0) in picks.items():
        sets[key] = (np.arange(r0, min(r0 + 256, n)), np.arange(c0, min(c0 + 256, n)))
    acc = {key: np.zeros((len(rr), len(cc))) for key, (rr, cc) in sets.items()}
    buf = np.empty((B, pitch), dtype=np.uint8)
    stats_ok = True
    t0 = time.perf_counter()
    for s0 in range(0, m, B):
        cnt = min(B, m - s0)
        if (s0 // B) % 16 == 15:
            progress("grm5 parity block %d/%d" % (s0 // B + 1, (m + B - 1) // B))
        else:
            mark(None, "grm5 parity block %d" % (s0 // B + 1))
        fill(ctypes.c_void_p(buf.ctypes.data), s0, cnt)
        body = buf[:cnt] if pitch == bpc else np.ascontiguousarray(buf[:cnt, :bpc])
        body = body.reshape(-1)
        st = O.snp_stats(body, n, cnt)
        stats_ok &= bool(np.array_equal(st.astype(gpu_stats.dtype), gpu_stats[s0:s0 + cnt]))
        for key, (rr, cc) in sets.items():
            Zr = O.decode(body, n, cnt, iid_index=rr)
            O.standardize_native(Zr, use_stats=True, stats=st)
            if np.array_equal(rr, cc):
                acc[key] += Zr.dot(Zr.T)
            else:
                Zc = O.decode(body, n, cnt, iid_index=cc)
                O.standardize_native(Zc, use_stats=True, stats=st)
                acc[key] += Zr.dot(Zc.T)
    out, worst, diag_scale = [], 0.0, 1.0
    for key, (blk, r0, c0) in picks.items():
        if r0 == c0:
            diag_scale = max(diag_scale, float(np.abs(np.diag(acc[key])).max()))
    for key, (blk, r0, c0) in picks.items():
        ref = acc[key]
        err = float(np.abs(blk[:ref.shape[0], :ref.shape[1]].astype(np.float64) - ref).max())
        rel = err / diag_scale
        worst = max(worst, rel)
        out.append({"block": key, "row0": int(r0), "col0": int(c0), "max_abs_err": err,
                    "max_abs_err_over_max_diag": rel})
    f64 = gpu_stats.dtype == np.float64
    tol = 1e-12 if f64 else 1e-5
    return {"check": "part blocks (first diagonal, first off-diagonal, last) over all %d SNPs x %d iids: GPU %s "
                     "(%d-SNP blocks accumulated in HBM) vs oracle f64 (stats over every iid, products accumulated "
                     "per SNP block)" % (m, n, "f64 (int8 MFMA residues + CRT)" if f64 else "f32 (fp16x2 MFMA)", B),
            "blocks": out, "max_abs_err_over_max_diag": worst, "stats_bit_exact": stats_ok, "tolerance": tol,
            "oracle_seconds": time.perf_counter() - t0, "pass": worst <= tol and stats_ok}


def input_sha256(sample, n):
    """SHA-256 of the packed bytes of the sampled columns (pin the synthetic input)."""
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(sample[:, :(n + 3) // 4]).tobytes()).hexdigest()


PMC_PROFILE = "r06fin2"  # this round's PMC passes (tools/profile_r06.sh -> profiles/<PMC_PROFILE>/traffic.json)


def pmc_traffic(kernel, leg, n_iid, block):
    """Per-launch HBM bytes of ``kernel`` from this round's committed PMC summary
    (profiles/PMC_PROFILE/traffic.json), when that profile was taken at this configuration
    ([n_iid, block] of the leg); else None."""
    path = os.path.join(ROOT, "profiles", PMC_PROFILE, "traffic.json")
    try:
        d = json.load(open(path))
        e = d[kernel][leg]
        if d.get("_config", {}).get(leg) == [n_iid, block]:
            return e["traffic_bytes"]
    except Exception:
        pass
    return None


def grm_entry(args, dist, r, dtype):
    n, m = args.grm_iid, args.grm_sid
    gf = n * (n + 1) * m / r["wall"] / 1e9
    f32 = dtype == "f32"
    per_launch = {"launches_on_rank": r["launches"], "snps_per_launch": r["snps_per_launch"],
                  "mean_launch_ms": r["syrk_ms"] / max(r["launches"], 1)}
    if f32:
        peak = SPLIT_PEAK_TFLOPS
        roof = {"bound": "mfma", "achieved": r["mean_tflops"], "peak": peak, "unit": "TFLOP/s",
                "frac": r["mean_tflops"] / peak, "per_launch_flops": n * (n + 1) * r["snps_per_launch"],
                "traffic": pmc_traffic("f32w::k_syrk_h2s", "grm", n, r["snps_per_launch"]),
                "traffic_note": "PMC HBM bytes per launch (profiles/<PMC_PROFILE>/traffic.json) against ~10.8 GB "
                                "algorithmic at 50k x 62.5k, split (DESIGN.md 3.4): K tiles 5.0 GB read (accumulate) + 5.0 GB "
                                "written; SegFlush slots (256 KiB per workgroup, 19,306 workgroups, a flush every 12,288 SNPs = "
                                "5 rounds: one store, four rounds of f32 atomics, one read back) ~25 GB written + ~25 GB read "
                                "between L2 and the memory side (the 256 MiB slot pool sits in the MALL, which the TCC "
                                "counters see as HBM traffic); codes 0.8 GB + their panel re-fetches "
                                "~5 GB.  The flush machinery costs 1.6-3% of the launch's time (profiles/r05sc), the f32 "
                                "accuracy it buys is DESIGN.md 3.4's table",
                "traffic_split_gb": {"K_read": 5.0, "K_write": 5.0, "slots_write": 25.3, "slots_read": 25.3,
                                     "codes_and_panel_refetch": 6.0, "source": "PMC r05z and r06fin: read 36.1 GB, write 30.7 GB per launch"},
                "kernel": "f32w::k_syrk_h2s<false> (warp-specialised: 8 MFMA waves + 4 loader waves per 256x256 "
                          "block): f32 GRM as 3 fp16 MFMA products of each value's fp16x2 "
                          "split, f32 accumulate (v_mfma_f32_32x32x16_f16); peak = 2.5 PF fp16 dense / 3; the timed "
                          "span also holds k_snp_stats, k_lut_bf3, k_lut_h2 and the range-gated bf16x3 launch (exits "
                          "at once for Unit) of each launch",
                "f32_mfma_peak": MFMA_F32_PEAK_TFLOPS,
                "mfma_util_executed": r["mean_tflops"] * r["exec_ratio"] / MFMA_BF16_PEAK_TFLOPS}
    else:
        nb = (n + 255) // 256
        R = r.get("crt_block_moduli") or r["crt_moduli"] or CRT_MODULI
        ops = R * 2 * 256 * 256 * (nb * (nb + 1) // 2) * r["my_m"]  # executed int8 ops over the rank's span
        achieved = ops / (r["syrk_ms"] * 1e-3) / 1e12 if r["syrk_ms"] else 0.0
        roof = {"bound": "mfma", "achieved": achieved, "peak": MFMA_I8_PEAK_TOPS, "unit": "TOP/s",
                "frac": achieved / MFMA_I8_PEAK_TOPS,
                "per_launch_ops": R * 2 * 256 * 256 * (nb * (nb + 1) // 2) * r["snps_per_launch"], "traffic": None,
                "f64_equiv_tflops": r["mean_tflops"], "f64_mfma_peak": MFMA_F64_PEAK_TFLOPS,
                "vs_f64_mfma_peak": r["mean_tflops"] / MFMA_F64_PEAK_TFLOPS,
                "moduli_per_block": R, "moduli_launch_wide": r["crt_moduli"], "moduli_max": CRT_MODULI,
                "kernel": "k_syrk_i8w (warp-specialised: 8 MFMA waves + 4 loader waves; v_mfma_i32_32x32x32_i8; "
                          "grid = 256-blocks of a tile chunk x 15 moduli, those "
                          "past the block's R exit at once) + k_crt (Garner over R digits) + k_crt_exp/k_crt_lut/"
                          "k_crt_bound/k_crt_r; achieved = executed int8 ops (R moduli x full 256-blocks) / the whole "
                          "timed span"}
    roof.update(per_launch)
    coll = {"reduce": "ncclReduce(sum, root 0)", "allreduce": "ncclAllReduce(sum)"}.get(r["collective"])
    if coll and not dist.rccl:
        coll = "host-staged %s (rehearsal group)" % r["collective"]
    return {"workload": "cfg4: %d iid x %d SNP, Unit, %s SYRK; SNPs split into %d contiguous shard(s), each "
                        "accumulated through shard.ShardedGrm in launches of <= 65536 SNPs (the reference's block_size "
                        "%d bounds host memory, snpreader.py:651)%s"
                        % (n, m, "f32 (fp16x2 MFMA)" if f32 else "f64 (int8 MFMA residues + CRT)", dist.world,
                           args.grm_block, (", %s%s of the K tiles" % ("RCCL " if dist.rccl else "", coll))
                           if coll else ""),
            "gflops": gf, "snps_per_s": m / r["wall"], "seconds": r["wall"], "scaling": "strong",
            "collective": coll, "allreduce_ms": r["allreduce_ms"],
            "collective_alone": dict(r["unoverlapped"], note="each collective alone over the whole K-tile buffer, "
                                     "after the timed region (reduce = ncclReduce onto rank 0, the half-bytes form "
                                     "for one caller; allreduce = the timed exchange, here unoverlapped)")
            if r["unoverlapped"] else None,
            "collective_overlap": (("the last SYRK launch in %d column groups, each group's tiles summed on the aux "
                                    "stream under the next group's SYRK" % args.grm_overlap_parts) if f32 else
                                   "the CRT path's column-aligned residue chunks of the last launch, each chunk's f64 "
                                   "tiles summed on the aux stream under the next chunk")
            + "; allreduce_ms = the exposed tail after the last SYRK"
            if (coll and dist.rccl and (args.grm_overlap_parts > 1 or not f32)) else None,
            "trace_K": r["trace"], "roofline": roof}


# ---------------------------------------------------------------------------- leg 4: the reference's call path
def write_bed(N, path, n, m, seed, miss):
    """Synthetic .bed/.bim/.fam: packed columns generated on the GPU (SnpGen MAF curve), copied
    back and written as the SNP-major body (untimed; the file then sits in the page cache)."""
    pitch = N.lib().snpmi_packed_pitch(n)
    bpc = (n + 3) // 4
    step = max(1, min(m, (1 << 30) // pitch))
    dev = Dev(N, pitch * step)
    host = np.empty((step, pitch), dtype=np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        for s0 in range(0, m, step):
            cnt = min(step, m - s0)
            synth(N, dev.p, pitch, n, s0, cnt, seed, miss)
            N.call("snpmi_memcpy_d2h", N.ptr(host), dev.p, cnt * pitch)
            f.write(np.ascontiguousarray(host[:cnt, :bpc]).tobytes())
    dev.free()
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))


def leg_file(N, args):
    """Bed / SnpData / SnpKernel calls exactly as a PySnpTools user makes them, on a synthetic
    args.file_iid x args.file_sid .bed in local storage (21.8% missing, SnpGen's rate), each with
    parity against the oracle on a sample.  PCIe-inclusive; never `value`."""
    import shutil

    from oracle import oracle as O
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Beta, Unit

    n, m = args.file_iid, args.file_sid
    tmp = tempfile.mkdtemp(prefix="snpmi_file_", dir=args.file_dir)
    saved_xp = os.environ.get("ARRAY_MODULE")
    out = {"workload": "synthetic %d iid x %d SNP .bed (%.2f GB packed, SnpGen MAF curve, 21.8%% missing) in local "
                       "storage, read through the page cache" % (n, m, m * ((n + 3) // 4) / 1e9)}
    try:
        base = os.path.join(tmp, "cfg")
        t0 = time.perf_counter()
        write_bed(N, base, n, m, args.seed + 300, 0.218)
        out["write_s"] = time.perf_counter() - t0
        body = O.read_bed_bytes(base + ".bed")
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid  # metadata outside the timed regions
        flops = n * (n + 1) * m
        # (1) Bed.read_kernel(Unit(), float32): K in HBM (ARRAY_MODULE=hbm), then K copied to the host
        os.environ["ARRAY_MODULE"] = "hbm"
        bed[:, :2000].read_kernel(Unit(), dtype=np.float32)  # warm-up: scratch + session tiles
        t0 = time.perf_counter()
        Kd = bed.read_kernel(Unit(), dtype=np.float32)
        t_hbm = time.perf_counter() - t0  # the first full-size call (grows the chunk buffers)
        del Kd
        t0 = time.perf_counter()
        Kd = bed.read_kernel(Unit(), dtype=np.float32)
        t_hbm_warm = time.perf_counter() - t0
        rows = 8
        k_rows = np.empty((rows, n), dtype=np.float32)
        for r in range(rows):
            N.call("snpmi_memcpy_d2h", N.ptr(k_rows[r]), ctypes.c_void_p(Kd.val.ptr + r * n * 4), n * 4)
        del Kd
        os.environ.pop("ARRAY_MODULE")
        t0 = time.perf_counter()
        Kh = bed.read_kernel(Unit(), dtype=np.float32)
        t_host = time.perf_counter() - t0
        same_k = bool(np.array_equal(Kh.val[:rows], k_rows))
        del Kh
        # oracle: K rows 0..7 over every SNP, in 4096-SNP blocks (f64 one-pass Unit)
        ref = np.zeros((rows, n))
        for s0 in range(0, m, 4096):
            sid = np.arange(s0, min(m, s0 + 4096), dtype=np.uint64)
            Z, _ = O.decode_standardize(body, n, m, sid_index=sid, dtype=np.float64, num_threads=cpu_threads())
            ref += Z[:rows].dot(Z.T)
        err = float(np.abs(k_rows - ref).max() / np.abs(np.diag(ref[:, :rows])).max())
        out["read_kernel_f32"] = {
            "call": "Bed(path).read_kernel(Unit(), dtype=np.float32)", "reference": "snpreader.py:528-561,623-668",
            "seconds_K_in_hbm": t_hbm, "tflops_K_in_hbm": flops / t_hbm / 1e12,
            "seconds_K_in_hbm_warm": t_hbm_warm, "tflops_K_in_hbm_warm": flops / t_hbm_warm / 1e12,
            "seconds_K_to_host": t_host, "tflops_K_to_host": flops / t_host / 1e12, "K_GB": n * n * 4 / 1e9,
            "parity": {"check": "K rows 0..%d vs oracle f64 over all %d SNPs; host K == HBM K" % (rows - 1, m),
                       "max_abs_err_over_max_diag": err, "host_equals_hbm": same_k,
                       "pass": err <= 1e-5 and same_k}}
        # (1b) the same call in float64, the reference's default dtype (snpreader.py:528): int8 CRT SYRK
        os.environ["ARRAY_MODULE"] = "hbm"
        bed[:, :2000].read_kernel(Unit())  # warm-up: f64 scratch
        t0 = time.perf_counter()
        Kd = bed.read_kernel(Unit())
        t_hbm64 = time.perf_counter() - t0
        k64 = np.empty((rows, n), dtype=np.float64)
        for r in range(rows):
            N.call("snpmi_memcpy_d2h", N.ptr(k64[r]), ctypes.c_void_p(Kd.val.ptr + r * n * 8), n * 8)
        del Kd
        os.environ.pop("ARRAY_MODULE")
        err64 = float(np.abs(k64 - ref).max() / np.abs(np.diag(ref[:, :rows])).max())
        out["read_kernel_f64"] = {
            "call": "Bed(path).read_kernel(Unit())  # float64, the reference's default",
            "reference": "snpreader.py:528-561,623-668", "seconds_K_in_hbm": t_hbm64,
            "tflops_K_in_hbm": flops / t_hbm64 / 1e12, "K_GB": n * n * 8 / 1e9,
            "parity": {"check": "K rows 0..%d vs oracle f64 over all %d SNPs" % (rows - 1, m),
                       "max_abs_err_over_max_diag": err64, "pass": err64 <= 1e-12}}
        # (2) Bed[:, :10000].read(float32, xp='hbm')
        B = min(10_000, m)
        sub = bed[:, :B]
        sub.read(dtype=np.float32, xp="hbm")
        t0 = time.perf_counter()
        vd = sub.read(dtype=np.float32, xp="hbm")
        t_read = time.perf_counter() - t0
        cols = np.empty((64, n), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(cols), vd.val.snpmi_ptr, cols.nbytes)
        del vd
        refc = O.decode(body, n, m, sid_index=np.arange(64), dtype=np.float32)
        out["read_hbm"] = {
            "call": "Bed(path)[:, :%d].read(dtype=np.float32, xp='hbm')" % B, "reference": "bed.py:318-345",
            "seconds": t_read, "snps_per_s": B / t_read, "values_GB": n * B * 4 / 1e9,
            "packed_GBps": B * ((n + 3) // 4) / t_read / 1e9,
            "parity": {"check": "first 64 columns vs oracle decode", "bit_exact":
                       bool(np.array_equal(cols.T, refc, equal_nan=True))}}
        # (3) the configs[2] workload: read + Beta(1,25) standardize, values in HBM
        bed.read(dtype=np.float32, xp="hbm").standardize(Beta(1, 25))  # warm-up at full size
        t0 = time.perf_counter()
        sd = bed.read(dtype=np.float32, xp="hbm")
        t_rd = time.perf_counter() - t0
        sd.standardize(Beta(1, 25))
        t_all = time.perf_counter() - t0
        cols = np.empty((256, n), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(cols), sd.val.snpmi_ptr, cols.nbytes)
        del sd
        refb, _ = O.decode_standardize(body, n, m, sid_index=np.arange(256, dtype=np.uint64), is_beta=True, a=1.0,
                                       b=25.0, dtype=np.float32)
        rel = float(np.max(np.abs(cols.T.astype(np.float64) - refb) / np.maximum(np.abs(refb), 1e-30)))
        out["read_standardize_beta"] = {
            "call": "Bed(path).read(dtype=np.float32, xp='hbm').standardize(Beta(1, 25))",
            "reference": "bed.py:318-345, beta.py:33-50, standardizer.py:176-211",
            "seconds": t_all, "read_seconds": t_rd, "snps_per_s": m / t_all, "values_GB": n * m * 4 / 1e9,
            "parity": {"check": "first 256 columns vs oracle one-pass Beta(1,25) (f32)", "max_rel_err": rel,
                       "bit_exact": bool(np.array_equal(cols.T, refb)), "pass": rel <= 1e-5}}
        # (4) read + Unit standardize, values in HBM: the reference's two calls (the dense kernel
        # k_std_cols_f timed with HIP events on the library stream -> its roofline; round 3's kernel
        # beside it through the "std" hook), and the fused call its read().standardize() call sites
        # now make (_as_snpdata, SnpKernel.read_snps)
        from pysnptools_amd.snpreader.snpreader import _read_and_standardize

        ev = Events(N, 2)
        vals_gb = n * m * 4 / 1e9
        std_ms = {}
        for variant in (1, 0, 0):  # round 3's kernel, then the shipped one (warm, timed)
            sd = bed.read(dtype=np.float32, xp="hbm")
            N.call("snpmi_set_kernel_variant", b"std", variant)
            try:
                ev.record(0)
                sd.standardize(Unit())
                ev.record(1)
            finally:
                N.call("snpmi_set_kernel_variant", b"std", 0)
            std_ms[variant] = ev.ms(0, 1)
            if variant == 0:
                two = np.empty((256, n), dtype=np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(two), sd.val.snpmi_ptr, two.nbytes)
            del sd
        t0 = time.perf_counter()
        sd = bed.read(dtype=np.float32, xp="hbm")
        sd.standardize(Unit())
        t_two = time.perf_counter() - t0
        del sd
        os.environ["ARRAY_MODULE"] = "hbm"
        _read_and_standardize(bed, Unit(), "F", np.float32)  # warm-up
        t0 = time.perf_counter()
        one, _ = _read_and_standardize(bed, Unit(), "F", np.float32)
        t_one = time.perf_counter() - t0
        os.environ.pop("ARRAY_MODULE")
        fused = np.empty((256, n), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(fused), one.val.snpmi_ptr, fused.nbytes)
        del one
        ev.destroy()
        refu, _ = O.decode_standardize(body, n, m, sid_index=np.arange(256, dtype=np.uint64), dtype=np.float32)
        ach = 2 * vals_gb / (std_ms[0] * 1e-3)
        out["read_standardize_unit"] = {
            "call": "Bed(path).read(dtype=np.float32, xp='hbm').standardize(Unit())",
            "reference": "bed.py:318-345, unit.py:28-51, standardizer.py:90-133", "values_GB": vals_gb,
            "seconds_two_calls": t_two, "snps_per_s_two_calls": m / t_two,
            "standardize_ms": std_ms[0], "standardize_ms_round3_kernel": std_ms[1],
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("k_std_cols_f<float>", "std", n, m),
                         "traffic_source": "profiles/%s/traffic.json (tools/exp_std_dense.py, same shape)" % PMC_PROFILE,
                         "per_call_bytes": 2 * vals_gb * 1e9,
                         "kernel": "k_std_cols_f<float,1024,16,false>: one workgroup per column, the column held "
                                   "in registers between the stats and the table apply (read once, written once = "
                                   "2 x 4 B per value), plus the flag memset + 4-B readback of the call"},
            "fused_call": "_read_and_standardize(bed, Unit()) = what _as_snpdata / SnpKernel.read_snps run: "
                          "snpmi_bed_read_standardize_f32 (stats from code counts + table decode, values written once)",
            "seconds_fused": t_one, "snps_per_s_fused": m / t_one,
            "parity": {"check": "first 256 columns: two calls vs oracle decode + one-pass Unit (f32), fused vs two "
                                "calls", "bit_exact": bool(np.array_equal(two.T, refu)),
                       "fused_bit_exact": bool(np.array_equal(fused, two)),
                       "pass": bool(np.array_equal(two.T, refu)) and bool(np.array_equal(fused, two))}}
    finally:
        if saved_xp is None:
            os.environ.pop("ARRAY_MODULE", None)
        else:
            os.environ["ARRAY_MODULE"] = saved_xp
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def decode_entry(r, label):
    """The decode leg's roofline object (k_decode_f<float>, HBM bound)."""
    timed_tight = r["out_ld"] == r["tight"]
    side = {"achieved": r["side_gbs"], "frac": r["side_gbs"] / HBM_PEAK_GBS if r["side_gbs"] else None,
            "mean_launch_ms": r["side_ms"], "ld": r["side_ld"],
            "note": "the same kernel, %d full-block launches in the same process, into a block buffer with %s"
                    % (r["side_launches"], "tight columns (ld = round_up(n,16), what Bed.read(xp='hbm') writes)"
                       if not timed_tight else "a %d-float (%d MB) column pitch (the block spread over that many times "
                       "more HBM pages, DESIGN.md 3.1)" % (r["side_ld"], r["side_ld"] * 4 >> 20))}
    return {"bound": "hbm", "achieved": r["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": r["achieved_gbs"] / HBM_PEAK_GBS,
            "layout": "tight columns (ld = round_up(n,16), the library's read layout)" if timed_tight else
                      "column pitch %d floats" % r["out_ld"],
            "frac_tight": r["achieved_gbs"] / HBM_PEAK_GBS if timed_tight else side["frac"],
            "frac_spread": side["frac"] if timed_tight else r["achieved_gbs"] / HBM_PEAK_GBS,
            "side": side,
            "kernel": "k_decode_f<float> (after k_snp_stats%s)" % label,
            "per_launch_bytes": r["full_block_bytes"], "mean_launch_ms": r["dec_mean_ms"],
            "measured_stream_GBps": {"copy_16B_nt (1 read : 1 write)": r["copy_gbs"],
                                     "hipMemset fill (write only)": r["fill_gbs"]},
            "step": {"bytes": r["step_bytes"], "achieved": r["step_bytes"] * r["steps"] / r["wall"] / 1e9,
                     "frac": r["step_bytes"] * r["steps"] / r["wall"] / 1e9 / HBM_PEAK_GBS,
                     "note": "whole timed step (host wall): k_snp_stats read + decode read + write of every "
                             "column, launch gaps included"}}


def main(argv=None):
    global WD, RANK
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args, argv))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (one process per GPU)" % (args.gpus, world))
    if os.environ.get("SNPMI_BENCH_DRYRUN"):
        # launcher check without a GPU (tests/test_bench_launch.py): report the rank layout and stop
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                         "MASTER_PORT", "SNPMI_RCCL_ID_FILE")}), flush=True)
        return
    from pysnptools_amd import _native as N
    from pysnptools_amd import dist as D

    try:
        # not the "current" group: bench.py times its legs explicitly, and rank 0's file leg calls
        # Bed.read_kernel alone -- routed through the group it would wait in an all-reduce the other
        # ranks never join
        dist = D.init_from_env(force_rccl=args.force_rccl, timeout=args.dist_timeout, set_current=False)
    except TimeoutError as e:  # a stuck RCCL init cannot be cancelled: leave at once, non-zero
        sys.stderr.write("bench.py: %s\n" % e)
        sys.stderr.flush()
        os._exit(3)
    except Exception as e:
        # an RCCL init that FAILS (rather than hangs) on every rank: rather than no line at all, run
        # the job in the host group (host-staged sums and all-gathers, its own rendezvous file) and
        # say so in the line (config.rccl_init_error); a rank whose init succeeded meanwhile never
        # joins it, and the host group's bounded rendezvous ends the job as before
        if world <= 1 or os.environ.get("SNPMI_DIST_HOST"):
            raise
        RCCL_FALLBACK["error"] = "%s: %s" % (type(e).__name__, e)
        sys.stderr.write("bench.py: RCCL init failed (%s); running in the host group instead\n" % RCCL_FALLBACK["error"])
        sys.stderr.flush()
        env = dict(os.environ, SNPMI_DIST_HOST="1", SNPMI_RCCL_ID_FILE=D.id_file() + ".host")
        dist = D.init_from_env(timeout=args.dist_timeout, env=env, set_current=False)
    RANK = dist.rank
    if dist.world > 1 or dist.rccl:
        # a collective one rank never joins would block the others forever: bounded, diagnosed exit
        WD = D.Watchdog(dist, args.watchdog, on_fire=partial_line if dist.rank == 0 else None)
    try:
        run_legs(N, args, dist)
    except Exception as e:
        if WD is not None:  # dump, tell the other ranks (they are waiting in a collective), exit 4
            import traceback

            traceback.print_exc()
            WD.fail("%s on rank %d: %s" % (type(e).__name__, dist.rank, e))
        raise
    if WD is not None:
        WD.stop()
        if dist.rank == 0:
            WD.clear()
    dist.close()


def run_legs(N, args, dist):
    box = box_info(N, dist)
    selfcheck = None
    if args.selfcheck == "on":
        progress("selfcheck (group size, K-tile all-reduce, all-gather)", limit=min(args.watchdog, 180.0))
        selfcheck = leg_selfcheck(N, args, dist)
        PARTIAL["selfcheck"] = selfcheck
    progress("decode + Unit standardize (value)")
    r1 = leg_standardize(N, args, dist)
    value = args.n_sid * args.steps / r1["wall"]
    PARTIAL.update(value=value, n_gpus=dist.n_gpus, steps=args.steps, warmup=args.warmup,
                   ms_per_step=r1["wall"] / args.steps * 1e3, selfcheck=selfcheck, box=box)
    grm = grm64 = grm5 = dec_c = e2e = beta = filed = None
    if dist.rank == 0:
        progress("decode_c / e2e")
        dec_c = leg_decode_c(N, args)
        if args.e2e == "on":
            e2e = leg_e2e(N, args)
    dist.barrier()
    if args.beta == "on":
        progress("beta (configs[2])")
        rb = leg_standardize(N, args, dist, n=args.beta_iid, n_sid=args.beta_sid, std=N.STD_BETA, a=1.0, b=25.0,
                             miss=0.218, seed=args.seed + 3)
    if not args.skip_grm:
        progress("grm cfg4 f32 / f64")
        with ClockSampler(box) as clk:
            r2 = leg_grm(N, args, dist, "f32")
        grm = grm_entry(args, dist, r2, "f32")
        grm["sclk_mhz"] = clk.summary()
        PARTIAL["grm"] = grm
        if args.grm_f64 == "on":
            with ClockSampler(box) as clk:
                r2d = leg_grm(N, args, dist, "f64")
            grm64 = grm_entry(args, dist, r2d, "f64")
            grm64["sclk_mhz"] = clk.summary()
            PARTIAL["grm_f64"] = grm64
    if args.grm5 == "on":
        progress("grm5 cfg5 (part %d)" % dist.rank)
        with ClockSampler(box) as clk5:
            r3 = leg_grm5(N, args, dist)
        n5, m5, P = args.grm5_iid, r3["m"], r3["P"]
        flops_part = n5 * (n5 + 1) * m5 / P  # this part's share of the SYRK work
        busy_s = sum(r3["block_ms"]) * 1e-3
        syrk_tf = flops_part / busy_s / 1e12
        gather = (" + RCCL all-gather" if dist.rccl else
                  (" + host all-gather (rehearsal group)" if dist.world > 1 else ""))
        f64_5 = r3["dtype"] == np.float64
        if f64_5:  # the CRT path: executed int8 ops against the int8 peak, beside the f64-equivalent rate
            nloc5 = r3["n_local_blocks"]
            R5 = r3.get("crt_block_moduli") or r3.get("crt_moduli") or CRT_MODULI
            ops5 = R5 * 2 * 256 * 256 * nloc5 * m5
            roof5 = {"bound": "mfma", "achieved": ops5 / busy_s / 1e12, "peak": MFMA_I8_PEAK_TOPS, "unit": "TOP/s",
                     "frac": ops5 / busy_s / 1e12 / MFMA_I8_PEAK_TOPS, "traffic": None,
                     "f64_equiv_tflops": syrk_tf, "f64_mfma_peak": MFMA_F64_PEAK_TFLOPS, "moduli_per_block": R5,
                     "moduli_launch_wide": r3.get("crt_moduli"),
                     "kernel": "k_syrk_i8w in part mode (int8 residues of the quantised LUT, R moduli per block) + "
                               "k_crt into the part's f64 blocks; time = the blocks' compute-stream spans (stats + CRT "
                               "SYRK%s)" % (" + all-gather" if gather else "")}
        grm5 = {"workload": "cfg5: %d iid x %d SNP, Unit, %s, %.1f%% missing; K as 256x256 blocks in "
                            "%d parts (the 8-GPU plan), this process = part %d; all %d blocks (of %d SNPs, the first a quarter) timed: each "
                            "rank's 1/%d share generated on %d host threads into pinned memory, uploaded on the copy "
                            "stream under the previous block's SYRK%s, stats + SYRK into the part's blocks in HBM "
                            "(shard.PartitionedGrm); no reduction"
                            % (n5, m5, "f64 (int8 MFMA residues + CRT)" if f64_5 else "f32 (fp16x2 MFMA)",
                               100 * args.grm5_miss, P, dist.rank, r3["blocks"], args.grm5_block, dist.world,
                               r3["threads"], gather),
                "seconds": r3["wall"], "blocks": r3["blocks"], "gpu_busy_seconds": busy_s,
                "exposed_wait_seconds": max(0.0, r3["wall"] - busy_s),
                "block_ms_mean": float(np.mean(r3["block_ms"])), "block_ms_first": r3["block_ms"][0],
                "block_ms_max": float(np.max(r3["block_ms"])),
                "syrk_tflops": syrk_tf, "parts": P, "scaling": "strong",
                "job_note": "the P parts run concurrently on P GPUs at N = P, so `seconds` is the 8-GPU job time at "
                            "N = 8; at N < P it is one part's share of that job, measured whole (`part_*` rates; "
                            "`single_gpu_job_*_projected` = all P parts one after another on one GPU)",
                "blocks_on_rank0": r3["n_local_blocks"],
                "K_bytes_per_rank": r3["n_local_blocks"] * 256 * 256 * r3["dtype"].itemsize,
                "roofline": {"bound": "mfma", "achieved": syrk_tf, "peak": SPLIT_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": syrk_tf / SPLIT_PEAK_TFLOPS, "traffic": None,
                             "kernel": "f32w::k_syrk_h2s<true> (warp-specialised; fp16x2 split, 3 fp16 MFMA products, f32 "
                                       "accumulate), this part's blocks only; time = the blocks' compute-stream "
                                       "spans (stats + SYRK%s)" % (" + all-gather" if gather else "")}}
        if f64_5:
            grm5["roofline"] = roof5
            grm5["f64_equiv_tflops"] = grm5.pop("syrk_tflops")
        if dist.world >= P:  # every part runs: the job measured whole
            grm5.update({"gflops_per_gpu": flops_part / r3["wall"] / 1e9, "snps_per_s": m5 / r3["wall"]})
        else:
            grm5.update({"part_gflops": flops_part / r3["wall"] / 1e9, "part_snps_per_s": m5 / r3["wall"],
                         "single_gpu_job_seconds_projected": P * r3["wall"],
                         "single_gpu_job_snps_per_s_projected": m5 / (P * r3["wall"]),
                         "projection_note": "projection, not a measurement: part %d of %d measured whole, times %d "
                                            "(the parts are the same size within %.1f%%)"
                                            % (dist.rank, P, P, 100.0 * grm5_part_spread(n5, P))})
        if r3.get("parity_sample") is not None:
            grm5["parity"] = grm5_parity(args, r3["parity_sample"][0], r3["parity_sample"][1], r3["threads"])
        elif dist.rank == 0:
            grm5["parity"] = {"check": "skipped at N > 1 for %d SNPs (> --grm5-parity-max-sid): part 0 of the same "
                                       "8-part plan is checked over all SNPs at N = 1" % m5, "pass": True}
        if dist.rank == 0 and r3.get("gather_exact") is not None:
            grm5["parity"]["gathered_block_bit_exact"] = r3["gather_exact"]
            grm5["parity"]["pass"] = grm5["parity"]["pass"] and r3["gather_exact"]
        grm5["sclk_mhz"] = clk5.summary()
        PARTIAL["grm5"] = grm5
    if dist.rank == 0 and args.file == "on":
        progress("file leg")
        filed = leg_file(N, args)
    if dist.rank == 0:
        progress("cpu baselines + parity")
        cpu = parity = None
        if not args.skip_cpu and r1["sample"] is not None:
            ref, cpu = cpu_baseline_standardize(args, r1["sample"], timed=dist.world == 1)
            same = np.array_equal(r1["gpu_cols"][:, :args.n_iid].T, ref)
            parity = {"check": "first %d SNP columns x %d iids: GPU stats+decode vs oracle decode+one-pass "
                               "Unit (f32)" % (ref.shape[1], ref.shape[0]), "bit_exact": bool(same),
                      "input_sha256": input_sha256(r1["sample"], args.n_iid),
                      "input_hashed": "packed bytes (ceil(N/4) per column) of SNP columns 0..%d of the synthetic "
                                      "matrix (counter-based generator, seed %d)" % (len(r1["sample"]) - 1, args.seed)}
            if grm is not None:
                grm["cpu_baseline"] = cpu_baseline_grm(args, "f32") if dist.world == 1 else None
                if r2.get("parity_sample") is not None:
                    grm["parity"] = grm_parity(args, *r2["parity_sample"], tol=1e-5)
            if grm64 is not None:
                grm64["cpu_baseline"] = cpu_baseline_grm(args, "f64") if dist.world == 1 else None
                if r2d.get("parity_sample") is not None:
                    grm64["parity"] = grm_parity(args, *r2d["parity_sample"], tol=1e-10)
        if args.beta == "on":
            nb_, mb_ = args.beta_iid, args.beta_sid
            beta = {"workload": "configs[2]: Beta(1,25) standardize + NaN impute of the %d iid x %d SNP matrix "
                                "(packed resident in HBM, SnpGen MAF curve, 21.8%% missing), %d contiguous shard(s), "
                                "block %d SNPs, f32 F-order" % (nb_, mb_, dist.world, args.block),
                    "snps_per_s": mb_ * args.steps / rb["wall"], "seconds_per_pass": rb["wall"] / args.steps,
                    "block_buffer_ld": rb["out_ld"], "roofline": decode_entry(rb, ", Beta(1,25) LUT")}
            if not args.skip_cpu and rb["sample"] is not None:
                refb, cpub = cpu_baseline_standardize(args, rb["sample"], timed=dist.world == 1, n=nb_, is_beta=True,
                                                      a=1.0, b=25.0)
                got = rb["gpu_cols"][:, :nb_].T.astype(np.float64)
                rel = float(np.max(np.abs(got - refb) / np.maximum(np.abs(refb), 1e-30)))
                beta["parity"] = {"check": "first %d SNP columns x %d iids: GPU vs oracle one-pass Beta(1,25) (f32)"
                                           % (refb.shape[1], nb_), "max_rel_err": rel,
                                  "input_sha256": input_sha256(rb["sample"], nb_),
                                  "bit_exact": bool(np.array_equal(rb["gpu_cols"][:, :nb_].T, refb)),
                                  "pass": rel <= 1e-5}
                beta["cpu_baseline"] = cpub
        n = args.n_iid
        line = {
            "metric": METRIC, "value": value, "unit": "SNPs/s", "n_gpus": dist.n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": r1["wall"] / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "decode+Unit standardize of the %d iid x %d SNP matrix (packed BED resident in "
                                   "HBM, SnpGen MAF curve, 1%% missing), SNPs split into %d contiguous shard(s), "
                                   "block %d SNPs, f32 F-order block buffer with a %d-float column pitch"
                                   % (n, args.n_sid, dist.world, args.block, r1["out_ld"]),
                       "n_iid": n, "n_sid": args.n_sid, "n_sid_per_gpu": r1["m"], "block": args.block,
                       "block_buffer_ld": r1["out_ld"],
                       "parallelism": "snp-shard x%d" % dist.world,
                       "process_group": "rccl" if dist.rccl else ("host rehearsal (SNPMI_DIST_HOST: socket barriers, "
                                                                  "ranks share one GPU, host-staged sums and "
                                                                  "all-gathers)" if dist.world > 1 else "none"),
                       **({"rccl_init_error": RCCL_FALLBACK["error"],
                           "process_group_note": "RCCL init failed on every rank: the host group carried this "
                                                 "run's collectives (host-staged, not xGMI)"}
                          if RCCL_FALLBACK else {})},
            "weak": ({"value": args.n_sid * args.steps * dist.world / r1["weak_wall"], "unit": "SNPs/s",
                      "workload": "every rank streams 1M SNPs per step (its shard %d times)" % dist.world}
                     if r1["weak_wall"] else None),
            "roofline": dict(decode_entry(r1, ""), traffic=pmc_traffic("k_decode_f<float>", "dec", n, args.block)),
            "cpu_baseline": cpu,
            "parity": parity,
            "decode_c": dec_c,
            "e2e": e2e,
            "beta": beta,
            "grm": grm,
            "grm_f64": grm64,
            "grm5": grm5,
            "file": filed,
            "selfcheck": selfcheck,
            "box": dict(box, fill_GBps=r1["fill_gbs"], copy_GBps=r1["copy_gbs"],
                        note="the box this line was measured on: device ids, the hipMemset fill and 1:1 copy ceilings "
                             "measured in this process (decode leg buffers), and the SCLK sampled from sysfs during "
                             "each GRM leg (grm*.sclk_mhz) -- compare runs on different boxes against these"),
        }
        if args.hook or args.decode_variant:  # an A/B run, not the default configuration
            line["config"]["ab_hooks"] = list(args.hook) + (["decode=%d" % args.decode_variant] if args.decode_variant else [])
        print(json.dumps(line), flush=True)
        PARTIAL["_printed"] = True
    # every rank leaves together (rank 0 ran the CPU baselines and the file leg alone)
    progress("final barrier", limit=args.watchdog_final)
    dist.barrier()


if __name__ == "__main__":
    main()
