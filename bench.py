"""Benchmark of the BED decode -> standardize -> GRM hot path on MI355X.

Metric (BASELINE.json): "SNPs/sec standardized (500k x 1M) + GRM GF/s at 1/2/4/8 GPUs".

  value      = SNPs/s standardized, whole job: every rank decodes + Unit-standardizes its own
               synthetic 500k-iid x 1M-SNP BED matrix (the UKBB shape of configs[4]), resident in
               HBM as packed 2-bit codes, in blocks of 2048 SNPs into an f32 F-order block buffer
               (weak scaling: per-GPU work fixed).  A step = one pass over the 1M SNPs.
  roofline   = the decode kernel (k_decode_f<float>), HBM bound: algorithmic bytes per launch =
               block * (ceil(N/4) + 4N) / its mean HIP-event duration, vs 8.0 TB/s.
  grm        = SnpKernel GRM of configs[3] (50k iid x 500k SNP, Unit, block 10k, f32): SNP blocks
               round-robin over ranks, one RCCL all-reduce of the upper-triangle K tiles.  The f32
               products run on the fp16 MFMA pipe as 3 fp16 products of each value's fp16x2 split
               (f32-level accuracy, f32 accumulate; bf16x3 = 6 bf16 products when a SNP's LUT is
               outside fp16's range).  gflops uses N(N+1)M (SYRK work); roofline
               vs 2.5 PF fp16 dense / 3 = 833.3 TF (the f32-MFMA peak is 157.3).
  cpu_baseline = the oracle's C/OpenMP decode + one-pass Unit standardize (the CPU restatement
               of bed-reader's read + standardize_f32) on a sample of the same packed columns,
               rank 0 only; grm.cpu_baseline = NumPy/OpenBLAS Z.dot(Z.T) (snpreader.py:655).

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import contextlib
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SNPs/sec standardized (500k×1M) + GRM GF/s at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0
MFMA_F32_PEAK_TFLOPS = 157.3
MFMA_BF16_PEAK_TFLOPS = 2500.0
# f32 GRM on the fp16 MFMA pipe (same dense rate as bf16): each f32 product = 3 fp16 MFMA
# products of the fp16x2 split (k_syrk_h2; Unit LUTs always fit fp16's range)
SPLIT_PRODUCTS = 3
SPLIT_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS


def parse():
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
    p.add_argument("--grm5", choices=["auto", "on", "off"], default="auto",
                   help="cfg5 tile-partitioned GRM leg (auto: when WORLD_SIZE >= 4)")
    p.add_argument("--grm5-iid", type=int, default=500_000)
    p.add_argument("--grm5-sid", type=int, default=8192)
    p.add_argument("--skip-cpu", action="store_true")
    p.add_argument("--fused", choices=["on", "off"], default="off",
                   help="decode leg: fused stats+decode kernel k_decode_std_lds_f32 (needs a packed column <= "
                        "150 KiB); off = k_snp_stats + k_decode_f, measured faster at 500k iids (2.63 vs 2.40 M SNPs/s)")
    p.add_argument("--decode-variant", type=int, default=0, help="snpmi_set_kernel_variant('decode', v) (A/B runs)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--seed", type=int, default=5)
    p.add_argument("--force-rccl", action="store_true", help="build the RCCL communicator even at world size 1")
    return p.parse_args()


@contextlib.contextmanager
def stdout_to_stderr():
    """RCCL prints a version banner on the C stdout (fd 1) around communicator setup; the bench's
    stdout must carry only its one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


class Dist:
    """Control plane for one process per GPU WITHOUT torch: importing torch would load its own
    libamdhip64.so.7 (ROCm 7.0) next to libsnpmi's (ROCm 7.2) -- same SONAME, two runtimes.
    torch.distributed.run only launches the processes; the ncclUniqueId is handed from rank 0
    to the others through a node-local file keyed by the launcher's pid, and barriers /
    max-over-ranks are RCCL all-reduces of a scalar."""

    def __init__(self, gpus, N, force_rccl=False):
        self.N = N
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        assert self.world == gpus or self.world == 1, "--gpus must match WORLD_SIZE"
        N.call("snpmi_set_device", self.local_rank)
        self.rccl = False
        if self.world > 1 or force_rccl:
            import tempfile

            key = "snpmi_rccl_%d_%s.id" % (os.getppid(), os.environ.get("MASTER_PORT", "0"))
            path = os.path.join(tempfile.gettempdir(), key)
            uid = (ctypes.c_uint8 * 128)()
            if self.rank == 0:
                with stdout_to_stderr():
                    N.call("snpmi_rccl_unique_id", uid, 128)
                with open(path + ".tmp", "wb") as f:
                    f.write(bytes(uid))
                os.replace(path + ".tmp", path)
            else:
                t0 = time.time()
                while not os.path.exists(path):
                    if time.time() - t0 > 300:
                        raise TimeoutError("rank %d: no RCCL id from rank 0 at %s" % (self.rank, path))
                    time.sleep(0.05)
                with open(path, "rb") as f:
                    uid = (ctypes.c_uint8 * 128).from_buffer_copy(f.read(128))
            with stdout_to_stderr():
                N.call("snpmi_rccl_init", self.world, self.rank, uid, 128)
            self.rccl = True
            self.barrier()
            if self.rank == 0:
                os.remove(path)

    def barrier(self):
        if self.rccl:
            self.N.call("snpmi_rccl_barrier")

    def max(self, x):
        if not self.rccl:
            return x
        v = (ctypes.c_double * 1)(float(x))
        self.N.call("snpmi_rccl_host_allreduce_f64", v, 1, 1)
        return float(v[0])

    def close(self):
        if self.rccl:
            with stdout_to_stderr():
                self.N.call("snpmi_rccl_destroy")


class Dev:
    def __init__(self, N, nbytes):
        self.N = N
        self.p = ctypes.c_void_p()
        N.call("snpmi_dev_alloc", ctypes.byref(self.p), int(nbytes))

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

    def record(self, i):
        self.N.call("snpmi_event_record", self.ev[i])

    def ms(self, a, b):
        out = ctypes.c_float()
        self.N.call("snpmi_event_elapsed_ms", self.ev[a], self.ev[b], ctypes.byref(out))
        return float(out.value)

    def destroy(self):
        for e in self.ev:
            self.N.call("snpmi_event_destroy", e)


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


# ---------------------------------------------------------------------------- leg 1: decode + standardize
def use_fused(args, n):
    """k_decode_std_lds_f32 holds one packed column in LDS: up to 150 KiB (N <= 614,400)."""
    if args.fused != "on":
        return False
    return ((n + 63) // 64) * 16 <= 150 * 1024
def leg_standardize(N, args, dist):
    n, m, B = args.n_iid, args.n_sid, args.block
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, dist.rank * m, m, args.seed, 0.01)
    nblk = (m + B - 1) // B
    lut, stats, out = Dev(N, B * 16), Dev(N, B * 8), Dev(N, B * ld * 4)
    ev = Events(N, 2 + 2 * nblk)
    fused = use_fused(args, n)
    N.call("snpmi_set_kernel_variant", b"decode", args.decode_variant)

    def run_block(src, cnt, timed, k):
        if fused:  # stats + decode in one kernel (column staged in LDS, packed bytes read once)
            if timed:
                ev.record(2 + 2 * k)
            N.call("snpmi_dev_decode_standardize", src, pitch, n, cnt, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
                   stats.p, lut.p, out.p, ld)
        else:
            N.call("snpmi_dev_snp_stats", src, pitch, n, cnt, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
            if timed:
                ev.record(2 + 2 * k)
            N.call("snpmi_dev_decode", src, pitch, n, cnt, lut.p, N.DT_F32, 0, out.p, ld)
        if timed:
            ev.record(3 + 2 * k)

    def step(timed):
        dec_ms = 0.0
        if timed:
            ev.record(0)
        for k in range(nblk):
            s0 = k * B
            cnt = min(B, m - s0)
            run_block(ctypes.c_void_p(packed.p.value + s0 * pitch), cnt, timed, k)
        if timed:
            ev.record(1)
        N.call("snpmi_stream_sync")
        if timed:
            dec_ms = sum(ev.ms(2 + 2 * k, 3 + 2 * k) for k in range(nblk))
        return dec_ms

    for _ in range(args.warmup):
        step(False)
    dist.barrier()
    N.call("snpmi_stream_sync")
    t0 = time.perf_counter()
    dec_ms_total = 0.0
    step_ms = []
    for _ in range(args.steps):
        dec_ms_total += step(True)
        step_ms.append(ev.ms(0, 1))
    N.call("snpmi_stream_sync")
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    launches = args.steps * nblk
    dec_mean_ms = dec_ms_total / launches
    full_block_bytes = B * ((n + 3) // 4 + 4 * n)
    total_bytes = m * ((n + 3) // 4 + 4 * n)
    achieved_gbs = (total_bytes / nblk) / (dec_mean_ms * 1e-3) / 1e9
    # measured copy peak (untimed): device-to-device copies of the block buffer's size
    cbytes = min(B * ld * 4, pitch * m)
    N.call("snpmi_dev_memcpy_d2d", out.p, packed.p, cbytes)
    N.call("snpmi_stream_sync")
    ev.record(0)
    for _ in range(5):
        N.call("snpmi_dev_memcpy_d2d", out.p, packed.p, cbytes)
    ev.record(1)
    N.call("snpmi_stream_sync")
    copy_gbs = 2 * 5 * cbytes / (ev.ms(0, 1) * 1e-3) / 1e9
    # write-only stream (the decode writes 16 B per 1 B it reads): hipMemset fill of the buffer
    ev.record(0)
    for _ in range(5):
        N.call("snpmi_dev_memset", out.p, 0, B * ld * 4)
    ev.record(1)
    N.call("snpmi_stream_sync")
    fill_gbs = 5 * B * ld * 4 / (ev.ms(0, 1) * 1e-3) / 1e9
    sample = gpu_cols = None
    if dist.rank == 0 and not args.skip_cpu:
        # parity sample: the first 512 columns, re-decoded by the same kernels (untimed)
        ncols = min(512, m)
        sample = np.empty((ncols, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
        run_block(packed.p, ncols, False, 0)
        gpu_cols = np.empty((ncols, ld), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(gpu_cols), out.p, gpu_cols.nbytes)
    res = dict(wall=wall, step_ms=step_ms, dec_mean_ms=dec_mean_ms, achieved_gbs=achieved_gbs, fused=fused,
               copy_gbs=copy_gbs, fill_gbs=fill_gbs,
               full_block_bytes=full_block_bytes, launches=launches, nblk=nblk, pitch=pitch, sample=sample,
               gpu_cols=gpu_cols)
    ev.destroy()
    for d in (packed, lut, stats, out):
        d.free()
    return res


def cpu_baseline_standardize(args, sample, pitch, timed=True):
    """Oracle C/OpenMP decode + one-pass Unit standardize on a bounded sample (rank 0); with
    timed=False (N > 1: the baseline is reported at N = 1 only) one untimed pass for parity."""
    from oracle import oracle as O

    n = args.n_iid
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    bpc = (n + 3) // 4
    body = np.ascontiguousarray(sample[:, :bpc]).reshape(-1)
    ncols = sample.shape[0]
    if not timed:
        ref, _ = O.decode_standardize(body, n, ncols, dtype=np.float32, num_threads=threads)
        return ref, None
    done, t0 = 0, time.perf_counter()
    while True:
        ref, _ = O.decode_standardize(body, n, ncols, dtype=np.float32, num_threads=threads)
        done += ncols
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or done >= 64 * ncols:
            break
    return ref, {"value": done / el, "unit": "SNPs/s", "cores": threads, "kind": "port",
            "sample": "%d reps x %d SNP columns x %d iids (first packed columns of the same synthetic matrix), "
                      "f32 Unit, oracle/bed_oracle.c oracle_decode_standardize_f32, %.1f s" % (done // ncols, ncols, n, el)}


# ---------------------------------------------------------------------------- leg 2: GRM
def leg_grm(N, args, dist, rccl):
    n, m, B = args.grm_iid, args.grm_sid, args.grm_block
    pitch = N.lib().snpmi_packed_pitch(n)
    from pysnptools_amd.shard import rank_span_blocks, snp_blocks

    blocks = snp_blocks(m, B)
    mine = rank_span_blocks(m, B, dist.rank, dist.world)
    my_m = sum(c for _, c in mine)
    packed = Dev(N, max(1, my_m) * pitch)
    off = 0
    for s0, c in mine:  # generate exactly the global SNP ids this rank owns
        synth(N, ctypes.c_void_p(packed.p.value + off * pitch), pitch, n, s0, c, args.seed + 100, 0.01)
        off += c
    tile_bytes = N.lib().snpmi_grm_tile_bytes(n, N.DT_F32)
    tiles = Dev(N, tile_bytes)
    lut, stats = Dev(N, B * 16), Dev(N, B * 8)
    ev = Events(N, 2 + 2 * max(1, len(mine)) + 2)

    def run(timed, limit=None):
        off = 0
        todo = mine if limit is None else mine[:limit]
        if not todo:
            N.call("snpmi_dev_memset", tiles.p, 0, tile_bytes)
        for k, (s0, c) in enumerate(todo):
            src = ctypes.c_void_p(packed.p.value + off * pitch)
            N.call("snpmi_dev_snp_stats", src, pitch, n, c, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
            if timed:
                ev.record(2 + 2 * k)
            N.call("snpmi_dev_syrk_packed", src, pitch, n, c, lut.p, N.DT_F32, tiles.p, int(k > 0))
            if timed:
                ev.record(3 + 2 * k)
            off += c
        if rccl and timed:
            ev.record(len(ev.ev) - 2)
            N.call("snpmi_rccl_allreduce_sum", tiles.p, tile_bytes // 4, N.DT_F32)
            ev.record(len(ev.ev) - 1)
        N.call("snpmi_stream_sync")

    run(False, limit=1)  # warm-up: one block
    dist.barrier()
    t0 = time.perf_counter()
    run(True)
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    syrk_ms = [ev.ms(2 + 2 * k, 3 + 2 * k) for k in range(len(mine))]
    allreduce_ms = ev.ms(len(ev.ev) - 2, len(ev.ev) - 1) if rccl else 0.0
    # spot parity at scale: diag(K) == sum over SNPs of z^2 == count of polymorphic SNPs-ish is
    # not exact; instead check symmetry-free invariant: trace(K) = sum_j n_obs_j (Unit: sum z^2 = n_obs)
    tr = ctypes.c_double()
    N.call("snpmi_dev_grm_trace", tiles.p, n, N.DT_F32, ctypes.byref(tr))
    flops_full_block = n * (n + 1) * B
    nb = (n + 255) // 256
    exec_ratio = SPLIT_PRODUCTS * 2 * 256 * 256 * (nb * (nb + 1) // 2) / (n * (n + 1))  # executed bf16 / algorithmic
    res = dict(wall=wall, syrk_ms=syrk_ms, allreduce_ms=allreduce_ms, trace=tr.value, exec_ratio=exec_ratio,
               # throughput over this rank's launches (the last block of a shard can be partial)
               mean_tflops=(n * (n + 1) * my_m / (np.sum(syrk_ms) * 1e-3) / 1e12) if syrk_ms else 0.0,
               nblocks=len(blocks))
    if dist.rank == 0 and not args.skip_cpu and my_m > 0:
        # parity sample (untimed): K rows 0..63 of the GRM of this rank's first 512 SNPs
        cm, rows = min(512, my_m), 64
        N.call("snpmi_dev_snp_stats", packed.p, pitch, n, cm, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
        N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, cm, lut.p, N.DT_F32, tiles.p, 0)
        ri = np.arange(rows, dtype=np.uint64)
        dri, dout = Dev(N, rows * 8), Dev(N, rows * n * 4)
        N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
        N.call("snpmi_dev_grm_extract", tiles.p, n, N.DT_F32, dri.p, rows, None, n, 1, 1.0, dout.p)
        krows = np.empty((rows, n), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(krows), dout.p, krows.nbytes)
        sample = np.empty((cm, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
        res["parity_sample"] = (krows, sample, cm, (mine[0][0] if mine else 0))
        dri.free()
        dout.free()
    ev.destroy()
    for d in (packed, tiles, lut, stats):
        d.free()
    return res


# ---------------------------------------------------------------------------- leg 3: cfg5 partitioned GRM
def leg_grm5(N, args, dist):
    """configs[4] shape: 500k iids, K (500 GB upper triangle f32)
    partitioned over ranks as 256x256 blocks.  Per SNP block each rank uploads ITS 1/p of the
    packed columns from pinned host memory, ncclAllGather rebuilds the packed block on every
    rank, then stats + the fused SYRK fill only the rank's own K blocks -- no reduction.
    One timed block of --grm5-sid SNPs (GRM time is linear in M)."""
    n, p = args.grm5_iid, dist.world
    m = (args.grm5_sid + p - 1) // p * p
    ms = m // p
    pitch = N.lib().snpmi_packed_pitch(n)
    nloc = N.lib().snpmi_grm_part_blocks(n, dist.rank, p)
    packed = Dev(N, pitch * m)
    mine = packed.p.value + dist.rank * ms * pitch
    # the rank's shard of the .bed, staged in page-locked memory (untimed, like reading the file)
    host = ctypes.c_void_p()
    N.call("snpmi_host_alloc", ctypes.byref(host), ms * pitch)
    synth(N, mine, pitch, n, dist.rank * ms, ms, args.seed + 200, 0.01)
    N.call("snpmi_memcpy_d2h", host, mine, ms * pitch)
    N.call("snpmi_dev_memset", packed.p, 0, pitch * m)
    lut, stats = Dev(N, m * 16), Dev(N, m * 8)
    blocks = Dev(N, max(nloc, 1) * 256 * 256 * 4)
    ev = Events(N, 4)
    N.call("snpmi_stream_sync")
    dist.barrier()
    t0 = time.perf_counter()
    ev.record(0)
    N.call("snpmi_memcpy_h2d", mine, host, ms * pitch)
    ev.record(1)
    if dist.rccl:
        N.call("snpmi_rccl_allgather", mine, packed.p, ms * pitch)
    ev.record(2)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, dist.rank, p, blocks.p, 0)
    ev.record(3)
    N.call("snpmi_stream_sync")
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    res = {"wall": wall, "h2d_ms": ev.ms(0, 1), "allgather_ms": ev.ms(1, 2), "syrk_ms": ev.ms(2, 3),
           "n_local_blocks": nloc, "m": m}
    if dist.rank == 0 and not args.skip_cpu and nloc > 0:
        r0, c0 = ctypes.c_uint64(), ctypes.c_uint64()
        N.call("snpmi_grm_part_coords", n, 0, p, 0, ctypes.byref(r0), ctypes.byref(c0))
        blk = np.empty((256, 256), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(blk), blocks.p, blk.nbytes)
        sample = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
        # the gathered block must equal the whole block generated in one piece
        synth(N, packed.p, pitch, n, 0, m, args.seed + 200, 0.01)
        whole = np.empty_like(sample)
        N.call("snpmi_memcpy_d2h", N.ptr(whole), packed.p, whole.nbytes)
        res["gather_exact"] = bool(np.array_equal(sample, whole))
        del whole
        res["parity_sample"] = (blk, sample, r0.value, c0.value)
    ev.destroy()
    N.call("snpmi_host_free", host)
    for d in (packed, lut, stats, blocks):
        d.free()
    return res


def grm5_parity(args, m, blk, sample, row0, col0):
    """Oracle (f64) for one 256x256 block of the partitioned K: decode only its 512 iids."""
    from oracle import oracle as O

    n = args.grm5_iid
    bpc = (n + 3) // 4
    body = np.ascontiguousarray(sample[:, :bpc]).reshape(-1)
    rows = np.arange(row0, min(row0 + 256, n))
    cols = np.arange(col0, min(col0 + 256, n))
    # stats use every iid; the block needs only its rows/cols
    full_stats = O.snp_stats(body, n, m)
    Zr = O.decode(body, n, m, iid_index=rows)
    Zc = O.decode(body, n, m, iid_index=cols)
    O.standardize_native(Zr, use_stats=True, stats=full_stats)
    O.standardize_native(Zc, use_stats=True, stats=full_stats)
    ref = Zr.dot(Zc.T)
    scale = max(np.abs(np.diag(ref)).max() if row0 == col0 else np.abs(ref).max(), 1.0)
    err = float(np.abs(blk[:len(rows), :len(cols)].astype(np.float64) - ref).max() / scale)
    return {"check": "rank 0 block 0 (rows %d.., cols %d..) over %d SNPs x %d iids: GPU f32 vs oracle f64"
                     % (row0, col0, m, n), "max_abs_err_over_scale": err, "pass": err <= 1e-5}


def cpu_baseline_grm(args):
    """NumPy Z.dot(Z.T) (OpenBLAS syrk, the reference's snpdata.py:203-206 / snpreader.py:655)."""
    n, b = 10_000, 2048
    rng = np.random.default_rng(0)
    Z = rng.standard_normal((n, b)).astype(np.float32)
    t0 = time.perf_counter()
    reps = 0
    while True:
        Z.dot(Z.T)
        reps += 1
        el = time.perf_counter() - t0
        if el > 4.0 or reps >= 8:
            break
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    return {"value": reps * n * (n + 1) * b / el / 1e9, "unit": "GF/s", "cores": threads, "kind": "port",
            "sample": "%d x Z.dot(Z.T), Z = %d x %d f32 (NumPy/OpenBLAS), %.1f s" % (reps, n, b, el)}


def grm_parity(args, krows, sample, cm, sid0):
    """Oracle (f64, reference one-pass Unit + NumPy Z Z^T) vs the GPU's f32 K rows."""
    from oracle import oracle as O

    n = args.grm_iid
    bpc = (n + 3) // 4
    Z = O.decode(np.ascontiguousarray(sample[:, :bpc]).reshape(-1), n, cm, dtype=np.float64)
    O.standardize_native(Z)
    rows = krows.shape[0]
    ref = Z[:rows].dot(Z.T)
    scale = np.abs(np.diag(ref[:, :rows])).max()
    err = float(np.abs(krows.astype(np.float64) - ref).max() / scale)
    return {"check": "K rows 0..%d over %d SNPs (first of this rank's blocks), %d iids: GPU f32 MFMA vs oracle f64"
                     % (rows - 1, cm, n), "max_abs_err_over_max_diag": err, "pass": err <= 1e-5}


def pmc_traffic(kernel, leg, n_iid, block):
    """Per-launch HBM bytes of ``kernel`` from the committed PMC summary, when its profile was
    taken at this configuration (tools/profile.sh + tools/traffic_summary.py); else None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))
        e = d[kernel][leg]
        if d.get("_config", {}).get(leg) == [n_iid, block]:
            return e["traffic_bytes"]
    except Exception:
        pass
    return None


def main():
    args = parse()
    from pysnptools_amd import _native as N

    dist = Dist(args.gpus, N, args.force_rccl)
    rccl = dist.rccl

    r1 = leg_standardize(N, args, dist)
    total_snps = args.n_sid * dist.world * args.steps
    value = total_snps / r1["wall"]
    grm = None
    if not args.skip_grm:
        r2 = leg_grm(N, args, dist, rccl)
        n, m = args.grm_iid, args.grm_sid
        gf = n * (n + 1) * m / r2["wall"] / 1e9
        grm = {"workload": "cfg4: %d iid x %d SNP, Unit, block %d, f32 (fp16x2 MFMA) SYRK, SNPs split into %d equal "
                           "contiguous shard(s) streamed in blocks%s" % (n, m, args.grm_block, dist.world,
                                                                         ", RCCL all-reduce of K tiles" if rccl else ""),
               "gflops": gf, "snps_per_s": m / r2["wall"], "seconds": r2["wall"], "scaling": "strong",
               "allreduce_ms": r2["allreduce_ms"], "trace_K": r2["trace"],
               "roofline": {"bound": "mfma", "achieved": r2["mean_tflops"], "peak": SPLIT_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": r2["mean_tflops"] / SPLIT_PEAK_TFLOPS,
                            "traffic": pmc_traffic("f32w::k_syrk_h2", "grm", n, args.grm_block),
                            "kernel": "f32w::k_syrk_h2<false,4>: f32 GRM as 3 fp16 MFMA products of each "
                                      "value's fp16x2 split, f32 accumulate (v_mfma_f32_32x32x16_f16); "
                                      "peak = 2.5 PF fp16 dense / 3; time per block includes k_lut_bf3, "
                                      "k_lut_h2 and the range-gated bf16x3 launch (exits at once for Unit)",
                            "per_launch_flops": n * (n + 1) * args.grm_block,
                            "f32_mfma_peak": MFMA_F32_PEAK_TFLOPS,
                            "mfma_util_executed": r2["mean_tflops"] * r2["exec_ratio"] / MFMA_BF16_PEAK_TFLOPS,
                            "bf16x3_peak": MFMA_BF16_PEAK_TFLOPS / 6}}
    grm5 = None
    run5 = args.grm5 == "on" or (args.grm5 == "auto" and dist.world >= 4 and not args.skip_grm)
    if run5:
        r3 = leg_grm5(N, args, dist)
        n5, m5 = args.grm5_iid, r3["m"]
        gf5 = n5 * (n5 + 1) * m5 / r3["wall"] / 1e9
        grm5 = {"workload": "cfg5: %d iid x %d SNP (one block of the 1M), Unit, f32 MFMA; each rank uploads 1/%d "
                            "of the packed block from pinned host, RCCL all-gather, K as 256x256 blocks "
                            "partitioned over %d rank(s), no reduction" % (n5, m5, dist.world, dist.world),
                "h2d_ms": r3["h2d_ms"], "allgather_ms": r3["allgather_ms"], "syrk_ms": r3["syrk_ms"],
                "gflops": gf5, "seconds": r3["wall"], "scaling": "strong",
                "blocks_on_rank0": r3["n_local_blocks"], "K_bytes_per_rank": r3["n_local_blocks"] * 256 * 256 * 4,
                "roofline": {"bound": "mfma", "achieved": gf5 / 1e3 / dist.world, "peak": SPLIT_PEAK_TFLOPS,
                             "unit": "TFLOP/s per GPU", "frac": gf5 / 1e3 / dist.world / SPLIT_PEAK_TFLOPS,
                             "traffic": None, "kernel": "f32w::k_syrk_h2<true,4> (fp16x2 split, 3 fp16 "
                                                        "MFMA products, f32 accumulate; wall incl. H2D + all-gather)"},
                "projected_seconds_1M_snps": r3["wall"] * 1_000_000 / m5}
        if r3.get("parity_sample") is not None:
            grm5["parity"] = grm5_parity(args, m5, *r3["parity_sample"])
            grm5["parity"]["gathered_block_bit_exact"] = r3["gather_exact"]
            grm5["parity"]["pass"] = grm5["parity"]["pass"] and r3["gather_exact"]
    if dist.rank == 0:
        cpu = None
        parity = None
        if not args.skip_cpu and r1["sample"] is not None:
            ref, cpu = cpu_baseline_standardize(args, r1["sample"], r1["pitch"], timed=dist.world == 1)
            same = np.array_equal(r1["gpu_cols"][:, :args.n_iid].T, ref)
            parity = {"check": "first %d SNP columns x %d iids: GPU stats+decode vs oracle decode+one-pass "
                               "Unit (f32)" % (ref.shape[1], ref.shape[0]), "bit_exact": bool(same)}
            if grm is not None:
                grm["cpu_baseline"] = cpu_baseline_grm(args) if dist.world == 1 else None
                if r2.get("parity_sample") is not None:
                    grm["parity"] = grm_parity(args, *r2["parity_sample"])
        n = args.n_iid
        line = {
            "metric": METRIC, "value": value, "unit": "SNPs/s", "n_gpus": dist.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": r1["wall"] / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "decode+Unit standardize, %d iid x %d SNP per GPU (packed BED resident in HBM, "
                                   "SnpGen MAF curve, 1%% missing), block %d SNPs, f32 F-order" % (
                                       n, args.n_sid, args.block),
                       "n_iid": n, "n_sid_per_gpu": args.n_sid, "block": args.block,
                       "parallelism": "snp-shard x%d" % dist.world},
            "roofline": {"bound": "hbm", "achieved": r1["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": r1["achieved_gbs"] / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("k_decode_std_lds_f32" if r1["fused"] else "k_decode_f<float>", "dec",
                                                n, args.block),
                         "kernel": ("k_decode_std_lds_f32 (stats + decode, packed column staged in LDS)"
                                    if r1["fused"] else "k_decode_f<float> (after k_snp_stats)"),
                         "per_launch_bytes": r1["full_block_bytes"],
                         "mean_launch_ms": r1["dec_mean_ms"],
                         "measured_stream_GBps": {"copy_16B_nt (1 read : 1 write)": r1["copy_gbs"],
                                                  "hipMemset fill (write only)": r1["fill_gbs"]}},
            "cpu_baseline": cpu,
            "parity": parity,
            "grm": grm,
            "grm5": grm5,
        }
        print(json.dumps(line), flush=True)
    dist.barrier()  # every rank leaves together (rank 0 ran the CPU baselines alone)
    dist.close()


if __name__ == "__main__":
    main()
