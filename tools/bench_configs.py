"""Time every BASELINE.json config on one MI355X and its CPU baseline on the same box
(BASELINE.md §2-3).  Prints one JSON line per (config, backend); GPU legs are device-resident
(packed bytes generated in HBM), CPU legs run the oracle's C/OpenMP decode+standardize and
NumPy Z·Zᵀ (the reference's own GRM call) at all host threads (capped at 16) and at 1 thread,
on the sizes / slices BASELINE.md §2 prescribes (extrapolations are labelled).
Usage: python tools/bench_configs.py [--only 1,2,3,4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def emit(**kw):
    print(json.dumps(kw), flush=True)


def gpu_decode_std(N, n, m, seed, miss, kind, a, b, block_bytes=4 << 30, reps=2):
    """Blocks of ~block_bytes of f32 output (>= 2048 SNPs): at small N a fixed SNP count makes
    short launches whose gaps dominate (cfg2 at 8192-SNP blocks: 70 us per launch)."""
    from bench import Dev, Events, synth

    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, seed, miss)
    B = min(m, max(2048, block_bytes // (4 * ld)))
    lut, st, out = Dev(N, B * 16), Dev(N, B * 8), Dev(N, B * ld * 4)
    ev = Events(N, 2)
    best = None
    for r in range(reps + 1):
        ev.record(0)
        for s0 in range(0, m, B):
            cnt = min(B, m - s0)
            src = ctypes.c_void_p(packed.p.value + s0 * pitch)
            N.call("snpmi_dev_snp_stats", src, pitch, n, cnt, 0, kind, a, b, 0, N.DT_F32, st.p, lut.p)
            N.call("snpmi_dev_decode", src, pitch, n, cnt, lut.p, N.DT_F32, 0, out.p, ld)
        ev.record(1)
        t = ev.ms(0, 1) / 1e3
        if r > 0:
            best = t if best is None else min(best, t)
    sample = np.empty((min(m, 2048), pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(sample), packed.p, sample.nbytes)
    for d in (packed, lut, st, out):
        d.free()
    ev.destroy()
    return best, sample, B


def cpu_decode_std(sample, n, is_beta, a, b, threads, budget=6.0):
    from oracle import oracle as O

    body = np.ascontiguousarray(sample[:, :(n + 3) // 4]).reshape(-1)
    cols = sample.shape[0]
    done, t0 = 0, time.perf_counter()
    while True:
        O.decode_standardize(body, n, cols, is_beta=is_beta, a=a, b=b, dtype=np.float32, num_threads=threads)
        done += cols
        el = time.perf_counter() - t0
        if el > budget or done >= 8 * cols:
            return done / el, done


def cpu_grm(n, b, dtype, threads):
    from threadpoolctl import threadpool_limits

    Z = np.random.default_rng(0).standard_normal((n, b)).astype(dtype)
    with threadpool_limits(limits=threads):
        Z.dot(Z.T)
        t0 = time.perf_counter()
        Z.dot(Z.T)
        el = time.perf_counter() - t0
    return n * (n + 1) * b / el / 1e9, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="1,2,3,4")
    args = ap.parse_args()
    only = {int(x) for x in args.only.split(",")}
    from pysnptools_amd import _native as N

    allt = min(16, os.cpu_count() or 1)
    if 1 in only:
        from oracle import oracle as O
        from pysnptools_amd.snpreader import Bed
        from pysnptools_amd.standardizer import Unit

        for name, n, m in (("n300", 300, 1015), ("toydata", 500, 10000)):
            path = os.path.join(ROOT, "tests", "golden", "data", name + ".bed")
            bed = Bed(path, count_A1=False)
            bed.read(dtype=np.float32).standardize(Unit())
            t0 = time.perf_counter()
            bed.read(dtype=np.float32).standardize(Unit())
            tg = time.perf_counter() - t0
            t0 = time.perf_counter()
            K = bed.read_kernel(Unit(), dtype=np.float64).val
            tk = time.perf_counter() - t0
            body = O.read_bed_bytes(path)
            t0 = time.perf_counter()
            Kref, _ = O.grm_from_bed(body, n, m)
            tkc = time.perf_counter() - t0
            err = float(np.abs(K - Kref).max() / np.abs(np.diag(Kref)).max())
            emit(cfg=1, workload="%s %dx%d Bed.read(f32).standardize(Unit()) + read_kernel(f64), file-backed" % (name, n, m),
                 backend="1xMI355X", read_std_s=tg, snps_per_s=m / tg, grm_s=tk, grm_vs_oracle=err,
                 cpu_grm_s_numpy_f64=tkc)
    if 2 in only or 3 in only:
        for cfg, n, m, seed, miss, kind, a, b, lab in (
                (2, 10_000, 100_000, 2, 0.01, N.STD_UNIT, 0.0, 0.0, "Unit"),
                (3, 100_000, 1_000_000, 3, 0.218, N.STD_BETA, 1.0, 25.0, "Beta(1,25)+NaN impute")):
            if cfg not in only:
                continue
            t, sample, B = gpu_decode_std(N, n, m, seed, miss, kind, a, b)
            nbytes = m * ((n + 3) // 4 + 4 * n)
            emit(cfg=cfg, workload="%d iid x %d SNP, %s, f32, HBM-resident packed, %d-SNP blocks" % (n, m, lab, B),
                 backend="1xMI355X", seconds=t, snps_per_s=m / t, GBps=nbytes / t / 1e9, hbm_frac=nbytes / t / 8e12)
            for th in (allt, 1):
                v, done = cpu_decode_std(sample, n, kind == N.STD_BETA, a, b, th)
                emit(cfg=cfg, workload="same, CPU oracle decode+one-pass standardize on the first %d columns "
                                       "(%d SNPs timed; rate extrapolates linearly in M)" % (sample.shape[0], done),
                     backend="CPU port", threads=th, snps_per_s=v, projected_full_s=m / v)
    if 4 in only:
        for dt in (np.float32, np.float64):
            for th in (allt, 1):
                gf, el = cpu_grm(10_000 if th > 1 else 4_000, 2048 if th > 1 else 1024, dt, th)
                emit(cfg=4, workload="NumPy Z.dot(Z.T) %s (the reference's GRM call) on a slice; cfg4 projection = "
                                     "50k*50001*500k flops / rate" % np.dtype(dt).name,
                     backend="CPU NumPy/OpenBLAS", threads=th, GFps=gf,
                     projected_cfg4_s=50_000 * 50_001 * 500_000 / (gf * 1e9),
                     projected_cfg5_s=500_000 * 500_001 * 1_000_000 / (gf * 1e9))


if __name__ == "__main__":
    main()
