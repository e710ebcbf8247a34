"""Dense standardize A/B on HBM-resident f32 values (the reference's Bed.read().standardize(Unit())
with values in HBM): a synthetic --n x --m packed matrix (SnpGen MAF curve, 21.8% missing) decoded
once into tight F-order f32 columns, then standardized in place by the round-4 kernel
(k_std_cols_f, hook "std" 0) and by round 3's (hook 1), Unit and Beta(1,25), each timed with HIP
events on the library stream; the two results compared bit for bit on sampled columns.  Prints
JSON lines; algorithmic bytes = 2 x 4 B per value.  Also the profiling target of
tools/profile_r04.sh (--only 0 runs the round-4 kernel alone)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--m", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", type=int, default=None, help="run just this hook value (profiling)")
    args = ap.parse_args()
    import bench
    from pysnptools_amd import _native as N

    n, m = args.n, args.m
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, 321, 0.218)
    lut = np.tile(np.array([0.0, np.nan, 1.0, 2.0], dtype=np.float32), m)
    dlut = bench.Dev(N, lut.nbytes)
    N.call("snpmi_memcpy_h2d", dlut.p, N.ptr(lut), lut.nbytes)
    vals = bench.Dev(N, n * m * 4)
    stats = np.empty((m, 2), dtype=np.float32)
    ev = bench.Events(N, 2)
    variants = [args.only] if args.only is not None else [1, 0]
    samples = {}
    for kind, beta in (("unit", 0), ("beta", 1)):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"std", v)
            ts = []
            for _ in range(args.reps):
                N.call("snpmi_dev_decode", packed.p, pitch, n, m, dlut.p, N.DT_F32, 0, vals.p, n)
                N.call("snpmi_stream_sync")
                ev.record(0)
                N.call("snpmi_standardize_f32", vals.p, n, m, 0, beta, 1.0 if beta else np.nan,
                       25.0 if beta else np.nan, 1, 0, N.ptr(stats), 0)
                ev.record(1)
                ts.append(ev.ms(0, 1))
            N.call("snpmi_set_kernel_variant", b"std", 0)
            smp = np.empty((64, n), dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(smp), ctypes.c_void_p(vals.p.value + (m // 2) * n * 4), smp.nbytes)
            samples[(kind, v)] = (smp, stats.copy())
            gb = 2.0 * n * m * 4 / 1e9
            print(json.dumps({"n": n, "m": m, "std": kind, "hook_std": v, "ms_min": min(ts), "ms_all": ts,
                              "TBps": gb / (min(ts) * 1e-3) / 1e3, "frac_of_8TBps": gb / (min(ts) * 1e-3) / 8e3}),
                  flush=True)
        if len(variants) == 2:
            a, b = samples[(kind, 0)], samples[(kind, 1)]
            print(json.dumps({"std": kind, "bit_equal_round3": bool(np.array_equal(a[0].view(np.uint32),
                                                                                b[0].view(np.uint32))
                                                                   and np.array_equal(a[1], b[1]))}), flush=True)
    ev.destroy()
    for d in (packed, dlut, vals):
        d.free()


if __name__ == "__main__":
    main()
