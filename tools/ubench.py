"""A/B microbenchmarks of single kernels (interleaved rounds in ONE process, HIP events).

The ablation variants of rounds 1-5 were deleted in round 6 (DESIGN.md records what they measured):
the variants left are the shipped kernels' hooks -- decode 0-17 (block shapes / staging switches of
the shipped decode and repack), syrk 0 (default chain), 36 (bf16x3 alone), 20 (f32 MFMA), 5
(128x128 small-N kernels); the loader-wave forms of the SYRKs are tools/ab_crt.py's.

  python tools/ubench.py decode [--n 500000 --m 8192 --variants 0,1,2,3,4,5,6]
  python tools/ubench.py syrk   [--n 50000 --m 10000]      (variants 0,36,20 by default)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pysnptools_amd import _native as N  # noqa: E402
from bench import Dev, Events, synth  # noqa: E402


def decode(args):
    n, m = args.n, args.m
    dt, esz = {"f32": (N.DT_F32, 4), "f64": (N.DT_F64, 8)}[args.dtype]
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    lut, st, out = Dev(N, m * 4 * esz), Dev(N, m * 2 * esz), Dev(N, m * ld * esz)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
    variants = [int(v) for v in args.variants.split(",")]
    ev = Events(N, 2)
    res = {v: [] for v in variants}
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            if v >= 0:
                N.call("snpmi_set_kernel_variant", b"decode", v)
                ev.record(0)
                N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
                N.call("snpmi_dev_decode", packed.p, pitch, n, m, lut.p, dt, 0, out.p, ld)
                ev.record(1)
            else:
                ev.record(0)
                N.call("snpmi_dev_decode_standardize", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
                       st.p, lut.p, out.p, ld)
                ev.record(1)
            res[v].append(ev.ms(0, 1))
            if rnd == 0:
                chk = np.empty(4 * ld, dtype=np.float32 if esz == 4 else np.float64)
                N.call("snpmi_memcpy_d2h", N.ptr(chk), ctypes.c_void_p(out.p.value + (m - 4) * ld * esz), chk.nbytes)
                if ref is None:
                    ref = chk.copy()
                assert np.array_equal(chk, ref), "variant %d output differs" % v
    nbytes = m * ((n + 3) // 4 + esz * n)
    for v in variants:
        t = np.median(res[v])
        print(json.dumps({"kernel": "stats+decode" if v >= 0 else "fused", "dtype": args.dtype, "variant": v, "median_ms": t, "min_ms": min(res[v]),
                          "GBps": nbytes / t / 1e6, "frac_8TBs": nbytes / t / 1e6 / 8000}))


def stats(args):
    """k_snp_stats alone, cycling over --m SNPs in blocks of 2048 so each launch reads its codes
    from HBM (the whole buffer is larger than the 256 MB Infinity Cache); variant 6 = one wave
    per SNP, 0 = four waves per SNP for columns >= 16 KiB."""
    n, m, B = args.n, args.m, 2048
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    lut, st = Dev(N, B * 16), Dev(N, B * 8)
    variants = [int(v) for v in args.variants.split(",")]
    ev = Events(N, 2)
    res = {v: [] for v in variants}
    nblk = m // B
    k = 0
    for rnd in range(args.rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"decode", v)
            for _ in range(nblk):
                src = ctypes.c_void_p(packed.p.value + (k % nblk) * B * pitch)
                k += 1
                ev.record(0)
                N.call("snpmi_dev_snp_stats", src, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
                ev.record(1)
                res[v].append(ev.ms(0, 1))
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    nbytes = B * ((n + 3) // 4)
    for v in variants:
        t = np.median(res[v])
        print(json.dumps({"kernel": "snp_stats", "variant": v, "n": n, "block": B, "median_ms": t,
                          "GBps": nbytes / t / 1e6}))


def decode_c(args):
    """C-order decode (k_decode_c): out[i][j], ld = m; the same bytes as the F-order decode."""
    n, m = args.n, args.m
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    lut, st, out = Dev(N, m * 16), Dev(N, m * 8), Dev(N, m * n * 4)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
    variants = [int(v) for v in args.variants.split(",")]
    ev = Events(N, 2)
    res = {v: [] for v in variants}
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"decode", v)
            ev.record(0)
            N.call("snpmi_dev_decode", packed.p, pitch, n, m, lut.p, N.DT_F32, 1, out.p, m)
            ev.record(1)
            res[v].append(ev.ms(0, 1))
            if rnd == 0:  # every variant must write the same values (first and last 64 rows)
                got = np.empty((128, m), dtype=np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(got[:64]), out.p, 64 * m * 4)
                N.call("snpmi_memcpy_d2h", N.ptr(got[64:]), out.at((n - 64) * m * 4), 64 * m * 4)
                if ref is None:
                    ref = got
                assert np.array_equal(got, ref), "variant %d differs" % v
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    nbytes = m * ((n + 3) // 4 + 4 * n)
    for v in variants:
        t = np.median(res[v])
        print(json.dumps({"kernel": "decode_c", "variant": v, "n": n, "m": m, "median_ms": t, "GBps": nbytes / t / 1e6,
                          "frac_8TBs": nbytes / t / 1e6 / 8000}))


def repack(args):
    """iid gather of packed columns (k_repack_lds): --index rev2 (every other iid, reversed; the
    round-1 figure), random (n/2 draws with replacement) or sorted (a random half, in order)."""
    n, m = args.n, args.m
    pitch = N.lib().snpmi_packed_pitch(n)
    rng = np.random.default_rng(0)
    if args.index == "random":
        idx = rng.choice(n, size=n // 2, replace=True).astype(np.uint64)
    elif args.index == "sorted":
        idx = np.sort(rng.choice(n, size=n // 2, replace=False)).astype(np.uint64)
    else:
        idx = np.arange(n - 1, -1, -2, dtype=np.uint64)
    n_out = len(idx)
    pitch_out = N.lib().snpmi_packed_pitch(n_out)
    packed, dst, didx = Dev(N, pitch * m), Dev(N, pitch_out * m), Dev(N, n_out * 8)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    N.call("snpmi_memcpy_h2d", didx.p, N.ptr(idx), idx.nbytes)
    ev = Events(N, 2)
    variants = [int(v) for v in args.variants.split(",")]
    ts = {v: [] for v in variants}
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"decode", v)
            N.call("snpmi_dev_memset", dst.p, 0xA5, pitch_out * m)
            ev.record(0)
            N.call("snpmi_dev_repack", packed.p, pitch, n, didx.p, n_out, m, dst.p, pitch_out)
            ev.record(1)
            ts[v].append(ev.ms(0, 1))
            if rnd == 0:  # every variant must produce the same bytes
                got = np.empty((m, pitch_out), dtype=np.uint8)
                N.call("snpmi_memcpy_d2h", N.ptr(got), dst.p, got.nbytes)
                if ref is None:
                    ref = got
                assert np.array_equal(got[:, :(n_out + 3) // 4], ref[:, :(n_out + 3) // 4]), "variant %d differs" % v
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    nbytes = m * ((n + 3) // 4 + (n_out + 3) // 4)
    for v in variants:
        t = np.median(ts[v])
        print(json.dumps({"kernel": "repack", "variant": v, "index": args.index, "n": n, "n_out": n_out, "m": m,
                          "median_ms": t, "GBps": nbytes / t / 1e6, "frac_8TBs": nbytes / t / 1e6 / 8000,
                          "note": "time = plan (+ window scan, one host sync) + gather; decode variant 8 = no "
                                  "windowed kernel"}))


def syrk_dense(args):
    """decode the block to f32/f64 in HBM (ld = round_up(n,256)) + dense-loader SYRK."""
    n, m = args.n, args.m
    dt = N.DT_F64 if args.dtype == "f64" else N.DT_F32
    esz = 8 if dt == N.DT_F64 else 4
    pitch = N.lib().snpmi_packed_pitch(n)
    ldz = (n + 255) // 256 * 256
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    lut, st, Z = Dev(N, m * 4 * esz), Dev(N, m * 2 * esz), Dev(N, m * ldz * esz)
    N.call("snpmi_dev_memset", Z.p, 0, m * ldz * esz)
    tiles = Dev(N, N.lib().snpmi_grm_tile_bytes(n, dt))
    ev = Events(N, 4)
    variants = [int(v) for v in args.variants.split(",")]
    ts = {v: [] for v in variants}
    td = []
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            # v < 0: default kernels with the genotype re-encoding off (dense stage-image path)
            N.call("snpmi_set_kernel_variant", b"syrk", max(v, 0))
            N.call("snpmi_set_kernel_variant", b"dense_codes", 0 if v < 0 else 1)
            ev.record(0)
            N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
            N.call("snpmi_dev_decode", packed.p, pitch, n, m, lut.p, dt, 0, Z.p, ldz)
            ev.record(1)
            N.call("snpmi_dev_syrk_dense", Z.p, ldz, n, m, dt, tiles.p, 0)
            ev.record(2)
            td.append(ev.ms(0, 1))
            ts[v].append(ev.ms(1, 2))
            if rnd == 0:
                chk = np.empty(1 << 22, dtype=np.float64 if esz == 8 else np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(chk), tiles.p, chk.nbytes)
                ref = chk.copy() if ref is None else ref
                err = np.abs(chk.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1)
                assert err < 1e-5, "variant %d differs: %g" % (v, err)
    d = np.median(td)
    peak = 78.6 if esz == 8 else 157.3
    for v in variants:
        t = np.median(ts[v])
        print(json.dumps({"kernel": "decode+syrk_dense_" + args.dtype, "variant": v, "n": n, "m": m, "decode_ms": d,
                          "syrk_ms": t, "TFLOPs_syrk": n * (n + 1) * m / t / 1e9,
                          "frac_syrk": n * (n + 1) * m / t / 1e9 / peak,
                          "TFLOPs_total": n * (n + 1) * m / (t + d) / 1e9}))


def syrk(args):
    n, m = args.n, args.m
    dt = N.DT_F64 if args.dtype == "f64" else N.DT_F32
    esz = 8 if dt == N.DT_F64 else 4
    peak = 78.6 if dt == N.DT_F64 else 157.3
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
    lut, st = Dev(N, m * 4 * esz), Dev(N, m * 2 * esz)
    tiles = Dev(N, N.lib().snpmi_grm_tile_bytes(n, dt))
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
    ev = Events(N, 2)
    variants = [int(v) for v in args.variants.split(",")]
    ts = {v: [] for v in variants}
    errs = {}
    ref = None
    nt_bytes = N.lib().snpmi_grm_tile_bytes(n, dt)
    for rnd in range(args.rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"syrk", v)
            ev.record(0)
            N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, dt, tiles.p, int(args.acc and rnd > 0))
            ev.record(1)
            ts[v].append(ev.ms(0, 1))
            if rnd == 0:
                N.call("snpmi_stream_sync")
                chk = np.empty(min(nt_bytes // esz, 1 << 22), dtype=np.float64 if esz == 8 else np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(chk), tiles.p, chk.nbytes)
                if ref is None:
                    ref = chk.copy()
                err = np.abs(chk.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1)
                errs[v] = float(err)
                assert args.noassert or v in (10, 11, 12, 13, 14, 15, 39, 63, 73, 74) or err < 1e-5, "variant %d differs: %g" % (v, err)
    for v in variants:
        t = np.median(ts[v])
        print(json.dumps({"kernel": "syrk_" + args.dtype, "variant": v, "n": n, "m": m, "accumulate": args.acc,
                          "median_ms": t, "err_vs_first": errs.get(v),
                          "TFLOPs": n * (n + 1) * m / t / 1e9, "frac": n * (n + 1) * m / t / 1e9 / peak}))


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("what")
    p.add_argument("--n", type=int, default=500000)
    p.add_argument("--m", type=int, default=8192)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--dtype", default="f32")
    p.add_argument("--index", default="rev2", choices=["rev2", "random", "sorted"])
    p.add_argument("--variants", default="0,1,2,3,4,5,6")
    p.add_argument("--acc", type=int, default=0, help="syrk: accumulate into the tiles (rounds after the first)")
    p.add_argument("--noassert", type=int, default=0)
    p.add_argument("--set-variant", default=None, help="kernel=variant applied once before the run")
    a = p.parse_args()
    if a.what in ("syrk", "syrk_dense") and a.variants == "0,1,2,3,4,5,6":
        a.variants = "0,36,20"
    if a.set_variant:
        k, v = a.set_variant.split("=")
        N.call("snpmi_set_kernel_variant", k.encode(), int(v))
    {"decode": decode, "stats": stats, "decode_c": decode_c, "repack": repack, "syrk": syrk, "syrk_dense": syrk_dense}[a.what](a)
