"""Accuracy of the f32 GRM kernels at large M (diagnostic, prints JSON lines).

K rows 0..R-1 of an n x m synthetic matrix (SnpGen MAF curve, --miss missing) from:
  * the default f32 path (fp16x2 split on the fp16 MFMA), launches of --chunk SNPs,
  * the bf16x3 path (syrk variant 36) and the f32-MFMA path (variant 20),
  * "reference f32": NumPy float32 Z_b[:R] @ Z_b.T per block of 10k SNPs, accumulated in float32
    (what snpreader.py:651-655 computes with dtype=float32),
against the f64 oracle.  Reports max|dK| / max diag and where the maximum sits.
"""
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
    ap.add_argument("--miss", type=float, default=0.218)
    ap.add_argument("--seed", type=int, default=305)
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--chunks", default="65536")
    ap.add_argument("--segs", default="0,4096,8192,16384", help="syrk 'seg' settings (SNPs per f32 chain)")
    ap.add_argument("--variants", default="0,36,20")
    ap.add_argument("--diags", default="1,0", help="hook 'diag': 1 = exact f64 diagonal (round 4 default), 0 = off")
    args = ap.parse_args()
    import bench
    from oracle import oracle as O
    from pysnptools_amd import _native as N
    from pysnptools_amd.shard import ShardedGrm

    n, m, R = args.n, args.m, args.rows
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, args.seed, args.miss)
    host = np.empty((m, pitch), dtype=np.uint8)
    N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
    body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
    del host
    ref = np.zeros((R, n))
    ref32 = np.zeros((R, n), dtype=np.float32)
    for s0 in range(0, m, 10_000):
        sid = np.arange(s0, min(m, s0 + 10_000), dtype=np.uint64)
        Z, _ = O.decode_standardize(body, n, m, sid_index=sid, dtype=np.float64, num_threads=16)
        ref += Z[:R].dot(Z.T)
        Z32 = Z.astype(np.float32)  # f64 stats rounded once, as the f32 path's LUT
        ref32 += Z32[:R].dot(Z32.T)
    scale = np.abs(np.diag(ref[:, :R])).max()

    def report(name, K, **extra):
        d = np.abs(K.astype(np.float64) - ref)
        off = d.copy()
        off[np.arange(R), np.arange(R)] = 0  # the diagonal entries of rows 0..R-1
        io, jo = np.unravel_index(np.argmax(off), off.shape)
        extra = dict(extra, offdiag_max_abs_err_over_max_diag=float(off.max() / scale), offdiag_at=[int(io), int(jo)],
                     offdiag_ref_there=float(ref[io, jo]))
        i, j = np.unravel_index(np.argmax(d), d.shape)
        print(json.dumps({"path": name, "max_abs_err_over_max_diag": float(d.max() / scale),
                          "at": [int(i), int(j)], "ref_there": float(ref[i, j]), "max_diag": float(scale),
                          "mean_abs_err_over_max_diag": float(d.mean() / scale),
                          "diag_rel_err": float(np.max(np.abs(np.diag(K[:, :R]) - np.diag(ref[:, :R]))
                                                       / np.abs(np.diag(ref[:, :R])))), **extra}), flush=True)

    report("reference_f32_numpy_blocks_10k", ref32)
    stats = bench.Dev(N, m * 8)
    ri = np.arange(R, dtype=np.uint64)
    dri, dout = bench.Dev(N, R * 8), bench.Dev(N, R * n * 4)
    N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
    ev = [ctypes.c_void_p(), ctypes.c_void_p()]
    for e in ev:
        N.call("snpmi_event_create", ctypes.byref(e))
    for dg, seg in [(int(d_), int(x)) for d_ in args.diags.split(",") for x in args.segs.split(",")]:
        N.call("snpmi_set_kernel_variant", b"diag", dg)
        N.call("snpmi_set_kernel_variant", b"seg", seg)
        labels = {0: "fp16x2", 36: "bf16x3", 20: "f32_mfma"}
        for variant in [int(v) for v in args.variants.split(",")]:
            label = labels[variant]
            N.call("snpmi_set_kernel_variant", b"syrk", variant)
            for chunk in [int(c) for c in args.chunks.split(",")]:
                g = ShardedGrm(n, np.float32, None, "none")
                g.add_packed(packed.p, pitch, min(m, 256), N.STD_UNIT, 0.0, 0.0, 0, stats.p)  # warm-up
                g.abort()
                g = ShardedGrm(n, np.float32, None, "none")
                N.call("snpmi_event_record", ev[0])
                for s0 in range(0, m, chunk):
                    c = min(chunk, m - s0)
                    g.add_packed(packed.at(s0 * pitch), pitch, c, N.STD_UNIT, 0.0, 0.0, 0, stats.at(s0 * 8))
                N.call("snpmi_event_record", ev[1])
                ms = ctypes.c_float()
                N.call("snpmi_event_elapsed_ms", ev[0], ev[1], ctypes.byref(ms))
                t, _ = g.tiles()
                N.call("snpmi_dev_grm_extract", t, n, N.DT_F32, dri.p, R, None, n, 1, 1.0, dout.p)
                K = np.empty((R, n), dtype=np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
                g.abort()
                report("%s_chunk%d_seg%d_diag%d" % (label, chunk, seg, dg), K, ms=ms.value,
                       tflops=n * (n + 1) * m / (ms.value * 1e-3) / 1e12)
    N.call("snpmi_set_kernel_variant", b"seg", 12288)
    N.call("snpmi_set_kernel_variant", b"syrk", 0)
    N.call("snpmi_set_kernel_variant", b"diag", 1)


if __name__ == "__main__":
    main()
