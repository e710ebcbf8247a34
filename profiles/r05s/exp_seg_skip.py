"""Adaptive SegFlush sweep (round 5): for each threshold factor (hook "seg_skip"; 0 = flush at every
due point) one f32 SYRK launch over m SnpGen-shaped SNPs (21.8% missing) through
snpmi_dev_syrk_packed (exact diagonal + threshold + fp16x2 SYRK): due points flushed / kept, the
launch time (HIP events, best of `rounds`), and K rows 0..7 vs the f64 oracle (max |dK| / max diag).
Usage: python tools/exp_seg_skip.py n m fac,fac,... [seg,seg,...]   One JSON line per (seg, factor)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import bench
    from oracle import oracle as O
    from pysnptools_amd import _native as N

    n, m = int(sys.argv[1]), int(sys.argv[2])
    facs = [int(x) for x in sys.argv[3].split(",")]
    segs = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [N.kernel_variant("seg")]
    rounds, R = 3, 8
    pitch = N.lib().snpmi_packed_pitch(n)
    p = bench.Dev(N, pitch * m)
    bench.synth(N, p.p, pitch, n, 0, m, 305, 0.218)
    lut, st = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    N.call("snpmi_dev_snp_stats", p.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
    tiles = bench.Dev(N, N.lib().snpmi_grm_tile_bytes(n, N.DT_F32))
    ref = np.zeros((R, n))
    chunk = 4096
    host = np.empty((chunk, pitch), dtype=np.uint8)
    for s0 in range(0, m, chunk):
        c = min(chunk, m - s0)
        N.call("snpmi_memcpy_d2h", N.ptr(host), p.at(s0 * pitch), c * pitch)
        body = np.ascontiguousarray(host[:c, :(n + 3) // 4]).reshape(-1)
        Z, _ = O.decode_standardize(body, n, c, dtype=np.float64, num_threads=16)
        ref += Z[:R].dot(Z.T)
    scale = np.abs(np.diag(ref[:, :R])).max()
    ri = np.arange(R, dtype=np.uint64)
    dri, dout = bench.Dev(N, R * 8), bench.Dev(N, R * n * 4)
    N.call("snpmi_memcpy_h2d", dri.p, N.ptr(ri), ri.nbytes)
    ev = bench.Events(N, 2)
    fl, kept = ctypes.c_uint64(), ctypes.c_uint64()
    default, seg_default = N.kernel_variant("seg_skip"), N.kernel_variant("seg")
    N.call("snpmi_set_kernel_variant", b"seg_stats", 1)
    try:
        for seg, fac in [(g, f) for g in segs for f in facs]:
            N.call("snpmi_set_kernel_variant", b"seg", seg)
            N.call("snpmi_set_kernel_variant", b"seg_skip", fac)
            ms = []
            for r in range(rounds):
                N.call("snpmi_seg_flush_stats", ctypes.byref(fl), ctypes.byref(kept), 1)
                ev.record(0)
                N.call("snpmi_dev_syrk_packed", p.p, pitch, n, m, lut.p, N.DT_F32, tiles.p, 0)
                ev.record(1)
                ms.append(ev.ms(0, 1))
            N.call("snpmi_seg_flush_stats", ctypes.byref(fl), ctypes.byref(kept), 1)
            N.call("snpmi_dev_grm_extract", tiles.p, n, N.DT_F32, dri.p, R, None, n, 1, 1.0, dout.p)
            K = np.empty((R, n), dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
            err = float(np.abs(K.astype(np.float64) - ref).max() / scale)
            print(json.dumps({"n": n, "m": m, "seg": N.kernel_variant("seg"), "seg_skip": fac,
                              "flushed": fl.value, "kept": kept.value,
                              "kept_frac": kept.value / max(1, fl.value + kept.value), "ms": ms,
                              "best_ms": min(ms), "err_rel_maxdiag": err}), flush=True)
    finally:
        N.call("snpmi_set_kernel_variant", b"seg_skip", default)
        N.call("snpmi_set_kernel_variant", b"seg", seg_default)
        N.call("snpmi_set_kernel_variant", b"seg_stats", 0)


if __name__ == "__main__":
    main()
