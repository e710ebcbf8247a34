"""Whole-K extraction A/B (hook "extract": 0 = k_grm_extract_sym, each upper 64x64 block read once
and written twice; 1 = round 3's k_grm_extract_rows): HIP-event time per call on the library
stream for K of n iids in HBM (f32 and f64), and the two outputs compared bit for bit.  Prints
JSON lines (algorithmic bytes = the upper-triangle tiles read once + n^2 written)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pysnptools_amd import _native as N

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
    reps = 5
    for code, es, name in ((N.DT_F32, 4, "f32"), (N.DT_F64, 8, "f64")):
        tb = N.lib().snpmi_grm_tile_bytes(n, code)
        tiles = bench.Dev(N, tb)
        N.call("snpmi_dev_memset", tiles.p, 0x3f, tb)  # any finite pattern
        outs = [bench.Dev(N, n * n * es), bench.Dev(N, n * n * es)]
        outs += [outs[0]] * 3  # A/B shapes 2-4 write over the shipped kernel's output
        ev = bench.Events(N, 2)
        res = {}
        for v in (1, 0, 2, 3, 4, 1, 0, 2, 3, 4):
            N.call("snpmi_set_kernel_variant", b"extract", v)
            ts = []
            for _ in range(reps):
                ev.record(0)
                N.call("snpmi_dev_grm_extract", tiles.p, n, code, None, n, None, n, 1, 1.0, outs[min(v, 2) if v < 2 else 0].p)
                ev.record(1)
                ts.append(ev.ms(0, 1))
            res[v] = min(ts)
        N.call("snpmi_set_kernel_variant", b"extract", 0)
        a = np.empty(n * 64, dtype=np.uint8)
        same = True
        for off in (0, (n * n * es) // 2, n * n * es - a.nbytes):
            b0, b1 = np.empty_like(a), np.empty_like(a)
            N.call("snpmi_memcpy_d2h", N.ptr(b0), outs[0].at(off), a.nbytes)
            N.call("snpmi_memcpy_d2h", N.ptr(b1), outs[1].at(off), a.nbytes)
            same &= bool(np.array_equal(b0, b1))
        algo = tb + n * n * es  # the upper-triangle tiles read once + K written
        print(json.dumps({"n": n, "dtype": name, "sym_ms": res[0], "rows_ms": res[1], "algorithmic_GB": algo / 1e9,
                          "shapes_ms": {"128x128/512thr": res[2], "64x64 (f64: 512thr)": res[3], "128x128/1024thr": res[4]},
                          "sym_TBps": algo / (res[0] * 1e-3) / 1e12, "frac_of_8TBps": algo / (res[0] * 1e-3) / 8e12,
                          "rows_TBps": algo / (res[1] * 1e-3) / 1e12, "sample_bit_equal": same}), flush=True)
        ev.destroy()
        for d in [tiles] + outs[:2]:
            d.free()


if __name__ == "__main__":
    main()
