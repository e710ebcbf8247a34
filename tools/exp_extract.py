"""Whole-K extraction A/B (hook "extract": 0 = k_grm_extract_sym, each upper 64x64 block read once
and written twice; 1 = round 3's k_grm_extract_rows; 2-4 other block shapes; 5-7 the pipelined
kernel): HIP-event time per call on the library
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
        # a non-uniform fill: a random chunk whose length is no multiple of a tile, repeated
        dt = np.float32 if es == 4 else np.float64
        chunk = np.random.default_rng(5).standard_normal(4_000_037).astype(dt)
        for off in range(0, tb, chunk.nbytes):
            N.call("snpmi_memcpy_h2d", tiles.at(off), N.ptr(chunk), min(chunk.nbytes, tb - off))
        outs = [bench.Dev(N, n * n * es), bench.Dev(N, n * n * es)]
        ev = bench.Events(N, 2)
        res = {}
        variants = (1, 0, 2, 3, 4, 5, 6, 7)
        for v in variants + variants:
            N.call("snpmi_set_kernel_variant", b"extract", v)
            ts = []
            for _ in range(reps):
                ev.record(0)
                N.call("snpmi_dev_grm_extract", tiles.p, n, code, None, n, None, n, 1, 1.0, outs[v == 1].p)
                ev.record(1)
                ts.append(ev.ms(0, 1))
            res[v] = min(ts)
        # every variant's K vs the row kernel's on 64 sampled rows (each row crosses every block
        # column straight and mirrored)
        rows = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(9).integers(0, n, 62)]))
        ref = np.empty((len(rows), n), dtype=dt)
        for k, r in enumerate(rows):
            N.call("snpmi_memcpy_d2h", N.ptr(ref[k]), outs[1].at(int(r) * n * es), n * es)
        same = {}
        for v in variants[1:]:
            N.call("snpmi_set_kernel_variant", b"extract", v)
            N.call("snpmi_dev_grm_extract", tiles.p, n, code, None, n, None, n, 1, 1.0, outs[0].p)
            got = np.empty_like(ref)
            for k, r in enumerate(rows):
                N.call("snpmi_memcpy_d2h", N.ptr(got[k]), outs[0].at(int(r) * n * es), n * es)
            same[v] = bool(np.array_equal(got, ref))
        N.call("snpmi_set_kernel_variant", b"extract", 0)
        algo = tb + n * n * es  # the upper-triangle tiles read once + K written
        print(json.dumps({"n": n, "dtype": name, "sym_ms": res[0], "rows_ms": res[1], "algorithmic_GB": algo / 1e9,
                          "shapes_ms": {"128x128/512thr": res[2], "64x64 (f64: 512thr)": res[3], "128x128/1024thr": res[4],
                                        "pipe default shape": res[5], "pipe 128x128/1024thr": res[6],
                                        "pipe 64x64 (f32: 256thr, f64: 512thr)": res[7]},
                          "sym_TBps": algo / (res[0] * 1e-3) / 1e12, "frac_of_8TBps": algo / (res[0] * 1e-3) / 8e12,
                          "best_frac": algo / (min(res.values()) * 1e-3) / 8e12,
                          "rows_TBps": algo / (res[1] * 1e-3) / 1e12, "sampled_rows_bit_equal_to_rows_kernel": same}),
              flush=True)
        ev.destroy()
        for d in [tiles] + outs[:2]:
            d.free()


if __name__ == "__main__":
    main()
