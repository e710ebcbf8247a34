"""Same-process A/B of the f64 GRM's residue SYRK forms (hook "crt": 0 = k_syrk_i8r, loader in
every wave; 1 = k_syrk_i8w, warp-specialised loader waves), interleaved rounds, HIP events on the
library stream, K tiles compared bit for bit.

  python tools/ab_crt.py [--n 50000 --m 62500 --rounds 3 --forms 0,1]

One snpmi_dev_syrk_packed(f64) call = the bound / moduli kernels + per residue chunk k_syrk_i8* +
k_crt, i.e. what the bench's grm_f64 leg times per 62.5k-SNP launch.  Prints one JSON line per form.
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=50000)
    p.add_argument("--m", type=int, default=62500)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--forms", default="0,1")
    p.add_argument("--miss", type=float, default=0.01)
    p.add_argument("--part", default=None, help="P/W: the cfg5 part kernel, part P of W (e.g. 0/8), into its blocks")
    p.add_argument("--dtype", choices=["f32", "f64"], default="f64",
                   help="f64: the residue SYRK forms (hook crt); f32: the fp16x2 SYRK forms (hook h2)")
    p.add_argument("--hook", default=None,
                   help="override the A/B hook, e.g. crt_block (f64: 0 = launch-wide R, 1 = moduli per 256-block)")
    p.add_argument("--set", action="append", default=[], help="KERNEL=V: a hook applied once before the A/B (e.g. seg=0)")
    a = p.parse_args()
    for kv in a.set:
        k, v = kv.split("=")
        N.call("snpmi_set_kernel_variant", k.encode(), int(v))
    hook = a.hook.encode() if a.hook else (b"crt" if a.dtype == "f64" else b"h2")
    dt, esz = (N.DT_F64, 8) if a.dtype == "f64" else (N.DT_F32, 4)
    n, m = a.n, a.m
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 105, a.miss)
    lut, st = Dev(N, m * 4 * esz), Dev(N, m * 2 * esz)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, dt, st.p, lut.p)
    part = tuple(int(x) for x in a.part.split("/")) if a.part else None
    nloc = N.lib().snpmi_grm_part_blocks(n, part[0], part[1]) if part else 0
    tb = nloc * 65536 * esz if part else N.lib().snpmi_grm_tile_bytes(n, dt)
    tiles = Dev(N, tb)
    forms = [int(f) for f in a.forms.split(",")]
    ev = Events(N, 2)
    res = {f: [] for f in forms}
    sums = {}
    sum_r, nl = ctypes.c_uint64(), ctypes.c_uint64()
    blk_r = {}
    for rnd in range(a.rounds + 1):  # round 0: warm-up (scratch allocations, code objects)
        for f in forms:
            N.call("snpmi_set_kernel_variant", hook, f)
            N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 1)
            N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 1)
            ev.record(0)
            if part:
                N.call("snpmi_dev_syrk_packed_part" + ("_f64" if esz == 8 else ""), packed.p, pitch, n, m, lut.p,
                       part[0], part[1], tiles.p, 0)
            else:
                N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, dt, tiles.p, 0)
            ev.record(1)
            N.call("snpmi_stream_sync")
            if rnd:
                res[f].append(ev.ms(0, 1))
            else:
                # the first and last 32M tile elements (512 MiB) compared with form 0's, bit for bit
                k = min(tb // esz, 1 << 25)
                h = np.empty(2 * k, dtype=np.float64 if esz == 8 else np.float32)
                N.call("snpmi_memcpy_d2h", N.ptr(h[:k]), tiles.p, k * esz)
                N.call("snpmi_memcpy_d2h", N.ptr(h[k:]), ctypes.c_void_p(tiles.p.value + tb - k * esz), k * esz)
                sums[f] = h
                N.call("snpmi_crt_block_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 0)
                blk_r[f] = sum_r.value / nl.value if nl.value else None
                N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 0)
            print(json.dumps({"round": rnd, "form": f, "ms": ev.ms(0, 1)}), file=sys.stderr, flush=True)
    N.call("snpmi_set_kernel_variant", hook, 1)
    # executed MFMA work: f64 = R int8 SYRKs per block (5.0 POP/s dense); f32 = 3 fp16 products (2.5 PF/s)
    R_launch, peak = (sum_r.value / max(nl.value, 1), 5000.0) if a.dtype == "f64" else (3.0, 2500.0)
    nb = (n + 255) // 256
    base = sums[forms[0]]
    for f in forms:
        t = float(np.median(res[f]))
        R = (blk_r.get(f) or R_launch) if a.dtype == "f64" else R_launch
        ops = R * 2 * 256 * 256 * (nloc if part else nb * (nb + 1) // 2) * m
        names = {b"crt": {0: "k_syrk_i8r", 1: "k_syrk_i8w", 2: "k_syrk_i8w plain"}, b"h2": {0: "k_syrk_h2<.,4>", 1: "k_syrk_h2s"},
                 b"crt_block": {0: "launch-wide R", 1: "R per 256-block"}}.get(hook, {})
        print(json.dumps({"form": f, "hook": hook.decode(), "kernel": names.get(f, "ablation %d" % f), "dtype": a.dtype,
                          "n": n, "m": m, "median_ms": t, "all_ms": res[f],
                          "moduli": R if a.dtype == "f64" else None,
                          "moduli_launch_wide": R_launch if a.dtype == "f64" else None,
                          "frac_mfma_peak_executed": ops / t / 1e9 / peak, "syrk_tflops": n * (n + 1) * m / t / 1e9 / (part[1] if part else 1), "part": a.part,
                          "tiles_equal_form0": bool(np.array_equal(sums[f], base))}), flush=True)


if __name__ == "__main__":
    main()
