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
    a = p.parse_args()
    n, m = a.n, a.m
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = Dev(N, pitch * m)
    synth(N, packed.p, pitch, n, 0, m, 105, a.miss)
    lut, st = Dev(N, m * 32), Dev(N, m * 16)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F64, st.p, lut.p)
    tb = N.lib().snpmi_grm_tile_bytes(n, N.DT_F64)
    tiles = Dev(N, tb)
    forms = [int(f) for f in a.forms.split(",")]
    ev = Events(N, 2)
    res = {f: [] for f in forms}
    sums = {}
    sum_r, nl = ctypes.c_uint64(), ctypes.c_uint64()
    for rnd in range(a.rounds + 1):  # round 0: warm-up (scratch allocations, code objects)
        for f in forms:
            N.call("snpmi_set_kernel_variant", b"crt", f)
            N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 1)
            ev.record(0)
            N.call("snpmi_dev_syrk_packed", packed.p, pitch, n, m, lut.p, N.DT_F64, tiles.p, 0)
            ev.record(1)
            N.call("snpmi_stream_sync")
            if rnd:
                res[f].append(ev.ms(0, 1))
            else:
                h = np.empty(tb // 8, dtype=np.float64)
                N.call("snpmi_memcpy_d2h", N.ptr(h), tiles.p, tb)
                sums[f] = (float(np.sum(h)), float(np.sum(h * np.arange(h.size) % 977)))
                N.call("snpmi_crt_moduli_stats", ctypes.byref(sum_r), ctypes.byref(nl), 0)
    N.call("snpmi_set_kernel_variant", b"crt", 0)
    R = sum_r.value / max(nl.value, 1)
    nb = (n + 255) // 256
    ops = R * 2 * 256 * 256 * (nb * (nb + 1) // 2) * m
    base = sums[forms[0]]
    for f in forms:
        t = float(np.median(res[f]))
        print(json.dumps({"form": f, "kernel": "k_syrk_i8r" if f == 0 else "k_syrk_i8w", "n": n, "m": m,
                          "median_ms": t, "all_ms": res[f], "moduli": R, "int8_tops": ops / t / 1e9,
                          "frac_int8_peak": ops / t / 1e9 / 5000.0, "f64_equiv_tflops": n * (n + 1) * m / t / 1e9,
                          "tiles_equal_form0": sums[f] == base}), flush=True)


if __name__ == "__main__":
    main()
