"""Does the packed column pitch slow the fp16x2 SYRK?  The cfg5 part kernel runs at ~4% fewer
TFLOP/s than the cfg4 kernel (profiles/r04r); one difference is the code-row stride (125 KB at
500k iids vs 12.5 KB at 50k).  Same kernel (snpmi_dev_syrk_packed, f32), n = 50,000 iids, the
same codes stored with the tight pitch and with a 10x pitch, alternating rounds, K compared.
Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pysnptools_amd import _native as N

    n, m, rounds = 50_000, 31_250, 4
    tight = N.lib().snpmi_packed_pitch(n)
    wide = tight * 10
    res = {}
    bufs = {}
    for name, pitch in (("tight", tight), ("wide", wide)):
        p = bench.Dev(N, pitch * m)
        bench.synth(N, p.p, pitch, n, 0, m, 5, 0.218)  # codes by (sid, iid): the same values at any pitch
        bufs[name] = (p, pitch)
    lut, st = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    tiles = bench.Dev(N, N.lib().snpmi_grm_tile_bytes(n, N.DT_F32))
    ev = bench.Events(N, 2)
    samples = {}
    for r in range(rounds + 1):
        for name, (p, pitch) in bufs.items():
            N.call("snpmi_dev_snp_stats", p.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
            ev.record(0)
            N.call("snpmi_dev_syrk_packed", p.p, pitch, n, m, lut.p, N.DT_F32, tiles.p, 0)
            ev.record(1)
            t = ev.ms(0, 1)
            if r:
                res.setdefault(name, []).append(t)
            s = np.empty(1 << 20, dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(s), tiles.p, s.nbytes)
            samples[name] = s
    fl = n * (n + 1) * m
    print(json.dumps({"n": n, "m": m, "pitch_tight": tight, "pitch_wide": wide, "tight_ms": res["tight"],
                      "wide_ms": res["wide"], "tight_TF": fl / min(res["tight"]) / 1e9,
                      "wide_TF": fl / min(res["wide"]) / 1e9, "slowdown": min(res["wide"]) / min(res["tight"]),
                      "sample_bit_equal": bool(np.array_equal(samples["tight"], samples["wide"]))}), flush=True)
    ev.destroy()
    for p, _ in bufs.values():
        p.free()
    for d in (lut, st, tiles):
        d.free()


if __name__ == "__main__":
    main()
