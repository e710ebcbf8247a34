"""Experiment: C-order decode (k_decode_c_reg<float>, 2048 SNPs x 500k iids) into row pitches of
2048 (tight) ... 32768 floats, alternating, one process: does spreading the rows over more HBM pages
help the C-order writes as the 32 MB column pitch helps the F-order decode?"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402

n, B = 500_000, 2048
pitch = N.lib().snpmi_packed_pitch(n)
packed = bench.Dev(N, pitch * B)
bench.synth(N, packed.p, pitch, n, 0, B, 1, 0.01)
lut, st = bench.Dev(N, B * 16), bench.Dev(N, B * 8)
N.call("snpmi_dev_snp_stats", packed.p, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
lds = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2048,4096,8192,16384,32768").split(",")]
ev = bench.Events(N, 2)
res = {ld: [] for ld in lds}
ref = None
for rnd in range(3):
    for ld in lds:
        out = bench.Dev(N, n * ld * 4)
        N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 1, out.p, ld)
        N.call("snpmi_stream_sync")
        ts = []
        for _ in range(6):
            ev.record(0)
            N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 1, out.p, ld)
            ev.record(1)
            N.call("snpmi_stream_sync")
            ts.append(ev.ms(0, 1))
        res[ld].append(float(np.median(ts)))
        if rnd == 0:  # rows 0..63 must not depend on the pitch
            rows = np.empty((64, B), dtype=np.float32)
            for i in range(64):
                N.call("snpmi_memcpy_d2h", N.ptr(rows[i]), out.at(i * ld * 4), B * 4)
            ref = rows if ref is None else ref
            assert np.array_equal(rows, ref)
        out.free()
nbytes = B * ((n + 3) // 4 + 4 * n)
for ld in lds:
    t = float(np.median(res[ld]))
    print(json.dumps({"kernel": "k_decode_c_reg<float>", "row_ld": ld, "median_ms": t, "per_round": res[ld],
                      "GBps": nbytes / t / 1e6, "frac_8TBs": nbytes / t / 1e6 / 8000}), flush=True)
