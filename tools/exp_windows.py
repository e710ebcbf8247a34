"""Experiment: decode speed along one large allocation.

Times the 2048-SNP decode (500k iids, f32 F order) into 4 GB windows of a --big-gb allocation at
--step-gb offsets, and into a "spread" layout (column pitch --spread-ld floats, so the same 2048
columns land all over the allocation).  If a window's speed is a property of where its physical
pages sit (e.g. unevenly spread over the HBM stacks), the spread layout should run at the rate of
the best windows."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-iid", type=int, default=500_000)
    p.add_argument("--block", type=int, default=2048)
    p.add_argument("--big-gb", type=float, default=64.0)
    p.add_argument("--step-gb", type=float, default=2.0)
    p.add_argument("--spread-ld", default="8000000,4000000,1000000")
    p.add_argument("--reps", type=int, default=4)
    p.add_argument("--rounds", type=int, default=2)
    a = p.parse_args()
    n, B = a.n_iid, a.block
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = bench.Dev(N, pitch * B)
    bench.synth(N, packed.p, pitch, n, 0, B, 1, 0.01)
    big_bytes = int(a.big_gb * (1 << 30))
    big = bench.Dev(N, big_bytes)
    lut, stats = bench.Dev(N, B * 16), bench.Dev(N, B * 8)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    ev = bench.Events(N, 2)
    win = B * ld * 4
    cases = []
    off = 0
    step = int(a.step_gb * (1 << 30))
    while off + win <= big_bytes:
        cases.append(("window@%.1fGB" % (off / (1 << 30)), off, ld))
        off += step
    for sl in (int(x) for x in a.spread_ld.split(",") if x):
        if (B - 1) * sl * 4 + n * 4 <= big_bytes:
            cases.append(("spread_ld%d" % sl, 0, sl))
    for name, o, l in cases:  # first touch
        N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, big.at(o), l)
    N.call("snpmi_stream_sync")
    t = {c[0]: [] for c in cases}
    for _ in range(a.rounds):
        for name, o, l in cases:
            ev.record(0)
            for _ in range(a.reps):
                N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, big.at(o), l)
            ev.record(1)
            N.call("snpmi_stream_sync")
            t[name].append(ev.ms(0, 1) / a.reps)
    nbytes = B * ((n + 3) // 4 + 4 * n)
    for name, o, l in cases:
        m = float(np.mean(t[name]))
        print(json.dumps({"case": name, "ld": l, "mean_ms": round(m, 4), "GBps": round(nbytes / (m * 1e-3) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
