"""Experiment: the iid gather (snpmi_dev_repack, 500k -> 250k iids, 8192 SNPs) into destination column
pitches from tight (62.5 KB) to 8 MB, alternating in one process (does spreading the 0.5 GB of output
over more HBM pages help, as for the decode, DESIGN 3.1?).  Time = plan + gather (same plan cost)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402

n, m = 500_000, 8192
pitch = N.lib().snpmi_packed_pitch(n)
idx = np.arange(n - 1, -1, -2, dtype=np.uint64)
n_out = len(idx)
tight = N.lib().snpmi_packed_pitch(n_out)
packed = bench.Dev(N, pitch * m)
bench.synth(N, packed.p, pitch, n, 0, m, 3, 0.01)
didx = bench.Dev(N, n_out * 8)
N.call("snpmi_memcpy_h2d", didx.p, N.ptr(idx), idx.nbytes)
pitches = [tight, 1 << 20, 4 << 20, 8 << 20]
ev = bench.Events(N, 2)
res = {p: [] for p in pitches}
ref = None
for rnd in range(3):
    for p in pitches:
        dst = bench.Dev(N, p * m)
        N.call("snpmi_dev_repack", packed.p, pitch, n, didx.p, n_out, m, dst.p, p)
        N.call("snpmi_stream_sync")
        ts = []
        for _ in range(6):
            ev.record(0)
            N.call("snpmi_dev_repack", packed.p, pitch, n, didx.p, n_out, m, dst.p, p)
            ev.record(1)
            N.call("snpmi_stream_sync")
            ts.append(ev.ms(0, 1))
        res[p].append(float(np.median(ts)))
        if rnd == 0:
            cols = np.empty((16, (n_out + 3) // 4), dtype=np.uint8)
            for j in range(16):
                N.call("snpmi_memcpy_d2h", N.ptr(cols[j]), dst.at((m - 16 + j) * p), cols.shape[1])
            ref = cols if ref is None else ref
            assert np.array_equal(cols, ref)
        dst.free()
nbytes = m * ((n + 3) // 4 + (n_out + 3) // 4)
for p in pitches:
    t = float(np.median(res[p]))
    print(json.dumps({"kernel": "repack (plan + k_repack_win16)", "dst_pitch": p, "median_ms": t, "per_round": res[p],
                      "GBps": nbytes / t / 1e6}), flush=True)
