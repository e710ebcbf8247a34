"""Experiment: k_snp_stats of block k+1 on the aux stream beside block k's decode (bench.py
--overlap-stats) vs the serial stats -> decode order, in ONE process on the SAME buffers, so output
placement is not a variable.  Alternates the two orders over rounds; per order
prints the mean step time over --blocks blocks of 2048 SNPs at 500k iids and the rate in SNPs/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-iid", type=int, default=500_000)
    p.add_argument("--block", type=int, default=2048)
    p.add_argument("--blocks", type=int, default=48)
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--out-ld", type=int, default=0, help="F-order column pitch in floats (0 = tight)")
    p.add_argument("--miss", type=float, default=0.01)
    a = p.parse_args()
    n, B = a.n_iid, a.block
    m = B * a.blocks
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = max(a.out_ld, (n + 15) // 16 * 16) // 16 * 16
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, 7, a.miss)
    out = bench.Dev(N, B * ld * 4)
    lut, stats = bench.Dev(N, 2 * B * 16), bench.Dev(N, 2 * B * 8)
    sev = bench.Events(N, 4)
    rec = [False, False]

    def step(overlap):
        for k in range(a.blocks):
            src = packed.at(k * B * pitch)
            if not overlap:
                N.call("snpmi_dev_snp_stats", src, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
                N.call("snpmi_dev_decode", src, pitch, n, B, lut.p, N.DT_F32, 0, out.p, ld)
                continue
            sl = k & 1
            if rec[sl]:
                N.call("snpmi_stream_wait_event", sev.ev[2 + sl], 2)
            N.call("snpmi_set_stream", 2)
            N.call("snpmi_dev_snp_stats", src, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
                   stats.at(sl * B * 8), lut.at(sl * B * 16))
            N.call("snpmi_set_stream", 0)
            sev.record(sl, 2)
            N.call("snpmi_stream_wait_event", sev.ev[sl], 0)
            N.call("snpmi_dev_decode", src, pitch, n, B, lut.at(sl * B * 16), N.DT_F32, 0, out.p, ld)
            sev.record(2 + sl)
            rec[sl] = True
        N.call("snpmi_stream_sync")

    # parity of the two orders: the last block's output is the same
    res = {}
    for ov in (False, True):
        step(ov)
        last = np.empty(n, dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(last), out.at((B - 1) * ld * 4), n * 4)
        res[ov] = last
    assert np.array_equal(res[False], res[True]), "overlap changes the output"
    times = {False: [], True: []}
    for r in range(a.rounds):
        for ov in ((False, True) if r % 2 == 0 else (True, False)):
            t0 = time.perf_counter()
            step(ov)
            times[ov].append(time.perf_counter() - t0)
    for ov in (False, True):
        t = np.array(times[ov])
        print(json.dumps({"overlap_stats": ov, "n_iid": n, "block": B, "blocks": a.blocks, "ld": ld,
                          "mean_ms_per_block": float(t.mean() / a.blocks * 1e3),
                          "min_ms_per_block": float(t.min() / a.blocks * 1e3),
                          "snps_per_s": float(m / t.mean())}), flush=True)


if __name__ == "__main__":
    main()
