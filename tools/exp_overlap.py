"""A/B in one process (same buffers): stats + decode serial on the compute stream vs the stats
pass of block k+1 on the copy stream beside the decode of block k (bench.py --stats-overlap).
500k iids, 2048-SNP blocks over --n-sid SNPs resident in HBM; prints ms per block for each mode."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-iid", type=int, default=500_000)
    ap.add_argument("--n-sid", type=int, default=200_704)
    ap.add_argument("--block", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    n, B, m = a.n_iid, a.block, a.n_sid
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, 5, 0.01)
    luts = [bench.Dev(N, B * 16), bench.Dev(N, B * 16)]
    stats, out = bench.Dev(N, B * 8), bench.Dev(N, B * ld * 4)
    sync = bench.Events(N, 4)
    nblk = (m + B - 1) // B

    def serial():
        for k in range(nblk):
            s0 = k * B
            c = min(B, m - s0)
            N.call("snpmi_dev_snp_stats", packed.at(s0 * pitch), pitch, n, c, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
                   stats.p, luts[0].p)
            N.call("snpmi_dev_decode", packed.at(s0 * pitch), pitch, n, c, luts[0].p, N.DT_F32, 0, out.p, ld)

    def stats_on_copy(k):
        s0, s = k * B, k & 1
        if k >= 2:
            N.call("snpmi_stream_wait_event", sync.ev[2 + s], 1)
        N.call("snpmi_dev_snp_stats_on", packed.at(s0 * pitch), pitch, n, min(B, m - s0), 0, N.STD_UNIT, 0.0, 0.0,
               0, N.DT_F32, stats.p, luts[s].p, 1)
        sync.record(s, on_copy=1)

    def overlapped():
        stats_on_copy(0)
        for k in range(nblk):
            if k + 1 < nblk:
                stats_on_copy(k + 1)
            s0, s = k * B, k & 1
            N.call("snpmi_stream_wait_event", sync.ev[s], 0)
            N.call("snpmi_dev_decode", packed.at(s0 * pitch), pitch, n, min(B, m - s0), luts[s].p, N.DT_F32, 0,
                   out.p, ld)
            sync.record(2 + s)

    res = {"serial": [], "overlap": []}
    for r in range(a.rounds + 1):
        for name, fn in (("serial", serial), ("overlap", overlapped)):
            N.call("snpmi_stream_sync")
            t0 = time.perf_counter()
            fn()
            N.call("snpmi_stream_sync")
            if r > 0:
                res[name].append((time.perf_counter() - t0) / nblk * 1e3)
    for name, v in res.items():
        print(json.dumps({"mode": name, "ms_per_block": sorted(v)[len(v) // 2], "all": [round(x, 4) for x in v],
                          "n_iid": n, "n_sid": m, "block": B}), flush=True)


if __name__ == "__main__":
    main()
