"""k_snp_stats A/B (HBM read bound): per-launch time of the stats + LUT kernel on blocks of
--block packed SNP columns at --n iids, for decode-hook variants (0 = default, 7 = 4 loads in
flight, 9 = 16, 8 = 2 waves per SNP, 6 = 1 wave per SNP), interleaved rounds on distinct
blocks (a launch's input is not in the MALL from the previous launch).  JSON lines."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--block", type=int, default=2048)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,7,9,8")
    args = ap.parse_args()
    import bench
    from pysnptools_amd import _native as N

    n, B = args.n, args.block
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * B * args.blocks)
    bench.synth(N, packed.p, pitch, n, 0, B * args.blocks, 5, 0.01)
    lut, stats = bench.Dev(N, B * 16), bench.Dev(N, B * 8)
    ev = bench.Events(N, 2 * args.blocks)
    variants = [int(v) for v in args.variants.split(",")]
    res = {v: [] for v in variants}
    ref = None
    for r in range(args.rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"decode", v)
            for k in range(args.blocks):
                ev.record(2 * k)
                N.call("snpmi_dev_snp_stats", packed.at(k * B * pitch), pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0,
                       N.DT_F32, stats.p, lut.p)
                ev.record(2 * k + 1)
            N.call("snpmi_stream_sync")
            res[v].extend(ev.ms(2 * k, 2 * k + 1) for k in range(1, args.blocks))
            out = np.empty(B * 4, dtype=np.float32)
            N.call("snpmi_memcpy_d2h", N.ptr(out), lut.p, out.nbytes)
            if ref is None:
                ref = out
            assert np.array_equal(out, ref), "variant %d differs" % v
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    nbytes = B * ((n + 3) // 4)
    for v in variants:
        us = float(np.median(res[v])) * 1e3
        print(json.dumps({"bench": "k_snp_stats", "variant": v, "n": n, "block": B, "median_us": us,
                          "mean_us": float(np.mean(res[v])) * 1e3, "GBps": nbytes / (us * 1e-6) / 1e9,
                          "frac_of_8TBps": nbytes / (us * 1e-6) / 8e12}), flush=True)


if __name__ == "__main__":
    main()
