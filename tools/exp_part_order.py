"""cfg5 part-kernel block order A/B (hook part_order: 0 = 64-block supertiles, 1 = triangular
order, 2 = 16-block supertiles; keyed 0 / 67 / 16 below): HIP-event time of snpmi_dev_syrk_packed_part on one SnpGen-shaped
block of --m SNPs at --n iids, part 0 of 8, alternating rounds, and sampled blocks compared bit
for bit.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pysnptools_amd import _native as N

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    n, m, P = a.n, a.m, a.parts
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    lut, stats = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    nloc = N.lib().snpmi_grm_part_blocks(n, 0, P)
    blocks = bench.Dev(N, nloc * 256 * 256 * 4)
    bench.synth(N, packed.p, pitch, n, 0, m, 77, 0.218)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    ev = bench.Events(N, 2)
    picks = sorted({0, 1, nloc // 3, nloc // 2, nloc - 2, nloc - 1})
    res, samples = {0: [], 67: [], 16: []}, {}
    for r in range(a.rounds + 1):
        for v in (67, 16, 0):
            N.call("snpmi_set_kernel_variant", b"part_order", {0: 0, 67: 1, 16: 2}[v])
            ev.record(0)
            N.call("snpmi_dev_syrk_packed_part", packed.p, pitch, n, m, lut.p, 0, P, blocks.p, 0)
            ev.record(1)
            t = ev.ms(0, 1)
            N.call("snpmi_set_kernel_variant", b"part_order", 0)
            if r:  # round 0 = warm-up (code objects, order table)
                res[v].append(t)
            s = np.empty((len(picks), 256, 256), dtype=np.float32)
            for k, b in enumerate(picks):
                N.call("snpmi_memcpy_d2h", N.ptr(s[k]), blocks.at(b * 256 * 256 * 4), 256 * 256 * 4)
            samples[v] = s
    flops = n * (n + 1) * m / P
    print(json.dumps({"n": n, "m": m, "parts": P, "local_blocks": nloc,
                      "supertile64_ms": res[0], "supertile16_ms": res[16], "triangular_ms": res[67],
                      "supertile64_TF": flops / (min(res[0]) * 1e-3) / 1e12,
                      "supertile16_TF": flops / (min(res[16]) * 1e-3) / 1e12,
                      "triangular_TF": flops / (min(res[67]) * 1e-3) / 1e12,
                      "speedup_64_vs_triangular": min(res[67]) / min(res[0]),
                      "speedup_64_vs_16": min(res[16]) / min(res[0]),
                      "sampled_blocks_bit_equal": bool(np.array_equal(samples[0], samples[67]) and
                                                       np.array_equal(samples[16], samples[67]))}), flush=True)
    ev.destroy()
    for d in (packed, lut, stats, blocks):
        d.free()


if __name__ == "__main__":
    main()
