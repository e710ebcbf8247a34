"""Why does the cfg5 part kernel run ~4% below the replicated one?  Same n = 150,000 iids (enough blocks per part that the last round of workgroups does not dominate), same
codes: k_syrk_h2<LOCAL> over all blocks (parts = 1) vs over part 0 of 8 (every 8th block of the
supertile order, as cfg5), time per block, alternating rounds.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pysnptools_amd import _native as N

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 150_000
    m, rounds = 16_384, 3
    parts = (1, 8) if n <= 200_000 else (8,)  # 500k x 1 part = 500 GB of blocks
    pitch = N.lib().snpmi_packed_pitch(n)
    p = bench.Dev(N, pitch * m)
    bench.synth(N, p.p, pitch, n, 0, m, 5, 0.218)
    lut, st = bench.Dev(N, m * 16), bench.Dev(N, m * 8)
    N.call("snpmi_dev_snp_stats", p.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, st.p, lut.p)
    res = {}
    ev = bench.Events(N, 2)
    blocks = {P: N.lib().snpmi_grm_part_blocks(n, 0, P) for P in parts}
    bufs = {P: bench.Dev(N, blocks[P] * 256 * 256 * 4) for P in parts}
    for r in range(rounds + 1):
        for P in parts:
            ev.record(0)
            N.call("snpmi_dev_syrk_packed_part", p.p, pitch, n, m, lut.p, 0, P, bufs[P].p, 0)
            ev.record(1)
            if r:
                res.setdefault(P, []).append(ev.ms(0, 1))
    out = {"n": n, "m": m}
    for P in parts:
        us = min(res[P]) * 1e3 / blocks[P]
        out["parts%d" % P] = {"blocks": blocks[P], "ms": res[P], "us_per_block": us,
                              "TFLOPs": 2 * 256 * 256 * m / (us * 1e-6) / 1e12}
    if 1 in parts:
        out["part8_vs_all_per_block"] = out["parts8"]["us_per_block"] / out["parts1"]["us_per_block"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
