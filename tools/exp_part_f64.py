"""cfg5 f64 part SYRK (snpmi_dev_syrk_packed_part_f64: the CRT kernel over part 0 of P) at n iids x m
SNPs, for each syrk variant given (ubench library: 88 = the round-5 (blocks, moduli) grid, 0 = the
XCD-grouped moduli), alternating rounds; best ms and the K bits vs the first variant.
Usage: SNPMI_LIB=tools/libsnpmi_ubench.so python tools/exp_part_f64.py n m P v,v,... rounds"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import bench
    from pysnptools_amd import _native as N

    n, m, P = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    variants = [int(v) for v in sys.argv[4].split(",")]
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    pitch = N.lib().snpmi_packed_pitch(n)
    p = bench.Dev(N, pitch * m)
    bench.synth(N, p.p, pitch, n, 0, m, 5, 0.218)
    lut, st = bench.Dev(N, m * 32), bench.Dev(N, m * 16)
    N.call("snpmi_dev_snp_stats", p.p, pitch, n, m, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F64, st.p, lut.p)
    nloc = N.lib().snpmi_grm_part_blocks(n, 0, P)
    blocks = bench.Dev(N, nloc * 256 * 256 * 8)
    ev = bench.Events(N, 2)
    ms = {v: [] for v in variants}
    ref, same = None, {}
    for r in range(rounds):
        for v in variants:
            N.call("snpmi_set_kernel_variant", b"syrk", v)
            ev.record(0)
            N.call("snpmi_dev_syrk_packed_part_f64", p.p, pitch, n, m, lut.p, 0, P, blocks.p, 0)
            ev.record(1)
            ms[v].append(ev.ms(0, 1))
            if r == 0:
                chk = np.empty(1 << 20, dtype=np.float64)
                N.call("snpmi_memcpy_d2h", N.ptr(chk), blocks.p, chk.nbytes)
                ref = chk.copy() if ref is None else ref
                same[v] = bool(np.array_equal(chk.view(np.uint64), ref.view(np.uint64)))
    N.call("snpmi_set_kernel_variant", b"syrk", 0)
    for v in variants:
        print(json.dumps({"n": n, "m": m, "parts": P, "blocks": nloc, "variant": v, "ms": ms[v], "best_ms": min(ms[v]),
                          "bits_equal_first": same[v]}), flush=True)


if __name__ == "__main__":
    main()
