"""Per-configuration kernel averages from a rocprofv3 kernel trace of the default bench
(tools/profile_r04.sh step 1): the decode's full launches, the cfg4 SYRK launches, the cfg5 timed
blocks, the dense standardize, the f64 CRT SYRK and the whole-K extraction.  Usage:
    python tools/trace_summary.py <run_kernel_trace.csv> <bench_under_rocprof.json> > summary.json"""
import csv
import json
import sys
from collections import Counter


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    for r in rows:
        r["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def named(s):
        return [r for r in rows if s in r["Kernel_Name"]]

    out = {}
    dec = named("k_decode_f<float")
    if dec:
        grid = Counter(r["Grid_Size_X"] for r in dec).most_common(1)[0][0]
        full = [r["us"] for r in dec if r["Grid_Size_X"] == grid]
        out["k_decode_f<float> launches of the most common grid (full launches)"] = {
            "launches": len(full), "avg_us": sum(full) / len(full), "grid_x": int(grid),
            "bench_roofline_avg_us": bench.get("roofline", {}).get("avg_launch_us")}
    g4 = named("k_syrk_h2s<false>")
    if g4:
        mx = max(r["us"] for r in g4)
        full = [r["us"] for r in g4 if r["us"] >= 0.8 * mx]
        g = bench.get("grm", {}).get("roofline", {})
        fl = g.get("per_launch_flops")
        avg = sum(full) / len(full)
        out["f32w::k_syrk_h2s<false> cfg4 launches (>= 0.8 of the longest)"] = {
            "launches": len(full), "avg_us": avg, "flops": fl, "TFLOPs": fl / (avg * 1e-6) / 1e12 if fl else None}
    g5 = named("k_syrk_h2s<true>")
    blocks = bench.get("grm5", {}).get("blocks")
    if g5 and blocks:
        timed = g5[-blocks:]
        busy = sum(r["us"] for r in timed) * 1e-6
        n5 = 500_000
        wl = bench["grm5"].get("workload", "")
        try:
            n5 = int(wl.split("cfg5: ")[1].split(" iid")[0])
            m5 = int(wl.split(" iid x ")[1].split(" SNP")[0])
        except (IndexError, ValueError):
            m5 = 1_000_000
        P = bench["grm5"].get("parts", 8)
        fl = n5 * (n5 + 1) * m5 / P
        out["f32w::k_syrk_h2s<true> cfg5 timed blocks (part 0 of %d)" % P] = {
            "launches": len(timed), "sum_s": busy, "avg_us_full_blocks": sorted(r["us"] for r in timed)[len(timed) // 2],
            "flops_part": fl, "TFLOPs": fl / busy / 1e12, "bench_seconds": bench["grm5"].get("seconds")}
    std = named("k_std_cols_f<float, 1024, 16, false>")
    if std:
        out["k_std_cols_f<float,1024,16,false> (file leg, 50k x 100k f32)"] = {
            "launches": len(std), "avg_us": sum(r["us"] for r in std) / len(std), "algorithmic_bytes": 40_000_000_000,
            "TBps": 40e9 / (sum(r["us"] for r in std) / len(std) * 1e-6) / 1e12}
    crt = named("k_syrk_i8w")
    if crt:
        out["k_syrk_i8w (f64 CRT) all launches"] = {"launches": len(crt), "avg_us": sum(r["us"] for r in crt) / len(crt)}
    ex = named("k_grm_extract_sym<double")
    if ex:
        out["k_grm_extract_sym<double,64> (50k K, file leg)"] = {"launches": len(ex),
                                                               "avg_us": sum(r["us"] for r in ex) / len(ex)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
