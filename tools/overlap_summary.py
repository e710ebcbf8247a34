"""Copy/kernel overlap from a rocprofv3 --kernel-trace --memory-copy-trace CSV pair.

For every host<->device copy lasting at least --min-us microseconds (the ROCm 7.2 copy trace has
no byte count): how much of its interval ran while a kernel was executing (union of kernel
intervals), per direction, plus totals.  Evidence that the copy stream overlaps
the compute stream (bench.py e2e leg, snpmi_bed_read_* / snpmi_grm_bed_* chunk pipelines).
Usage: python tools/overlap_summary.py <trace-dir> [--min-us 500]
"""
import bisect
import csv
import glob
import json
import os
import sys


def intervals(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        out.append((s, e, r))
    return out


def union(iv):
    iv = sorted((s, e) for s, e, _ in iv)
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    return merged


def covered(merged, starts, s, e):
    tot = 0
    i = max(0, bisect.bisect_right(starts, s) - 1)
    while i < len(merged) and merged[i][0] < e:
        a, b = merged[i]
        tot += max(0, min(b, e) - max(a, s))
        i += 1
    return tot


def main(d, min_us):
    kp = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    cp = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    kern = union(intervals(kp, "k"))
    starts = [a for a, _ in kern]
    rows = []
    for s, e, r in intervals(cp, "c"):
        if (e - s) < min_us * 1e3:
            continue
        ov = covered(kern, starts, s, e)
        rows.append({"direction": r.get("Direction", "").replace("MEMORY_COPY_", ""), "stream": r.get("Stream_Id"),
                     "us": (e - s) / 1e3, "overlapped_frac": ov / max(e - s, 1)})
    res = {}
    for dname in sorted(set(x["direction"] for x in rows)):
        sel = [x for x in rows if x["direction"] == dname]
        tot_t = sum(x["us"] for x in sel)
        res[dname] = {"copies": len(sel), "copy_us": tot_t,
                      "overlapped_frac_time_weighted": sum(x["us"] * x["overlapped_frac"] for x in sel) / tot_t,
                      "first": sel[:4]}
    # the other way round: how much of each kernel's time ran under a copy (kernels hidden by DMA)
    cop = union([(s, e, None) for s, e, r in intervals(cp, "c") if "DEVICE_TO_DEVICE" not in r.get("Direction", "")])
    cstarts = [a for a, _ in cop]
    byk = {}
    for s, e, r in intervals(kp, "k"):
        name = r["Kernel_Name"].replace("snpmi::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        k = byk.setdefault(name, [0, 0, 0])
        k[0] += 1
        k[1] += e - s
        k[2] += covered(cop, cstarts, s, e)
    res["kernels_under_copies"] = {n: {"launches": v[0], "us": v[1] / 1e3, "overlapped_frac": v[2] / max(v[1], 1)}
                                   for n, v in byk.items() if v[1] > 1e5}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], float(a[a.index("--min-us") + 1]) if "--min-us" in a else 500.0)
