"""Summarise a rocprofv3 --pmc CSV pass per kernel: mean counter value per dispatch, the
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) and MFMA busy per SIMD.

Usage: python tools/pmc_summary.py <dir-with-run_counter_collection.csv> [--match substr ...]
Counter semantics (MI355X_MICROARCH.md §rocprofv3 PMC slots / cycle constants): SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed
over the chip's SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, match):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if match and not any(m in name for m in match):
            continue
        key = name.replace("snpmi::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r and "End_Timestamp" in r:
            dur.setdefault(key, {})[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        ds = list(dur.get(k, {}).values())
        if ds:
            t = sum(ds) / len(ds)
            e["kernel_s"] = t
            if "GRBM_GUI_ACTIVE" in e:
                e["clock_GHz"] = e["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
                if "SQ_VALU_MFMA_BUSY_CYCLES" in e:
                    e["mfma_busy_per_simd"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out[k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    args = sys.argv[1:]
    match = args[args.index("--match") + 1:] if "--match" in args else []
    main(args[0], match)
