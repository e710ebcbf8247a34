"""Summarise tools/run_r05_ab_libs.sh output: per variant the k_syrk_h2 FETCH/WRITE GB per launch and
the bench grm leg seconds / roofline fraction.  Usage: python tools/ab_summary.py gpurun_out/<tag>"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for v in sorted(x for x in os.listdir(d) if os.path.isdir(os.path.join(d, x))):
    row = [v]
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(d, v, "grm_" + C, "run_counter_collection.csv")
        if os.path.exists(f):
            row.append("%s %s" % (C[:5], [round(float(r["Counter_Value"]) * 1024 / 1e9, 2)
                                          for r in csv.DictReader(open(f)) if "k_syrk_h2" in r["Kernel_Name"]]))
    ts = []
    for f in sorted(glob.glob(os.path.join(d, "t_%s_*.json" % v))):
        try:
            g = json.loads(open(f).read().strip().splitlines()[-1])["grm"]
            ts.append("%.4f s / %.4f" % (g["seconds"], g["roofline"]["frac"]))
        except Exception as e:  # noqa: BLE001
            ts.append(repr(e)[:60])
    print(" | ".join(row + ts))
