"""Time .fam/.bim metadata parsing at UK-Biobank shape.

Writes a synthetic 500k-line .fam and 1M-line .bim, then times
  * this build: Bed(...).iid / .sid / .pos through the threaded C parser (libsnpmi), and
  * the reference-style parse: pandas read_csv (whitespace, all columns as str) + the
    chrom map / float conversion of snpreader/bed.py:170-194 -- what bed-reader's Python
    metadata layer does.
Prints one JSON line.  Host-only (no GPU needed).
Usage: python tools/bench_meta.py [--n-iid 500000] [--n-sid 1000000] [--threads 16]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_files(d, n, m):
    rng = np.random.default_rng(0)
    fam = os.path.join(d, "u.fam")
    with open(fam, "w") as f:
        ids = np.arange(n) + 1000000
        f.write("".join("%d %d 0 0 %d -9\n" % (i, i, 1 + (i & 1)) for i in ids))
    bim = os.path.join(d, "u.bim")
    chrom = np.sort(rng.integers(1, 27, m))
    names = np.where(chrom == 23, "X", np.where(chrom == 26, "MT", chrom.astype(str)))
    bp = rng.integers(1, 250_000_000, m)
    with open(bim, "w") as f:
        f.write("".join("%s\trs%d\t0\t%d\tA\tG\n" % (names[j], j, bp[j]) for j in range(m)))
    open(os.path.join(d, "u.bed"), "wb").write(bytes([0x6C, 0x1B, 0x01]))
    return os.path.join(d, "u.bed"), fam, bim


def pandas_style(fam, bim):
    import pandas as pd

    t = pd.read_csv(fam, sep=r"\s+", header=None, dtype=str, keep_default_na=False, engine="c")
    iid = np.array([t[0].to_numpy(dtype=str), t[1].to_numpy(dtype=str)]).T
    b = pd.read_csv(bim, sep=r"\s+", header=None, dtype=str, keep_default_na=False, engine="c")
    sid = b[1].to_numpy(dtype=str)
    chrom = b[0].to_numpy(dtype=str).astype(object)
    for k, v in {"X": 23, "Y": 24, "XY": 25, "MT": 26}.items():
        chrom[chrom == k] = v
    pos = np.array([chrom.astype(float), b[2].to_numpy(dtype=str).astype(float),
                    b[3].to_numpy(dtype=str).astype(float)]).T
    pos[pos == 0] = np.nan
    return iid, sid, pos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-iid", type=int, default=500_000)
    ap.add_argument("--n-sid", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    from pysnptools_amd.snpreader import Bed

    with tempfile.TemporaryDirectory() as d:
        bed, fam, bim = write_files(d, args.n_iid, args.n_sid)
        t0 = time.perf_counter()
        b = Bed(bed, count_A1=False, num_threads=args.threads, skip_format_check=True)
        iid, sid, pos = b.iid, b.sid, b.pos
        t_c = time.perf_counter() - t0
        t0 = time.perf_counter()
        iid2, sid2, pos2 = pandas_style(fam, bim)
        t_p = time.perf_counter() - t0
        same = bool(np.array_equal(iid, iid2) and np.array_equal(sid, sid2) and
                    np.array_equal(pos, pos2, equal_nan=True))
        print(json.dumps({"bench": "fam/bim metadata", "n_iid": args.n_iid, "n_sid": args.n_sid,
                          "threads": args.threads, "c_parser_s": t_c, "pandas_reference_style_s": t_p,
                          "speedup": t_p / t_c, "identical": same,
                          "bytes": os.path.getsize(fam) + os.path.getsize(bim)}))


if __name__ == "__main__":
    main()
