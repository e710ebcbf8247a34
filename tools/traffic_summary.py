"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE) into per-launch HBM traffic.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16-B-per-lane streaming stores; both counters are in KiB.  The bf16x3 SYRK (k_syrk_bf3) reads
4-B-per-lane packed codes (64-B runs) and 16-B LUT rows, an access width the guide leaves
uncalibrated: its FETCH_SIZE is reported raw (x1), marked "read_scale": 1.
Usage: python tools/traffic_summary.py <prof_dir> <out.json> [dec_n,dec_block grm_n,grm_snps_per_launch]
"""
import collections
import csv
import json
import os
import sys

KERNELS = {"k_decode_std_lds_f32": "k_decode_std_lds_f32", "k_decode_f<float, 4>": "k_decode_f<float>", "k_decode_f<float": "k_decode_f<float>",
           "f32k::k_syrk<true": "f32k::k_syrk<true>", "k_syrk256<1, false>": "f32w::k_syrk256",
           "k_syrk256<1, true>": "f32w::k_syrk256<local>", "k_syrk256d<false": "f32w::k_syrk256d",
           "k_syrk256d<true": "f32w::k_syrk256d<local>", "k_snp_stats<float>": "k_snp_stats<float>",
           "k_syrk_bf3<false": "f32w::k_syrk_bf3", "k_syrk_bf3<true": "f32w::k_syrk_bf3<local>",
           "k_syrk_h2<false": "f32w::k_syrk_h2", "k_syrk_h2<true": "f32w::k_syrk_h2<local>",
           "k_syrk_h2s<false": "f32w::k_syrk_h2s", "k_syrk_h2s<true": "f32w::k_syrk_h2s<local>",
           "k_std_cols_f<float": "k_std_cols_f<float>", "k_diag_sq": "k_diag_sq"}


def short(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def load(path, counter):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        s = short(r["Kernel_Name"])
        if s and r["Counter_Name"] == counter:
            by[s].append(float(r["Counter_Value"]) * 1024.0)
    return by


def main(prof, out, dec_cfg=(500000, 2048), grm_cfg=(50000, 10000), std_cfg=(50000, 100000)):
    res = {}
    for leg in ("dec", "grm", "std"):
        if not os.path.isdir(os.path.join(prof, leg + "_FETCH_SIZE")):
            continue
        f = load(os.path.join(prof, leg + "_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
        w = load(os.path.join(prof, leg + "_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
        for k in f:
            # full launches only: the largest write volume (drops the partial tail block)
            wv = sorted(w.get(k, [0.0]))
            fv = sorted(f[k])
            full_w = [x for x in wv if x >= 0.95 * wv[-1]]
            full_f = [x for x in fv if x >= 0.95 * fv[-1]]
            scale = 1.0 if ("bf3" in k or "h2" in k) else 2.0
            read_b = scale * sum(full_f) / len(full_f)
            write_b = sum(full_w) / len(full_w)
            res.setdefault(k, {})[leg] = {"read_bytes": read_b, "write_bytes": write_b,
                                          "traffic_bytes": read_b + write_b, "launches": len(fv),
                                          "read_scale": scale}
    res["_config"] = {"dec": list(dec_cfg), "grm": list(grm_cfg), "std": list(std_cfg)}  # the script's settings
    res["_source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/profile.sh); "
                      "read = 2*FETCH_SIZE (gfx950 correction), per full launch")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    cfg = [tuple(int(x) for x in a.split(",")) for a in sys.argv[3:6]]
    main(sys.argv[1], sys.argv[2], *cfg)
