"""End-to-end (file-backed, PCIe-inclusive) timings of the mirrored API on one GPU.

Writes a synthetic cfg4-shaped .bed (default 50k iids x 100k SNPs, SnpGen MAF curve, 1%
missing; packed bytes generated on the GPU and written once), then times what a PySnpTools
user calls:
  * Bed(...).read_kernel(Unit(), dtype=float32)  -> snpmi_grm_bed_f32 (gather from the page
    cache, H2D of packed codes, fused decode+standardize+SYRK, K copied back)
  * Bed(...)[:, :B].read(dtype=float32)           -> snpmi_bed_read_f32 (values cross PCIe)
and reports them beside the device-resident figures bench.py measures.  Prints JSON lines.
Usage: python tools/bench_file.py [--n-iid 50000] [--n-sid 100000] [--dir /tmp]
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_bed(N, path, n, m, seed):
    from bench import Dev, synth

    pitch = N.lib().snpmi_packed_pitch(n)
    bpc = (n + 3) // 4
    step = max(1, (1 << 30) // pitch)
    dev = Dev(N, pitch * min(step, m))
    host = np.empty((min(step, m), pitch), dtype=np.uint8)
    with open(path + ".bed", "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        for s0 in range(0, m, step):
            cnt = min(step, m - s0)
            synth(N, dev.p, pitch, n, s0, cnt, seed, 0.01)
            N.call("snpmi_memcpy_d2h", N.ptr(host), dev.p, cnt * pitch)
            f.write(np.ascontiguousarray(host[:cnt, :bpc]).tobytes())
    dev.free()
    with open(path + ".fam", "w") as f:
        f.write("".join("f%d i%d 0 0 0 0\n" % (i, i) for i in range(n)))
    with open(path + ".bim", "w") as f:
        f.write("".join("1\ts%d\t0\t%d\tA\tC\n" % (j, j + 1) for j in range(m)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-iid", type=int, default=50_000)
    ap.add_argument("--n-sid", type=int, default=100_000)
    ap.add_argument("--read-block", type=int, default=10_000)
    ap.add_argument("--dir", default=tempfile.gettempdir())
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--part-iid", type=int, default=100_000, help="cfg5 rehearsal: iids of the partitioned leg")
    ap.add_argument("--part-sid", type=int, default=20_000)
    ap.add_argument("--part-world", type=int, default=8)
    args = ap.parse_args()
    from pysnptools_amd import _native as N
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    n, m = args.n_iid, args.n_sid
    with tempfile.TemporaryDirectory(dir=args.dir) as d:
        base = os.path.join(d, "cfg4")
        t0 = time.perf_counter()
        write_bed(N, base, n, m, args.seed)
        t_write = time.perf_counter() - t0
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid  # metadata outside the timed region
        # warm the page cache and the library (first call allocates scratch)
        bed[:, :2000].read_kernel(Unit(), dtype=np.float32)
        t0 = time.perf_counter()
        K = bed.read_kernel(Unit(), dtype=np.float32)
        t_grm = time.perf_counter() - t0
        flops = n * (n + 1) * m
        print(json.dumps({"bench": "file-backed GRM (Bed.read_kernel, f32)", "n_iid": n, "n_sid": m,
                          "seconds": t_grm, "TFLOPs_end_to_end": flops / t_grm / 1e12,
                          "packed_GB": m * ((n + 3) // 4) / 1e9, "K_GB": n * n * 4 / 1e9,
                          "bed_write_s": t_write, "trace": float(np.trace(K.val))}), flush=True)
        del K
        # the same with K left in HBM (ARRAY_MODULE=hbm: no 10 GB copy-out, util/__init__.py:652-730 seam)
        os.environ["ARRAY_MODULE"] = "hbm"
        bed[:, :2000].read_kernel(Unit(), dtype=np.float32)
        t0 = time.perf_counter()
        Kd = bed.read_kernel(Unit(), dtype=np.float32)
        t_grm_d = time.perf_counter() - t0
        kd = Kd.val[17, 17]
        print(json.dumps({"bench": "file-backed GRM (Bed.read_kernel, f32), K resident in HBM (ARRAY_MODULE=hbm)",
                          "n_iid": n, "n_sid": m, "seconds": t_grm_d, "TFLOPs_end_to_end": flops / t_grm_d / 1e12,
                          "K_GB": n * n * 4 / 1e9, "K17_17": float(kd)}), flush=True)
        t0 = time.perf_counter()
        Kd.standardize()  # DiagKtoN in place in HBM
        t_diag = time.perf_counter() - t0
        print(json.dumps({"bench": "KernelData.standardize(DiagKtoN()) on the HBM-resident K", "n_iid": n,
                          "seconds": t_diag, "GB_per_s": 2 * n * n * 4 / t_diag / 1e9}), flush=True)
        del Kd
        B = args.read_block
        bed[:, :B].read(dtype=np.float32)
        t0 = time.perf_counter()
        vd = bed[:, :B].read(dtype=np.float32)
        t_read_d = time.perf_counter() - t0
        t0 = time.perf_counter()
        vd.standardize(Unit())
        t_std_d = time.perf_counter() - t0
        print(json.dumps({"bench": "file-backed read into HBM (Bed[:, :B].read, f32, F, ARRAY_MODULE=hbm) + "
                                   "standardize in place", "n_iid": n, "snps": B, "read_seconds": t_read_d,
                          "read_snps_per_s": B / t_read_d, "packed_GB_per_s": B * ((n + 3) // 4) / t_read_d / 1e9,
                          "standardize_seconds": t_std_d}), flush=True)
        del vd
        os.environ.pop("ARRAY_MODULE")
        # the reference's default dtype (snpreader.py:528 read_kernel(..., dtype=np.float64))
        t0 = time.perf_counter()
        K = bed.read_kernel(Unit())
        t_grm64 = time.perf_counter() - t0
        print(json.dumps({"bench": "file-backed GRM (Bed.read_kernel, f64 default)", "n_iid": n, "n_sid": m,
                          "seconds": t_grm64, "TFLOPs_end_to_end": flops / t_grm64 / 1e12, "K_GB": n * n * 8 / 1e9}),
              flush=True)
        del K
        B = args.read_block
        sub = bed[:, :B]
        sub.read(dtype=np.float32)
        t0 = time.perf_counter()
        v = sub.read(dtype=np.float32)
        t_read = time.perf_counter() - t0
        print(json.dumps({"bench": "file-backed read (Bed[:, :B].read, f32, F)", "n_iid": n, "snps": B,
                          "seconds": t_read, "snps_per_s": B / t_read, "out_GB_per_s": v.val.nbytes / t_read / 1e9}),
              flush=True)
        # in-memory SnpData.standardize (host array -> GPU -> host, in place)
        v.standardize(Unit())
        t0 = time.perf_counter()
        v.standardize(Unit())
        t_std = time.perf_counter() - t0
        print(json.dumps({"bench": "SnpData.standardize(Unit()) in memory, f32", "n_iid": n, "snps": B,
                          "seconds": t_std, "snps_per_s": B / t_std,
                          "GB_per_s_each_way": v.val.nbytes / t_std / 1e9}), flush=True)
    # cfg5 rehearsal from a file: K partitioned over W ranks (shard.grm_partitioned); rank 0's
    # share timed on this GPU (every rank streams the whole file and owns ~1/W of the blocks)
    from pysnptools_amd.shard import grm_partitioned

    n5, m5, W = args.part_iid, args.part_sid, args.part_world
    with tempfile.TemporaryDirectory(dir=args.dir) as d:
        base = os.path.join(d, "cfg5")
        write_bed(N, base, n5, m5, args.seed + 1)
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid
        grm_partitioned(bed[:, :1000], Unit(), 0, W)  # warm-up (scratch, page cache of the head)
        t0 = time.perf_counter()
        blocks, coords, _ = grm_partitioned(bed, Unit(), 0, W)
        t5 = time.perf_counter() - t0
        flops = n5 * (n5 + 1) * m5 / W
        print(json.dumps({"bench": "file-backed partitioned GRM (cfg5 form, shard.grm_partitioned), rank 0 of %d, "
                                   "blocks copied to host memory" % W,
                          "n_iid": n5, "n_sid": m5, "seconds": t5, "blocks_on_rank": len(coords),
                          "K_GB_on_rank": blocks.nbytes / 1e9, "TFLOPs_end_to_end_per_rank": flops / t5 / 1e12}),
              flush=True)
        # the same with the blocks kept in HBM (accumulated in place): the streamed work alone,
        # which is what scales with N^2 M (the one-off copy-out scales with N^2 only)
        grm_partitioned(bed[:, :1000], Unit(), 0, W, out="hbm")
        t0 = time.perf_counter()
        hb, coords, _ = grm_partitioned(bed, Unit(), 0, W, out="hbm")
        t6 = time.perf_counter() - t0
        print(json.dumps({"bench": "file-backed partitioned GRM (cfg5 form), rank 0 of %d, blocks resident in HBM" % W,
                          "n_iid": n5, "n_sid": m5, "seconds": t6, "TFLOPs_end_to_end_per_rank": flops / t6 / 1e12,
                          "copy_out_s": t5 - t6,
                          "projected_500k_x_1M_s_per_rank": t6 * (500_000 / n5) ** 2 * (1_000_000 / m5),
                          "projection": "streamed time x (N ratio)^2 x (M ratio); K blocks of a rank at 500k: 62.6 GB, "
                                        "kept in HBM"}), flush=True)


if __name__ == "__main__":
    main()
