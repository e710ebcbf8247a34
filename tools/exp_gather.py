"""A/B of the host gather behind file reads (api.hip gather_columns, hook "gather": 0 = memcpy from
the mmap, 1 = pread per column) on a synthetic 50k x 100k .bed in the page cache: the full
Bed.read(float32, xp='hbm') (1.25 GB of packed codes cross PCIe), Bed[:, :10000].read(xp='hbm')
and Bed.read_kernel(Unit(), float32) with K in HBM; alternating variants, one JSON line per run."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pysnptools_amd import _native as N
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    n, m = 50_000, 100_000
    os.environ["ARRAY_MODULE"] = "hbm"
    with tempfile.TemporaryDirectory() as d:
        base = os.path.join(d, "cfg")
        bench.write_bed(N, base, n, m, 304, 0.218)
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid
        bed.read(dtype=np.float32)  # warm: scratch at full size
        bed.read_kernel(Unit(), dtype=np.float32)
        for rnd in range(3):
            for v in (0, 1):
                N.call("snpmi_set_kernel_variant", b"gather", v)
                t0 = time.perf_counter()
                x = bed.read(dtype=np.float32)
                t_full = time.perf_counter() - t0
                del x
                t0 = time.perf_counter()
                x = bed[:, :10000].read(dtype=np.float32)
                t_10k = time.perf_counter() - t0
                del x
                t0 = time.perf_counter()
                K = bed.read_kernel(Unit(), dtype=np.float32)
                t_k = time.perf_counter() - t0
                del K
                print(json.dumps({"round": rnd, "gather": ["mmap", "pread"][v], "read_full_s": t_full,
                                  "packed_GBps_full": m * ((n + 3) // 4) / t_full / 1e9, "read_10k_s": t_10k,
                                  "read_kernel_f32_s": t_k}), flush=True)
        N.call("snpmi_set_kernel_variant", b"gather", 0)


if __name__ == "__main__":
    main()
