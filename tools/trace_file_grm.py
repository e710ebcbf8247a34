"""Time Bed(path).read_kernel(Unit(), dtype) (TF_DTYPE, default float32) with K in HBM (TF_HOST=1: K to NumPy) (the bench's `file` leg, the
reference's own call: snpreader.py:528-561,623-668) on a synthetic 50k x 100k .bed, with
host-side timestamps; run under rocprofv3 --kernel-trace --memory-copy-trace to see where the
wall time beyond the SYRK goes.  Prints one JSON line per call."""
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

    n, m = int(os.environ.get("TF_N", 50_000)), int(os.environ.get("TF_M", 100_000))
    dtype = np.dtype(os.environ.get("TF_DTYPE", "float32"))
    to_host = os.environ.get("TF_HOST", "0") == "1"  # K copied to a NumPy array instead of left in HBM
    with tempfile.TemporaryDirectory() as d:
        base = os.path.join(d, "cfg")
        bench.write_bed(N, base, n, m, 304, 0.218)
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid
        if not to_host:
            os.environ["ARRAY_MODULE"] = "hbm"
        bed[:, :2000].read_kernel(Unit(), dtype=dtype)
        for rep in range(3):
            t0 = time.perf_counter()
            K = bed.read_kernel(Unit(), dtype=dtype)
            t = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "dtype": dtype.name, "K_to_host": to_host, "seconds": t, "tflops": n * (n + 1) * m / t / 1e12,
                              "t0_ns": time.perf_counter_ns()}), flush=True)
            del K


if __name__ == "__main__":
    main()
