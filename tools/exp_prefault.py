"""A/B of the host-K page pre-touch (api.hip HostPrefault, hook "prefault": 0 off, 1 on) on
Bed(path).read_kernel(Unit(), dtype) with K returned as a NumPy array (the reference's default
return, snpreader.py:623-668) on a synthetic 50k x 100k .bed; alternating, one JSON line per call.
The hook existed only for this A/B (no effect, profiles/r03j/host_k_prefault_ab.jsonl) and was removed
from the library afterwards; the script documents how the numbers were taken."""
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
    with tempfile.TemporaryDirectory() as d:
        base = os.path.join(d, "cfg")
        bench.write_bed(N, base, n, m, 304, 0.218)
        bed = Bed(base + ".bed", count_A1=False)
        bed.iid, bed.sid
        for dt in (np.float32, np.float64):
            bed.read_kernel(Unit(), dtype=dt)  # warm at full size
            for rnd in range(3):
                for v in (0, 1):
                    N.call("snpmi_set_kernel_variant", b"prefault", v)
                    t0 = time.perf_counter()
                    K = bed.read_kernel(Unit(), dtype=dt)
                    t = time.perf_counter() - t0
                    k0 = float(K.val[0, 0])
                    del K
                    print(json.dumps({"dtype": np.dtype(dt).name, "round": rnd, "prefault": v, "seconds": t,
                                      "K00": k0}), flush=True)
        N.call("snpmi_set_kernel_variant", b"prefault", 1)


if __name__ == "__main__":
    main()
