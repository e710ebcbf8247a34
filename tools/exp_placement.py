"""Experiment: does k_decode_f's rate depend on WHERE its 4 GB output buffer lives?

Round 1 saw the bench's decode land on discrete per-process levels (0.66 .. 0.79 ms per 2048-SNP
block at 500k iids); round 2 saw 0.598 ms in one process and 0.76 in the next on the same box.
This times the same decode (one 2048-SNP block, 500k iids, f32 F order) into several output
buffers of one process, interleaved over rounds, so placement is the only variable:
  hipMalloc 4 GB buffers (as bench.py), sub-ranges of one large buffer, and
  hipExtMallocWithFlags(hipDeviceMallocContiguous) buffers.
Prints one JSON line per buffer: mean / min ms per launch and GB/s.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-iid", type=int, default=500_000)
    p.add_argument("--block", type=int, default=2048)
    p.add_argument("--packed-gb", type=float, default=125.0)
    p.add_argument("--plain", type=int, default=6)
    p.add_argument("--sub", type=int, default=4)
    p.add_argument("--contig", type=int, default=2)
    p.add_argument("--ext-flags", default="", help="comma list of hipExtMallocWithFlags flags to add buffers for "
                                                   "(1 fine-grained, 3 uncached, 4 contiguous); --per-flag each")
    p.add_argument("--per-flag", type=int, default=2)
    p.add_argument("--outputs-first", action="store_true")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--variants", default="0", help="comma list of decode variants (ubench build: 21-23)")
    p.add_argument("--lds", default="", help="comma list of extra F-order column pitches (floats) to time")
    a = p.parse_args()
    n, B = a.n_iid, a.block
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    lds = [ld] + [int(x) for x in a.lds.split(",") if x]
    ob = B * max(lds) * 4  # every pitch fits every buffer
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    bufs = []

    def alloc_outputs():
        for i in range(a.plain):
            bufs.append(("hipMalloc_%d" % i, bench.Dev(N, ob).p))
        if a.sub:
            big = bench.Dev(N, ob * a.sub)
            for i in range(a.sub):
                bufs.append(("sub_%d" % i, ctypes.c_void_p(big.p.value + i * ob)))
        for i in range(a.contig):
            q = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(q), ctypes.c_size_t(ob), ctypes.c_uint(4))
            if rc == 0:
                bufs.append(("contiguous_%d" % i, q))
            else:
                print(json.dumps({"contiguous_alloc_rc": rc}), flush=True)
        for fl in [int(x) for x in a.ext_flags.split(",") if x]:
            for i in range(a.per_flag):
                q = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(q), ctypes.c_size_t(ob), ctypes.c_uint(fl))
                if rc == 0:
                    bufs.append(("flags%d_%d" % (fl, i), q))
                else:
                    print(json.dumps({"ext_flags": fl, "alloc_rc": rc}), flush=True)

    if a.outputs_first:
        alloc_outputs()
    packed = bench.Dev(N, int(a.packed_gb * 1e9) if a.packed_gb > 0 else pitch * B)
    bench.synth(N, packed.p, pitch, n, 0, B, 1, 0.01)
    if not a.outputs_first:
        alloc_outputs()
    lut, stats = bench.Dev(N, B * 16), bench.Dev(N, B * 8)
    N.call("snpmi_dev_snp_stats", packed.p, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
    ev = bench.Events(N, 2)
    variants = [int(v) for v in a.variants.split(",")]
    cases = [(name, q, v, l) for name, q in bufs for v in variants for l in lds]
    times = {c[:1] + c[2:]: [] for c in cases}
    for name, q in bufs:  # warm every buffer once (first-touch page mapping)
        N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, q, ld)
    N.call("snpmi_stream_sync")
    for r in range(a.rounds):
        for name, q, v, l in cases:
            if v >= 0:
                N.call("snpmi_set_kernel_variant", b"decode", v)
            ev.record(0)
            for _ in range(a.reps):
                if v < 0:  # variant -1: hipMemset of the same bytes (the fill ceiling on this buffer)
                    N.call("snpmi_dev_memset", q, 0, B * l * 4)
                else:
                    N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, q, l)
            ev.record(1)
            N.call("snpmi_stream_sync")
            times[(name, v, l)].append(ev.ms(0, 1) / a.reps)
    # parity: every variant's output (first, middle, last column of the first buffer) equals the
    # shipped kernel's
    q0 = bufs[0][1]
    ref = None
    cols = [0, B // 2, B - 1]
    for v in [0] + [x for x in variants if x >= 0 and x not in (23, 58, 59, 64, 65, 70, 71, 83, 87)]:  # store-only ablations
        N.call("snpmi_set_kernel_variant", b"decode", v)
        N.call("snpmi_dev_memset", q0, 0, B * ld * 4)
        N.call("snpmi_dev_decode", packed.p, pitch, n, B, lut.p, N.DT_F32, 0, q0, ld)
        got = np.empty((len(cols), n), dtype=np.float32)
        for i, c in enumerate(cols):
            N.call("snpmi_memcpy_d2h", N.ptr(got[i]), ctypes.c_void_p(q0.value + c * ld * 4), n * 4)
        if ref is None:
            ref = got
        elif not np.array_equal(got, ref):
            print(json.dumps({"variant": v, "parity": False}), flush=True)
            raise SystemExit(1)
    N.call("snpmi_set_kernel_variant", b"decode", 0)
    nbytes = B * ((n + 3) // 4 + 4 * n)
    for name, q, v, l in cases:
        t = np.array(times[(name, v, l)])
        print(json.dumps({"buf": name, "addr": hex(q.value), "variant": v, "ld": l,
                          "mean_ms": round(float(t.mean()), 4), "min_ms": round(float(t.min()), 4),
                          "max_ms": round(float(t.max()), 4), "GBps": round(nbytes / (t.mean() * 1e-3) / 1e9, 1),
                          "outputs_first": a.outputs_first}), flush=True)


if __name__ == "__main__":
    main()
