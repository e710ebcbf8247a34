"""cfg4 at its full size against the f64 oracle: 50,000 iids x 500,000 SNPs (bench.py's cfg4 input:
the same device generator, seed and missing rate), the f32 (fp16x2 + SegFlush + exact diagonal)
and f64 (int8 CRT) GRMs through shard.ShardedGrm in launches of <= 65536 SNPs, exactly as the
bench's `grm` / `grm_f64` legs run them; K rows 0..7 and 8 random rows vs the oracle's f64
Z_rows . Z^T accumulated over 8192-SNP chunks (stats over every iid).  Prints one JSON line.
Test infrastructure: the oracle is the checker here, never the thing measured."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def check():
    """Returns the JSON dict (see the module doc)."""
    import bench
    from oracle import oracle as O
    from pysnptools_amd import _native as N
    from pysnptools_amd.shard import ShardedGrm

    n, m = 50_000, 500_000
    args = bench.parse([])
    assert (args.grm_iid, args.grm_sid) == (n, m)
    rows = np.unique(np.concatenate([np.arange(8), np.random.default_rng(3).integers(8, n, 8)])).astype(np.uint64)
    R = len(rows)
    pitch = N.lib().snpmi_packed_pitch(n)
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, args.seed + 100, 0.01)  # = leg_grm's input at N = 1
    got = {}
    for name, npdt, code, es in (("f32", np.float32, N.DT_F32, 4), ("f64", np.float64, N.DT_F64, 8)):
        stats = bench.Dev(N, m * 2 * es)
        g = ShardedGrm(n, npdt, None, "none")
        t0 = time.perf_counter()
        g.add_packed(packed.p, pitch, m, N.STD_UNIT, 0.0, 0.0, 0, stats.p)
        N.call("snpmi_stream_sync")
        sec = time.perf_counter() - t0
        t, _ = g.tiles()
        dri, dout = bench.Dev(N, R * 8), bench.Dev(N, R * n * es)
        N.call("snpmi_memcpy_h2d", dri.p, N.ptr(rows), rows.nbytes)
        N.call("snpmi_dev_grm_extract", t, n, code, dri.p, R, None, n, 1, 1.0, dout.p)
        K = np.empty((R, n), dtype=npdt)
        N.call("snpmi_memcpy_d2h", N.ptr(K), dout.p, K.nbytes)
        g.abort()
        for d in (stats, dri, dout):
            d.free()
        got[name] = (K.astype(np.float64), sec)
        print("[check] %s GRM %.2f s" % (name, sec), file=sys.stderr, flush=True)
    ref = np.zeros((R, n))
    chunk = 8192
    host = np.empty((chunk, pitch), dtype=np.uint8)
    t0 = time.perf_counter()
    ri = rows.astype(np.int64)
    for s0 in range(0, m, chunk):
        c = min(chunk, m - s0)
        N.call("snpmi_memcpy_d2h", N.ptr(host), packed.at(s0 * pitch), c * pitch)
        body = np.ascontiguousarray(host[:c, :(n + 3) // 4]).reshape(-1)
        Z, _ = O.decode_standardize(body, n, c, dtype=np.float64, num_threads=16)
        ref += Z[ri].dot(Z.T)
        if (s0 // chunk) % 8 == 7:
            print("[check] oracle %d / %d SNPs, %.0f s" % (s0 + c, m, time.perf_counter() - t0), file=sys.stderr,
                  flush=True)
    packed.free()
    scale = float(np.abs(ref[np.arange(R), ri]).max())
    out = {"check": "cfg4 full size (50k iids x 500k SNPs, bench.py's cfg4 input), K rows %s vs the f64 oracle"
                    % ri.tolist(), "oracle_seconds": time.perf_counter() - t0, "max_diag": scale}
    for name, (K, sec) in got.items():
        err = np.abs(K - ref)
        out[name] = {"grm_seconds": sec, "max_abs_err_over_max_diag": float(err.max() / scale),
                     "max_rel_err_diag": float(np.max(np.abs(K[np.arange(R), ri] - ref[np.arange(R), ri]) /
                                                      ref[np.arange(R), ri])),
                     "rms_err_over_max_diag": float(np.sqrt(np.mean(err ** 2)) / scale)}
    return out


def main():
    print(json.dumps(check()), flush=True)


if __name__ == "__main__":
    main()
