"""bench.py's multi-GPU plans on one GPU (no RCCL): each leg is run as every rank of a world of
2 / 3 / 8 in turn (a stand-in for the Dist control plane without collectives), and the per-rank
results must add up to the single-rank run -- the SNP shards of the decode leg cover the matrix
once, and the per-rank partial K tiles summed ELEMENTWISE equal the single-rank tiles (what the
RCCL reduce would produce; a tile-placement or shard-offset bug that kept the trace would fail).
Small shapes; the kernels are the real ones."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402

pytestmark = pytest.mark.gpu


class FakeDist:
    def __init__(self, rank, world):
        self.rank, self.world, self.rccl, self.n_gpus = rank, world, False, 1
        self.can_reduce = False
        self.local_rank, self.device = rank, 0

    def barrier(self):
        pass

    def max(self, x):
        return x


def _args(*extra):
    return bench.parse(["--n-iid", "4099", "--n-sid", "20000", "--block", "2048", "--grm-iid", "5000",
                        "--grm-sid", "23000", "--grm-block", "5000", "--steps", "1", "--warmup", "0",
                        "--skip-cpu"] + list(extra))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_decode_leg_shards_cover_the_matrix(world):
    args = _args()
    seen = []
    for r in range(world):
        res = bench.leg_standardize(N, args, FakeDist(r, world))
        lo, hi = bench.shard(args.n_sid, r, world)
        assert res["m"] == hi - lo
        seen.append((lo, hi))
    assert seen[0][0] == 0 and seen[-1][1] == args.n_sid
    assert all(a[1] == b[0] for a, b in zip(seen, seen[1:]))


def _tiles_to_k(tiles, n):
    """Full symmetric n x n K (f64) from the upper-triangle 128x128 tile buffer."""
    nt = (n + 127) // 128
    K = np.zeros((nt * 128, nt * 128))
    t = tiles.reshape(-1, 128, 128)
    for tj in range(nt):
        for ti in range(tj + 1):
            blk = t[tj * (tj + 1) // 2 + ti]
            K[ti * 128:(ti + 1) * 128, tj * 128:(tj + 1) * 128] = blk
            K[tj * 128:(tj + 1) * 128, ti * 128:(ti + 1) * 128] = blk.T
    return K[:n, :n]


_WHOLE = {}


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_grm_leg_partial_tiles_sum_to_whole(world, dtype):
    """Every rank's tiles (its contiguous SNP span through shard.ShardedGrm) summed elementwise ==
    the single-rank tiles, and the single-rank K == the oracle's on a SNP sample (parity leg)."""
    args = _args()
    if dtype not in _WHOLE:
        _WHOLE[dtype] = bench.leg_grm(N, args, FakeDist(0, 1), dtype, keep_tiles=True)
    whole = _WHOLE[dtype]
    parts = [bench.leg_grm(N, args, FakeDist(r, world), dtype, keep_tiles=True) for r in range(world)]
    assert sum(p["my_m"] for p in parts) == args.grm_sid
    assert [p["collective"] for p in parts] == ["none"] * world
    n = args.grm_iid
    Kw = _tiles_to_k(whole["tiles"].astype(np.float64), n)
    Ks = sum(_tiles_to_k(p["tiles"].astype(np.float64), n) for p in parts)
    scale = np.abs(np.diag(Kw)).max()
    tol = 2e-6 if dtype == "f32" else 1e-12
    err = np.abs(Ks - Kw).max() / scale
    assert err <= tol, err
    # the sum is not dominated by one rank: every rank contributed a non-trivial partial K
    assert all(np.abs(np.diag(_tiles_to_k(p["tiles"].astype(np.float64), n))).max() > 0.01 * scale for p in parts)
    # trace(K) of Unit-standardized SNPs = the observed entries of the polymorphic SNPs <= N * M
    assert 0 < whole["trace"] <= n * args.grm_sid * (1 + 1e-5)
    assert abs(np.trace(Kw) - whole["trace"]) <= 1e-6 * whole["trace"]


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_grm_leg_parity_vs_oracle(dtype):
    args = bench.parse(["--grm-iid", "5000", "--grm-sid", "3000", "--steps", "1", "--warmup", "0"])
    r = bench.leg_grm(N, args, FakeDist(0, 1), dtype)
    p = bench.grm_parity(args, *r["parity_sample"], tol=1e-5 if dtype == "f32" else 1e-10)
    assert p["pass"], p


@pytest.mark.parametrize("collective", ["reduce", "allreduce"])
def test_bench_with_rccl_communicator_world1(collective):
    """The whole bench (every leg, parity checks, JSON line) with an RCCL communicator at world size
    1 (--force-rccl): the collective calls of the N > 1 plan run with their real buffers and sizes
    -- the in-place all-reduce of the K tiles (f32 and f64), the packed-block all-gather of the
    partitioned GRM, the RCCL barrier and max-over-ranks -- and the line keeps its schema.  The K
    tiles go through ncclReduce onto rank 0 (default) or ncclAllReduce (--grm-collective)."""
    import json
    import subprocess

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--force-rccl", "--steps", "1", "--warmup", "0",
           "--n-iid", "4099", "--n-sid", "6000", "--grm-iid", "5000", "--grm-sid", "12000", "--grm-block", "5000",
           "--grm5-iid", "20000", "--grm5-sid", "4096", "--grm5-block", "2048", "--e2e-sid", "4096", "--e2e-passes", "1",
           "--cpu-seconds", "0.2", "--grm-collective", collective, "--beta-iid", "5001", "--beta-sid", "6000",
           "--file-iid", "3001", "--file-sid", "5000", "--cpu-grm-iid", "3000", "--cpu-grm-sid", "64"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout  # stdout carries the JSON line only (RCCL banners go to stderr)
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["parity"]["bit_exact"]
    assert 0 < d["roofline"]["frac_tight"] and d["cpu_baseline"]["cpu_counts"]["usable"] >= 1
    assert d["roofline"]["layout"].startswith("tight") and d["roofline"]["frac"] == d["roofline"]["frac_tight"]
    assert len(d["parity"]["input_sha256"]) == 64 and len(d["beta"]["parity"]["input_sha256"]) == 64
    assert d["beta"]["parity"]["pass"] and d["beta"]["snps_per_s"] > 0, d["beta"]
    f = d["file"]
    assert f["read_kernel_f32"]["parity"]["pass"], f["read_kernel_f32"]["parity"]
    assert f["read_hbm"]["parity"]["bit_exact"] and f["read_standardize_beta"]["parity"]["pass"], f
    assert f["read_standardize_unit"]["parity"]["pass"], f["read_standardize_unit"]
    assert d["grm"]["cpu_baseline"]["projected_seconds"] > 0
    for k in ("grm", "grm_f64"):
        assert d[k]["parity"]["pass"], d[k]["parity"]
        assert d[k]["allreduce_ms"] > 0
        assert d[k]["collective"] == ("ncclReduce(sum, root 0)" if collective == "reduce" else "ncclAllReduce(sum)")
    g5 = d["grm5"]
    assert g5["parity"]["pass"] and g5["parity"]["stats_bit_exact"], g5["parity"]
    # 4096 SNPs: a 512-SNP first block, then 2048-SNP blocks (shard.block_spans)
    assert g5["blocks"] == 3 and g5["seconds"] > 0 and g5["gpu_busy_seconds"] > 0
    assert "+ RCCL all-gather" in g5["workload"]


def test_decode_leg_wide_block_buffer_same_values():
    """A 32 MB-pitch block buffer (--out-ld 8000000; the default timed layout is tight, the spread
    pitch is the side figure) holds the same values as tight columns: 131072 iids x 2048-SNP blocks
    (1 GB), first 512 columns compared bit for bit, and against the oracle's decode + one-pass Unit;
    each run times the other layout on the side."""
    from oracle import oracle as O

    base = ["--n-iid", "131072", "--n-sid", "4096", "--block", "2048", "--steps", "1", "--warmup", "0"]
    wide = bench.leg_standardize(N, bench.parse(base + ["--out-ld", "8000000"]), FakeDist(0, 1))
    tight = bench.leg_standardize(N, bench.parse(base + ["--out-ld", "0"]), FakeDist(0, 1))
    assert wide["out_ld"] == 8_000_000 and tight["out_ld"] == 131072
    assert wide["side_ld"] == 131072 and tight["side_ld"] == 8_000_000
    assert wide["side_gbs"] > 0 and tight["side_gbs"] > 0
    assert np.array_equal(wide["gpu_cols"], tight["gpu_cols"])
    n, ncols = 131072, wide["gpu_cols"].shape[0]
    body = np.ascontiguousarray(wide["sample"][:, :(n + 3) // 4]).reshape(-1)
    ref, _ = O.decode_standardize(body, n, ncols, dtype=np.float32)
    assert np.array_equal(wide["gpu_cols"][:, :n].T, ref)
