"""bench.py's multi-GPU plans on one GPU (no RCCL): each leg is run as every rank of a world of
2 / 3 / 8 in turn (a stand-in for the Dist control plane without collectives), and the per-rank
results must add up to the single-rank run -- the SNP shards of the decode leg cover the matrix
once, and the traces of the per-rank partial GRMs sum to the trace of the whole GRM (what the
RCCL all-reduce would produce).  Small shapes; the kernels are the real ones."""
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


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_grm_leg_partial_traces_sum_to_whole(world, dtype):
    args = _args()
    whole = bench.leg_grm(N, args, FakeDist(0, 1), dtype)
    parts = [bench.leg_grm(N, args, FakeDist(r, world), dtype) for r in range(world)]
    assert sum(p["my_m"] for p in parts) == args.grm_sid
    tol = 2e-6 if dtype == "f32" else 1e-12
    total = sum(p["trace"] for p in parts)
    assert abs(total - whole["trace"]) <= tol * abs(whole["trace"]), (total, whole["trace"])
    # trace(K) of Unit-standardized SNPs = the observed entries of the polymorphic SNPs <= N * M
    assert 0 < whole["trace"] <= args.grm_iid * args.grm_sid * (1 + 1e-5)


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
           "--grm5-iid", "20000", "--grm5-sid", "2048", "--e2e-sid", "4096", "--e2e-passes", "1",
           "--cpu-seconds", "0.2", "--grm-collective", collective]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout  # stdout carries the JSON line only (RCCL banners go to stderr)
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["parity"]["bit_exact"]
    for k in ("grm", "grm_f64"):
        assert d[k]["parity"]["pass"], d[k]["parity"]
        assert d[k]["allreduce_ms"] > 0
        assert d[k]["collective"] == ("ncclReduce(sum, root 0)" if collective == "reduce" else "ncclAllReduce(sum)")
    assert d["grm5"]["parity"]["pass"] and d["grm5"]["parity"]["gathered_block_bit_exact"]
    assert d["grm5"]["allgather_ms"] > 0
    st5 = d["grm5"]["streamed"]  # two blocks, the second upload under the first SYRK
    assert st5["blocks"] == 2 and len(st5["block_ms"]) == 2 and st5["seconds"] > 0
    assert "+ RCCL all-gather" in d["grm5"]["workload"]


def test_decode_leg_wide_block_buffer_same_values():
    """The decode leg's 32 MB-pitch block buffer (--out-ld 8000000, used for blocks >= 1 GB) holds
    the same values as tight columns: 131072 iids x 2048-SNP blocks (1 GB), first 512 columns
    compared bit for bit, and against the oracle's decode + one-pass Unit."""
    from oracle import oracle as O

    base = ["--n-iid", "131072", "--n-sid", "4096", "--block", "2048", "--steps", "1", "--warmup", "0"]
    wide = bench.leg_standardize(N, bench.parse(base + ["--out-ld", "8000000"]), FakeDist(0, 1))
    tight = bench.leg_standardize(N, bench.parse(base + ["--out-ld", "0"]), FakeDist(0, 1))
    assert wide["out_ld"] == 8_000_000 and tight["out_ld"] == 131072
    assert np.array_equal(wide["gpu_cols"], tight["gpu_cols"])
    n, ncols = 131072, wide["gpu_cols"].shape[0]
    body = np.ascontiguousarray(wide["sample"][:, :(n + 3) // 4]).reshape(-1)
    ref, _ = O.decode_standardize(body, n, ncols, dtype=np.float32)
    assert np.array_equal(wide["gpu_cols"][:, :n].T, ref)
