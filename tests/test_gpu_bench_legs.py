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
