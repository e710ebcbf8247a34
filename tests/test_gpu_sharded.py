"""SNP-sharded GRM (shard.grm_sharded / ShardedGrm) through the package, on
the reference fixtures N300 (300 x 1015) and toydata (500 x 10000) against the f64 oracle.

* Simulated worlds 2 / 3 / 8 on one GPU (collective "none"): every rank's partial K and partial
  stats, summed, equal the single-process GRM and the oracle -- elementwise.
* A real RCCL communicator at world size 1 (dist.init_from_env(force_rccl=True)): ncclReduce and
  ncclAllReduce of the session tiles, the stats all-reduce, DiagKtoN on the root.
* Bed.read_kernel under an open process group routes through grm_sharded (the reference's own
  entry point, snpreader.py:528-561, reaching the multi-GPU path)."""
import os

import numpy as np
import pytest

from conftest import DATA
from oracle import oracle as O
from pysnptools_amd import dist as D
from pysnptools_amd import shard
from pysnptools_amd.snpreader import Bed
from pysnptools_amd.standardizer import Beta, Unit

pytestmark = pytest.mark.gpu

FIX = {"n300": (300, 1015), "toydata": (500, 10000)}


def _bed(name):
    return Bed(os.path.join(DATA, name + ".bed"), count_A1=False)


def _oracle(name, std, iid_index=None, sid_index=None):
    n, m = FIX[name]
    body = O.read_bed_bytes(os.path.join(DATA, name + ".bed"))
    sid = np.arange(m) if sid_index is None else np.asarray(sid_index)
    Z = O.decode(body, n, m, iid_index=iid_index, sid_index=sid, dtype=np.float64)
    beta = isinstance(std, Beta)
    st = O.standardize_native(Z, is_beta=beta, a=std.a if beta else np.nan, b=std.b if beta else np.nan)
    return Z.dot(Z.T), st


def _err(K, ref):
    return np.abs(np.asarray(K, dtype=np.float64) - ref).max() / np.abs(np.diag(ref)).max()


@pytest.mark.parametrize("name", ["n300", "toydata"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_simulated_ranks_sum_to_oracle(name, dtype, world):
    bed = _bed(name)
    Kref, sref = _oracle(name, Unit())
    Ksum = np.zeros_like(Kref)
    ssum = np.zeros_like(sref)
    for r in range(world):
        K, trained, f = shard.grm_sharded(bed, Unit(), rank=r, world=world, dtype=dtype, collective="none")
        assert K.dtype == dtype and np.isnan(f)
        lo, hi = shard.rank_span(bed.sid_count, r, world)
        st = trained.stats.astype(np.float64)
        assert np.all(st[:lo] == 0) and np.all(st[hi:] == 0)  # only the owned SNPs
        Ksum += K
        ssum += st
    tol = 1e-5 if dtype == np.float32 else 1e-10
    assert _err(Ksum, Kref) <= tol
    if dtype == np.float64:
        np.testing.assert_array_equal(ssum, sref)  # exact: stats from integer code counts
    else:
        np.testing.assert_array_equal(ssum.astype(np.float32), sref.astype(np.float32))


@pytest.mark.parametrize("world", [2, 3])
def test_simulated_ranks_subsets_beta(world):
    """iid + reversed sid subsets (test.py:820,842 shapes) and Beta(1,25)."""
    bed = _bed("n300")
    rows, cols = np.arange(299, 0, -2), np.arange(1014, 0, -3)
    Kref, sref = _oracle("n300", Beta(1, 25), iid_index=rows, sid_index=cols)
    Ksum, ssum = 0, 0
    for r in range(world):
        K, trained, _ = shard.grm_sharded(bed[rows, cols], Beta(1, 25), rank=r, world=world, dtype=np.float64,
                                          collective="none")
        Ksum = Ksum + K
        ssum = ssum + trained.stats
    assert _err(Ksum, Kref) <= 1e-10
    np.testing.assert_allclose(ssum, sref, rtol=0, atol=0)


def test_collective_needs_a_communicator():
    with pytest.raises(RuntimeError, match="RCCL communicator"):
        shard.grm_sharded(_bed("n300"), Unit(), rank=0, world=2, collective="reduce")


@pytest.fixture
def rccl1():
    d = D.init_from_env(force_rccl=True, env={"RANK": "0", "WORLD_SIZE": "1"}, timeout=120)
    try:
        yield d
    finally:
        d.close()
    assert D.current() is None


@pytest.mark.parametrize("collective", ["reduce", "allreduce"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_rccl_world1(rccl1, collective, dtype):
    assert rccl1.rccl and rccl1.n_gpus == 1 and rccl1.world == 1
    bed = _bed("toydata")
    Kref, sref = _oracle("toydata", Unit())
    K, trained, f = shard.grm_sharded(bed, Unit(), dtype=dtype, collective=collective, diag_k_to_n=True)
    Kd, fref = O.diag_k_to_n(Kref)
    assert abs(f - fref) <= 1e-6 * fref
    assert _err(K, Kd) <= (1e-5 if dtype == np.float32 else 1e-10)
    np.testing.assert_array_equal(trained.stats.astype(np.float64), sref.astype(dtype).astype(np.float64))
    # the golden GRM of the reference (toydata.kernel.npz, pysnptools/examples)
    gold = np.load(os.path.join(DATA, "toydata.kernel.npz"))["val"]
    assert _err(K / f, gold) <= (1e-5 if dtype == np.float32 else 1e-10)


def test_read_kernel_routes_through_the_process_group(rccl1):
    """Under an open process group of world > 1, Bed.read_kernel runs grm_sharded with an all-reduce.
    The communicator here has one rank, so a group that claims two ranks computes rank 0's half of
    the SNPs and the all-reduce over the one real rank leaves it as is: the half-SNP partial GRM."""
    fake = D.Dist(rank=0, world=2, local_rank=0, device=rccl1.device, rccl=True, n_gpus=1)
    saved = D._CURRENT
    D._CURRENT = fake
    try:
        K = _bed("n300").read_kernel(Unit(), dtype=np.float64).val
        Kp, _, _ = shard.grm_sharded(_bed("n300"), Unit(), rank=0, world=2, dtype=np.float64, collective="none")
    finally:
        D._CURRENT = saved
    lo, hi = shard.rank_span(1015, 0, 2)
    Kref, _ = _oracle("n300", Unit(), sid_index=np.arange(lo, hi))
    np.testing.assert_array_equal(K, Kp)
    assert _err(K, Kref) <= 1e-10
