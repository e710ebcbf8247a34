"""The package's multi-GPU paths at world 2 and 3 on ONE GPU, through the host
rehearsal group (tests/_gpu_dist_worker.py): every rank's result of the reference's own
entry points under an open group matches the f64 oracle ELEMENTWISE --

* cfg4: ``Bed.read_kernel`` (routed through ``shard.grm_sharded`` + the all-reduce of the K
  tiles, which the rehearsal group stages through host memory) in f32 and f64 on every rank;
  ``grm_sharded`` with a reduce onto rank 1 + DiagKtoN (K only on rank 1), stats merged by
  ``_sum_stats``;
* cfg5: ``shard.grm_partitioned`` under the group -- each rank reads 1/world of every SNP block
  from the .bed and the all-gather rebuilds it -- bit-identical to the same parts computed by one
  process without a group (``PartitionedGrm`` at world 1), and the parts reassembled equal the
  oracle; iid subset, Unit and Beta(1,25), blocks of 97 SNPs (partial last block, shares of 33 /
  49 columns)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import DATA, ROOT
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIX = {"n300": (300, 1015), "toydata": (500, 10000)}


def _oracle(name, beta=False, iid_index=None, diag=False):
    n, m = FIX[name]
    body = O.read_bed_bytes(os.path.join(DATA, name + ".bed"))
    Z = O.decode(body, n, m, iid_index=iid_index, dtype=np.float64)
    st = O.standardize_native(Z, is_beta=beta, a=1.0 if beta else np.nan, b=25.0 if beta else np.nan)
    return Z.dot(Z.T), st


def _err(K, ref):
    return np.abs(np.asarray(K, dtype=np.float64) - ref).max() / np.abs(np.diag(ref)).max()


@pytest.fixture(scope="module", params=[2, 3])
def world_run(request, tmp_path_factory):
    world = request.param
    out = tmp_path_factory.mktemp("w%d" % world)
    env = dict(os.environ, SNPMI_DIST_HOST="1", WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               SNPMI_RCCL_ID_FILE=str(out / "hub.id"))
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_gpu_dist_worker.py"), str(out)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    res = [p.communicate(timeout=240) for p in procs]
    assert all(p.returncode == 0 for p in procs), [e[-3000:] for _, e in res]
    return world, out


def _load(out, key, r):
    p = os.path.join(str(out), "%s.r%d.npy" % (key, r))
    return np.load(p) if os.path.exists(p) else None


@pytest.mark.parametrize("name", ["n300", "toydata"])
def test_read_kernel_under_group_every_rank(world_run, name):
    world, out = world_run
    Kref, _ = _oracle(name)
    for dt, tol in (("float32", 1e-5), ("float64", 1e-10)):
        Ks = [_load(out, "%s_readkernel_%s" % (name, dt), r) for r in range(world)]
        for r, K in enumerate(Ks):
            assert K is not None and K.dtype == np.dtype(dt), (r, dt)
            assert _err(K, Kref) <= tol, (r, dt, _err(K, Kref))
        for K in Ks[1:]:
            np.testing.assert_array_equal(K, Ks[0])  # the all-reduce leaves one K on every rank


@pytest.mark.parametrize("name", ["n300", "toydata"])
def test_reduce_onto_rank1_with_diag_k_to_n(world_run, name):
    world, out = world_run
    Kref, sref = _oracle(name)
    Kd, fref = O.diag_k_to_n(Kref)
    for r in range(world):
        K = _load(out, "%s_reduce1" % name, r)
        assert (K is not None) == (r == 1), r
        np.testing.assert_array_equal(_load(out, "%s_reduce1_stats" % name, r), sref)  # exact code-count stats
    assert _err(_load(out, "%s_reduce1" % name, 1), Kd) <= 1e-10
    f = float(_load(out, "%s_reduce1_factor" % name, 1)[0])
    assert abs(f - fref) <= 1e-12 * fref


@pytest.mark.parametrize("name", ["n300", "toydata"])
@pytest.mark.parametrize("beta", [False, True])
def test_partitioned_allgather_plan(world_run, name, beta):
    from pysnptools_amd import shard
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Beta, Unit
    from pysnptools_amd.standardizer.standardizer import _std_args

    world, out = world_run
    tag = "beta" if beta else "unit"
    n, m = FIX[name]
    rows = np.arange(n - 1, 0, -2)
    Kref, sref = _oracle(name, beta=beta, iid_index=rows)
    bed = Bed(os.path.join(DATA, name + ".bed"), count_A1=False)
    std = Beta(1, 25) if beta else Unit()
    parts = []
    for r in range(world):
        blocks = _load(out, "%s_part_%s_blocks" % (name, tag), r)
        coords = _load(out, "%s_part_%s_coords" % (name, tag), r)
        stats = _load(out, "%s_part_%s_stats" % (name, tag), r)
        np.testing.assert_array_equal(stats, sref.astype(np.float32))
        # one process, no group: the same part streamed whole (world-1 gather) -- bit-identical
        kind, a, b, _, _, _ = _std_args(std)
        b1, c1, s1 = shard._partitioned_bed(bed, rows, None, kind, a, b, False, None, None, r, world, 97, None, 4)
        np.testing.assert_array_equal(coords, c1)
        np.testing.assert_array_equal(blocks, b1)
        np.testing.assert_array_equal(stats, s1)
        parts.append((blocks, coords))
    K = shard.assemble_partitioned(parts, len(rows))
    assert _err(K, Kref) <= 1e-5
    # and the library's own single-process part path (snpmi_grm_part_bed_f32) agrees with the oracle
    b0, c0, _ = shard.grm_partitioned(bed[rows, :], std, rank=0, world=world)
    np.testing.assert_array_equal(c0, _load(out, "%s_part_%s_coords" % (name, tag), 0))
    K0 = shard.assemble_partitioned([(b0, c0)] + parts[1:], len(rows))
    assert _err(K0, Kref) <= 1e-5


@pytest.mark.parametrize("name", ["n300", "toydata"])
def test_partitioned_f64_under_the_group(world_run, name):
    """cfg5 in float64 (the reference's default dtype) under the group: each rank's f64 blocks equal
    the same part computed by one process, and the parts assembled match the f64 oracle within
    1e-12 of max diag."""
    from pysnptools_amd import shard
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    world, out = world_run
    n, m = FIX[name]
    rows = np.arange(n - 1, 0, -2)
    Kref, sref = _oracle(name, iid_index=rows)
    bed = Bed(os.path.join(DATA, name + ".bed"), count_A1=False)
    parts = []
    for r in range(world):
        blocks = _load(out, "%s_part_f64_blocks" % name, r)
        coords = _load(out, "%s_part_f64_coords" % name, r)
        np.testing.assert_array_equal(_load(out, "%s_part_f64_stats" % name, r), sref)
        b1, c1, _ = shard._partitioned_bed(bed, rows, None, 1, 0.0, 0.0, False, None, None, r, world, 97, None, 4,
                                           np.float64)
        np.testing.assert_array_equal(coords, c1)
        np.testing.assert_array_equal(blocks, b1)
        parts.append((blocks, coords))
    assert _err(shard.assemble_partitioned(parts, len(rows)), Kref) <= 1e-12


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_partitioned_many_blocks_under_the_group(world_run, dtype):
    """A 2300-iid K (9 x 9 blocks): every part of the world-2/3 plan owns blocks; the parts tile K
    once and assemble to the f64 oracle (f32 1e-5, f64 1e-12 of max diag)."""
    from _gpu_dist_worker import SYNTH
    from pysnptools_amd import shard

    world, out = world_run
    n, m = SYNTH
    body = O.read_bed_bytes(os.path.join(str(out), "synth.bed"))
    Z = O.decode(body, n, m, dtype=np.float64)
    O.standardize_native(Z)
    Kref = Z.dot(Z.T)
    parts = [(_load(out, "synth_part_%s_blocks" % dtype, r), _load(out, "synth_part_%s_coords" % dtype, r))
             for r in range(world)]
    assert all(len(b) for b, _ in parts)
    assert sum(len(c) for _, c in parts) == 45
    assert _err(shard.assemble_partitioned(parts, n), Kref) <= (1e-12 if dtype == "float64" else 1e-5)


@pytest.mark.parametrize("name", ["n300", "synth"])
def test_partitioned_k_through_the_kernelreader_api(world_run, name):
    """with K partitioned over the group (set_grm_partition("always")), the
    reference's KernelReader entry points -- SnpKernel(bed, Unit())[rows, cols].read(),
    Bed.read_kernel, SnpKernel._read_with_standardizing (DiagKtoN) -- return on EVERY rank the K the
    oracle computes (f32 <= 1e-5, f64 <= 1e-12 of max diag, elementwise), and the blocks written by
    PartitionedKernel.write and read back by PartitionedKernel.load serve the same sub-matrix."""
    from _gpu_dist_worker import SYNTH, pk_indices

    world, out = world_run
    if name == "n300":
        n, m = FIX[name]
        body = O.read_bed_bytes(os.path.join(DATA, name + ".bed"))
    else:
        n, m = SYNTH
        body = O.read_bed_bytes(os.path.join(str(out), "synth.bed"))
    Z = O.decode(body, n, m, dtype=np.float64)
    O.standardize_native(Z)
    Kref = Z.dot(Z.T)
    rows, cols = pk_indices(n)
    sub = Kref[np.ix_(rows, cols)]
    scale = np.abs(np.diag(Kref)).max()
    factor = n / np.trace(Kref)
    for r in range(world):
        for dt, tol in (("float32", 1e-5), ("float64", 1e-12)):
            got = _load(out, "%s_pk_sub_%s" % (name, dt), r)
            assert got.dtype == np.dtype(dt) and got.shape == sub.shape
            assert np.abs(got - sub).max() / scale <= tol, (r, dt)
            full = _load(out, "%s_pk_full_%s" % (name, dt), r)
            assert np.abs(full - Kref).max() / scale <= tol, (r, dt)
            assert np.array_equal(full, full.T)
        np.testing.assert_allclose(_load(out, "%s_pk_factor" % name, r)[0], factor, rtol=1e-13)
        assert np.abs(_load(out, "%s_pk_diag" % name, r) - Kref * factor).max() / (scale * factor) <= 1e-12
        np.testing.assert_array_equal(_load(out, "%s_pk_loaded" % name, r), _load(out, "%s_pk_sub_float32" % name, r))
