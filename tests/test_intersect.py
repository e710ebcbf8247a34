"""intersect_apply / intersect_ids (util/__init__.py:18-265) against vectors made by the
reference itself (tools/make_golden.py), plus KernelNpz persistence and the
intersect-before-standardize SnpKernel path."""
import os
import tempfile

import numpy as np
import pytest

from conftest import DATA, GOLDEN
from pysnptools_amd.util import intersect_apply, intersect_ids


def G():
    return np.load(os.path.join(GOLDEN, "intersect.npz"), allow_pickle=False)


def lists(g, tag):
    s = lambda k: g[k].astype(str)
    return {"a": [None, s("bed_iid"), s("pheno_iid"), s("cov_iid")], "b": [s("sub_iid"), s("bed_iid"), s("pheno_iid")],
            "c": [s("pheno_iid"), None, s("sub_iid")]}[tag]


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_intersect_ids_vs_reference(tag):
    g = G()
    assert np.array_equal(intersect_ids(lists(g, tag)), g["ind_" + tag])


@pytest.mark.parametrize("tag", ["a", "b", "c"])
@pytest.mark.parametrize("sort", [True, False])
def test_intersect_apply_tuples_vs_reference(tag, sort):
    g = G()
    ls = lists(g, tag)
    outs = intersect_apply([None if x is None else (np.arange(len(x)), x) for x in ls], sort_by_dataset=sort)
    got = np.array([o[0] for o in outs if o is not None])
    assert np.array_equal(got, g["out_%s_%d" % (tag, sort)])


def test_intersect_apply_mixed_formats_and_identity():
    from pysnptools_amd.snpreader import Bed

    g = G()
    bed = Bed(os.path.join(DATA, "n300.bed"), count_A1=False)
    pheno = {"iid": g["pheno_iid"].astype(str), "vals": g["pheno_val"].copy()}
    cov = (g["cov_val"], g["cov_iid"].astype(str))
    out_bed, out_pheno, out_cov = intersect_apply([bed, pheno, cov])
    assert np.array_equal(out_bed.iid, out_pheno["iid"]) and np.array_equal(out_bed.iid, out_cov[1])
    ref = g["out_a_1"]  # [None, bed, pheno, cov] sorted by the bed order
    assert np.array_equal(out_bed.iid, bed.iid[ref[0]])
    same = [bed, (np.zeros(300), bed.iid)]
    assert intersect_apply(same) is same


@pytest.mark.gpu
def test_snpkernel_intersect_before_standardize_and_kernelnpz():
    """The SnpKernel is reindexed BEFORE standardizing: its K equals the GRM of the iid-subset
    reader (decoded through the iid gather), not a slice of the full K; KernelNpz round trip."""
    from pysnptools_amd.kernelreader import KernelNpz, SnpKernel
    from pysnptools_amd.snpreader import Bed
    from pysnptools_amd.standardizer import Unit

    g = G()
    bed = Bed(os.path.join(DATA, "n300.bed"), count_A1=False)
    sub = (np.zeros(260), g["sub_iid"].astype(str))
    k_out, sub_out = intersect_apply([SnpKernel(bed, Unit()), sub])
    assert isinstance(k_out, SnpKernel)
    K = k_out.read().val
    pos = {tuple(x): i for i, x in enumerate(bed.iid.tolist())}
    rows = np.array([pos[tuple(x)] for x in k_out.iid.tolist()])
    assert np.array_equal(rows, np.sort(rows)) and len(rows) == 260  # sorted by the first dataset (bed)
    assert np.array_equal(sub_out[1], k_out.iid)
    Kref = bed[rows, :].read_kernel(Unit()).val
    np.testing.assert_allclose(K, Kref, rtol=0, atol=1e-9 * np.abs(np.diag(Kref)).max())
    assert not np.allclose(K, bed.read_kernel(Unit()).val[np.ix_(rows, rows)])
    with tempfile.TemporaryDirectory() as d:
        kd = k_out.read()
        p = os.path.join(d, "k.kernel.npz")
        back = KernelNpz.write(p, kd)
        assert back.iid0 is back.iid1 and np.array_equal(back.iid, kd.iid)
        assert np.array_equal(back.read().val, kd.val)
        assert np.array_equal(back[3:7].read().val, kd.val[3:7, 3:7])


@pytest.mark.gpu
def test_kernelnpz_reads_reference_fixture():
    from pysnptools_amd.kernelreader import KernelNpz

    src = "toydata.kernel.npz"
    path = os.path.join(DATA, src)
    if not os.path.exists(path):
        pytest.skip("fixture not copied")
    k = KernelNpz(path)
    assert k.iid_count == 500 and k.iid0 is k.iid1
    t = np.load(os.path.join(GOLDEN, "toydata.npz"), allow_pickle=False)
    assert np.array_equal(k.read().val[:64], t["K_rows"])
