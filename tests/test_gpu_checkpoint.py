"""Checkpoint / resume of a blocked GRM (pysnptools_amd/checkpoint.py; SURVEY.md section 5: the
reference's K lives only in RAM while snpreader.py:643-655 accumulates it).  A run interrupted
after 5 of 8 SNP blocks (checkpoints every 2) resumes from block 4 and gives K bit-identical to an
uninterrupted checkpointed run, within 1e-10 (f64) / 1e-5 (f32) of max diag of Bed.read_kernel,
with the same trained stats; a checkpoint of another GRM is refused."""
import json
import os

import numpy as np
import pytest

from pysnptools_amd import checkpoint as C
from pysnptools_amd.snpreader import Bed, SnpData
from pysnptools_amd.standardizer import Beta, Unit

pytestmark = pytest.mark.gpu


def _bed(tmp_path, n=1003, m=5000, seed=3):
    rng = np.random.default_rng(seed)
    v = rng.binomial(2, rng.uniform(0.02, 0.5, m), size=(n, m)).astype(np.float64)
    v[rng.random(v.shape) < 0.01] = np.nan
    return Bed.write(str(tmp_path / "g.bed"), SnpData(iid=[["f", str(i)] for i in range(n)],
                                                      sid=["s%d" % j for j in range(m)], val=v), count_A1=False)


@pytest.mark.parametrize("dtype,tol,std", [(np.float64, 1e-10, Unit()), (np.float32, 1e-5, Beta(1, 25))])
def test_interrupted_grm_resumes_bit_identical(tmp_path, dtype, tol, std):
    bed = _bed(tmp_path)
    reader = bed[::-1, 7:]  # subsets on both axes go through the index plumbing
    ref = reader.read_kernel(std, dtype=dtype).val
    full, tr_full = C.read_kernel_checkpointed(reader, std, str(tmp_path / "a"), block_size=700, every=2, dtype=dtype)
    assert not os.path.exists(str(tmp_path / "a.json"))  # removed on completion
    ck = str(tmp_path / "b")
    with pytest.raises(C._Interrupted):
        C.read_kernel_checkpointed(reader, std, ck, block_size=700, every=2, dtype=dtype, _stop_after=5)
    with open(ck + ".json") as f:
        assert json.load(f)["next_block"] == 4
    resumed, tr = C.read_kernel_checkpointed(reader, std, ck, block_size=700, every=2, dtype=dtype)
    assert np.array_equal(resumed.val, full.val)
    assert np.array_equal(tr.stats, tr_full.stats)
    scale = np.abs(np.diag(ref)).max()
    assert np.abs(resumed.val.astype(np.float64) - ref).max() <= tol * scale
    assert not os.path.exists(ck + ".json") and not [p for p in os.listdir(tmp_path) if p.startswith("b.g")]


def test_checkpoint_of_another_grm_is_refused(tmp_path):
    bed = _bed(tmp_path, n=300, m=1200)
    ck = str(tmp_path / "c")
    with pytest.raises(C._Interrupted):
        C.read_kernel_checkpointed(bed, Unit(), ck, block_size=200, every=1, _stop_after=2)
    with pytest.raises(ValueError, match="another GRM"):
        C.read_kernel_checkpointed(bed, Unit(), ck, block_size=300, every=1)


def test_crash_before_the_commit_resumes_from_the_previous_generation(tmp_path, monkeypatch):
    """The save after block 4 writes its tiles and stats, then dies before the JSON rename (the
    commit): the resumed run must start from the previous committed generation (block 2) and give
    the uninterrupted K -- never blocks 2..3 twice -- and a corrupted generation is refused."""
    bed = _bed(tmp_path, n=700, m=4200)
    full, tr_full = C.read_kernel_checkpointed(bed, Unit(), str(tmp_path / "a"), block_size=700, every=2)
    ck = str(tmp_path / "b")
    real_replace = os.replace

    def failing_replace(src, dst):
        if dst == ck + ".json" and os.path.exists(ck + ".g4.stats.npy"):
            raise OSError("simulated crash before the commit")
        return real_replace(src, dst)

    monkeypatch.setattr(C.os, "replace", failing_replace)
    with pytest.raises(OSError, match="simulated crash"):
        C.read_kernel_checkpointed(bed, Unit(), ck, block_size=700, every=2)
    monkeypatch.setattr(C.os, "replace", real_replace)
    with open(ck + ".json") as f:
        saved = json.load(f)
    assert saved["next_block"] == 2 and saved["files"]["tiles"] == "b.g2.tiles.npy"
    assert os.path.exists(ck + ".g4.tiles.npy")  # the uncommitted generation is ignored, not used
    resumed, tr = C.read_kernel_checkpointed(bed, Unit(), ck, block_size=700, every=2)
    assert np.array_equal(resumed.val, full.val)
    assert np.array_equal(tr.stats, tr_full.stats)
    assert not [p for p in os.listdir(tmp_path) if p.startswith("b.")]  # everything removed on completion
    # a committed generation whose file was damaged is refused, not silently used
    with pytest.raises(C._Interrupted):
        C.read_kernel_checkpointed(bed, Unit(), ck, block_size=700, every=2, _stop_after=3)
    with open(ck + ".g2.tiles.npy", "r+b") as f:
        f.seek(-8, 2)
        f.write(b"\x00" * 8)
    with pytest.raises(ValueError, match="hash"):
        C.read_kernel_checkpointed(bed, Unit(), ck, block_size=700, every=2)
