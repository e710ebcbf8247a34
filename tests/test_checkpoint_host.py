"""Host logic of pysnptools_amd/checkpoint.py without a GPU: the fingerprint names everything that
changes K (file identity, sizes, dtype, block size, standardizer, subsets, trained stats), and a
checkpoint whose fingerprint differs is refused before any device call."""
import json
import os

import numpy as np
import pytest

from pysnptools_amd import checkpoint as C


def _meta(path, **kw):
    args = dict(bed_path=path, n=10, m=20, dtype=np.float32, block_size=5, kind=1, a=np.nan, b=np.nan,
                use_stats=False, rows=None, cols=None, count_a1=False, stats_in=None)
    args.update(kw)
    return C._fingerprint(**args)


def test_fingerprint_tracks_what_changes_k(tmp_path):
    bed = tmp_path / "x.bed"
    bed.write_bytes(b"\x6c\x1b\x01" + bytes(20))
    base = _meta(str(bed))
    assert json.loads(json.dumps(base)) == base  # survives the JSON round trip unchanged
    for kw in (dict(dtype=np.float64), dict(block_size=6), dict(kind=2, a=1.0, b=25.0), dict(count_a1=True),
               dict(rows=np.arange(5)), dict(cols=np.arange(3)), dict(use_stats=True),
               dict(stats_in=np.ones((20, 2), dtype=np.float32))):
        assert _meta(str(bed), **kw) != base, kw
    bed.write_bytes(b"\x6c\x1b\x01" + bytes(21))  # the file changed
    assert _meta(str(bed)) != base


def test_foreign_checkpoint_is_refused_before_any_device_call(tmp_path):
    bed = tmp_path / "x.bed"
    bed.write_bytes(b"\x6c\x1b\x01" + bytes(20))
    ck = str(tmp_path / "ck")
    with open(ck + ".json", "w") as f:
        json.dump(dict(_meta(str(bed), block_size=7), next_block=2), f)
    with pytest.raises(ValueError, match="another GRM"):
        C._restore(ck, _meta(str(bed)), np.float32)
    assert C._restore(str(tmp_path / "none"), _meta(str(bed)), np.float32) is None
    assert os.path.exists(ck + ".json")  # a refused checkpoint is left in place


def test_settings_only_difference_names_the_setting(tmp_path):
    """A checkpoint of the same GRM written under other kernel settings (here the exact-diagonal
    switch, which changes f32 K bits) is refused with an error naming the settings; one written
    before the settings were recorded likewise."""
    bed = tmp_path / "x.bed"
    bed.write_bytes(b"\x6c\x1b\x01" + bytes(20))
    meta = _meta(str(bed))
    assert set(meta["settings"]) == {"f32_seg", "f32_diag", "f32_syrk"}
    ck = str(tmp_path / "ck")
    other = dict(meta, settings=dict(meta["settings"], f32_diag=1 - meta["settings"]["f32_diag"]))
    with open(ck + ".json", "w") as f:
        json.dump(dict(other, next_block=2), f)
    with pytest.raises(ValueError, match="other GRM kernel settings"):
        C._restore(ck, meta, np.float32)
    legacy = {k: v for k, v in meta.items() if k != "settings"}
    with open(ck + ".json", "w") as f:
        json.dump(dict(legacy, next_block=2), f)
    with pytest.raises(ValueError, match="none recorded"):
        C._restore(ck, meta, np.float32)
