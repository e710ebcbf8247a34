"""configs[3] (cfg4) at its FULL size against the f64 oracle: 50,000 iids x 500,000 SNPs -- bench.py's
cfg4 input (same device generator, seed, missing rate) -- through shard.ShardedGrm in launches of
<= 65536 SNPs, as the bench's `grm` / `grm_f64` legs run it; 16 K rows (0..7 and 8 random) vs the
oracle's f64 products over all 500k SNPs (tools/check_cfg4_full.py; ~25 s on the box, the oracle
on 16 host threads).  Bars: f32 within 2e-6 of max diag (measured 5.6e-7, profiles/r04j), f64
within 1e-12 (measured 9.7e-16: the CRT path's integer products are exact)."""
import importlib.util
import os

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cfg4_full_size_vs_oracle():
    spec = importlib.util.spec_from_file_location("check_cfg4_full", os.path.join(ROOT, "tools", "check_cfg4_full.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    r = mod.check()
    assert r["f32"]["max_abs_err_over_max_diag"] <= 2e-6, r
    assert r["f32"]["max_rel_err_diag"] <= 1e-6, r
    assert r["f64"]["max_abs_err_over_max_diag"] <= 1e-12, r
    assert r["f64"]["max_rel_err_diag"] <= 1e-12, r
