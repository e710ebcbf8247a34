"""C-ABI checks that need no GPU: libsnpmi.so loads, exports every symbol include/snpmi.h
declares, and fails loudly (no CPU fallback) when no device is present."""
import os
import re

import numpy as np
import pytest

from conftest import DATA, ROOT, has_gpu_device
from pysnptools_amd import _native as N


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "snpmi.h")).read()
    return sorted(set(re.findall(r"\b(snpmi_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = N.lib()
    decl = declared_symbols()
    assert len(decl) >= 40
    for name in decl:
        assert hasattr(lib, name), name
    # the ctypes binding covers exactly the declared ABI
    assert sorted(N.symbols()) == decl


def test_exports_match_nm():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = sorted(set(re.findall(r" T (snpmi_[a-z0-9_]+)", out)))
    assert exported == declared_symbols()


def test_pure_helpers():
    assert N.lib().snpmi_version() == 1
    assert N.lib().snpmi_packed_pitch(300) == 128
    assert N.lib().snpmi_packed_pitch(500000) % 64 == 0
    assert N.lib().snpmi_grm_tile_bytes(300, N.DT_F32) == 6 * 128 * 128 * 4
    assert N.lib().snpmi_grm_tile_bytes(129, N.DT_F64) == 3 * 128 * 128 * 8


@pytest.mark.skipif(has_gpu_device(), reason="checks the no-device error path")
def test_no_cpu_fallback_without_device():
    assert N.device_count() == 0
    from pysnptools_amd.snpreader import Bed

    with pytest.raises(N.NativeError, match="no HIP device"):
        Bed(os.path.join(DATA, "n300.bed"), count_A1=False).read()
    v = np.ones((3, 2))
    with pytest.raises(N.NativeError):
        N.call("snpmi_standardize_f64", N.ptr(v), 3, 2, 0, 0, 0.0, 0.0, 1, 0, N.ptr(np.empty((2, 2))), 1)


def test_format_errors_are_host_side():
    """Bad magic / size mismatch are reported before any device work (bed.py:137-145)."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.bed")
        with open(p, "wb") as f:
            f.write(bytes([0x6C, 0x1B, 0x00]) + bytes(10))
        with pytest.raises(ValueError, match="SNP-major"):
            N.call("snpmi_bed_check", p.encode(), 4, 10)
        with open(p, "wb") as f:
            f.write(bytes([1, 2, 3]))
        with pytest.raises(ValueError, match="magic"):
            N.call("snpmi_bed_check", p.encode(), 4, 0)
        with open(p, "wb") as f:
            f.write(bytes([0x6C, 0x1B, 0x01]) + bytes(9))
        with pytest.raises(ValueError, match="size"):
            N.call("snpmi_bed_check", p.encode(), 4, 10)
        N.call("snpmi_bed_check", p.encode(), 4, 9)
    with pytest.raises(IOError):
        N.call("snpmi_bed_check", b"/nonexistent/file.bed", 1, 1)
