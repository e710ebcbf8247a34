"""Empty selections through the GPU path, as the reference's NumPy path gives them: no SNPs -> an
(n, 0) value matrix and an all-zero n x n kernel (snpreader.py:623-634: `Z.dot(Z.T)` of an (n, 0)
block), no iids -> a (0, m) matrix and a 0 x 0 kernel.  float32 and the reference's default
float64 (the int8-residue path), through `read`, `read().standardize`, `read_kernel` and
`SnpKernel(...).read()`."""
import os

import numpy as np
import pytest

from conftest import DATA
from pysnptools_amd.kernelreader import SnpKernel
from pysnptools_amd.snpreader import Bed
from pysnptools_amd.standardizer import Unit

pytestmark = pytest.mark.gpu


def _bed():
    return Bed(os.path.join(DATA, "toydata.bed"), count_A1=False)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_no_snps(dtype):
    bed = _bed()
    n = bed.iid_count
    sub = bed[:, :0]
    assert sub.sid_count == 0
    v = sub.read(dtype=dtype).val
    assert v.shape == (n, 0) and v.dtype == dtype
    z = sub.read(dtype=dtype).standardize(Unit()).val
    assert z.shape == (n, 0)
    K = sub.read_kernel(Unit(), dtype=dtype).val
    assert K.shape == (n, n) and K.dtype == dtype and not K.any()
    K2 = SnpKernel(sub, Unit()).read(dtype=dtype).val
    assert K2.shape == (n, n) and not K2.any()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_no_iids(dtype):
    bed = _bed()
    m = bed.sid_count
    sub = bed[:0, :]
    assert sub.iid_count == 0
    v = sub.read(dtype=dtype).val
    assert v.shape == (0, m) and v.dtype == dtype
    K = sub.read_kernel(Unit(), dtype=dtype).val
    assert K.shape == (0, 0) and K.dtype == dtype
