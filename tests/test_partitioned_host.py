"""Host logic of the partitioned-K reader (pysnptools_amd/kernelreader/partitionedkernel.py) without
a GPU: when SnpKernel / Bed.read_kernel partition K (set_grm_partition, use_partitioned), and which
reads a part without its process group may serve (_check_owned, against the library's layout)."""
import numpy as np
import pytest

from pysnptools_amd import _native as N
from pysnptools_amd.kernelreader import partitionedkernel as P
from pysnptools_amd.kernelreader.partitionedkernel import PartitionedKernel
from pysnptools_amd.shard import part_coords


class _Group:
    def __init__(self, world, others=0.0):
        self.world, self.rank, self.others = world, 0, others

    def max(self, x):  # the group's max over ranks: `others` = what the other ranks decided
        return max(x, self.others)


@pytest.fixture
def mode():
    old = P.grm_partition_mode()
    yield
    P.set_grm_partition(old)


def test_modes(mode, monkeypatch):
    with pytest.raises(ValueError):
        P.set_grm_partition("sometimes")
    P.set_grm_partition("never")
    assert not P.use_partitioned(500_000, np.float32, _Group(8))
    P.set_grm_partition("always")
    assert P.use_partitioned(300, np.float64, None)
    P.set_grm_partition("auto")
    assert not P.use_partitioned(500_000, np.float32, None)  # one process: nothing to partition over
    assert not P.use_partitioned(500_000, np.float32, _Group(1))

    def fake_call(name, *args):  # a 288 GB device with 280 GB free
        assert name == "snpmi_device_memory"
        args[0]._obj.value, args[1]._obj.value = 280 << 30, 288 << 30

    monkeypatch.setattr(P.N, "call", fake_call)
    assert P.use_partitioned(500_000, np.float32, _Group(8))        # 500 GB of f32 tiles
    assert P.use_partitioned(250_000, np.float64, _Group(8))        # 250 GB of f64 tiles + extraction
    assert not P.use_partitioned(50_000, np.float64, _Group(8))     # cfg4: 10 GB, replicated
    assert not P.use_partitioned(150_000, np.float32, _Group(2))    # 45 GB
    assert P.use_partitioned(150_000, np.float32, _Group(2, others=1.0))  # another rank is short: all partition


def _view(n, part, parts):
    """A PartitionedKernel shell (no device blocks) for the host-side ownership check."""
    pk = PartitionedKernel.__new__(PartitionedKernel)
    pk.n, pk.part, pk.parts, pk.dist = n, part, parts, None
    return pk


@pytest.mark.parametrize("n,parts", [(5000, 3), (9000, 8), (300, 2)])
def test_single_part_reads_only_its_blocks(n, parts):
    nb = (n + 255) // 256
    owner = {}
    for p in range(parts):
        for r0, c0 in part_coords(n, p, parts):
            owner[(r0 // 256, c0 // 256)] = p
    assert len(owner) == nb * (nb + 1) // 2
    rng = np.random.default_rng(n)
    for p in range(parts):
        pk = _view(n, p, parts)
        for (I, J), q in list(owner.items())[:40]:
            rows = np.arange(256 * I, min(256 * I + 256, n))[rng.permutation(min(256, n - 256 * I))[:5]]
            cols = np.arange(256 * J, min(256 * J + 256, n))[:7]
            for ri, ci in ((rows, cols), (cols, rows)):  # K is symmetric: (J, I) is block (I, J)
                if q == p:
                    pk._check_owned(N.index_array(ri), N.index_array(ci))
                else:
                    with pytest.raises(ValueError, match="outside part %d of %d" % (p, parts)):
                        pk._check_owned(N.index_array(ri), N.index_array(ci))
        pk._check_owned(np.zeros(0, dtype=np.uint64), None)  # nothing asked, nothing needed


def test_lone_part_refuses_whole_k_operations():
    """A part of a plan of several, read without its group, holds only its share of the diagonal:
    trace(K) and DiagKtoN must raise instead of scaling by a partial trace."""
    from pysnptools_amd.kernelstandardizer import DiagKtoN, DiagKtoNTrained, Identity

    pk = _view(5000, 1, 3)
    with pytest.raises(ValueError, match="needs all of them"):
        pk.trace()
    with pytest.raises(ValueError, match="needs all of them"):
        pk._read_with_standardizing(True, kernel_standardizer=DiagKtoN())
    assert PartitionedKernel.supports(DiagKtoN()) and PartitionedKernel.supports(DiagKtoNTrained(2.0))
    assert PartitionedKernel.supports(Identity()) and not PartitionedKernel.supports(object())
    with pytest.raises(ValueError, match="supports the DiagKtoN"):
        pk._read_with_standardizing(False, kernel_standardizer=object())
