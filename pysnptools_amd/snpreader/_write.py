"""BED writer (reference Bed.write -> bed-reader to_bed, bed.py:229-316).

SURVEY.md §8(f) row f2: the 2-bit encoder runs on the GPU (csrc/encode.hip, C ABI
snpmi_bed_write_*); the .fam/.bim text is written here.
Inverse LUT: count_A1=False 0->00, 1->10, 2->11, missing->01; count_A1=True swaps 0/2.
Values other than 0, 1, 2 or missing raise ValueError and leave no .bed behind.
"""
import numpy as np


def _fmt(x):
    """.bim number: Python float text ("1.0", "9270273.0"), as in the reference-written
    tests/datasets/distributed_bed_test1 pieces; NaN -> "0.0" (PLINK missing, bed.py:254)."""
    if x != x:
        return "0.0"
    return repr(float(x))


def write_bed_body(filename, val, count_A1):
    """Genotype half of bed-reader's to_bed: values -> .bed on the GPU (snpmi_bed_write_*)."""
    from pysnptools_amd import _native as N
    from pysnptools_amd import hbm

    if not isinstance(val, hbm.HbmArray):  # device values are encoded where they are
        val = np.asarray(val)
    if val.dtype not in (np.float32, np.float64, np.int8):
        val = val.astype(np.float64)
    if not (val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]):
        val = np.asfortranarray(val)
    n, m = val.shape
    order_c = 1 if val.flags["C_CONTIGUOUS"] and not val.flags["F_CONTIGUOUS"] else 0
    fn = "snpmi_bed_write_" + {np.dtype(np.float32): "f32", np.dtype(np.float64): "f64",
                               np.dtype(np.int8): "i8"}[val.dtype]
    N.call(fn, filename.encode(), N.ptr(val), n, m, order_c, int(bool(count_A1)), 0)


def write_bed(filename, snpdata, count_A1, reverse_chrom_map):
    base = filename[:-4] if filename.lower().endswith(".bed") else filename
    write_bed_body(filename, snpdata.val, count_A1)
    with open(base + ".fam", "w") as f:
        for fid, iid in snpdata.iid:
            f.write("{0} {1} 0 0 0 0\n".format(fid, iid))
    with open(base + ".bim", "w") as f:
        for sid, (chrom, cm, bp) in zip(snpdata.sid, snpdata.pos):
            c = reverse_chrom_map.get(chrom, None) if chrom == chrom else None
            f.write("{0}\t{1}\t{2}\t{3}\tA\tC\n".format(c if c is not None else _fmt(chrom), sid, _fmt(cm), _fmt(bp)))
