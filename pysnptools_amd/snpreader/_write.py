"""BED writer (reference Bed.write -> bed-reader to_bed, bed.py:229-316).

SURVEY.md §8(f) row f2 ("next"): the 2-bit encoder runs vectorised on the host for now;
it is used to write fixtures, not on the decode/standardize/GRM path.
Inverse LUT: count_A1=False 0->00, 1->10, 2->11, missing->01; count_A1=True swaps 0/2.
"""
import numpy as np


def _fmt(x):
    if x != x:
        return "0"
    return str(int(x)) if float(x).is_integer() else repr(float(x))


def encode_codes(val, count_A1=False):
    """iid x sid values -> SNP-major packed bytes [sid, ceil(iid/4)]."""
    val = np.asarray(val)
    n, m = val.shape
    if val.dtype == np.int8:
        miss = val == -127
        v = val.astype(np.int16)
    else:
        miss = np.isnan(val)
        v = np.where(miss, 0, val)
    ok = miss | (v == 0) | (v == 1) | (v == 2)
    if not np.all(ok):
        raise ValueError("Expect values to be 0, 1, 2 or missing")
    lut = np.array([3, 2, 0], dtype=np.uint8) if count_A1 else np.array([0, 2, 3], dtype=np.uint8)
    codes = np.where(miss, np.uint8(1), lut[np.clip(v, 0, 2).astype(np.intp)]).astype(np.uint8)  # n x m
    bpc = (n + 3) // 4
    padded = np.zeros((bpc * 4, m), dtype=np.uint8)
    padded[:n] = codes
    q = padded.reshape(bpc, 4, m)
    packed = q[:, 0] | (q[:, 1] << 2) | (q[:, 2] << 4) | (q[:, 3] << 6)
    return np.ascontiguousarray(packed.T)


def write_bed(filename, snpdata, count_A1, reverse_chrom_map):
    base = filename[:-4] if filename.lower().endswith(".bed") else filename
    packed = encode_codes(snpdata.val, count_A1)
    with open(filename, "wb") as f:
        f.write(bytes([0x6C, 0x1B, 0x01]))
        f.write(packed.tobytes())
    with open(base + ".fam", "w") as f:
        for fid, iid in snpdata.iid:
            f.write("{0} {1} 0 0 0 0\n".format(fid, iid))
    with open(base + ".bim", "w") as f:
        for sid, (chrom, cm, bp) in zip(snpdata.sid, snpdata.pos):
            c = reverse_chrom_map.get(chrom, None) if chrom == chrom else None
            f.write("{0}\t{1}\t{2}\t{3}\tA\tC\n".format(c if c is not None else _fmt(chrom), sid, _fmt(cm), _fmt(bp)))
