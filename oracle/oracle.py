"""CPU oracle for the BED decode -> slice -> standardize -> GRM path.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, by ``__graft_entry__.smoke()`` and by the
``cpu_baseline`` leg of bench.py -- never by ``pysnptools_amd`` (the product path has no
CPU fallback).  The C half lives in ``bed_oracle.c`` (see its header for the reference
file:line each function restates); this module binds it with ctypes and adds the NumPy
restatements that the reference itself runs in NumPy:

* ``standardize_python``  -- ``Standardizer._standardize_unit_python`` /
  ``_standardize_beta_python`` (standardizer.py:136-163, 176-211), the two-pass path.
* ``grm_blocked``         -- ``SnpReader._read_kernel`` block loop (snpreader.py:637-668):
  ``K += Z_b.dot(Z_b.T)`` over SNP blocks, float64 by default.
* ``diag_k_to_n``         -- ``DiagKtoN._standardize_kernel`` (diag_K_to_N.py:54-64).
* ``maf_table``           -- SnpGen's MAF distribution (snpreader/snpgen.py:140-151).
* ``encode``              -- bed-reader ``to_bed``'s 2-bit encoder (Bed.write, bed.py:300-314).

Pinning: tests/test_oracle.py checks every function here against the reference's own
fixtures and against golden vectors made by running the reference (tools/make_golden.py).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")


def build():
    """Compile liboracle.so with the Makefile next to this file."""
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")  # tools/sanitize.sh
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, u64, i32, f64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
        for name in ("oracle_decode_f64", "oracle_decode_f32", "oracle_decode_i8"):
            fn = getattr(L, name)
            fn.argtypes = [vp, u64, u64, i32, vp, u64, vp, u64, i32, vp, i32]
            fn.restype = i32
        for name in ("oracle_standardize_f64", "oracle_standardize_f32"):
            fn = getattr(L, name)
            fn.argtypes = [vp, u64, u64, i32, i32, f64, f64, i32, vp, i32]
            fn.restype = i32
        for name in ("oracle_decode_standardize_f64", "oracle_decode_standardize_f32"):
            fn = getattr(L, name)
            fn.argtypes = [vp, u64, u64, i32, vp, u64, i32, f64, f64, vp, vp, i32]
            fn.restype = i32
        for name in ("oracle_subset_f64_f64", "oracle_subset_f32_f64", "oracle_subset_f32_f32"):
            fn = getattr(L, name)
            fn.argtypes = [vp, u64, u64, u64, i32, vp, u64, vp, u64, i32, vp]
            fn.restype = i32
        L.oracle_snp_stats.argtypes = [vp, u64, u64, i32, vp, i32]
        L.oracle_snp_stats.restype = i32
        L.oracle_beta_pdf.argtypes = [f64, f64, f64]
        L.oracle_beta_pdf.restype = f64
        L.oracle_synth_bed.argtypes = [u64, u64, u64, u64, u64, vp, vp, i32, f64, vp, i32]
        L.oracle_synth_bed.restype = i32
        L.oracle_max_threads.restype = i32
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------- files
def read_bed_bytes(path):
    """Raw .bed body (after the 3-byte magic 6C 1B 01)."""
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size < 3 or raw[0] != 0x6C or raw[1] != 0x1B or raw[2] != 0x01:
        raise ValueError("not a SNP-major .bed file: %s" % path)
    return raw[3:]


def count_lines(path):
    with open(path, "rb") as f:
        return sum(1 for line in f if line.strip())


def bed_shape(bed_path):
    base = bed_path[:-4] if bed_path.endswith(".bed") else bed_path
    return count_lines(base + ".fam"), count_lines(base + ".bim")


# ----------------------------------------------------------------------------- decode
def decode(body, n_iid, n_sid, count_A1=False, iid_index=None, sid_index=None,
           order="F", dtype=np.float64, num_threads=0):
    """open_bed.read restated (bed.py:337-343)."""
    dtype = np.dtype(dtype)
    iid = np.arange(n_iid, dtype=np.uint64) if iid_index is None else np.ascontiguousarray(iid_index, dtype=np.uint64)
    sid = np.arange(n_sid, dtype=np.uint64) if sid_index is None else np.ascontiguousarray(sid_index, dtype=np.uint64)
    body = np.ascontiguousarray(body, dtype=np.uint8)
    if body.size < n_sid * ((n_iid + 3) // 4):
        raise ValueError("bed body too short")
    out = np.empty((len(iid), len(sid)), dtype=dtype, order=order)
    fn = {np.dtype(np.float64): lib().oracle_decode_f64, np.dtype(np.float32): lib().oracle_decode_f32,
          np.dtype(np.int8): lib().oracle_decode_i8}[dtype]
    rc = fn(_ptr(body), n_iid, n_sid, int(bool(count_A1)), _ptr(iid), len(iid), _ptr(sid), len(sid),
            1 if order == "C" else 0, _ptr(out), num_threads)
    if rc:
        raise IndexError("index out of range")
    return out


def decode_standardize(body, n_iid, n_sid, is_beta=False, a=np.nan, b=np.nan, count_A1=False,
                       sid_index=None, dtype=np.float32, num_threads=0):
    """Fused decode + one-pass standardize (F order), the CPU baseline kernel."""
    dtype = np.dtype(dtype)
    sid = np.arange(n_sid, dtype=np.uint64) if sid_index is None else np.ascontiguousarray(sid_index, dtype=np.uint64)
    out = np.empty((n_iid, len(sid)), dtype=dtype, order="F")
    stats = np.empty((len(sid), 2), dtype=dtype)
    fn = lib().oracle_decode_standardize_f64 if dtype == np.float64 else lib().oracle_decode_standardize_f32
    fn(_ptr(np.ascontiguousarray(body)), n_iid, n_sid, int(bool(count_A1)), _ptr(sid), len(sid),
       int(bool(is_beta)), float(a), float(b), _ptr(out), _ptr(stats), num_threads)
    return out, stats


def snp_stats(body, n_iid, n_sid, count_A1=False, num_threads=0):
    """One-pass (mean, std) per SNP in f64 from code counts, without decoding the matrix."""
    stats = np.empty((n_sid, 2), dtype=np.float64)
    lib().oracle_snp_stats(_ptr(np.ascontiguousarray(body)), n_iid, n_sid, int(bool(count_A1)), _ptr(stats),
                           num_threads)
    return stats


def encode(val, count_A1=False):
    """bed-reader to_bed's body encoder restated (called from bed.py:300-314): n_iid x n_sid values
    -> SNP-major packed bytes [n_sid, ceil(n_iid/4)].  count_A1=False: 0->00, 1->10, 2->11,
    missing->01 (count_A1=True swaps 0/2); pad codes 00.  Pinned against the reference-written
    generate/gen1.bed, gen4.bed (N % 4 == 2) and the N300 .bed (tests/test_oracle.py)."""
    val = np.asarray(val)
    n, m = val.shape
    if val.dtype == np.int8:
        miss = val == -127
        v = val.astype(np.int16)
    else:
        miss = np.isnan(val)
        v = np.where(miss, 0, val)
    if not np.all(miss | (v == 0) | (v == 1) | (v == 2)):
        raise ValueError("Expect values to be 0, 1, 2 or missing")
    lut = np.array([3, 2, 0], dtype=np.uint8) if count_A1 else np.array([0, 2, 3], dtype=np.uint8)
    codes = np.where(miss, np.uint8(1), lut[np.clip(v, 0, 2).astype(np.intp)]).astype(np.uint8)
    bpc = (n + 3) // 4
    padded = np.zeros((bpc * 4, m), dtype=np.uint8)
    padded[:n] = codes
    q = padded.reshape(bpc, 4, m)
    packed = q[:, 0] | (q[:, 1] << 2) | (q[:, 2] << 4) | (q[:, 3] << 6)
    return np.ascontiguousarray(packed.T)


# ----------------------------------------------------------------------------- standardize
def standardize_native(val, is_beta=False, a=np.nan, b=np.nan, use_stats=False, stats=None, num_threads=0):
    """bed-reader standardize_f32/f64 restated (standardizer.py:114,120); in place; returns stats."""
    assert val.dtype in (np.float32, np.float64)
    assert val.flags["C_CONTIGUOUS"] or val.flags["F_CONTIGUOUS"]
    order_c = 1 if val.flags["C_CONTIGUOUS"] and not val.flags["F_CONTIGUOUS"] else 0
    if val.ndim == 2 and val.shape[1] == 1:
        order_c = 0
    rows, cols = val.shape
    st = np.empty((cols, 2), dtype=val.dtype) if stats is None else np.array(stats, dtype=val.dtype, order="C")
    fn = lib().oracle_standardize_f64 if val.dtype == np.float64 else lib().oracle_standardize_f32
    fn(_ptr(val), rows, cols, order_c, int(bool(is_beta)), float(a), float(b), int(bool(use_stats)),
       _ptr(st), num_threads)
    return st


def beta_pdf(x, a, b):
    return lib().oracle_beta_pdf(float(x), float(a), float(b))


def standardize_python(val, is_beta=False, a=np.nan, b=np.nan, use_stats=False, stats=None):
    """The reference's two-pass NumPy path (standardizer.py:136-163 Unit, 176-211 Beta)."""
    import warnings

    imiss = np.isnan(val)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if use_stats:
            mean = np.asarray(stats)[:, 0].astype(val.dtype)
            std = np.asarray(stats)[:, 1].astype(val.dtype)
        elif is_beta:
            n_obs = (~imiss).sum(0)
            mean = np.nansum(val, axis=0) * 1.0 / n_obs
            std = np.sqrt(np.nansum((val - mean) ** 2, axis=0) / n_obs)
            std[std == 0] = np.inf
        else:
            std = np.nanstd(val, axis=0)
            mean = np.nanmean(val, axis=0)
            std[std == 0.0] = np.inf
        out_stats = np.stack([mean, std], axis=1).astype(val.dtype)
        if is_beta:
            from scipy.stats import beta as _beta

            maf = mean / 2.0
            maf[maf > 0.5] = 1.0 - maf[maf > 0.5]
            w = _beta.pdf(maf, a, b)
            val -= mean
            val *= w
            val[imiss] = 0.0
            if use_stats:
                val[:, std == np.inf] = 0.0
        else:
            val -= mean
            val /= std
            val[imiss] = 0
    return out_stats


# ----------------------------------------------------------------------------- subset / GRM
def subset(val, row_index, col_index, order="A", dtype=np.float64):
    """sub_matrix restated (util/__init__.py:271-393)."""
    dtype = np.dtype(dtype)
    eff = ("F" if val.flags["F_CONTIGUOUS"] else "C") if order == "A" else order
    v3 = val if val.ndim == 3 else val.reshape(val.shape[0], val.shape[1], 1, order="A")
    ri = np.ascontiguousarray(row_index, dtype=np.uint64)
    ci = np.ascontiguousarray(col_index, dtype=np.uint64)
    out = np.full((len(ri), len(ci), v3.shape[2]), np.nan, dtype=dtype, order=eff)
    key = (val.dtype, dtype)
    fn = {(np.dtype(np.float64), np.dtype(np.float64)): lib().oracle_subset_f64_f64,
          (np.dtype(np.float32), np.dtype(np.float64)): lib().oracle_subset_f32_f64,
          (np.dtype(np.float32), np.dtype(np.float32)): lib().oracle_subset_f32_f32}.get(key)
    if fn is None:
        out[...] = v3[np.ix_(ri, ci)].astype(dtype)
    else:
        in_c = 0 if v3.flags["F_CONTIGUOUS"] else 1
        if fn(_ptr(np.asarray(v3, order="K")), v3.shape[0], v3.shape[1], v3.shape[2], in_c, _ptr(ri), len(ri),
              _ptr(ci), len(ci), 0 if eff == "F" else 1, _ptr(out)):
            raise IndexError("index out of range")
    return out if val.ndim == 3 else out.reshape(out.shape[0], out.shape[1], order="A")


def grm_blocked(Z_blocks, dtype=np.float64):
    """K = sum_b Z_b Z_b^T (snpreader.py:643-655)."""
    K = None
    for Z in Z_blocks:
        Z = np.asarray(Z, dtype=dtype)
        part = Z.dot(Z.T)
        K = part if K is None else K + part
    return K


def grm_from_bed(body, n_iid, n_sid, is_beta=False, a=np.nan, b=np.nan, count_A1=False,
                 block_size=None, dtype=np.float64, iid_index=None, standardize=True):
    """Reference GRM of a BED matrix: decode -> (native one-pass) standardize -> blocked syrk."""
    block = n_sid if not block_size else block_size
    parts, stats = [], []
    for s0 in range(0, n_sid, block):
        sid = np.arange(s0, min(n_sid, s0 + block), dtype=np.uint64)
        Z = decode(body, n_iid, n_sid, count_A1, iid_index=iid_index, sid_index=sid, dtype=dtype)
        if standardize:
            stats.append(standardize_native(Z, is_beta, a, b))
        parts.append(Z)
    K = grm_blocked(parts, dtype=dtype)
    return K, (np.concatenate(stats) if stats else None)


def diag_k_to_n(K):
    """DiagKtoN._standardize_kernel (diag_K_to_N.py:54-64); returns (K, factor)."""
    factor = float(K.shape[0]) / np.diag(K).sum()
    if abs(factor - 1.0) > 1e-15:
        K = K * factor
    return K, factor


# ----------------------------------------------------------------------------- synthetic data
def maf_table(n_iid):
    """SnpGen's MAF curve (snpgen.py:140-151): 100 log-spaced points, weight exp(w0 log x + w1)."""
    w = np.array([-0.6482249, -8.49790398])
    x = np.logspace(np.log10(0.1 / n_iid), np.log10(0.5), 100, base=10)
    y = np.exp(w[0] * np.log(x) + w[1])
    cdf = np.cumsum(y / y.sum())
    cdf[-1] = 1.0
    return x, cdf


def synth_bed(seed, n_iid, sid0, n_sid, miss_rate, pitch=None, num_threads=0):
    """CPU twin of the device generator; returns uint8 [n_sid, pitch]."""
    bpc = (n_iid + 3) // 4
    pitch = bpc if pitch is None else pitch
    x, cdf = maf_table(n_iid)
    out = np.empty((n_sid, pitch), dtype=np.uint8)
    rc = lib().oracle_synth_bed(seed, n_iid, sid0, n_sid, pitch, _ptr(x), _ptr(cdf), len(x), float(miss_rate),
                                _ptr(out), num_threads)
    assert rc == 0
    return out
