"""HBM-resident arrays: the array module behind ``ARRAY_MODULE='hbm'`` / ``xp='hbm'``.

The reference keeps ``SnpData.val`` and ``KernelData.val`` on the GPU through its array-module
seam (util/__init__.py:652-730; used at snpreader.py:638-643, pstdata.py:139-148,
kerneldata.py:73,91, unit.py:32-38), with CuPy as the device module.  This module is that seam
for libsnpmi: an :class:`HbmArray` is a buffer in the GPU's HBM (``snpmi_dev_alloc``) with a
shape, dtype and order, and every libsnpmi entry point accepts it wherever it accepts a NumPy
array (the C ABI takes host or device pointers, include/snpmi.h).  So with
``ARRAY_MODULE=hbm``:

* ``Bed(...).read()`` decodes straight into HBM (only the 2-bit codes cross PCIe);
* ``SnpData.standardize(...)`` runs in place in HBM;
* ``read_kernel(...)`` leaves K in HBM (no N x N copy back: 10 GB at N = 50k f32);
* ``KernelData.standardize(DiagKtoN())`` traces and scales K in place;
* ``util.asnumpy(a)`` / ``a.get()`` copy to the host; ``__cuda_array_interface__`` hands the
  buffer to other GPU libraries without a copy.

Differences from the CuPy seam, by design: values keep their float32/float64 dtype (CuPy's
``xp.array(input, dtype=float64)`` promotion at pstdata.py:146 is not reproduced), and an
HbmArray is a storage type, not a general array library -- indexing other than a single
element goes through a host copy.
"""
import ctypes

import numpy as np

from pysnptools_amd import _native as N

float32 = np.float32
float64 = np.float64
int8 = np.int8


class _Flags(dict):
    def __getattr__(self, k):
        return self[k.upper()]


class HbmArray(object):
    """A C- or F-contiguous 2-D/3-D array in device memory owned by libsnpmi."""

    __array_priority__ = 100

    def __init__(self, shape, dtype=np.float64, order="C", _base=None, _ptr=None):
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        if order not in ("C", "F"):
            raise ValueError("order must be 'C' or 'F'")
        self.order = order
        self._base = _base
        if _ptr is not None:
            self._ptr = _ptr
        else:
            p = ctypes.c_void_p()
            N.call("snpmi_dev_alloc", ctypes.byref(p), max(self.nbytes, 1))
            self._ptr = p.value

    # ------------------------------------------------------------------ array protocol
    @property
    def ndim(self):
        return len(self.shape)

    @property
    def size(self):
        return int(np.prod(self.shape, dtype=np.int64)) if self.shape else 1

    @property
    def itemsize(self):
        return self.dtype.itemsize

    @property
    def nbytes(self):
        return self.size * self.itemsize

    @property
    def strides(self):
        dims = self.shape if self.order == "C" else self.shape[::-1]
        st, acc = [], self.itemsize
        for d in reversed(dims):
            st.append(acc)
            acc *= d
        st = st[::-1]
        return tuple(st if self.order == "C" else st[::-1])

    @property
    def flags(self):
        trivial = self.ndim <= 1 or sum(1 for s in self.shape if s != 1) <= 1
        return _Flags(C_CONTIGUOUS=self.order == "C" or trivial, F_CONTIGUOUS=self.order == "F" or trivial,
                      OWNDATA=self._base is None, WRITEABLE=True)

    @property
    def ptr(self):
        """Device address (int)."""
        return self._ptr

    @property
    def snpmi_ptr(self):
        return ctypes.c_void_p(self._ptr)

    @property
    def __cuda_array_interface__(self):
        return {"shape": self.shape, "typestr": self.dtype.str, "data": (self._ptr, False), "version": 3,
                "strides": None if self.order == "C" else self.strides}

    @property
    def T(self):
        """Transposed view (shares the buffer): C <-> F."""
        return HbmArray(self.shape[::-1], self.dtype, "F" if self.order == "C" else "C", _base=self, _ptr=self._ptr)

    def get(self, order=None):
        """Copy to a NumPy array on the host (cupy.ndarray.get)."""
        out = np.empty(self.shape, dtype=self.dtype, order=self.order)
        if self.nbytes:
            N.call("snpmi_memcpy_d2h", N.ptr(out), self.snpmi_ptr, self.nbytes)
        return out if order is None else np.asarray(out, order=order)

    def __array__(self, dtype=None, copy=None):
        a = self.get()
        return a if dtype is None else a.astype(dtype)

    def __len__(self):
        return self.shape[0]

    def __getitem__(self, key):
        """A single element is copied back alone; anything else indexes a host copy."""
        if isinstance(key, tuple) and len(key) == self.ndim and all(isinstance(k, (int, np.integer)) for k in key):
            idx = [int(k) + (s if int(k) < 0 else 0) for k, s in zip(key, self.shape)]
            if not all(0 <= i < s for i, s in zip(idx, self.shape)):
                raise IndexError("index %s out of bounds for shape %s" % (key, self.shape))
            off = int(np.dot(idx, self.strides))
            one = np.empty(1, dtype=self.dtype)
            N.call("snpmi_memcpy_d2h", N.ptr(one), ctypes.c_void_p(self._ptr + off), self.itemsize)
            return one[0]
        return self.get()[key]

    def copy(self, order="K"):
        """Device-to-device copy (same layout)."""
        out = HbmArray(self.shape, self.dtype, self.order)
        if self.nbytes:
            N.call("snpmi_dev_memcpy_d2d", out.snpmi_ptr, self.snpmi_ptr, self.nbytes)
            N.call("snpmi_stream_sync")
        return out if order in ("K", "A", self.order) else asarray(self, order=order)

    def astype(self, dtype, order="K", copy=True):
        """dtype conversion on the device (float32 -> float64 through the subset kernel with
        identity indices); other conversions via the host."""
        dtype = np.dtype(dtype)
        target = self.order if order in ("K", "A") else order
        if dtype == self.dtype and target == self.order:
            return self.copy() if copy else self
        if self.ndim == 2 and self.dtype in (np.float32, np.float64) and dtype in (np.float32, np.float64) \
                and not (self.dtype == np.float64 and dtype == np.float32):
            from pysnptools_amd.util import sub_matrix

            return sub_matrix(self, np.arange(self.shape[0]), np.arange(self.shape[1]), order=target, dtype=dtype)
        return asarray(self.get().astype(dtype, order=target))

    def __repr__(self):
        return "HbmArray(shape=%s, dtype=%s, order=%s, ptr=0x%x)" % (self.shape, self.dtype, self.order, self._ptr)

    def __del__(self):
        try:
            if self._base is None and self._ptr:
                N.call("snpmi_dev_free", ctypes.c_void_p(self._ptr))
        except Exception:
            pass
        self._ptr = 0


ndarray = HbmArray


def empty(shape, dtype=np.float64, order="C"):
    return HbmArray(shape, dtype, order)


def zeros(shape, dtype=np.float64, order="C"):
    a = HbmArray(shape, dtype, order)
    if a.nbytes:
        N.call("snpmi_dev_memset", a.snpmi_ptr, 0, a.nbytes)
        N.call("snpmi_stream_sync")
    return a


def asarray(a, dtype=None, order=None):
    """HbmArray of ``a`` (copied to the device if it is on the host; returned as is if it is
    already an HbmArray of that dtype and order)."""
    if isinstance(a, HbmArray):
        if (dtype is None or np.dtype(dtype) == a.dtype) and (order in (None, "K", "A") or order == a.order):
            return a
        return a.astype(dtype or a.dtype, order=order or "K")
    h = np.asarray(a, dtype=dtype)
    if order in ("C", "F"):
        h = np.asarray(h, order=order)
    if not (h.flags["C_CONTIGUOUS"] or h.flags["F_CONTIGUOUS"]):
        h = np.ascontiguousarray(h)
    lay = "F" if (h.flags["F_CONTIGUOUS"] and not h.flags["C_CONTIGUOUS"]) else "C"
    out = HbmArray(h.shape, h.dtype, lay)
    if h.nbytes:
        N.call("snpmi_memcpy_h2d", out.snpmi_ptr, N.ptr(h), h.nbytes)
    return out


def array(a, dtype=None, order=None):
    """A new HbmArray holding a copy of ``a``."""
    if isinstance(a, HbmArray):
        out = a.copy()
        return out if dtype is None and order in (None, "K", "A") else asarray(out, dtype=dtype, order=order)
    return asarray(a, dtype=dtype, order=order)


def asnumpy(a):
    return a.get() if isinstance(a, HbmArray) else np.asarray(a)


def is_hbm(a):
    return isinstance(a, HbmArray)
