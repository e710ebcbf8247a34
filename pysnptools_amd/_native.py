"""ctypes binding of libsnpmi.so (include/snpmi.h) -- the only way this package computes.

There is deliberately no CPU fallback: if the HIP library cannot be loaded, or no GPU is
visible, every compute call raises.  ``SNPMI_LIB`` overrides the library path.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SNPMI_LIB", os.path.join(_HERE, "libsnpmi.so"))

E_ARG, E_INDEX, E_FORMAT, E_IO, E_HIP, E_NOMEM, E_RCCL = 1, 2, 3, 4, 5, 6, 7
STD_NONE, STD_UNIT, STD_BETA = 0, 1, 2
DT_F32, DT_F64, DT_I8 = 0, 1, 2

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int
_f64 = ctypes.c_double
_cp = ctypes.c_char_p
_dp = ctypes.POINTER(ctypes.c_double)
_u64p = ctypes.POINTER(ctypes.c_uint64)

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "snpmi_version": [],
    "snpmi_device_count": [ctypes.POINTER(ctypes.c_int)],
    "snpmi_set_device": [_i32],
    "snpmi_get_device": [ctypes.POINTER(ctypes.c_int)],
    "snpmi_release_cache": [],
    "snpmi_device_info": [_i32, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64),
                          ctypes.POINTER(ctypes.c_int)],
    "snpmi_device_ids": [_i32, _vp, _vp, ctypes.POINTER(ctypes.c_int)],
    "snpmi_set_kernel_variant": [_cp, _i32],
    "snpmi_get_kernel_variant": [_cp, ctypes.POINTER(ctypes.c_int)],
    "snpmi_bed_check": [_cp, _u64, _u64],
    "snpmi_bed_read_f32": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_bed_read_f64": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_bed_read_i8": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_text_scan": [_cp, _i32, _i32, ctypes.POINTER(ctypes.c_uint64), _vp, _i32],
    "snpmi_text_strings": [_cp, _i32, _u64, _u64, _vp, _i32],
    "snpmi_text_f64": [_cp, _i32, _u64, _vp, _i32],
    "snpmi_bed_write_f32": [_cp, _vp, _u64, _u64, _i32, _i32, _i32],
    "snpmi_bed_write_f64": [_cp, _vp, _u64, _u64, _i32, _i32, _i32],
    "snpmi_bed_write_i8": [_cp, _vp, _u64, _u64, _i32, _i32, _i32],
    "snpmi_standardize_f32": [_vp, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _i32, _vp, _i32],
    "snpmi_standardize_f64": [_vp, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _i32, _vp, _i32],
    "snpmi_subset_f64_f64": [_vp, _u64, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_subset_f32_f64": [_vp, _u64, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_subset_f32_f32": [_vp, _u64, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _vp, _i32],
    "snpmi_bed_read_standardize_f32": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _i32, _f64, _f64, _i32,
                                       _vp, _vp, _i32],
    "snpmi_bed_read_standardize_f64": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _i32, _f64, _f64, _i32,
                                       _vp, _vp, _i32],
    "snpmi_grm_bed_f32": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32, _dp, _vp,
                          _i32],
    "snpmi_grm_bed_f64": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32, _dp, _vp,
                          _i32],
    "snpmi_grm_dense_f32": [_vp, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp, _i32, _dp, _vp],
    "snpmi_grm_dense_f64": [_vp, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp, _i32, _dp, _vp],
    "snpmi_grm_begin": [_u64, _i32],
    "snpmi_grm_add_bed_f32": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32],
    "snpmi_grm_add_bed_f64": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32],
    "snpmi_grm_add_bed_reduce_f32": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32,
                                     _i32, _i32, _i32],
    "snpmi_grm_add_bed_reduce_f64": [_cp, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _f64, _i32, _vp, _i32,
                                     _i32, _i32, _i32],
    "snpmi_grm_add_packed_f32": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp],
    "snpmi_grm_add_packed_f64": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp],
    "snpmi_grm_add_packed_reduce_f32": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp, _i32, _i32, _i32,
                                        _vp],
    "snpmi_grm_add_packed_reduce_f64": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _vp, _i32, _i32, _i32,
                                        _vp],
    "snpmi_grm_add_dense_f32": [_vp, _u64, _u64, _i32],
    "snpmi_grm_add_dense_f64": [_vp, _u64, _u64, _i32],
    "snpmi_grm_session_tiles": [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)],
    "snpmi_grm_session_sum": [_i32, _i32, _i32],
    "snpmi_grm_end": [_i32, _dp, _vp],
    "snpmi_diag_k_to_n_snps_f32": [_vp, _u64, _u64, _dp],
    "snpmi_diag_k_to_n_snps_f64": [_vp, _u64, _u64, _dp],
    "snpmi_scale_f32": [_vp, _u64, _f64],
    "snpmi_scale_f64": [_vp, _u64, _f64],
    "snpmi_diag_k_to_n_f32": [_vp, _u64, _dp],
    "snpmi_diag_k_to_n_f64": [_vp, _u64, _dp],
    "snpmi_packed_pitch": [_u64],
    "snpmi_grm_tile_bytes": [_u64, _i32],
    "snpmi_dev_alloc": [ctypes.POINTER(ctypes.c_void_p), _u64],
    "snpmi_dev_free": [_vp],
    "snpmi_host_alloc": [ctypes.POINTER(ctypes.c_void_p), _u64],
    "snpmi_host_free": [_vp],
    "snpmi_dev_memset": [_vp, _i32, _u64],
    "snpmi_memcpy_h2d": [_vp, _vp, _u64],
    "snpmi_memcpy_d2h": [_vp, _vp, _u64],
    "snpmi_dev_memcpy_d2d": [_vp, _vp, _u64],
    "snpmi_stream_sync": [],
    "snpmi_event_create": [ctypes.POINTER(ctypes.c_void_p)],
    "snpmi_event_destroy": [_vp],
    "snpmi_event_record": [_vp],
    "snpmi_event_elapsed_ms": [_vp, _vp, ctypes.POINTER(ctypes.c_float)],
    "snpmi_memcpy_async": [_vp, _vp, _u64, _i32, _i32],
    "snpmi_event_record_on": [_vp, _i32],
    "snpmi_set_stream": [_i32],
    "snpmi_stream_wait_event": [_vp, _i32],
    "snpmi_event_sync": [_vp],
    "snpmi_dev_synth_bed": [_vp, _u64, _u64, _u64, _u64, _u64, _f64, _vp, _vp, _i32],
    "snpmi_host_synth_bed": [_vp, _u64, _u64, _u64, _u64, _u64, _f64, _vp, _vp, _i32, _i32],
    "snpmi_bed_gather_packed": [_cp, _u64, _u64, _vp, _u64, _u64, _vp, _i32],
    "snpmi_dev_snp_stats": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _i32, _vp, _vp],
    "snpmi_dev_decode": [_vp, _u64, _u64, _u64, _vp, _i32, _i32, _vp, _u64],
    "snpmi_dev_decode_standardize": [_vp, _u64, _u64, _u64, _i32, _i32, _f64, _f64, _i32, _i32, _vp, _vp, _vp, _u64],
    "snpmi_dev_encode": [_vp, _i32, _i32, _u64, _u64, _u64, _i32, _vp, _u64, ctypes.POINTER(ctypes.c_uint64)],
    "snpmi_dev_repack": [_vp, _u64, _u64, _vp, _u64, _u64, _vp, _u64],
    "snpmi_dev_syrk_packed": [_vp, _u64, _u64, _u64, _vp, _i32, _vp, _i32],
    "snpmi_grm_part_blocks": [_u64, _i32, _i32],
    "snpmi_grm_part_coords": [_u64, _i32, _i32, _u64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)],
    "snpmi_grm_part_coords_all": [_u64, _i32, _i32, _vp],
    "snpmi_dev_syrk_packed_part": [_vp, _u64, _u64, _u64, _vp, _i32, _i32, _vp, _i32],
    "snpmi_grm_part_bed_f32": [ctypes.c_char_p, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, ctypes.c_double,
                               ctypes.c_double, _i32, _vp, _i32, _i32, _vp, _i32],
    "snpmi_grm_part_bed_f64": [ctypes.c_char_p, _u64, _u64, _i32, _vp, _u64, _vp, _u64, _i32, ctypes.c_double,
                               ctypes.c_double, _i32, _vp, _i32, _i32, _vp, _i32],
    "snpmi_dev_syrk_packed_part_f64": [_vp, _u64, _u64, _u64, _vp, _i32, _i32, _vp, _i32],
    "snpmi_grm_part_extract_f32": [_vp, _u64, _i32, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _vp],
    "snpmi_grm_part_extract_f64": [_vp, _u64, _i32, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _vp],
    "snpmi_grm_part_trace_f32": [_vp, _u64, _i32, _i32, _dp],
    "snpmi_grm_part_trace_f64": [_vp, _u64, _i32, _i32, _dp],
    "snpmi_device_memory": [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)],
    "snpmi_dev_syrk_dense": [_vp, _u64, _u64, _u64, _i32, _vp, _i32],
    "snpmi_dev_grm_extract": [_vp, _u64, _i32, _vp, _u64, _vp, _u64, _i32, _f64, _vp],
    "snpmi_dev_grm_trace": [_vp, _u64, _i32, _dp],
    "snpmi_crt_moduli_stats": [_u64p, _u64p, _i32],
    "snpmi_crt_block_moduli_stats": [_u64p, _u64p, _i32],
    "snpmi_rccl_unique_id": [_vp, _u64],
    "snpmi_rccl_init": [_i32, _i32, _vp, _u64],
    "snpmi_rccl_allreduce_sum": [_vp, _u64, _i32],
    "snpmi_rccl_reduce_sum": [_vp, _u64, _i32, _i32],
    "snpmi_rccl_allgather": [_vp, _vp, _u64],
    "snpmi_rccl_host_allreduce_f64": [_vp, _u64, _i32],
    "snpmi_rccl_barrier": [],
    "snpmi_rccl_comm_count": [ctypes.POINTER(ctypes.c_int)],
    "snpmi_rccl_destroy": [],
    "snpmi_rccl_trace": [_vp, _u64],
    "snpmi_last_error": [],
}
_RESTYPES = {"snpmi_last_error": ctypes.c_char_p, "snpmi_packed_pitch": ctypes.c_uint64,
             "snpmi_grm_tile_bytes": ctypes.c_uint64, "snpmi_grm_part_blocks": ctypes.c_uint64}

_lib = None
_load_error = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libsnpmi.so (raises ImportError with the reason if it cannot be loaded)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise ImportError(_load_error)
    try:
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        _load_error = ("pysnptools_amd: cannot load the HIP library %s (%s). Build it with "
                       "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C pysnptools_amd/csrc`. "
                       "There is no CPU fallback." % (LIB_PATH, e))
        raise ImportError(_load_error)
    for name, args in _SIGS.items():
        if "SNPMI_LIB" in os.environ and not hasattr(L, name):
            continue  # an A/B build of an earlier revision (SNPMI_LIB): calls to what it lacks raise
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = L
    return L


def symbols():
    return sorted(_SIGS)


def last_error():
    msg = lib().snpmi_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc):
    if rc == 0:
        return
    msg = last_error()
    if rc == E_INDEX:
        raise IndexError(msg)
    if rc == E_FORMAT:
        raise ValueError(msg)
    if rc == E_IO:
        raise IOError(msg)
    if rc == E_ARG:
        raise ValueError(msg)
    if rc == E_NOMEM:
        raise MemoryError(msg)
    raise NativeError("libsnpmi error %d: %s" % (rc, msg))


def call(name, *args):
    check(getattr(lib(), name)(*args))


def kernel_variant(name):
    """Current value of a ``snpmi_set_kernel_variant`` switch (e.g. "f64", "seg")."""
    v = ctypes.c_int(0)
    call("snpmi_get_kernel_variant", name.encode() if isinstance(name, str) else name, ctypes.byref(v))
    return v.value


TRACE_FIELDS = ("calls", "allreduce", "reduce", "allgather", "host", "bytes", "sig", "last_kind", "last_count",
                "in_blocking_call", "blocking_calls_done", "comm")
TRACE_KINDS = {0: None, 1: "allreduce", 2: "reduce", 3: "allgather", 4: "host_allreduce"}


def rccl_trace():
    """This process's RCCL call counters (snpmi_rccl_trace) as a dict; safe from a watchdog thread."""
    out = (ctypes.c_uint64 * len(TRACE_FIELDS))()
    check(lib().snpmi_rccl_trace(out, len(TRACE_FIELDS)))
    d = dict(zip(TRACE_FIELDS, (int(x) for x in out)))
    d["sig"] = "%016x" % d["sig"]
    d["last_kind"] = TRACE_KINDS.get(d["last_kind"], d["last_kind"])
    return d


def device_count():
    n = ctypes.c_int(0)
    call("snpmi_device_count", ctypes.byref(n))
    return n.value


def ptr(a):
    """Raw data pointer of a NumPy array or an HbmArray (device address; the C ABI takes host or
    device buffers), None for None."""
    if a is None:
        return None
    dev = getattr(a, "snpmi_ptr", None)
    if dev is not None:
        return dev
    return ctypes.c_void_p(a.ctypes.data)


def index_array(idx):
    """NumPy uintp (uint64) contiguous array, or None."""
    if idx is None:
        return None
    return np.ascontiguousarray(idx, dtype=np.uint64)


_DT = {np.dtype(np.float32): ("f32", DT_F32), np.dtype(np.float64): ("f64", DT_F64), np.dtype(np.int8): ("i8", DT_I8)}


def suffix(dtype):
    return _DT[np.dtype(dtype)][0]


def dt_code(dtype):
    return _DT[np.dtype(dtype)][1]
