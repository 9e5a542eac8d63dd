"""ctypes binding of libratslam_hip.so (declared in include/ratslam_abi.h).

The library is loaded from this package directory only (built in-tree by
``pyratslam_amd._build``).  There is no fallback: if the shared object is
missing or no HIP device is visible, the drop-in classes raise.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libratslam_hip.so')

RS_OK = 0
RS_ERR_ARG = 1
RS_ERR_TYPE = 2
RS_ERR_LUT_KEY = 3
RS_ERR_HIP = 4
RS_ERR_RCCL = 5
RS_ERR_STATE = 6
RS_ERR_NOMEM = 7
RS_ERR_CTL_RANGE = 8
RS_PREC_F32 = 0
RS_PREC_F64 = 1
RS_PC_DBG_POISON = 1
RS_PC_DBG_SKIP_EXPORT = 2
RS_PC_DBG_HALO_SETTLE = 3
RS_PC_DBG_HALO_AMBIG = 4
RS_VT_FROZEN = 0
RS_VT_SEQUENTIAL = 1
RS_UNIQUE_ID_BYTES = 128
RS_DT_F32 = 0
RS_DT_F64 = 1
FILTER_LEN = 7

_c_int_p = ctypes.POINTER(ctypes.c_int)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_f64p = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p


class PcParams(ctypes.Structure):
    """``rs_pc_params`` (ratslam_abi.h)."""
    _fields_ = [
        ('precision', ctypes.c_int),
        ('global_inhibition', ctypes.c_double),
        ('ge', ctypes.c_double * FILTER_LEN),
        ('gi', ctypes.c_double * FILTER_LEN),
        ('k_scale', ctypes.c_double),
        ('nfilters', ctypes.c_int),
        ('xy_filters', _f64p),
    ]


# name -> (restype, argtypes); every exported symbol of ratslam_abi.h
SIGNATURES = {
    'rs_version': (ctypes.c_int, []),
    'rs_last_error': (ctypes.c_char_p, []),
    'rs_device_count': (ctypes.c_int, []),
    'rs_dev_malloc': (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    'rs_dev_free': (ctypes.c_int, [_vp]),
    'rs_dev_copy': (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    'rs_host_alloc': (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_vp)]),
    'rs_host_free': (ctypes.c_int, [_vp]),
    'rs_pc_create': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(PcParams), ctypes.c_int, ctypes.POINTER(_vp)]),
    'rs_pc_destroy': (ctypes.c_int, [_vp]),
    'rs_pc_shape': (ctypes.c_int, [_vp, _c_int_p, _c_int_p, _c_int_p]),
    'rs_pc_update': (ctypes.c_int, [_vp, _i32p, _i32p, _i32p, _f64p, _i32p]),
    'rs_pc_run': (ctypes.c_int, [_vp, ctypes.c_int, _i32p, _i32p, _i32p, _f64p, _i32p]),
    'rs_pc_set_odometry_tables': (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_double, _f64p, _f64p,
                                                 ctypes.c_int, ctypes.c_int, _i32p, ctypes.c_int,
                                                 ctypes.c_int, _f64p]),
    'rs_pc_update_odom': (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_double, _i32p]),
    'rs_pc_odom_control': (ctypes.c_int, [ctypes.c_int, ctypes.c_double, ctypes.c_double, _f64p,
                                          _f64p, ctypes.c_int, ctypes.c_int, _i32p, ctypes.c_int,
                                          ctypes.c_int, _f64p, ctypes.c_int, _f64p, _i32p, _i32p,
                                          _i32p, _f64p, _i32p]),
    'rs_pc_run_odom': (ctypes.c_int, [_vp, ctypes.c_int, _f64p, _i32p, _c_int_p]),
    'rs_pc_excite': (ctypes.c_int, [_vp]),
    'rs_pc_inject': (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    'rs_pc_get_max': (ctypes.c_int, [_vp, _i32p]),
    'rs_pc_read': (ctypes.c_int, [_vp, _f64p]),
    'rs_pc_read_pinned': (ctypes.c_int, [_vp, _vp]),
    'rs_pc_update_odom_read': (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_double, _i32p, _vp]),
    'rs_pc_write': (ctypes.c_int, [_vp, _f64p]),
    'rs_pc_total': (ctypes.c_int, [_vp, _f64p]),
    'rs_pc_last_ms': (ctypes.c_int, [_vp, _f64p]),
    'rs_pc_set_profiling': (ctypes.c_int, [_vp, ctypes.c_int]),
    'rs_pc_kernel_ms': (ctypes.c_int, [_vp, _f64p]),
    'rs_pc_step_form': (ctypes.c_char_p, [_vp]),
    'rs_pc_debug': (ctypes.c_int, [_vp, ctypes.c_int]),
    'rs_pc_debug_value': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    'rs_vt_create': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                    ctypes.c_int64, ctypes.c_int, ctypes.POINTER(_vp)]),
    'rs_vt_destroy': (ctypes.c_int, [_vp]),
    'rs_vt_count': (ctypes.c_int, [_vp, _i64p]),
    'rs_vt_add': (ctypes.c_int, [_vp, ctypes.c_int, _u8p, _i64p]),
    'rs_vt_read': (ctypes.c_int, [_vp, ctypes.c_int64, _u8p]),
    'rs_vt_match_batch': (ctypes.c_int, [_vp, ctypes.c_int, _u8p, ctypes.c_int, _u64p, _i64p, _u8p]),
    'rs_vt_match_stream': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _u64p, _i64p]),
    'rs_vt_match': (ctypes.c_int, [_vp, _u8p, _u64p, _i64p, _c_int_p]),
    'rs_vt_scores': (ctypes.c_int, [_vp, ctypes.c_int, _u8p, ctypes.c_int64, ctypes.c_int64, _u64p]),
    'rs_vt_set_subsample': (ctypes.c_int, [_vp, ctypes.c_int64, _i32p]),
    'rs_vt_match_frames': (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, _u64p, _i64p, _u8p]),
    'rs_vt_scan_local': (ctypes.c_int, [_vp, ctypes.c_int, _u8p, _u64p]),
    'rs_vt_resolve': (ctypes.c_int, [_vp, ctypes.c_int, _u64p, ctypes.c_int, _u64p, _i64p, _u8p]),
    'rs_vt_last_ms': (ctypes.c_int, [_vp, _f64p]),
    'rs_vt_set_timing': (ctypes.c_int, [_vp, ctypes.c_int]),
    'rs_vt_scan_form': (ctypes.c_char_p, [_vp]),
    'rs_vt_set_threshold': (ctypes.c_int, [_vp, ctypes.c_double]),
    'rs_sad_scores': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int64, _vp, ctypes.c_int, _vp, _vp]),
    'rs_comm_unique_id': (ctypes.c_int, [_u8p]),
    'rs_vt_attach_comm': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _u8p]),
    'rs_vt_set_shard': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    'rs_vt_rank': (ctypes.c_int, [_vp, _c_int_p, _c_int_p]),
}

_lib = None
_lock = threading.Lock()


class HipLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or reported a runtime error."""


def load(path=LIB_PATH):
    """Load (once) and return the ctypes handle; raises if the .so is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise HipLibraryError(
                f'{path} not found: build it with `python -m pyratslam_amd._build` '
                '(there is no CPU fallback)')
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(status):
    """Map an rs_* status code to the exception the reference would raise."""
    if status == RS_OK:
        return
    msg = (_lib.rs_last_error() or b'').decode(errors='replace') if _lib else ''
    if status == RS_ERR_ARG:
        raise ValueError(msg)
    if status == RS_ERR_TYPE:
        raise TypeError(msg)
    if status == RS_ERR_LUT_KEY:
        raise KeyError(msg)
    if status == RS_ERR_NOMEM:
        raise MemoryError(msg)
    raise HipLibraryError(f'rs status {status}: {msg}')


def require_device():
    """Load the library and make sure a HIP device is visible."""
    lib = load()
    n = lib.rs_device_count()
    if n <= 0:
        raise HipLibraryError('no HIP device visible: the pyratslam_amd hot path runs only on '
                              'an AMD GPU (gfx950); there is no CPU fallback')
    return lib


def ptr(a, ctype):
    """ctypes pointer to a contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def as_c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class DeviceBuffer:
    """A block of HBM owned by the caller (rs_dev_malloc); ``ptr`` is the device
    address, usable wherever the C ABI accepts device-resident inputs."""

    def __init__(self, nbytes, device=0):
        self._lib = require_device()
        p = ctypes.c_void_p()
        check(self._lib.rs_dev_malloc(int(device), int(nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p, int(nbytes)

    def upload(self, array):
        import numpy as np
        a = np.ascontiguousarray(array)
        if a.nbytes > self.nbytes:
            raise ValueError('%d bytes do not fit a %d-byte buffer' % (a.nbytes, self.nbytes))
        check(self._lib.rs_dev_copy(self.ptr, ctypes.c_void_p(a.ctypes.data), a.nbytes))
        return self

    def offset(self, byte_offset):
        """A view of the buffer from ``byte_offset`` on (``ptr`` / ``nbytes``), kept
        valid by a reference to this buffer."""
        if not 0 <= byte_offset <= self.nbytes:
            raise ValueError('offset %d outside the %d-byte buffer' % (byte_offset, self.nbytes))
        return DeviceView(self, int(byte_offset))

    def close(self):
        if getattr(self, 'ptr', None) is not None and self.ptr.value:
            self._lib.rs_dev_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceView:
    """``DeviceBuffer.offset``: a sub-range of a device buffer."""

    def __init__(self, base, byte_offset):
        self._base = base
        self.ptr = ctypes.c_void_p(base.ptr.value + byte_offset)
        self.nbytes = base.nbytes - byte_offset
