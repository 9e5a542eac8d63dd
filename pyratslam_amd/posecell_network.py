"""Drop-in ``PoseCellNetwork`` backed by the MI355X kernels of libratslam_hip.

API of ``/root/reference/ratslam/posecell_network.py:22-353``: ``PoseCellNetwork(shape)``,
``update(v)`` -> ``max_pc`` (also stored as ``.max_pc``), ``inject(energy, loc)``,
``get_pc_max()``, ``.posecells`` (float64 ndarray, C order (X, Y, TH)), ``.shape``,
plus the filter helpers the reference exposes.  ``step(v)`` is an alias of
``update`` (the name BASELINE.json's north_star uses) and ``run(odometry)``
performs many updates with one host round trip.

The pose-cell volume lives on the GPU; ``.posecells`` copies it to the host
on access (and uploads on assignment).  The per-step control scalars are
derived on the host exactly as the reference derives them (``filters``), the
volume work runs in ``pc_excite`` + ``pc_path`` (``csrc/posecell.hip``).
"""
import ctypes
import math
import threading
import weakref

import numpy as np

from . import _lib
from . import filters as F

PC_DIM_XY = 21           # posecell_network.py:8 (unused by the reference too)
PC_DIM_TH = 36
PC_E_SIGMA = F.PC_E_SIGMA
PC_I_SIGMA = F.PC_I_SIGMA
PC_E_DIM = F.PC_E_DIM
PC_I_DIM = F.PC_I_DIM
PC_GLOBAL_INHIB = F.PC_GLOBAL_INHIB
PC_CELL_X_SIZE = F.PC_CELL_X_SIZE
PC_C_SIZE_TH = 2.0 * np.pi / PC_DIM_TH

_PRECISIONS = {'float32': _lib.RS_PREC_F32, np.float32: _lib.RS_PREC_F32,
               'float64': _lib.RS_PREC_F64, np.float64: _lib.RS_PREC_F64}


class _PinnedArrays:
    """Float64 arrays in pinned, GPU-visible host memory (rs_host_alloc), handed out
    one per ``.posecells`` read: the GPU writes the volume straight into the array
    the caller gets (rs_pc_read_pinned), so the readback needs no host-side copy.
    Each array owns its block until it is garbage-collected, when the block goes
    back to the free list (the caller's arrays never alias one another).  At most
    ``cap`` blocks exist at once: a caller that keeps every volume (a history list)
    gets ordinary pageable arrays past that (``array`` returns None), so pinned host
    memory stays bounded."""

    CAP = 8

    def __init__(self, lib, n, cap=CAP):
        self._lib, self._n, self._cap = lib, n, cap
        self._free = []
        self._blocks = 0
        # reentrant: a cyclic GC run inside a locked section can finalise one of this
        # pool's arrays on the same thread, and _release takes the lock again
        self._lock = threading.RLock()

    def array(self, shape):
        with self._lock:
            ptr = self._free.pop() if self._free else None
            if ptr is None:
                if self._blocks >= self._cap:
                    return None, None
                self._blocks += 1
        if ptr is None:
            p = ctypes.c_void_p()
            st = self._lib.rs_host_alloc(8 * self._n, ctypes.byref(p))
            if st != _lib.RS_OK:
                with self._lock:
                    self._blocks -= 1
                _lib.check(st)
            ptr = p.value
        view = (ctypes.c_double * self._n).from_address(ptr)
        weakref.finalize(view, self._release, ptr).atexit = False  # the process frees it at exit
        return np.frombuffer(view, dtype=np.float64).reshape(shape), ptr

    def _release(self, ptr):
        with self._lock:
            if not self._closed:
                self._free.append(ptr)
                return
        self._lib.rs_host_free(ctypes.c_void_p(ptr))  # an array that outlived its network

    _closed = False

    def close(self):
        empty = []   # allocated before the lock is taken
        with self._lock:
            self._closed = True
            free, self._free = self._free, empty
        for ptr in free:
            self._lib.rs_host_free(ctypes.c_void_p(ptr))


def round_up(x):  # posecell_network.py:19-20
    return math.ceil(x) if x > 0 else math.floor(x)


class PoseCellNetwork:
    """Continuous-attractor pose-cell network on one GPU.

    ``precision``: 'float32' (default; activations within 1e-5 of the float64
    reference) or 'float64'.  ``device``: HIP device ordinal.  ``readback``: 'lazy'
    (default: ``.posecells`` exports the volume when read) or 'eager' (every
    ``update()`` also exports the new volume into a pinned array before its one host
    sync, and the next ``.posecells`` read returns that array: the ROS node's
    update-then-publish step, ros_simulate.py:134-145, as one round trip).
    Extra keyword arguments are accepted and ignored, like the reference (:24).
    """

    def __init__(self, shape, precision='float32', device=0, readback='lazy', **kwargs):
        if readback not in ('lazy', 'eager'):
            raise ValueError("readback must be 'lazy' or 'eager', got %r" % (readback,))
        self._eager = readback == 'eager'
        self._fresh = None   # eager: the volume exported by the last update()
        if len(shape) != 3:
            raise TypeError('PoseCellNetwork shape must be (X, Y, TH), got %r' % (shape,))
        self.shape = tuple(int(s) for s in shape)
        self.precision = 'float32' if _PRECISIONS[precision] == _lib.RS_PREC_F32 else 'float64'
        self.device = int(device)
        self.global_inhibition = PC_GLOBAL_INHIB
        self.pc_vtrans_scale = PC_CELL_X_SIZE
        self.pc_vrot_scale = 2.0 * np.pi / self.shape[2]
        self.kernel_3d = F.kernel_3d()
        # the reference's unused attributes (posecell_network.py:30-32)
        self.kernel_2d = F.diff_gaussian(order=2)
        self.kernel_1d = F.diff_gaussian(order=1)
        self.kernel_1d_sep = F.diff_gaussian_separable()
        self.filter_table = F.FilterTable()
        self.filter_dict_2d = self.filter_table.dict
        self.filter_dict_2d_precision = F.LUT_PRECISION
        self.max_pc = None
        self._max_valid = False
        self._mutex = threading.Lock()
        self._h = None
        self._pinned = None
        self._lib = _lib.require_device()
        ge, gi, scale = F.separable_factors()
        self._table = np.ascontiguousarray(self.filter_table.filters, dtype=np.float64)
        params = _lib.PcParams()
        params.precision = _PRECISIONS[precision]
        params.global_inhibition = self.global_inhibition
        params.ge[:] = list(ge)
        params.gi[:] = list(gi)
        params.k_scale = scale
        params.nfilters = self._table.shape[0]
        params.xy_filters = _lib.ptr(self._table, ctypes.c_double)
        h = ctypes.c_void_p()
        _lib.check(self._lib.rs_pc_create(*self.shape, ctypes.byref(params), self.device,
                                          ctypes.byref(h)))
        self._h = h
        # fast path of update(): raw addresses, preallocated output
        self._update = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p)(('rs_pc_update', self._lib))
        self._out3 = np.empty(3, dtype=np.int32)
        self._out3_addr = self._out3.ctypes.data
        self._upload_odometry_tables()
        self._update_odom = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                             ctypes.c_double, ctypes.c_void_p)(
            ('rs_pc_update_odom', self._lib))
        self._update_odom_read = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                                  ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p)(
            ('rs_pc_update_odom_read', self._lib))

    def _upload_odometry_tables(self):
        """Tables for the library-side control of update()/run() (filters.odometry_tables)."""
        self._odo_tables = F.odometry_tables(self.shape[2], self.filter_table)
        _lib.check(self._lib.rs_pc_set_odometry_tables(self._h, *F.table_args(self._odo_tables)))

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        st = 0
        if self._h is not None and self._h.value:
            st = self._lib.rs_pc_destroy(self._h)   # (reports an error of queued work)
        self._h = None
        if getattr(self, '_pinned', None) is not None:
            self._pinned.close()
            self._pinned = None
        _lib.check(st)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- state ------------------------------------------------------------------
    @property
    def posecells(self):
        """Copy of the activity volume, float64 C order (X, Y, TH) (posecell_network.py:27).

        The GPU writes it straight into a fresh pinned host array (no host-side copy;
        ros_simulate.py:140,145 reads it after every update)."""
        with self._mutex:
            if self._fresh is not None:   # exported by the last update() (readback='eager')
                out, self._fresh = self._fresh, None
                return out
            out, ptr = self._pinned_array()
            if out is None:   # the pinned pool is all held by the caller: pageable copy
                out = np.empty(self.shape, dtype=np.float64)
                _lib.check(self._lib.rs_pc_read(self._h, _lib.ptr(out, ctypes.c_double)))
            else:
                _lib.check(self._lib.rs_pc_read_pinned(self._h, ctypes.c_void_p(ptr)))
        return out

    def _pinned_array(self):
        if self._pinned is None:
            self._pinned = _PinnedArrays(self._lib, int(np.prod(self.shape)))
        return self._pinned.array(self.shape)

    @posecells.setter
    def posecells(self, value):
        v = np.asarray(value)
        if v.shape != self.shape:
            raise TypeError('posecells must have shape %r, got %r' % (self.shape, v.shape))
        v = np.ascontiguousarray(v, dtype=np.float64)
        with self._mutex:
            self._fresh = None
            _lib.check(self._lib.rs_pc_write(self._h, _lib.ptr(v, ctypes.c_double)))
            self._max_valid = False

    def total(self):
        t = ctypes.c_double()
        with self._mutex:
            _lib.check(self._lib.rs_pc_total(self._h, ctypes.byref(t)))
        return t.value

    # -- reference API ----------------------------------------------------------
    def inject(self, energy, loc):
        """posecells[loc] += energy for one cell ``loc = (x, y, th)`` (posecell_network.py:322-324)."""
        if isinstance(loc, list):
            raise TypeError('inject expects a tuple (x, y, th); the reference would fancy-index '
                            'whole planes with a list (posecell_network.py:324)')
        x, y, th = (int(v) for v in loc)
        X, Y, TH = self.shape
        # numpy indexing semantics: negative indices count from the end
        x, y, th = x + X if x < 0 else x, y + Y if y < 0 else y, th + TH if th < 0 else th
        if not (0 <= x < X and 0 <= y < Y and 0 <= th < TH):
            raise IndexError('inject location %r outside grid %r' % (loc, self.shape))
        with self._mutex:
            self._fresh = None
            _lib.check(self._lib.rs_pc_inject(self._h, float(energy), x, y, th))
            self._max_valid = False

    def get_pc_max(self):
        """Argmax cell (first maximum in C order) (posecell_network.py:317-319)."""
        with self._mutex:
            if self._max_valid:
                return self.max_pc
            out = np.empty(3, dtype=np.int32)
            _lib.check(self._lib.rs_pc_get_max(self._h, _lib.ptr(out, ctypes.c_int32)))
        return tuple(int(v) for v in out)

    def update(self, v=(0.0, 0.0)):
        """One network step (posecell_network.py:326-353); returns and stores max_pc.

        One FFI call: the library derives path_integration's control from (vtrans,
        vrot) bit-identically to filters.step_control (rs_pc_update_odom)."""
        vtrans, vrot = float(v[0]), float(v[1])
        out = self._out3
        with self._mutex:
            self._fresh = None
            arr, ptr = self._pinned_array() if self._eager else (None, None)
            if arr is not None:
                st = self._update_odom_read(self._h, vtrans, vrot, self._out3_addr, ptr)
                if st == _lib.RS_OK:
                    self._fresh = arr
            else:
                st = self._update_odom(self._h, vtrans, vrot, self._out3_addr)
            if st == _lib.RS_OK:
                self.max_pc = (int(out[0]), int(out[1]), int(out[2]))
                self._max_valid = True
                return self.max_pc
            if st == _lib.RS_ERR_LUT_KEY:
                # steps 1-4 ran in the library; raise the reference's KeyError((k, k))
                self._max_valid = False
                F.step_control(vtrans, vrot, self.shape[2], self.filter_table)
                raise KeyError('path-integration LUT miss')  # pragma: no cover
            if st != _lib.RS_ERR_CTL_RANGE:
                _lib.check(st)
        return self._update_host_control(vtrans, vrot)

    def _update_host_control(self, vtrans, vrot):
        """update() with the control computed here in NumPy (filters.step_control) and
        handed to rs_pc_update: for odometry outside the library's control tables."""
        try:
            ox, oy, rows, zf, _ = F.step_control(vtrans, vrot, self.shape[2], self.filter_table)
        except KeyError:
            # the reference raises inside path_integration, after steps 1-4 ran
            with self._mutex:
                _lib.check(self._lib.rs_pc_excite(self._h))
                self._max_valid = False
            raise
        out = self._out3
        with self._mutex:
            st = self._update(self._h, ox.ctypes.data, oy.ctypes.data, rows.ctypes.data,
                              zf.ctypes.data, self._out3_addr)
            if st:
                _lib.check(st)
            self.max_pc = (int(out[0]), int(out[1]), int(out[2]))
            self._max_valid = True
        return self.max_pc

    step = update

    def run(self, odometry):
        """``update`` for every row (vtrans, vrot) of ``odometry``; one host round trip.

        Returns an int32 array (n, 3) of max_pc per step.  A LUT KeyError at step
        s leaves the state the reference would (steps < s done, then steps 1-4 of s).
        """
        od = np.ascontiguousarray(np.asarray(odometry, dtype=np.float64).reshape(-1, 2))
        n = od.shape[0]
        if n == 1 and not self._eager:
            # one step (the ROS node's queue drain, usually): update()'s prebound call,
            # the same library step and the same KeyError / host-control fallbacks
            return np.array([self.update(od[0])], dtype=np.int32)
        out = np.empty((n, 3), dtype=np.int32)
        bad = ctypes.c_int(-1)
        with self._mutex:
            self._fresh = None
            st = self._lib.rs_pc_run_odom(self._h, n, _lib.ptr(od, ctypes.c_double),
                                          _lib.ptr(out, ctypes.c_int32), ctypes.byref(bad))
            if st in (_lib.RS_OK, _lib.RS_ERR_LUT_KEY):
                todo = n if st == _lib.RS_OK else bad.value
                if todo > 0:
                    self.max_pc = tuple(int(v) for v in out[todo - 1])
                    self._max_valid = True
                if st == _lib.RS_ERR_LUT_KEY:
                    self._max_valid = False
            elif st != _lib.RS_ERR_CTL_RANGE:
                _lib.check(st)
        if st == _lib.RS_ERR_CTL_RANGE:
            return self._run_host_control(od)
        if st == _lib.RS_ERR_LUT_KEY:
            F.step_control(od[bad.value, 0], od[bad.value, 1], self.shape[2], self.filter_table)
            raise KeyError('LUT miss at step %d' % bad.value)  # pragma: no cover
        return out

    def _run_host_control(self, od):
        """run() with the control computed here (filters.batch_control) and handed to
        rs_pc_run: for odometry outside the library's control tables."""
        n = od.shape[0]
        ox, oy, rows, zf, first_bad = F.batch_control(od, self.shape[2], self.filter_table)
        todo = n if first_bad is None else first_bad
        out = np.empty((n, 3), dtype=np.int32)
        with self._mutex:
            if todo > 0:
                _lib.check(self._lib.rs_pc_run(
                    self._h, todo, _lib.ptr(ox, ctypes.c_int32), _lib.ptr(oy, ctypes.c_int32),
                    _lib.ptr(rows, ctypes.c_int32), _lib.ptr(zf, ctypes.c_double),
                    _lib.ptr(out, ctypes.c_int32)))
                self.max_pc = tuple(int(v) for v in out[todo - 1])
                self._max_valid = True
            if first_bad is not None:
                _lib.check(self._lib.rs_pc_excite(self._h))
                self._max_valid = False
        if first_bad is not None:
            F.step_control(od[first_bad, 0], od[first_bad, 1], self.shape[2], self.filter_table)
            raise KeyError('LUT miss at step %d' % first_bad)  # pragma: no cover
        return out

    def device_ms(self):
        """Device time (HIP events) of the last update/run, in ms; recorded only while
        profiling is enabled (``set_profiling``), else 0."""
        ms = ctypes.c_double()
        _lib.check(self._lib.rs_pc_last_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def step_form(self):
        """Step kernels in use: 'rows', 'tiles', 'cols', 'halo' or 'stream' (rs_pc_step_form)."""
        return self._lib.rs_pc_step_form(self._h).decode()

    def set_profiling(self, enable=True, per_kernel=True):
        """HIP events around each update()/run() (device_ms) and, with per_kernel, around
        every launch too (kernel_ms; those events add gaps between the kernels)."""
        _lib.check(self._lib.rs_pc_set_profiling(self._h, 0 if not enable else (1 if per_kernel else 2)))

    def kernel_ms(self):
        """Kernel times of the last run (profiling on, per_kernel=True), as
        rs_pc_kernel_ms returns them: (excite_ms, path_ms) summed over the steps for
        the two-launch forms (rows, tiles, cols, tc, stream); for the halo form
        (step_ms, finish_ms): the step kernels summed, then the one pc_halo_finish."""
        ms = np.zeros(2)
        _lib.check(self._lib.rs_pc_kernel_ms(self._h, _lib.ptr(ms, ctypes.c_double)))
        return float(ms[0]), float(ms[1])

    # -- filter helpers of the reference class (host-side, NumPy) -----------------
    def diff_gaussian(self, dim_e, dim_i, sigma_e, sigma_i, order=3):
        return F.diff_gaussian(dim_e, dim_i, sigma_e, sigma_i, order)

    def diff_gaussian_separable(self, dim_e, dim_i, sigma_e, sigma_i):
        return F.diff_gaussian_separable(dim_e, dim_i, sigma_e, sigma_i)

    def diff_gaussian_offset_2d(self, sigma_e, sigma_i, shape=(7, 7), origin=(0, 0)):
        return F.filter_2d(origin, sigma_e, sigma_i, shape)

    def diff_gaussian_offset_1d(self, sigma_e, sigma_i, size=7, origin=0):
        return np.array(F.filter_1d(origin, sigma_e, sigma_i, size))

    def build_diff_gaussian_set_2d(self, sigma_e, sigma_i, shape=(7, 7), precision=1):
        if precision != 1 or (sigma_e, sigma_i, tuple(shape)) != (PC_E_SIGMA, PC_I_SIGMA, (7, 7)):
            span = range(-5 * precision, 5 * precision)
            return {(x, y): F.filter_2d((x // (precision * 10), y // (precision * 10)),
                                        sigma_e, sigma_i, shape) for x in span for y in span}
        return dict(self.filter_dict_2d)

    def filters_from_origins_approx(self, origins, shape=(7, 7)):
        """LUT lookup per layer (posecell_network.py:244-250); KeyError on a miss."""
        origins = np.asarray(origins)
        keys = np.trunc(origins[0] * self.filter_dict_2d_precision).astype(np.int64)
        rows = self.filter_table.rows_for_keys(keys)
        return np.ascontiguousarray(np.moveaxis(self.filter_table.filters[rows], 0, -1))
