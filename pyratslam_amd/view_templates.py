"""Drop-in ``ViewTemplate`` / ``ViewTemplates`` backed by libratslam_hip.

API of ``/root/reference/ratslam/view_templates.py``: ``ViewTemplates(x_range,
y_range, x_step, y_step, im_x, im_y, match_threshold)`` with ``.match(input,
pc_x, pc_y, pc_th)`` -> ``ViewTemplate`` (``.get_index()``, ``.location()``,
``.template``, ``.match(other)``) and the ``.templates`` list.

The library lives on the GPU (``csrc/view_templates.hip``); each match scans it
with the wrapped-uint8 row-shift score and applies the reference's strict
threshold / first-argmin / append-on-miss rule.  ``match_batch`` runs many
matches with the exact sequential semantics in one call.
``ShardedViewTemplates`` spreads the library over ranks (one GPU each).

Frames are ``uint8`` on the ROS path (``ros_simulate.py:100-101``): the library
then lives on the GPU and a score wraps mod 256 like numpy's uint8 subtraction.
float32 / float64 frames follow the reference's float semantics instead (a true
sum of |T - Q| in numpy's summation order, ``rs_sad_scores`` on the GPU): once a
float frame is matched the library is scored pair-wise per match (a fidelity
path for float callers, not the throughput path).  The subsampling mask is the
reference's, with Python-2 integer division (:44-54).
"""
import ctypes
import threading

import numpy as np

from . import _lib

MAX_OFFSET = 8  # view_templates.py:14
_FLOAT_CODES = {np.dtype(np.float32): _lib.RS_DT_F32, np.dtype(np.float64): _lib.RS_DT_F64}


def sad_scores(templates, queries, max_offset=MAX_OFFSET, device=0):
    """``ViewTemplate.match`` (view_templates.py:16-28) of every (query, template)
    pair of float arrays on the GPU: (nq, nt) scores in numpy's result dtype of the
    two arrays (float32 or float64), bit-exact to the reference's numpy arithmetic."""
    t = np.asarray(templates)
    q = np.asarray(queries)
    dt = np.result_type(t.dtype, q.dtype)
    if dt not in _FLOAT_CODES:
        raise TypeError('ViewTemplate.match takes uint8 (wrapping) or float32/float64 arrays; '
                        'got %s and %s' % (t.dtype, q.dtype))
    if t.ndim != 3 or q.ndim != 3 or t.shape[1:] != q.shape[1:]:
        raise ValueError('template / query shapes %r, %r differ' % (t.shape[1:], q.shape[1:]))
    t = np.ascontiguousarray(t, dtype=dt)
    q = np.ascontiguousarray(q, dtype=dt)
    out = np.empty((q.shape[0], t.shape[0]), dtype=dt)
    lib = _lib.require_device()
    _lib.check(lib.rs_sad_scores(int(device), _FLOAT_CODES[dt], t.shape[1], t.shape[2], int(max_offset),
                                 t.shape[0], ctypes.c_void_p(t.ctypes.data), q.shape[0],
                                 ctypes.c_void_p(q.ctypes.data), ctypes.c_void_p(out.ctypes.data)))
    return out


def _wrapped_scores(templates, queries, device=0):
    """uint8 pair scores through a temporary device library (float-mode libraries
    that also hold uint8 templates)."""
    t = np.ascontiguousarray(templates, dtype=np.uint8)
    lib = ViewTemplates._from_shape(t.shape[1:], np.inf, device=device, capacity=len(t))
    try:
        lib.add(t)
        return lib.scores(queries)
    finally:
        lib.close()


def py2_mask(x_range, y_range, x_step, y_step, im_x, im_y):
    """``ViewTemplates.__init__`` mask and template shape (view_templates.py:42-57)."""
    pix = np.arange(im_x * im_y)
    r, c = np.divmod(pix, im_x)
    keep = (r > y_range[0]) & (r < y_range[1]) & (c > x_range[0]) & (c < x_range[1])
    keep &= ((r - y_range[0]) % y_step != 0) & ((c - x_range[0]) % x_step != 0)
    shape = ((x_range[1] - x_range[0]) // x_step, (y_range[1] - y_range[0]) // y_step)
    return keep.reshape((im_x, im_y)), shape


class ViewTemplate:
    """One stored view (view_templates.py:4-37)."""

    def __init__(self, pc_x, pc_y, pc_th, index, template, _owner=None):
        self.pc_x = pc_x
        self.pc_y = pc_y
        self.pc_th = pc_th
        self.template = template
        self.index = index
        self.max_offset = MAX_OFFSET
        self._owner = _owner
        self._solo = None

    def match(self, new_template):
        """Row-shift score against ``new_template`` (view_templates.py:16-28), on the
        GPU: uint8 arrays wrap mod 256 (numpy uint8 arithmetic, a numpy.uint64
        score); float arrays give numpy's true sum of |T - Q| in their dtype."""
        if self.template is None:
            owner = self._owner
            raise ValueError('the bytes of template %d live on rank %d (template g is stored on '
                             'rank g %% %d): score it there' % (self.index, self.index % owner.nranks,
                                                                owner.nranks))
        q = np.ascontiguousarray(new_template)
        t = np.asarray(self.template)
        dev = self._owner.device if self._owner is not None else 0
        if t.dtype != np.uint8 or q.dtype != np.uint8:
            return sad_scores(t[None], q[None], self.max_offset, dev)[0, 0]
        owner = self._owner
        if owner is not None and owner.nranks == 1 and not owner._float:
            return owner.scores(q[None], self.index, 1)[0, 0]
        if self._solo is None:
            t = np.ascontiguousarray(t)
            self._solo = ViewTemplates._from_shape(t.shape, np.inf, device=dev)
            self._solo.add(t[None])
        return self._solo.scores(q[None], 0, 1)[0, 0]

    def location(self):
        return (self.pc_x, self.pc_y, self.pc_th)

    def get_index(self):
        return self.index


class ViewTemplates:
    """Library of view templates on one GPU (view_templates.py:40-75)."""

    def __init__(self, x_range, y_range, x_step, y_step, im_x, im_y, match_threshold,
                 device=0, capacity=1024):
        self.mask, self.shape = py2_mask(x_range, y_range, x_step, y_step, im_x, im_y)
        self._init_device(self.shape, match_threshold, device, capacity)

    @classmethod
    def _from_shape(cls, shape, match_threshold, device=0, capacity=64):
        self = cls.__new__(cls)
        self.mask = None
        self.shape = tuple(int(s) for s in shape)
        self._init_device(self.shape, match_threshold, device, capacity)
        return self

    def _init_device(self, shape, match_threshold, device, capacity):
        self.shape = (int(shape[0]), int(shape[1]))
        self.match_threshold = match_threshold
        self.templates = []
        self.device = int(device)
        self.rank, self.nranks = 0, 1
        self._float = False      # float frames seen: pair-wise float scoring (module doc)
        self._mutex = threading.Lock()
        self._h = None
        self._lib = _lib.require_device()
        h = ctypes.c_void_p()
        _lib.check(self._lib.rs_vt_create(self.shape[0], self.shape[1], MAX_OFFSET, 0,
                                          int(capacity), self.device, ctypes.byref(h)))
        self._h = h
        # `min(match_val) > match_threshold` (view_templates.py:67), compared in float64 as
        # numpy compares the uint64 score with a Python number (inf: never, < 0: always)
        _lib.check(self._lib.rs_vt_set_threshold(h, float(match_threshold)))

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        st = 0
        if getattr(self, '_h', None) is not None and self._h.value:
            st = self._lib.rs_vt_destroy(self._h)   # (reports an error of queued work)
        self._h = None
        _lib.check(st)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return len(self.templates)

    def __getitem__(self, index):
        return self.templates[index]

    # -- helpers ----------------------------------------------------------------
    def subsample(self, image):
        """``input[self.mask].reshape(self.shape)`` (view_templates.py:64)."""
        im = np.asarray(image)
        if im.dtype != np.uint8 and im.dtype not in _FLOAT_CODES:
            raise TypeError('ViewTemplates matches uint8 (mono8, ros_simulate.py:100-101) or '
                            'float32/float64 frames; got %s' % im.dtype)
        if im.shape != self.mask.shape:
            raise ValueError('frame shape %r does not match the mask %r' % (im.shape, self.mask.shape))
        # input[mask] takes the kept pixels in C order: the same bytes as a take of the
        # mask's flat indices (one gather, no boolean pass over the frame; 12.6 -> ~3 us
        # per ROS frame), the indices cached per mask object
        cache = getattr(self, '_mask_take', None)
        if cache is None or cache[0] is not self.mask:
            cache = (self.mask, np.flatnonzero(self.mask.ravel()))
            self._mask_take = cache
        return im.reshape(-1).take(cache[1]).reshape(self.shape)

    def _check_templates(self, t):
        t = np.asarray(t)
        if t.dtype != np.uint8:
            raise TypeError('templates must be uint8, got %s' % t.dtype)
        if t.shape[-2:] != self.shape:
            raise ValueError('template shape %r != %r' % (t.shape[-2:], self.shape))
        return np.ascontiguousarray(t.reshape((-1,) + self.shape))

    def count(self):
        c = ctypes.c_int64()
        _lib.check(self._lib.rs_vt_count(self._h, ctypes.byref(c)))
        return c.value

    def _refuse_float(self, what):
        # after a float frame the Python template list holds templates the device
        # library does not (the float path scores pair-wise on the host's list)
        if self._float:
            raise TypeError('this library has matched float frames: %s works on uint8 '
                            'device libraries only; use match() / match_batch()' % what)

    def add(self, templates, locations=None):
        """Append templates unconditionally (indices len .. len+n-1)."""
        self._refuse_float('add()')
        t = self._check_templates(templates)
        first = ctypes.c_int64()
        with self._mutex:
            _lib.check(self._lib.rs_vt_add(self._h, t.shape[0], _lib.ptr(t, ctypes.c_uint8),
                                           ctypes.byref(first)))
            for i in range(t.shape[0]):
                loc = locations[i] if locations is not None else (0, 0, 0)
                self.templates.append(ViewTemplate(loc[0], loc[1], loc[2], first.value + i, t[i],
                                                   _owner=self))
        return first.value

    def scores(self, queries, t0=0, nt=None):
        """uint64 (nq, nt) scores of queries vs templates [t0, t0+nt) -- ViewTemplate.match."""
        self._refuse_float('scores()')
        q = self._check_templates(queries)
        nt = self.count() - t0 if nt is None else nt
        out = np.empty((q.shape[0], nt), dtype=np.uint64)
        with self._mutex:
            _lib.check(self._lib.rs_vt_scores(self._h, q.shape[0], _lib.ptr(q, ctypes.c_uint8),
                                              int(t0), int(nt), _lib.ptr(out, ctypes.c_uint64)))
        return out

    # -- matching ----------------------------------------------------------------
    def _record(self, q, pcs, idx, new):
        for i in range(q.shape[0]):
            if new[i]:
                assert idx[i] == len(self.templates), (idx[i], len(self.templates))
                p = pcs[i]
                self.templates.append(ViewTemplate(p[0], p[1], p[2], int(idx[i]), q[i].copy(),
                                                   _owner=self))
        return [self.templates[int(j)] for j in idx]

    def match_templates(self, queries, pcs=None, mode=_lib.RS_VT_SEQUENTIAL):
        """Match already-subsampled (nq, H, W) queries; returns (index, score, is_new)."""
        self._refuse_float('match_templates()')
        q = self._check_templates(queries)
        n = q.shape[0]
        idx = np.empty(n, dtype=np.int64)
        score = np.empty(n, dtype=np.uint64)
        new = np.zeros(n, dtype=np.uint8)
        with self._mutex:
            _lib.check(self._lib.rs_vt_match_batch(
                self._h, n, _lib.ptr(q, ctypes.c_uint8), mode, _lib.ptr(score, ctypes.c_uint64),
                _lib.ptr(idx, ctypes.c_int64), _lib.ptr(new, ctypes.c_uint8)))
            if mode == _lib.RS_VT_SEQUENTIAL:
                self._record(q, pcs if pcs is not None else [(0, 0, 0)] * n, idx, new)
        return idx, score, new.astype(bool)

    def match_stream(self, queries, nq=None):
        """Frozen-library matching of many batches with one host synchronisation
        (rs_vt_match_stream): ``queries`` is a uint8 (nb, nq, H, W) host array, or
        ``(nb, nq, _lib.DeviceBuffer)`` for batches already in HBM.  Returns
        ``(index, score)`` shaped (nb, nq); nothing is appended."""
        self._refuse_float('match_stream()')
        if isinstance(queries, tuple):
            nb, nq, buf = int(queries[0]), int(queries[1]), queries[2]
            if nb * nq * self.shape[0] * self.shape[1] > buf.nbytes:
                raise ValueError('%d x %d queries exceed the %d-byte device buffer'
                                 % (nb, nq, buf.nbytes))
            qptr, keep = buf.ptr, buf
        else:
            q = np.asarray(queries)
            if q.ndim != 4:
                raise ValueError('match_stream takes (nb, nq, H, W) queries, got %r' % (q.shape,))
            nb = q.shape[0]
            q = self._check_templates(q.reshape((-1,) + q.shape[2:])).reshape(q.shape)
            nq = q.shape[1]
            qptr, keep = ctypes.c_void_p(q.ctypes.data), q
        idx = np.empty((nb, nq), dtype=np.int64)
        score = np.empty((nb, nq), dtype=np.uint64)
        with self._mutex:
            _lib.check(self._lib.rs_vt_match_stream(self._h, nb, nq, qptr,
                                                    _lib.ptr(score, ctypes.c_uint64),
                                                    _lib.ptr(idx, ctypes.c_int64)))
        del keep
        return idx, score

    def match(self, input, pc_x, pc_y, pc_th):
        """Best template for a frame, or a new one (view_templates.py:63-75)."""
        t = self.subsample(input)
        if t.dtype != np.uint8 or self._float:
            return self._match_float(t, (pc_x, pc_y, pc_th))
        idx, _, _ = self.match_templates(t[None], [(pc_x, pc_y, pc_th)])
        return self.templates[int(idx[0])]

    def match_batch(self, images, pcs):
        """``[match(im, *pc) for im, pc in zip(images, pcs)]`` in one call."""
        q = [self.subsample(im) for im in images]
        if not q:
            return []
        if self._float or any(x.dtype != np.uint8 for x in q):
            return [self._match_float(x, pc) for x, pc in zip(q, pcs)]
        idx, _, _ = self.match_templates(np.stack(q), pcs)
        return [self.templates[int(i)] for i in idx]

    def _match_float(self, template, pc):
        """ViewTemplates.match (view_templates.py:63-75) on the float path: every
        stored template scored on the GPU in numpy's dtype of the pair, then the
        reference's own rule -- builtin min over the list against the threshold,
        numpy argmin for the best."""
        if self.nranks > 1:
            raise TypeError('float frames are not supported by a sharded library')
        with self._mutex:
            self._float = True
            match_val = [None] * len(self.templates)
            groups = {}
            for i, tm in enumerate(self.templates):
                groups.setdefault(np.asarray(tm.template).dtype, []).append(i)
            for dt, ids in groups.items():
                lib = np.stack([np.asarray(self.templates[i].template) for i in ids])
                if dt == np.uint8 and template.dtype == np.uint8:
                    sc = _wrapped_scores(lib, template[None], self.device)[0]
                else:
                    sc = sad_scores(lib, template[None], MAX_OFFSET, self.device)[0]
                for i, v in zip(ids, sc):
                    match_val[i] = v
            if len(match_val) == 0 or min(match_val) > self.match_threshold:
                new = ViewTemplate(pc[0], pc[1], pc[2], len(self.templates), np.array(template),
                                   _owner=self)
                self.templates.append(new)
                return new
            return self.templates[int(np.argmin(match_val))]

    # -- on-device subsampling --------------------------------------------------
    def _ensure_gather(self):
        if getattr(self, '_gather_ready', False):
            return
        if self.mask is None:
            raise ValueError('no subsampling mask: construct with the frame geometry')
        pix = np.ascontiguousarray(np.flatnonzero(self.mask.ravel()), dtype=np.int32)
        assert pix.size == self.shape[0] * self.shape[1]
        _lib.check(self._lib.rs_vt_set_subsample(self._h, self.mask.size,
                                                 _lib.ptr(pix, ctypes.c_int32)))
        self._gather_ready = True

    def match_frames(self, frames, pcs, mode=_lib.RS_VT_SEQUENTIAL):
        """``match`` for a batch of whole frames, subsampled on the GPU
        (view_templates.py:64 as a device gather through the mask's pixel offsets).

        ``frames``: uint8 (n, im_x, im_y) host array, or frames already in HBM as
        ``(n, _lib.DeviceBuffer)`` (n whole frames back to back), gathered in
        place.  Returns ``(index, score, is_new)`` like ``match_templates``.
        """
        self._refuse_float('match_frames()')
        self._ensure_gather()
        dev = isinstance(frames, tuple)
        if dev:
            n, buf = int(frames[0]), frames[1]
            if n * self.mask.size > buf.nbytes:
                raise ValueError('%d frames of %d bytes exceed the %d-byte device buffer'
                                 % (n, self.mask.size, buf.nbytes))
            fptr = buf.ptr
        else:
            f = np.asarray(frames)
            if f.dtype != np.uint8:
                raise TypeError('ViewTemplates matches uint8 frames (mono8, ros_simulate.py:100-101); '
                                'got %s' % f.dtype)
            if f.shape[1:] != self.mask.shape:
                raise ValueError('frame shape %r does not match the mask %r' % (f.shape[1:], self.mask.shape))
            f = np.ascontiguousarray(f)
            n = f.shape[0]
            fptr = ctypes.c_void_p(f.ctypes.data)
        idx = np.empty(n, dtype=np.int64)
        score = np.empty(n, dtype=np.uint64)
        new = np.zeros(n, dtype=np.uint8)
        with self._mutex:
            _lib.check(self._lib.rs_vt_match_frames(self._h, n, fptr, mode,
                                                    _lib.ptr(score, ctypes.c_uint64),
                                                    _lib.ptr(idx, ctypes.c_int64),
                                                    _lib.ptr(new, ctypes.c_uint8)))
            if mode == _lib.RS_VT_SEQUENTIAL:
                pcs = pcs if pcs is not None else [(0, 0, 0)] * n
                for i in range(n):
                    if new[i]:
                        if dev:  # the gathered bytes: read back from the owning rank
                            t = np.empty(self.shape, dtype=np.uint8)
                            if int(idx[i]) % self.nranks == self.rank:
                                _lib.check(self._lib.rs_vt_read(self._h, int(idx[i]),
                                                                _lib.ptr(t, ctypes.c_uint8)))
                            else:
                                t = None
                        else:
                            t = f[i][self.mask].reshape(self.shape)
                        p = pcs[i]
                        assert idx[i] == len(self.templates), (idx[i], len(self.templates))
                        self.templates.append(ViewTemplate(p[0], p[1], p[2], int(idx[i]), t,
                                                           _owner=self))
        return idx, score, new.astype(bool)

    def device_ms(self):
        """Scan kernel time (HIP events) of the last match, ms; -1 if it ran untimed."""
        ms = ctypes.c_double()
        _lib.check(self._lib.rs_vt_last_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def set_timing(self, enable=True):
        """HIP events around every scan (default off; rs_vt_set_timing).  While on, a
        call waits for its keys with a stream synchronisation instead of polling them."""
        _lib.check(self._lib.rs_vt_set_timing(self._h, int(bool(enable))))

    def scan_form(self):
        """Scan kernel family used for this shape ('plane', 'carry', 'sad', ...)."""
        return self._lib.rs_vt_scan_form(self._h).decode()


class ShardedViewTemplates(ViewTemplates):
    """Template library sharded round-robin over ranks (template g on rank g % n).

    ``reducer`` combines the per-rank first-argmin keys (uint64, key = score << 32
    | g, UINT64_MAX = none):
      * ``'rccl'``: an RCCL allreduce(min) on the GPU inside the library; every
        rank calls ``rs_comm_unique_id`` on rank 0's id (``unique_id`` bytes);
      * a callable ``f(keys: uint64 ndarray) -> uint64 ndarray`` returning the
        elementwise min over ranks (e.g. torch.distributed all_reduce MIN).
    Every rank sees all queries and keeps the full ``.templates`` metadata; the
    template bytes of g live only on rank g % n.
    """

    def __init__(self, x_range, y_range, x_step, y_step, im_x, im_y, match_threshold,
                 rank, nranks, reducer='rccl', unique_id=None, device=0, capacity=1024):
        self.mask, self.shape = py2_mask(x_range, y_range, x_step, y_step, im_x, im_y)
        self._init_device(self.shape, match_threshold, device, capacity)
        self._attach(rank, nranks, reducer, unique_id)

    @classmethod
    def from_shape(cls, shape, match_threshold, rank, nranks, reducer='rccl', unique_id=None,
                   device=0, capacity=1024):
        self = cls.__new__(cls)
        self.mask = None
        self._init_device(shape, match_threshold, device, capacity)
        self._attach(rank, nranks, reducer, unique_id)
        return self

    def _attach(self, rank, nranks, reducer, unique_id):
        self.rank, self.nranks = int(rank), int(nranks)
        self.reducer = reducer
        if reducer == 'rccl':
            if unique_id is None or len(unique_id) != _lib.RS_UNIQUE_ID_BYTES:
                raise ValueError('reducer="rccl" needs the %d-byte unique id from rank 0'
                                 % _lib.RS_UNIQUE_ID_BYTES)
            uid = np.frombuffer(bytes(unique_id), dtype=np.uint8).copy()
            _lib.check(self._lib.rs_vt_attach_comm(self._h, self.rank, self.nranks,
                                                   _lib.ptr(uid, ctypes.c_uint8)))
        elif callable(reducer):
            _lib.check(self._lib.rs_vt_set_shard(self._h, self.rank, self.nranks))
        else:
            raise ValueError('reducer must be "rccl" or a callable')

    @staticmethod
    def unique_id():
        """RCCL unique id (bytes) to broadcast from rank 0."""
        lib = _lib.require_device()
        buf = np.zeros(_lib.RS_UNIQUE_ID_BYTES, dtype=np.uint8)
        _lib.check(lib.rs_comm_unique_id(_lib.ptr(buf, ctypes.c_uint8)))
        return buf.tobytes()

    def match_templates(self, queries, pcs=None, mode=_lib.RS_VT_SEQUENTIAL):
        if self.reducer == 'rccl':
            return super().match_templates(queries, pcs, mode)
        q = self._check_templates(queries)
        n = q.shape[0]
        local = np.empty(n, dtype=np.uint64)
        idx = np.empty(n, dtype=np.int64)
        score = np.empty(n, dtype=np.uint64)
        new = np.zeros(n, dtype=np.uint8)
        with self._mutex:
            _lib.check(self._lib.rs_vt_scan_local(self._h, n, _lib.ptr(q, ctypes.c_uint8),
                                                  _lib.ptr(local, ctypes.c_uint64)))
            glob = np.ascontiguousarray(self.reducer(local), dtype=np.uint64)
            _lib.check(self._lib.rs_vt_resolve(
                self._h, n, _lib.ptr(glob, ctypes.c_uint64), mode, _lib.ptr(score, ctypes.c_uint64),
                _lib.ptr(idx, ctypes.c_int64), _lib.ptr(new, ctypes.c_uint8)))
            if mode == _lib.RS_VT_SEQUENTIAL:
                self._record(q, pcs if pcs is not None else [(0, 0, 0)] * n, idx, new)
        return idx, score, new.astype(bool)

    def add(self, templates, locations=None):
        # every rank calls add with the same templates; rank g % n keeps the bytes
        return super().add(templates, locations)
