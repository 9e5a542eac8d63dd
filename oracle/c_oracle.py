"""ctypes wrapper of oracle/lib/libratslam_oracle.so (the C/OpenMP restatement).

TEST INFRASTRUCTURE / CPU BASELINE ONLY -- see oracle/__init__.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'lib', 'libratslam_oracle.so')
_lib = None


def load(build=True):
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) and build:
            subprocess.check_call(['make', '-s', '-C', os.path.join(HERE, 'c')])
        _lib = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        i = ctypes.c_int
        _lib.ro_threads.restype = i
        _lib.ro_set_threads.argtypes = [i]
        _lib.ro_update.argtypes = [vp, vp, vp, ctypes.c_double, vp, vp, vp, vp, i, i, i, vp]
        _lib.ro_vt_scores.argtypes = [vp, ctypes.c_int64, vp, i, i, i, vp]
        _lib.ro_vt_best.argtypes = [vp, ctypes.c_int64, vp, i, i, i, i, vp, vp]
    return _lib


def _p(a):
    return a.ctypes.data


class PoseCellC:
    """Float64 pose-cell network stepping through the C kernels; control from the
    NumPy oracle (oracle.posecell.step_control)."""

    def __init__(self, shape):
        from . import posecell as P
        self.P = P
        self.shape = tuple(int(s) for s in shape)
        self.posecells = np.zeros(self.shape)
        self.tmp = np.zeros(self.shape)
        self.k3 = np.ascontiguousarray(P.dog_kernel_3d())
        self.lut = P.lut_2d()
        self.out = np.zeros(3, dtype=np.int32)
        load()

    def inject(self, energy, loc):
        self.posecells[tuple(int(v) for v in loc)] += energy

    def update(self, v):
        c = self.P.step_control(v[0], v[1], self.shape, self.lut)
        ox = np.ascontiguousarray(c['ox'], dtype=np.int32)
        oy = np.ascontiguousarray(c['oy'], dtype=np.int32)
        F = np.ascontiguousarray(c['filters'])
        zf = np.ascontiguousarray(c['zf'])
        _lib.ro_update(_p(self.posecells), _p(self.tmp), _p(self.k3), 0.2, _p(ox), _p(oy), _p(F),
                       _p(zf), *self.shape, _p(self.out))
        return tuple(int(x) for x in self.out)


def vt_best(library, queries, max_offset=8):
    """(best_score uint64[nq], best_index int64[nq]) over a frozen (T, H, W) uint8 library."""
    load()
    lib = np.ascontiguousarray(library, dtype=np.uint8)
    q = np.ascontiguousarray(queries, dtype=np.uint8)
    t, h, w = lib.shape
    s = np.empty(len(q), dtype=np.uint64)
    i = np.empty(len(q), dtype=np.int64)
    _lib.ro_vt_best(_p(lib), t, _p(q), len(q), h, w, max_offset, _p(s), _p(i))
    return s, i


def threads():
    return load().ro_threads()


def set_threads(n):
    load().ro_set_threads(int(n))
