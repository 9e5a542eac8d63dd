#!/usr/bin/env python3
"""Where a headline step's time goes outside the scan kernel (GPU box): one
rs_vt_match_stream call over 10 HBM-resident batches of 1,024 queries against 1,000
templates (the bench's step), timed from Python (ViewTemplates.match_stream), from a
C loop over the ABI (tools/vt_call_loop.cpp), and with the scan's own HIP-event time;
also the C loop with best_score omitted (half the host unpacking)."""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pyratslam_amd import _lib, synthetic  # noqa: E402
from pyratslam_amd.view_templates import ViewTemplates  # noqa: E402


def main():
    so = '/tmp/vt_call_loop.so'
    subprocess.check_call(['g++', '-O2', '-shared', '-fPIC', os.path.join(ROOT, 'tools', 'vt_call_loop.cpp'),
                           '-I' + os.path.join(ROOT, 'include'), '-L' + os.path.join(ROOT, 'pyratslam_amd'),
                           '-lratslam_hip', '-Wl,-rpath,' + os.path.join(ROOT, 'pyratslam_amd'), '-o', so])
    loop = ctypes.CDLL(so)
    Q, nb, T = 1024, 10, 1000
    vts = ViewTemplates._from_shape((64, 32), 45000, device=0, capacity=T)
    vts.add(synthetic.library(T, seed=1))
    qlib = synthetic.library(T, seed=1)
    qs = [synthetic.queries_fast(qlib, Q, seed=2 + 1000 * b)[0] for b in range(nb)]
    buf = _lib.DeviceBuffer(Q * qs[0][0].nbytes * nb, device=0).upload(np.stack(qs))
    score = np.empty(nb * Q, dtype=np.uint64)
    idx = np.empty(nb * Q, dtype=np.int64)
    us = ctypes.c_double()
    for _ in range(150):                       # clocks up
        vts.match_stream((nb, Q, buf))
    res = {}
    for rnd in range(3):
        t0 = time.perf_counter()
        for _ in range(100):
            vts.match_stream((nb, Q, buf))
        res.setdefault('python_us', []).append(round((time.perf_counter() - t0) * 1e4, 1))
        _lib.check(loop.vt_call_loop(vts._h, 100, nb, Q, buf.ptr,
                                     _lib.ptr(score, ctypes.c_uint64), _lib.ptr(idx, ctypes.c_int64),
                                     ctypes.byref(us)))
        res.setdefault('c_loop_us', []).append(round(us.value, 1))
        _lib.check(loop.vt_call_loop(vts._h, 100, nb, Q, buf.ptr,
                                     None, _lib.ptr(idx, ctypes.c_int64), ctypes.byref(us)))
        res.setdefault('c_loop_index_only_us', []).append(round(us.value, 1))
        vts.set_timing(True)
        ms = []
        for _ in range(50):
            vts.match_stream((nb, Q, buf))
            ms.append(vts.device_ms())
        vts.set_timing(False)
        res.setdefault('scan_events_us', []).append(round(1e3 * float(np.median(ms)), 1))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
