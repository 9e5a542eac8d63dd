#!/usr/bin/env python3
"""The ROS node's per-step drop-in cost (update() + .posecells), pinned direct
readback vs the copying rs_pc_read, at 21x21x36 and 64x64x36 (GPU box)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyratslam_amd import PoseCellNetwork, _lib, synthetic  # noqa: E402

for shape in ((21, 21, 36), (64, 64, 36)):
    net = PoseCellNetwork(shape)
    net.inject(1, tuple(s // 2 for s in shape))
    od = synthetic.odometry(2000, seed=0)
    buf = np.empty(shape, dtype=np.float64)

    def copying():
        _lib.check(net._lib.rs_pc_read(net._h, _lib.ptr(buf, ctypes.c_double)))
        return buf.copy()

    res = {}
    eager = PoseCellNetwork(shape, readback='eager')
    eager.inject(1, tuple(s // 2 for s in shape))
    for v in od[:100]:
        eager.update(v)
        eager.posecells
    t0 = time.perf_counter()
    for v in od[100:1100]:
        eager.update(v)
        eager.posecells
    res['eager'] = {'update_plus_read_us': round(1e3 * (time.perf_counter() - t0), 2)}
    eager.close()
    for name, read in (('pinned', lambda: net.posecells), ('copying', copying)):
        for v in od[:100]:
            net.update(v)
            read()
        t0 = time.perf_counter()
        for v in od[100:1100]:
            net.update(v)
            read()
        t1 = time.perf_counter()
        r0 = time.perf_counter()
        for _ in range(1000):
            read()
        r1 = time.perf_counter()
        res[name] = {'update_plus_read_us': round(1e3 * (t1 - t0), 2), 'read_us': round(1e3 * (r1 - r0), 2)}
    print(json.dumps({'shape': shape, **res}), flush=True)
    net.close()
