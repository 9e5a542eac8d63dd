#!/usr/bin/env python3
"""Per-call cost breakdown of PoseCellNetwork.update() (GPU box): the host
control (filters.step_control), the bare rs_pc_update call with precomputed
control, and the whole update(), in microseconds per call."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pyratslam_amd import PoseCellNetwork, synthetic
    from pyratslam_amd import filters as F
    shape = (64, 64, 36)
    n = 2000
    net = PoseCellNetwork(shape)
    net.inject(1, (32, 32, 18))
    od = synthetic.odometry(n + 100, seed=0)
    for v in od[:100]:
        net.update(v)
    t = time.perf_counter()
    ctl = [F.step_control(float(v[0]), float(v[1]), shape[2], net.filter_table) for v in od[100:]]
    t_ctl = (time.perf_counter() - t) / n
    t = time.perf_counter()
    for ox, oy, rows, zf, _ in ctl:
        net._update(net._h, ox.ctypes.data, oy.ctypes.data, rows.ctypes.data, zf.ctypes.data,
                    net._out3_addr)
    t_call = (time.perf_counter() - t) / n
    t = time.perf_counter()
    for v in od[100:]:
        net.update(v)
    t_upd = (time.perf_counter() - t) / n
    print({'step_control_us': 1e6 * t_ctl, 'rs_pc_update_us': 1e6 * t_call,
           'update_us': 1e6 * t_upd}, flush=True)
    net.close()


if __name__ == '__main__':
    main()
