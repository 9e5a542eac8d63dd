#!/usr/bin/env python3
"""A/B of pose-cell step forms on the GPU: steps/s, per-kernel HIP-event time and
max |difference| of the state after the same odometry vs the first form listed.

usage: python tools/pc_sweep.py --shape 128,128,72 --forms rows stream:1,8 stream:1,8,6 ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', default='128,128,72')
    ap.add_argument('--forms', nargs='+', default=['rows', 'stream'])
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--check-steps', type=int, default=40)
    ap.add_argument('--precision', default='float32')
    args = ap.parse_args()
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in args.shape.split(','))
    od = synthetic.odometry(args.steps + args.check_steps + 50, seed=0)
    ref_state, ref_max = None, None
    for form in args.forms:
        os.environ['RS_PC_FORM'] = form
        net = PoseCellNetwork(shape, precision=args.precision)
        net.inject(1, tuple(s // 2 for s in shape))
        mx = net.run(od[:args.check_steps])
        state = net.posecells
        if ref_state is None:
            ref_state, ref_max = state, mx
        err = float(np.abs(state - ref_state).max())
        same_max = bool(np.array_equal(np.asarray(mx), np.asarray(ref_max)))
        net.run(od[:50])
        t0 = time.perf_counter()
        net.run(od[50:50 + args.steps])
        dt = time.perf_counter() - t0
        net.set_profiling(True)
        n = min(args.steps, 200)
        net.run(od[:n])
        ex, pi = net.kernel_ms()
        print(json.dumps({'form': form, 'resolved': net.step_form(), 'shape': shape,
                          'us_per_step': 1e6 * dt / args.steps,
                          'excite_us': 1e3 * ex / n, 'path_us': 1e3 * pi / n,
                          'max_abs_diff_vs_first': err, 'argmax_same': same_max}), flush=True)
        net.close()


if __name__ == '__main__':
    main()
