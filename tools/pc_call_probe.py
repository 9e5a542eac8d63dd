#!/usr/bin/env python3
"""Per-call anatomy of update() on the GPU box: wall per call, the device span of the
call (HIP events around the whole call) and each kernel's event time, per form.

usage: python tools/pc_call_probe.py [--shape 64,64,36] [--calls 400] FORM [FORM ...]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(shape, calls):
    sys.path.insert(0, ROOT)
    import numpy as np
    from pyratslam_amd import PoseCellNetwork, synthetic
    od = synthetic.odometry(3 * calls, seed=0)
    net = PoseCellNetwork(shape)
    net.inject(1, tuple(s // 2 for s in shape))
    for v in od[:calls]:
        net.update(v)
    t0 = time.perf_counter()
    for v in od[calls:2 * calls]:
        net.update(v)
    wall = (time.perf_counter() - t0) / calls
    out = {'form': net.step_form(), 'wall_us': 1e6 * wall}
    for per_kernel in (False, True):
        net.set_profiling(True, per_kernel=per_kernel)
        dev, k0, k1 = [], [], []
        for v in od[2 * calls:2 * calls + calls // 2]:
            net.update(v)
            dev.append(net.device_ms())
            if per_kernel:
                k = net.kernel_ms()
                k0.append(k[0])
                k1.append(k[1])
        key = 'events_per_kernel' if per_kernel else 'events_call'
        out[key] = {'device_us': 1e3 * float(np.median(dev))}
        if per_kernel:
            out[key]['kernel0_us'] = 1e3 * float(np.median(k0))
            out[key]['kernel1_us'] = 1e3 * float(np.median(k1))
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('forms', nargs='*', default=['rows', 'halo'])
    ap.add_argument('--shape', default='64,64,36')
    ap.add_argument('--calls', type=int, default=400)
    ap.add_argument('--child', action='store_true', help=argparse.SUPPRESS)
    a = ap.parse_args()
    shape = tuple(int(s) for s in a.shape.split(','))
    if a.child:
        child(shape, a.calls)
        return
    for f in a.forms:
        env = dict(os.environ, RS_PC_FORM=f)
        p = subprocess.run([sys.executable, __file__, '--child', '--shape', a.shape, '--calls', str(a.calls)],
                           capture_output=True, text=True, timeout=300, env=env)
        if p.returncode != 0:
            print(p.stderr[-3000:], file=sys.stderr)
            raise SystemExit(p.returncode)
        if p.stderr.strip():
            print(p.stderr.strip()[-600:], file=sys.stderr, flush=True)
        print(p.stdout.strip().splitlines()[-1], flush=True)


if __name__ == '__main__':
    main()
