#!/usr/bin/env python3
"""Anatomy of one PoseCellNetwork.update() on the GPU box, per form: the Python
update() loop, the same calls from a C loop (tools/pc_call_loop.cpp: the library
alone, no ctypes), and the device span of a call (HIP events around it).  The HIP
API split (launches, synchronisation) comes from a rocprofv3 --hip-runtime-trace
run of `--mode calls`.

usage: python tools/pc_call_anatomy.py [--shape 64,64,36] [--calls 2000] FORM [FORM ...]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_loop():
    out = os.path.join(ROOT, 'gpurun_out', 'pc_call_loop.so')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(['g++', '-O2', '-shared', '-fPIC', os.path.join(ROOT, 'tools', 'pc_call_loop.cpp'),
                           '-I' + os.path.join(ROOT, 'include'), '-L' + os.path.join(ROOT, 'pyratslam_amd'),
                           '-lratslam_hip', '-Wl,-rpath,' + os.path.join(ROOT, 'pyratslam_amd'), '-o', out])
    return out


def child(shape, calls, loop_so, mode):
    sys.path.insert(0, ROOT)
    import numpy as np
    from pyratslam_amd import PoseCellNetwork, synthetic
    od = synthetic.odometry(4 * calls, seed=0)
    net = PoseCellNetwork(shape)
    net.inject(1, tuple(s // 2 for s in shape))
    for v in od[:calls]:
        net.update(v)
    if mode == 'calls':   # just the calls (for a rocprofv3 runtime trace)
        for v in od[calls:2 * calls]:
            net.update(v)
        return
    t0 = time.perf_counter()
    for v in od[calls:2 * calls]:
        net.update(v)
    py = (time.perf_counter() - t0) / calls
    lib = ctypes.CDLL(loop_so)
    lib.pc_call_loop.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    c_od = np.ascontiguousarray(od[2 * calls:3 * calls])
    us = np.zeros(1)
    st = lib.pc_call_loop(net._h, calls, c_od.ctypes.data, us.ctypes.data)
    assert st == 0, st
    amb = ctypes.c_int64(-1)
    if net.step_form() == 'halo':
        from pyratslam_amd import _lib
        _lib.check(net._lib.rs_pc_debug_value(net._h, _lib.RS_PC_DBG_HALO_AMBIG, ctypes.byref(amb)))
    net.set_profiling(True, per_kernel=False)
    dev = []
    for v in od[3 * calls:3 * calls + 200]:
        net.update(v)
        dev.append(net.device_ms() * 1e3)
    net.set_profiling(False)
    dev.sort()
    print(json.dumps({'form': net.step_form(), 'shape': list(shape), 'python_update_us': 1e6 * py,
                      'c_loop_update_us': float(us[0]), 'device_span_us_median': dev[len(dev) // 2],
                      'near_tie_calls': amb.value}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('forms', nargs='*', default=[''])
    ap.add_argument('--shape', default='64,64,36')
    ap.add_argument('--calls', type=int, default=2000)
    ap.add_argument('--mode', default='anatomy', choices=['anatomy', 'calls'])
    ap.add_argument('--child', action='store_true')
    ap.add_argument('--loop-so', default='')
    a = ap.parse_args()
    shape = tuple(int(s) for s in a.shape.split(','))
    if a.child:
        child(shape, a.calls, a.loop_so, a.mode)
        return
    so = build_loop() if a.mode == 'anatomy' else ''
    for spec in a.forms:
        # FORM[@VAR=V;...]: e.g. halo@ROC_ACTIVE_WAIT_TIMEOUT=100 (the HIP runtime's host
        # spin before it sleeps on the completion interrupt)
        form, _, extra = spec.partition('@')
        env = dict(os.environ, RS_PC_FORM=form)
        for kv in filter(None, extra.split(';')):
            k, v = kv.split('=', 1)
            env[k] = v
        print('#', spec, flush=True)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), '--child', '--shape', a.shape,
                               '--calls', str(a.calls), '--loop-so', so, '--mode', a.mode], env=env)


if __name__ == '__main__':
    main()
