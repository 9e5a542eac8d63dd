#!/usr/bin/env python3
"""Minimal workloads for rocprofv3 passes (tools/profile_r2.sh): one template
configuration's frozen scans, or one pose-cell grid's batched steps, and nothing
else, so every dispatch of the profiled kernel belongs to that configuration.

usage: python tools/scan_profile.py scan --templates 1000 --queries 1024 --launches 20
       python tools/scan_profile.py pc --shape 128,128,72 --steps 400
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def clock_warmup(ms, kind):
    """Bring the GPU to its steady clock (it ramps over the first tens of ms of load
    after idle) with kernels that are not the profiled one, so all of its dispatches
    run warm: 32x32-template scans (vt_scan_plane_kernel<32, ...>) before a 64x32
    scan profile, 64x32 scans before a pose-cell one."""
    import time
    if ms <= 0:
        return
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ViewTemplates
    shape = (32, 32) if kind == 'scan' else (64, 32)
    vts = ViewTemplates._from_shape(shape, 45000, capacity=1024)
    lib = synthetic.library(1024, h=shape[0], w=shape[1], seed=5)
    vts.add(lib)
    qs, _ = synthetic.queries_fast(lib, 8192, seed=6)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < ms * 1e-3:
        vts.match_templates(qs, mode=_lib.RS_VT_FROZEN)
    vts.close()


def scan(a):
    """The bench's own path: one rs_vt_match_stream call per launch over
    queries / 1024 HBM-resident batches of 1,024 queries (one plane-scan launch of
    all of them), calls back to back, so the profiled dispatches run as the bench's
    timed ones do."""
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ViewTemplates
    vts = ViewTemplates._from_shape((64, 32), 45000, capacity=a.templates)
    for lo in range(0, a.templates, 8192):
        vts.add(synthetic.library(min(8192, a.templates - lo), seed=1, first=lo))
    qlib = synthetic.library(min(a.templates, 4096), seed=1)
    bq = min(1024, a.queries)
    nb = max(1, a.queries // bq)
    qs, src = synthetic.queries_fast(qlib, nb * bq, seed=2)
    buf = _lib.DeviceBuffer(qs.nbytes).upload(qs)
    clock_warmup(a.clock_warmup_ms, 'scan')
    sidx, _ = vts.match_stream((nb, bq, buf.offset(0)))
    got = np.asarray(sidx).reshape(-1)
    ok = bool(np.all(got[src >= 0] == src[src >= 0]))
    vts.set_timing(True)
    ms = []
    for _ in range(a.launches):
        vts.match_stream((nb, bq, buf.offset(0)))
        ms.append(vts.device_ms())
    print(json.dumps({'templates': a.templates, 'queries': nb * bq, 'batches': nb, 'form': vts.scan_form(),
                      'scan_ms': float(np.mean(ms)), 'hits_correct': ok}), flush=True)


def pc(a):
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in a.shape.split(','))
    net = PoseCellNetwork(shape)
    net.inject(1, tuple(s // 2 for s in shape))
    od = synthetic.odometry(a.steps, seed=0)
    clock_warmup(a.clock_warmup_ms, 'pc')
    net.run(od)
    print(json.dumps({'shape': shape, 'form': net.step_form(),
                      'finite': bool(np.isfinite(net.posecells).all())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='what', required=True)
    s = sub.add_parser('scan')
    s.add_argument('--templates', type=int, default=1000)
    s.add_argument('--queries', type=int, default=1024)
    s.add_argument('--launches', type=int, default=20)
    p = sub.add_parser('pc')
    p.add_argument('--shape', default='64,64,36')
    p.add_argument('--steps', type=int, default=400)
    for x in (s, p):
        x.add_argument('--clock-warmup-ms', type=float, default=200.0)
        x.add_argument('--lib', default=None, help='a library build to load instead of the in-tree one (A/B)')
    a = ap.parse_args()
    if a.lib:
        from pyratslam_amd import _lib
        _lib.load(a.lib)
    scan(a) if a.what == 'scan' else pc(a)


if __name__ == '__main__':
    main()
