#!/usr/bin/env python3
"""A/B timing of the template scan across library builds (GPU box).

usage: python tools/scan_ab.py LIB.so [LIB2.so ...] [--reps 30] [--templates 1000] [--queries 1024]
Each library runs in its own process (ctypes loads one copy); the frozen-library
scan of the bench workload is timed with the library's own HIP events
(rs_vt_last_ms) and the packed results are compared across libraries.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, reps, T, Q, rounds):
    sys.path.insert(0, ROOT)
    import ctypes
    import numpy as np
    from pyratslam_amd import _lib, synthetic
    _lib.load(path)
    from pyratslam_amd.view_templates import ViewTemplates
    vts = ViewTemplates._from_shape((64, 32), 45000, device=0, capacity=T)
    vts.add(synthetic.library(T, seed=1))
    qs, _ = synthetic.queries(synthetic.library(min(T, 4096), seed=1), Q, seed=2)
    lib = vts._lib
    idx = np.empty(Q, dtype=np.int64)
    score = np.empty(Q, dtype=np.uint64)
    new = np.empty(Q, dtype=np.uint8)

    def run(staged):
        qp = None if staged else _lib.ptr(qs, ctypes.c_uint8)
        _lib.check(lib.rs_vt_match_batch(vts._h, Q, qp, _lib.RS_VT_FROZEN, _lib.ptr(score, ctypes.c_uint64),
                                         _lib.ptr(idx, ctypes.c_int64), _lib.ptr(new, ctypes.c_uint8)))
    run(False)
    ms = []
    for _ in range(rounds):
        for _ in range(3):
            run(True)
        for _ in range(reps):
            run(True)
            ms.append(vts.device_ms())
    ms = np.array(ms)
    print(json.dumps({'lib': os.path.basename(path), 'form': vts.scan_form(), 'median_ms': float(np.median(ms)),
                      'min_ms': float(ms.min()), 'max_ms': float(ms.max()),
                      'gcompares_s': T * Q / np.median(ms) / 1e6,
                      'checksum': int(score.astype(np.uint64).sum()) ^ int(idx.sum())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--reps', type=int, default=30)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--templates', type=int, default=1000)
    ap.add_argument('--queries', type=int, default=1024)
    ap.add_argument('--child', action='store_true')
    a = ap.parse_args()
    if a.child:
        child(a.libs[0], a.reps, a.templates, a.queries, a.rounds)
        return
    for _ in range(2):  # interleave the libraries twice against clock drift
        for path in a.libs:
            subprocess.check_call([sys.executable, __file__, path, '--child', '--reps', str(a.reps),
                                   '--rounds', str(a.rounds), '--templates', str(a.templates),
                                   '--queries', str(a.queries)], timeout=120)


if __name__ == '__main__':
    main()
