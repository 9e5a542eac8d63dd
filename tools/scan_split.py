#!/usr/bin/env python3
"""Plane-scan work split A/B (GPU box): time the frozen-library scan per
library size for several blocks-per-template-block values (RS_VT_NQC, read by
the library at every launch; 'auto' = the cost model in plane_split) and check
that every split returns the same packed results.

usage: python tools/scan_split.py [--templates 1000,25000,100000] [--nqc auto,1,8,16] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--templates', default='1000,12500,25000,100000')
    ap.add_argument('--nqc', default='auto,1,8,16')
    ap.add_argument('--queries', type=int, default=1024)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ViewTemplates
    Q = a.queries
    for T in (int(t) for t in a.templates.split(',')):
        vts = ViewTemplates._from_shape((64, 32), 45000, device=0, capacity=T)
        for lo in range(0, T, 8192):
            vts.add(synthetic.library(min(8192, T - lo), seed=1, first=lo))
        qs, src = synthetic.queries(synthetic.library(min(T, 4096), seed=1), Q, seed=2)
        lib = vts._lib
        idx = np.empty(Q, dtype=np.int64)
        score = np.empty(Q, dtype=np.uint64)
        new = np.empty(Q, dtype=np.uint8)
        ref = None
        for nqc in a.nqc.split(','):
            if nqc == 'auto':
                os.environ.pop('RS_VT_NQC', None)
            else:
                os.environ['RS_VT_NQC'] = nqc
            staged = False
            ms = []
            for r in range(a.reps + 1):
                qp = None if staged else _lib.ptr(qs, ctypes.c_uint8)
                _lib.check(lib.rs_vt_match_batch(vts._h, Q, qp, _lib.RS_VT_FROZEN,
                                                 _lib.ptr(score, ctypes.c_uint64),
                                                 _lib.ptr(idx, ctypes.c_int64),
                                                 _lib.ptr(new, ctypes.c_uint8)))
                staged = True
                if r:
                    ms.append(vts.device_ms())
            res = (idx.copy(), score.copy())
            same = ref is None or (np.array_equal(ref[0], res[0]) and np.array_equal(ref[1], res[1]))
            ref = ref or res
            hits = src >= 0
            print(json.dumps({'templates': T, 'nqc': nqc, 'scan_ms': float(np.median(ms)),
                              'gcompares_per_s': T * Q / (np.median(ms) * 1e-3) / 1e9,
                              'same_as_first': bool(same),
                              'hits_correct': bool(np.all(idx[hits] == src[hits]))}), flush=True)
        os.environ.pop('RS_VT_NQC', None)
        vts.close()


if __name__ == '__main__':
    main()
