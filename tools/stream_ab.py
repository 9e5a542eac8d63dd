#!/usr/bin/env python3
"""A/B of the bench's headline step (rs_vt_match_stream over 10 HBM-resident
batches of 1,024 queries against 1,000 templates) across library builds, each in
its own process, interleaved over rounds (GPU box).
usage: python tools/stream_ab.py LIB.so [LIB2.so ...] [--rounds 3] [--steps 60] [--host]
(--host: the same batches from one pageable host array, the bench's PCIe-inclusive leg)"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, steps, host=False):
    sys.path.insert(0, ROOT)
    import numpy as np
    from pyratslam_amd import _lib, synthetic
    _lib.load(path)
    from pyratslam_amd.view_templates import ViewTemplates
    vts = ViewTemplates._from_shape((64, 32), 45000, device=0, capacity=1000)
    lib = synthetic.library(1000, seed=1)
    vts.add(lib)
    qs = [synthetic.queries_fast(lib, 1024, seed=2 + 1000 * b)[0] for b in range(10)]
    if host:
        hq = np.ascontiguousarray(np.stack(qs))   # pageable
        arg = hq
    else:
        arg = (10, 1024, _lib.DeviceBuffer(10 * qs[0].nbytes, device=0).upload(np.stack(qs)))
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        vts.match_stream(arg)
    t0 = time.perf_counter()
    for _ in range(steps):
        vts.match_stream(arg)
    dt = (time.perf_counter() - t0) / steps
    idx, score = vts.match_stream(arg)
    h = hashlib.sha256(np.ascontiguousarray(idx).tobytes() + np.ascontiguousarray(score).tobytes()).hexdigest()[:16]
    print(json.dumps({'lib': path, 'ms_per_step': 1e3 * dt, 'gcompares_per_s': 10240 * 1000 / dt / 1e9,
                      'keys_sha16': h}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--child', action='store_true')
    ap.add_argument('--host', action='store_true')
    a = ap.parse_args()
    if a.child:
        child(a.libs[0], a.steps, a.host)
        return
    res = {l: [] for l in a.libs}
    keys, bad = {}, False
    for _ in range(a.rounds):
        for lib in a.libs:
            p = subprocess.run([sys.executable, __file__, lib, '--child', '--steps', str(a.steps)]
                               + (['--host'] if a.host else []),
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                raise SystemExit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res[lib].append(r['ms_per_step'])
            keys.setdefault(lib, r['keys_sha16'])
            if r['keys_sha16'] != keys[a.libs[0]]:
                print('stream_ab: INVALID A/B -- %s returns other keys than %s' % (lib, a.libs[0]), file=sys.stderr)
                bad = True
    for lib in a.libs:
        v = sorted(res[lib])
        print(json.dumps({'lib': lib, 'ms_per_step_median': v[len(v) // 2], 'all': [round(x, 4) for x in res[lib]],
                          'keys_sha16': keys[lib]}))
    if bad:
        raise SystemExit(1)


if __name__ == '__main__':
    main()
