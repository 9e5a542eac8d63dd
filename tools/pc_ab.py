#!/usr/bin/env python3
"""A/B timing of the pose-cell step across library builds (GPU box).

usage: python tools/pc_ab.py LIB.so[@ENV=V,...] [LIB2.so ...] [--shape 128,128,72] [--steps 2000] [--rounds 3]
       [--mode run|update|node]
(``@RS_PC_CTL=inline`` runs that library with the variable set; ``;`` separates several)
Each library runs in its own process (ctypes loads one copy), interleaved over
rounds so clock drift hits every build alike: batched run() steps/s after a clock
warm-up, and the state after the same odometry, compared across builds.  A build
whose state differs from the first one's by more than --tol (float32: the north_star
1e-5) computed something else: its timing is not a valid A/B, and the tool exits 1.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, shape, steps, check, precision, out, mode='run'):
    sys.path.insert(0, ROOT)
    import numpy as np
    from pyratslam_amd import _lib, synthetic
    _lib.load(path)
    from pyratslam_amd import PoseCellNetwork
    od = synthetic.odometry(steps + check + 50, seed=0)
    net = PoseCellNetwork(shape, precision=precision, readback='eager' if mode == 'node' else 'lazy')
    net.inject(1, tuple(s // 2 for s in shape))
    if mode != 'run':  # per-call update() ('update'), or update() + .posecells ('node')
        def one(v):
            net.update(v)
            if mode == 'node':
                net.posecells
        for v in od[:check]:
            one(v)
        np.save(out, net.posecells)   # the state every build reaches on the same odometry
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            for v in od[check:check + 50]:
                one(v)
        t0 = time.perf_counter()
        for v in od[check + 50:check + 50 + steps]:
            one(v)
        dt = time.perf_counter() - t0
        print(json.dumps({'lib': path, 'mode': mode, 'us_per_step': 1e6 * dt / steps, 'argmax': []}), flush=True)
        return
    mx = net.run(od[:check])
    np.save(out, net.posecells)
    t_end = time.perf_counter() + 0.3          # clock warm-up
    while time.perf_counter() < t_end:
        net.run(od[check:check + 50])
    net.run(od[check + 50:check + 50 + steps])  # a batch of the timed size (buffers sized), untimed
    t0 = time.perf_counter()
    net.run(od[check + 50:check + 50 + steps])
    dt = time.perf_counter() - t0
    print(json.dumps({'lib': path, 'form': net.step_form(), 'us_per_step': 1e6 * dt / steps,
                      'argmax': [list(map(int, m)) for m in mx[-3:]]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--shape', default='128,128,72')
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--check', type=int, default=40)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--precision', default='float32')
    ap.add_argument('--tol', type=float, default=None,
                    help='max |state difference| vs the first build (default 1e-5 float32, 1e-12 float64)')
    ap.add_argument('--child', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--out', default='')
    ap.add_argument('--mode', default='run', choices=('run', 'update', 'node'),
                    help="batched run() (default), per-call update(), or update() + .posecells (eager)")
    a = ap.parse_args()
    shape = tuple(int(s) for s in a.shape.split(','))
    if a.child:
        child(a.libs[0], shape, a.steps, a.check, a.precision, a.out, a.mode)
        return
    import numpy as np
    tol = a.tol if a.tol is not None else (1e-5 if a.precision == 'float32' else 1e-12)
    bad = []
    res = {lib: [] for lib in a.libs}
    for rnd in range(a.rounds):
        for i, lib in enumerate(a.libs):
            out = '/tmp/pc_ab_%d.npy' % i
            path, _, envs = lib.partition('@')
            # LIB@K=V;K2=V2 (';' between variables: a value may hold commas, tc:24,4)
            env = dict(os.environ, **dict(kv.split('=', 1) for kv in envs.split(';') if kv))
            p = subprocess.run([sys.executable, __file__, path, '--child', '--shape', a.shape, '--steps',
                                str(a.steps), '--check', str(a.check), '--precision', a.precision,
                                '--out', out, '--mode', a.mode], capture_output=True, text=True, timeout=300, env=env)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            r['lib'] = lib
            res[lib].append(r['us_per_step'])
            if rnd == 0:
                s0, s = np.load('/tmp/pc_ab_0.npy'), np.load(out)
                r['max_abs_diff_vs_first'] = float(np.abs(s - s0).max())
                if not r['max_abs_diff_vs_first'] <= tol:   # NaN fails too
                    bad.append((lib, r['max_abs_diff_vs_first']))
                print(json.dumps(r), flush=True)
    for lib in a.libs:
        v = sorted(res[lib])
        print(json.dumps({'lib': lib, 'us_per_step_min': v[0], 'us_per_step_median': v[len(v) // 2],
                          'all': [round(x, 2) for x in res[lib]]}), flush=True)
    if bad:
        print('pc_ab: INVALID A/B -- these builds end in a different state than %s (tol %g): %s'
              % (a.libs[0], tol, bad), file=sys.stderr, flush=True)
        raise SystemExit(1)


if __name__ == '__main__':
    main()
