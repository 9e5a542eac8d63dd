#!/usr/bin/env python3
"""Long-run check of the library's early host returns (GPU box): the same work in two
processes, one with the default waits (records, result words, per-block flags and
keys polled in pinned host memory) and one with every wait a stream synchronisation
(RS_PC_HALO_POLL=0 RS_PC_HALO_FLAGS=0 RS_VT_POLL=0 RS_VT_ZC=0).  Each process hashes
every peak, every volume it reads and every template index; the hashes must agree.

Work per process: at 21x21x36 and 64x64x36, N update()s each followed by a lazy
.posecells read, N more with readback='eager', and 300-step run() batches; and the
ROS replay stream (frames matched against a growing library).

usage: tools/wait_race_check.py [--steps N]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(steps):
    sys.path.insert(0, ROOT)
    import numpy as np
    from pyratslam_amd import PoseCellNetwork, replay, synthetic
    out = {}
    for shape in ((21, 21, 36), (64, 64, 36)):
        od = synthetic.odometry(steps, seed=3)
        for readback in ('lazy', 'eager'):
            h = hashlib.sha256()
            net = PoseCellNetwork(shape, readback=readback)
            net.inject(1, tuple(s // 2 for s in shape))
            for v in od:
                h.update(np.asarray(net.update(v), dtype=np.int64).tobytes())
                h.update(net.posecells.tobytes())
            for i in range(0, steps, 300):
                h.update(np.ascontiguousarray(net.run(od[i:i + 300])).tobytes())
                h.update(net.posecells.tobytes())
            out['%s %s' % (shape, readback)] = h.hexdigest()
            net.close()
    h = hashlib.sha256()
    r = replay.RatslamReplay(device=0).replay_events(synthetic.ros_stream(2000, seed=9))
    res = r.results()
    for k in ('pc_max', 'template_index', 'em_points'):
        h.update(np.ascontiguousarray(res[k]).tobytes())
    out['replay'] = h.hexdigest()
    out['templates'] = int(res['templates'])
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3000)
    ap.add_argument('--child', action='store_true')
    a = ap.parse_args()
    if a.child:
        child(a.steps)
        return
    runs = {}
    for name, extra in (('polled', {}), ('synchronised', {'RS_PC_HALO_POLL': '0', 'RS_PC_HALO_FLAGS': '0',
                                                          'RS_VT_POLL': '0', 'RS_VT_ZC': '0'})):
        env = dict(os.environ)
        env.update(extra)
        t0 = time.time()
        p = subprocess.run([sys.executable, os.path.abspath(__file__), '--child', '--steps', str(a.steps)],
                           env=env, capture_output=True, text=True, timeout=900)
        if p.returncode != 0:
            print(p.stderr[-3000:], file=sys.stderr)
            sys.exit(p.returncode)
        runs[name] = json.loads(p.stdout.strip().splitlines()[-1])
        print('%s: %.1f s' % (name, time.time() - t0), flush=True)
    same = runs['polled'] == runs['synchronised']
    print(json.dumps({'steps': a.steps, 'identical': same, 'runs': runs}, indent=1))
    sys.exit(0 if same else 1)


if __name__ == '__main__':
    main()
