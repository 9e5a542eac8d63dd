#!/usr/bin/env python3
"""Diagnostic for a one-off wrong first update at 128x128x72 (GPU box): fresh
handles, inject, one update, compared with the oracle's first step; interleaved
with rows-form handles (update() and batched run()) and a float64 handle, as the
test module runs them.  Prints the count of mismatches."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import posecell as P  # noqa: E402  (test infrastructure: the checker)
from pyratslam_amd import PoseCellNetwork  # noqa: E402


def odometry(n, seed, vmax=0.6, rmax=0.15):
    r = np.random.default_rng(seed)
    return np.stack([r.uniform(0, vmax, n), r.uniform(-rmax, rmax, n)], axis=1)


def main():
    shape = (128, 128, 72)
    od = odometry(40, 9)
    ref = P.PoseCellOracle(shape)
    ref.inject(1, (64, 64, 36))
    want = ref.update(od[0])
    bad = 0
    for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
        small = PoseCellNetwork((40, 100, 20))
        small.inject(1, (20, 50, 10))
        small.run(odometry(24, it))
        for v in odometry(5, it + 100):
            small.update(v)
        small.close()
        a = PoseCellNetwork(shape)
        b = PoseCellNetwork(shape, precision='float64')
        a.inject(1, (64, 64, 36))
        b.inject(1, (64, 64, 36))
        ga = a.update(od[0])
        gb = b.update(od[0])
        if ga != want or gb != want:
            bad += 1
            print('iteration %d: f32 %s f64 %s want %s' % (it, ga, gb, want), flush=True)
        a.close()
        b.close()
    print('mismatches: %d' % bad, flush=True)


if __name__ == '__main__':
    main()
