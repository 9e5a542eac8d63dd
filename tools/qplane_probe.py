#!/usr/bin/env python3
"""Query-plane kernel cost in rs_vt_match_stream under different neighbours
(run under rocprofv3 --kernel-trace): empty library (qplane back to back),
a 64-template library (short scans), the 1,000-template bench library."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ViewTemplates
    qlib = synthetic.library(1000, seed=1)
    qs = np.stack([synthetic.queries(qlib, 1024, seed=2 + b)[0] for b in range(8)])
    buf = _lib.DeviceBuffer(qs.nbytes).upload(qs)
    for t in (0, 64, 1000):
        vts = ViewTemplates._from_shape((64, 32), 45000, capacity=max(t, 64))
        if t:
            vts.add(qlib[:t])
        for _ in range(3):
            vts.match_stream((8, 1024, buf))
        vts.close()
    buf.close()
    print('done')


if __name__ == '__main__':
    main()
