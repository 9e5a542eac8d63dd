#!/usr/bin/env python3
"""Multi-rank check of the RCCL-sharded template library (GPU box).

Launch: python tools/rccl_check.py --gpus N [--same-device --host-reduce]
(it starts its own N rank processes; under torch.distributed.run it runs as one
of the launcher's ranks).  Each rank builds ShardedViewTemplates (template g on
rank g % N, RCCL allreduce(min, uint64) inside the library) through bench.py's
control plane (pyratslam_amd.dist: unique-id broadcast, barriers), runs a
frozen scan, a frozen rs_vt_match_stream over several batches (the bench's
path, one collective per batch on the side stream) and a sequential
(growing-library) batch, and rank 0 compares all of them with an unsharded
library on its own device.  --same-device puts every rank on device 0 (1-GPU
boxes; RCCL refuses two ranks on one GPU, so --host-reduce swaps the in-library
RCCL allreduce for the control plane's host min-reduction and checks everything
else).  Prints one JSON line on rank 0 and exits non-zero on any mismatch.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', '1')))
    ap.add_argument('--same-device', action='store_true')
    ap.add_argument('--host-reduce', action='store_true')
    ap.add_argument('--templates', type=int, default=700)
    args = ap.parse_args()
    from pyratslam_amd import launch
    if args.gpus > 1 and not launch.under_launcher():
        sys.exit(launch.spawn(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.dist import Dist
    from pyratslam_amd.view_templates import ShardedViewTemplates, ViewTemplates
    d = Dist(args.gpus)
    world = d.world
    dev = 0 if args.same_device else d.local
    if args.host_reduce:
        vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, world, reducer=d.min_keys,
                                              device=dev, capacity=256)
    else:
        uid = d.bcast_bytes(ShardedViewTemplates.unique_id() if d.rank == 0 else None)
        vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, world, reducer='rccl',
                                              unique_id=uid, device=dev, capacity=256)
    lib = synthetic.library(args.templates, seed=1)
    vts.add(lib)
    qs, src = synthetic.queries(lib, 300, seed=2)
    fi, fs, _ = vts.match_templates(qs, mode=_lib.RS_VT_FROZEN)
    batches = np.stack([synthetic.queries_fast(lib, 256, seed=10 + b)[0] for b in range(3)])
    si_stream = ss_stream = None
    if not args.host_reduce:
        si_stream, ss_stream = vts.match_stream(batches)
    # sequential: fresh queries (misses) grow the library in-batch
    q2, _ = synthetic.queries(lib, 200, seed=3, hit_frac=0.5)
    si, ss, sn = vts.match_templates(q2, mode=_lib.RS_VT_SEQUENTIAL)
    count = len(vts.templates)
    d.barrier()
    ok = True
    out = {'world': world, 'same_device': dev == 0 and world > 1,
           'reducer': 'host' if args.host_reduce else 'rccl'}
    if d.rank == 0:
        ref = ViewTemplates._from_shape((64, 32), 45000, device=dev, capacity=256)
        ref.add(lib)
        ri, rs_, _ = ref.match_templates(qs, mode=_lib.RS_VT_FROZEN)
        rbi, rbs = ref.match_stream(batches)
        r2i, r2s, r2n = ref.match_templates(q2, mode=_lib.RS_VT_SEQUENTIAL)
        out.update(frozen_equal=bool(np.array_equal(fi, ri) and np.array_equal(fs, rs_)),
                   stream_equal=None if si_stream is None else bool(
                       np.array_equal(si_stream, rbi) and np.array_equal(ss_stream, rbs)),
                   sequential_equal=bool(np.array_equal(si, r2i) and np.array_equal(ss, r2s)
                                         and np.array_equal(sn, r2n)),
                   count=count, count_ref=len(ref.templates),
                   hits_correct=bool(np.all(fi[src >= 0] == src[src >= 0])))
        ok = (out['frozen_equal'] and out['sequential_equal'] and out['stream_equal'] is not False
              and count == len(ref.templates))
        out['ok'] = ok
        print(json.dumps(out), flush=True)
        ref.close()
    vts.close()
    d.close()
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
