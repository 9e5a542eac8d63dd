#!/usr/bin/env python3
"""Multi-rank check of the RCCL-sharded template library (GPU box).

Launch: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
            --master-port P tools/rccl_check.py [--same-device]
Each rank builds ShardedViewTemplates (template g on rank g % N, RCCL
allreduce(min, uint64) inside the library) through bench.py's own control plane
(gloo: unique-id broadcast, barriers), runs a frozen scan and a sequential
(growing-library) batch, and rank 0 compares both with an unsharded library on
its own device.  --same-device puts every rank on device 0 (1-GPU boxes; RCCL
refuses two ranks on one GPU, so there --gloo swaps the in-library RCCL
allreduce for bench.py's host gloo min-reduction and checks everything else).
Prints one JSON line on rank 0 and exits non-zero on any mismatch.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ShardedViewTemplates, ViewTemplates
    world = int(os.environ.get('WORLD_SIZE', '1'))
    d = bench.Dist(world)
    dev = 0 if '--same-device' in sys.argv else d.local
    if '--gloo' in sys.argv:
        vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, world, reducer=d.min_keys,
                                              device=dev, capacity=256)
    else:
        uid = d.bcast_bytes(ShardedViewTemplates.unique_id() if d.rank == 0 else None)
        vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, world, reducer='rccl',
                                              unique_id=uid, device=dev, capacity=256)
    lib = synthetic.library(700, seed=1)
    vts.add(lib)
    qs, src = synthetic.queries(lib, 300, seed=2)
    fi, fs, _ = vts.match_templates(qs, mode=_lib.RS_VT_FROZEN)
    # sequential: fresh queries (misses) grow the library in-batch
    q2, _ = synthetic.queries(lib, 200, seed=3, hit_frac=0.5)
    si, ss, sn = vts.match_templates(q2, mode=_lib.RS_VT_SEQUENTIAL)
    count = len(vts.templates)
    d.barrier()
    ok = True
    out = {'world': world, 'same_device': dev == 0 and world > 1,
           'reducer': 'gloo' if '--gloo' in sys.argv else 'rccl'}
    if d.rank == 0:
        ref = ViewTemplates._from_shape((64, 32), 45000, device=dev, capacity=256)
        ref.add(lib)
        ri, rs_, _ = ref.match_templates(qs, mode=_lib.RS_VT_FROZEN)
        r2i, r2s, r2n = ref.match_templates(q2, mode=_lib.RS_VT_SEQUENTIAL)
        out.update(frozen_equal=bool(np.array_equal(fi, ri) and np.array_equal(fs, rs_)),
                   sequential_equal=bool(np.array_equal(si, r2i) and np.array_equal(ss, r2s)
                                         and np.array_equal(sn, r2n)),
                   count=count, count_ref=len(ref.templates),
                   hits_correct=bool(np.all(fi[src >= 0] == src[src >= 0])))
        ok = out['frozen_equal'] and out['sequential_equal'] and count == len(ref.templates)
        out['ok'] = ok
        print(json.dumps(out), flush=True)
        ref.close()
    vts.close()
    d.close()
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
