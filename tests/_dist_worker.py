"""One rank of tests/test_distributed_cpu.py (run by pyratslam_amd.launch or
torch.distributed.run): the sharding protocol of ShardedViewTemplates over the
torch-free control plane, with the per-rank scan played by the oracle (test
infrastructure; on the GPU it is rs_vt_scan_local)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NO_KEY = np.iinfo(np.uint64).max


def local_keys(shard, gids, queries):
    from oracle import view_templates as V
    keys = np.full(len(queries), NO_KEY, dtype=np.uint64)
    if len(shard) == 0:
        return keys
    for i, q in enumerate(queries):
        sc = V.vt_scores_library(shard, q)
        k = (sc.astype(np.uint64) << np.uint64(32)) | gids.astype(np.uint64)
        keys[i] = k.min()
    return keys


def main():
    import bench
    from pyratslam_amd import synthetic
    d = bench.Dist(int(os.environ['WORLD_SIZE']))
    try:
        d.barrier()
        uid = d.bcast_bytes(b'rank0-unique-id' if d.rank == 0 else None)
        assert uid == b'rank0-unique-id', uid
        assert d.max(float(d.rank) + 0.5) == d.world - 0.5
        lib = synthetic.library(48, seed=7)
        qs, _ = synthetic.queries(lib, 24, seed=8, hit_frac=0.75)
        gids = np.arange(d.rank, len(lib), d.world)        # template g on rank g % world
        glob = d.min_keys(local_keys(lib[gids], gids, qs))
        # unsigned order: keys >= 2^63 and UINT64_MAX ("no template") stay correct
        probe = np.array([NO_KEY, 5 + d.rank, (1 << 63) + d.rank, (1 << 40) | (3 - d.rank)],
                         dtype=np.uint64)
        pk = d.min_keys(probe)
        both = d.bcast_bytes(glob.tobytes() if d.rank == 0 else None)
        assert np.array_equal(np.frombuffer(both, dtype=np.uint64), glob)   # same on every rank
        d.barrier()
        if d.rank == 0:
            print(json.dumps({'world': d.world, 'keys': [int(k) for k in glob],
                              'probe': [int(k) for k in pk]}), flush=True)
    finally:
        d.close()


if __name__ == '__main__':
    main()
