"""N>1 host orchestration on CPU with torch.distributed gloo, world size 2.

Covers what runs on every rank besides the GPU scan: bench.py's control plane
(barrier, RCCL unique-id broadcast, max-over-ranks time, the host uint64 min
reducer with UINT64_MAX = "no template") and the sharding protocol of
ShardedViewTemplates -- template g on rank g % n at slot g // n, packed keys
(score << 32 | g), elementwise min over ranks == the unsharded first argmin.
The per-rank scan is played by the oracle here (test infrastructure); on the
GPU it is rs_vt_scan_local, checked against the same protocol in
tests/test_view_templates_gpu.py::test_sharded_ranks_simulated_on_one_gpu.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

NO_KEY = np.iinfo(np.uint64).max


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_keys(shard, gids, queries):
    from oracle import view_templates as V
    keys = np.full(len(queries), NO_KEY, dtype=np.uint64)
    if len(shard) == 0:
        return keys
    for i, q in enumerate(queries):
        sc = V.vt_scores_library(shard, q)
        k = (sc.astype(np.uint64) << np.uint64(32)) | gids.astype(np.uint64)
        keys[i] = k.min()
    return keys


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from pyratslam_amd import synthetic
    d = bench.Dist(world)
    try:
        d.barrier()
        uid = d.bcast_bytes(b'rank0-unique-id' if rank == 0 else None)
        assert uid == b'rank0-unique-id'
        assert d.max(float(rank) + 0.5) == world - 0.5
        lib = synthetic.library(48, seed=7)
        qs, src = synthetic.queries(lib, 24, seed=8, hit_frac=0.75)
        gids = np.arange(rank, len(lib), world)          # template g on rank g % world
        local = _local_keys(lib[gids], gids, qs)
        glob = d.min_keys(local)
        out[rank] = glob.copy()
        # "no template" (UINT64_MAX) survives the signed int64 gloo reduction
        probe = np.array([NO_KEY, 5, NO_KEY, (1 << 40) | 3], dtype=np.uint64)
        if rank == 1:
            probe = np.array([NO_KEY, NO_KEY, 7, (1 << 40) | 1], dtype=np.uint64)
        out['probe%d' % rank] = d.min_keys(probe).copy()
    finally:
        d.close()


def test_sharded_min_reduce_gloo_world2():
    from oracle import view_templates as V
    from pyratslam_amd import synthetic
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert np.array_equal(out[0], out[1])
    expect = np.array([NO_KEY, 5, 7, (1 << 40) | 1], dtype=np.uint64)
    assert np.array_equal(out['probe0'], expect) and np.array_equal(out['probe1'], expect)
    lib = synthetic.library(48, seed=7)
    qs, _ = synthetic.queries(lib, 24, seed=8, hit_frac=0.75)
    for i, q in enumerate(qs):
        sc = V.vt_scores_library(lib, q)
        key = int(out[0][i])
        assert key >> 32 == int(sc.min())
        assert key & 0xFFFFFFFF == int(np.argmin(sc))
