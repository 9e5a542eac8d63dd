"""Process-group control plane of the multi-GPU paths (bench.py, the replay,
tools/rccl_check.py): one process per GPU launched by torch.distributed.run
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment), a gloo group
for barriers, the RCCL unique-id broadcast and max-over-ranks timing.  The data
path never goes through it except ``min_keys``, the host fallback reducer of
the sharded template library when RCCL cannot run (two ranks on one GPU).
N = 1 needs no torch at all."""
import os

import numpy as np


class Dist:
    """Control plane: gloo process group for the barrier, the RCCL unique-id
    broadcast and the max-over-ranks time.  N = 1 needs no torch at all."""

    def __init__(self, gpus):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', '0'))
        if self.world != gpus:
            raise SystemExit('--gpus %d but WORLD_SIZE=%d: launch N>1 with '
                             'python -m torch.distributed.run --nproc-per-node N bench.py --gpus N'
                             % (gpus, self.world))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            dist.init_process_group('gloo', rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def min_keys(self, keys):
        import torch
        k = torch.from_numpy(keys.astype(np.uint64).view(np.int64).copy())
        k[k == -1] = np.iinfo(np.int64).max          # UINT64_MAX (no template) -> int64 max
        self.dist.all_reduce(k, op=self.dist.ReduceOp.MIN)
        out = k.numpy().copy()
        out[out == np.iinfo(np.int64).max] = -1
        return out.view(np.uint64)

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
