"""Spawn N rank processes of a script on one node (no PyTorch, no torchrun).

``python bench.py --gpus N`` calls ``spawn`` before it touches the GPU: the
parent starts N children of the same command line with RANK = LOCAL_RANK = r,
WORLD_SIZE = N, MASTER_ADDR = 127.0.0.1 and a fresh RS_DIST_DIR for the
control plane's rendezvous (dist.py), waits for them, and exits with the first
non-zero status (the other ranks are then terminated: a rank that lost its
peers would otherwise wait out its collective timeouts).  Rank 0's output is
the job's output.  Under torch.distributed.run (WORLD_SIZE already set) the
script runs as one of the launcher's ranks instead.
"""
import os
import shutil
import subprocess
import sys
import tempfile
import time


def under_launcher(env=None):
    env = os.environ if env is None else env
    return 'WORLD_SIZE' in env and 'RANK' in env


def spawn(nprocs, argv, env=None, poll_s=0.05):
    """Run ``python argv...`` as nprocs ranks; returns the job's exit status."""
    base = dict(os.environ if env is None else env)
    base.setdefault('MASTER_ADDR', '127.0.0.1')
    base.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')   # RCCL needs dmabuf IPC on these hosts
    rdir = tempfile.mkdtemp(prefix='rs_dist_')
    procs = []
    try:
        for r in range(nprocs):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                     LOCAL_WORLD_SIZE=str(nprocs), RS_DIST_DIR=rdir)
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
        status = 0
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    for q in live:          # the job failed: end its other ranks
                        q.terminate()
            time.sleep(poll_s)
        return status
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        shutil.rmtree(rdir, ignore_errors=True)
