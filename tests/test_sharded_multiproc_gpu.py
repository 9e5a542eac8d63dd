"""Sharded template library across real processes (one GPU box): three ranks under
torch.distributed.run, bench.py's control plane, template g on rank g % 3, the
per-rank scans combined by the host gloo min-reduction (RCCL refuses two ranks on
one GPU: 'Duplicate GPU detected'), compared bit-exactly with an unsharded library
on frozen and sequential (growing) batches.  tools/rccl_check.py is the same check
with the in-library RCCL allreduce on a multi-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_three_rank_sharded_match_equals_unsharded():
    from pyratslam_amd import _build
    _build.build()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '3',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()),
           os.path.join(ROOT, 'tools', 'rccl_check.py'), '--same-device', '--gloo']
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(lines[-1])
    assert out['world'] == 3 and out['ok'], out
    assert out['frozen_equal'] and out['sequential_equal'] and out['hits_correct'], out
