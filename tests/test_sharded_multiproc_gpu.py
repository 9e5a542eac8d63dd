"""Sharded template library across real processes, each a rank that
tools/rccl_check.py launches itself (pyratslam_amd.launch, no torchrun, no
PyTorch): template g on rank g % N, compared bit-exactly with an unsharded
library on frozen, streamed and sequential (growing) batches.

* one GPU (any box): three ranks on device 0, the per-rank keys combined by the
  control plane's host min-reduction (RCCL refuses two ranks on one GPU:
  'Duplicate GPU detected');
* two or more GPUs: two ranks, one per GPU, with the in-library RCCL
  allreduce(min, uint64) -- skipped where fewer than two devices are visible.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=150):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK'):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'rccl_check.py')] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads(lines[-1])


def test_three_rank_sharded_match_equals_unsharded():
    out = _run(['--gpus', '3', '--same-device', '--host-reduce'])
    assert out['world'] == 3 and out['ok'], out
    assert out['frozen_equal'] and out['sequential_equal'] and out['hits_correct'], out


def test_rccl_two_gpus_sharded_match_equals_unsharded():
    from pyratslam_amd import _lib
    if _lib.require_device().rs_device_count() < 2:
        pytest.skip('RCCL across ranks needs two visible GPUs')
    out = _run(['--gpus', '2'])
    assert out['world'] == 2 and out['reducer'] == 'rccl' and out['ok'], out
    assert out['frozen_equal'] and out['stream_equal'] and out['sequential_equal'], out
