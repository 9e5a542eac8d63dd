"""N>1 host orchestration on CPU, no PyTorch in the path: the launcher
(pyratslam_amd.launch, what ``python bench.py --gpus N`` uses) and the TCP
control plane (pyratslam_amd.dist) at world sizes 2 and 3, and the same control
plane under torch.distributed.run (the driver's launcher for the scaling bench).

Covers what runs on every rank besides the GPU scan: barriers, the RCCL
unique-id broadcast, the max-over-ranks time, the host uint64 min reducer
(unsigned order, UINT64_MAX = "no template") and the sharding protocol of
ShardedViewTemplates -- template g on rank g % n at slot g // n, packed keys
(score << 32 | g), elementwise min over ranks == the unsharded first argmin.
The per-rank scan is played by the oracle (tests/_dist_worker.py); on the GPU
it is rs_vt_scan_local (tests/test_view_templates_gpu.py, test_sharded_*).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NO_KEY = np.iinfo(np.uint64).max


def _env():
    env = dict(os.environ)
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT', 'RS_DIST_DIR'):
        env.pop(k, None)
    return env


def _json_line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads(lines[-1])


def _check_protocol(out, world):
    from oracle import view_templates as V
    from pyratslam_amd import synthetic
    assert out['world'] == world
    expect = [NO_KEY, 5, 1 << 63, (1 << 40) | (3 - (world - 1))]
    assert out['probe'] == [int(v) for v in expect]
    lib = synthetic.library(48, seed=7)
    qs, _ = synthetic.queries(lib, 24, seed=8, hit_frac=0.75)
    for i, q in enumerate(qs):
        sc = V.vt_scores_library(lib, q)
        key = out['keys'][i]
        assert key >> 32 == int(sc.min())
        assert key & 0xFFFFFFFF == int(np.argmin(sc))


@pytest.mark.parametrize('world', [2, 3])
def test_launcher_and_control_plane(world):
    code = ('import sys; sys.path.insert(0, %r); from pyratslam_amd import launch; '
            'sys.exit(launch.spawn(%d, [%r]))' % (ROOT, world, os.path.join(ROOT, 'tests', '_dist_worker.py')))
    r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=120)
    _check_protocol(_json_line(r), world)


def test_control_plane_under_torchrun():
    pytest.importorskip('torch')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.join(ROOT, 'tests', '_dist_worker.py')]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=180)
    _check_protocol(_json_line(r), 2)


def test_dist_selftest_and_failure_propagates():
    """dist's own self-test through the launcher; a failing rank fails the job
    (and the launcher ends the rank left waiting for it)."""
    code = ('import sys; sys.path.insert(0, %r); from pyratslam_amd import launch; '
            'sys.exit(launch.spawn(2, ["-m", "pyratslam_amd.dist"]))' % ROOT)
    r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=120)
    out = _json_line(r)
    assert out['world'] == 2 and out['uid'] == 'unique-id-of-rank-0' and out['max'] == 1.5
    assert out['min_keys'] == [int(NO_KEY), 5, 1 << 63, (3 << 32) | 6]
    bad = ('import os, sys; sys.path.insert(0, %r)\n'
           'from pyratslam_amd.dist import Dist\n'
           'd = Dist()\n'
           'if d.rank == 1: sys.exit(3)\n'
           'd.barrier()\n' % ROOT)
    path = os.path.join(ROOT, 'tests', '.fail_rank.py')
    with open(path, 'w') as f:
        f.write(bad)
    try:
        code = ('import sys; sys.path.insert(0, %r); from pyratslam_amd import launch; '
                'sys.exit(launch.spawn(2, [%r]))' % (ROOT, path))
        r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=_env(), capture_output=True,
                           text=True, timeout=120)
        assert r.returncode != 0
    finally:
        os.unlink(path)


def test_bench_spawns_its_own_ranks(monkeypatch):
    """``python bench.py --gpus N`` hands off to launch.spawn before touching the GPU."""
    import bench
    from pyratslam_amd import launch
    for k in ('RANK', 'WORLD_SIZE'):
        monkeypatch.delenv(k, raising=False)
    seen = {}

    def fake_spawn(n, argv, **kw):
        seen['n'], seen['argv'] = n, argv
        return 0
    monkeypatch.setattr(launch, 'spawn', fake_spawn)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4', '--steps', '3'])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert seen['n'] == 4 and seen['argv'][0].endswith('bench.py') and seen['argv'][1:] == [
        '--gpus', '4', '--steps', '3']


def test_rendezvous_file_is_owner_only(tmp_path, monkeypatch):
    """The rendezvous file holds the job's auth token: rank 0 creates it 0600
    (a world-readable file in a shared tempdir would let another local user join)."""
    import stat
    import threading
    from pyratslam_amd import dist
    monkeypatch.setenv('RS_DIST_DIR', str(tmp_path))
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setenv('RANK', '0')
    monkeypatch.setenv('MASTER_ADDR', '127.0.0.1')
    seen = {}
    path = dist.rendezvous_path()

    def watch():
        import time
        t_end = time.monotonic() + 20
        while time.monotonic() < t_end and not os.path.exists(path):
            time.sleep(0.01)
        seen['mode'] = stat.S_IMODE(os.stat(path).st_mode)
        port, token = open(path).read().split()
        import socket
        s = socket.create_connection(('127.0.0.1', int(port)))
        dist._send(s, ('%s 1' % token).encode())
        seen['ack'] = dist._recv(s)
        seen['sock'] = s

    t = threading.Thread(target=watch)
    t.start()
    d = dist.Dist(timeout=20)
    t.join()
    assert seen['mode'] == 0o600
    assert seen['ack'] == b'ok'
    seen['sock'].close()
    for c in d._peers.values():
        c.close()
