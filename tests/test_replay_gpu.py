"""Config 5 on the GPU: the synthetic stand-in for dataset_10Hz.bag replayed
through RatslamReplay with the MI355X PoseCellNetwork and ViewTemplates, vs the
golden run of the reference's own classes (tests/golden/ros_replay.npz)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import posecell as P
from test_replay import oracle_replay

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def golden():
    from pyratslam_amd import _build
    _build.build()
    return load_golden('ros_replay')


def _events(golden):
    from pyratslam_amd import synthetic
    return synthetic.ros_stream(int(golden['n']), seed=int(golden['seed']))


@pytest.mark.parametrize('batch,publish', [(True, False), (False, False), (False, True)])
def test_gpu_replay_matches_reference(golden, batch, publish):
    """publish=True: every update also reads .posecells (the node's publish,
    ros_simulate.py:140-145) through the eager readback."""
    from pyratslam_amd import replay
    r = replay.RatslamReplay(batch=batch, publish=publish).replay_events(_events(golden))
    if publish:
        assert r.published == len(r.pc_max) * int(np.prod(replay.POSE_SIZE))
    res = r.results()
    assert np.array_equal(res['pc_max'], golden['pc_max'])
    assert np.array_equal(res['template_index'], golden['template_index'])
    assert res['templates'] == int(golden['templates'])
    # the map integrates the odometry and stores the (identical) peak cells
    assert np.array_equal(res['em_points'], golden['em_points'])
    want = np.zeros(replay.POSE_SIZE)
    want.ravel()[golden['final_state_coo_idx']] = golden['final_state_coo_val']
    assert np.abs(r.pcn.posecells - want).max() < 1e-5


def test_gpu_bag_replay(tmp_path, golden):
    from pyratslam_amd import replay, synthetic
    path = synthetic.write_ros_bag(str(tmp_path / 'ds.bag'), _events(golden))
    res = replay.RatslamReplay().replay_bag(path).results()
    assert np.array_equal(res['pc_max'], golden['pc_max'])
    assert np.array_equal(res['template_index'], golden['template_index'])


def test_gpu_replay_with_template_feedback(golden):
    """The reference's commented-out feedback (ros_simulate.py:107-108,
    pcn.inject(.02, template.location())): GPU run vs the oracle run."""
    from pyratslam_amd import replay
    ev = _events(golden)
    g = replay.RatslamReplay(feedback_energy=0.02).replay_events(ev).results()
    o = oracle_replay(feedback_energy=0.02, batch=False).replay_events(ev).results()
    assert np.array_equal(g['pc_max'], o['pc_max'])
    assert np.array_equal(g['template_index'], o['template_index'])
    assert np.array_equal(g['em_points'], o['em_points'])


def test_replay_cli_synthetic(capsys):
    from pyratslam_amd import replay
    assert replay.main(['--synthetic', '40']) == 0
    assert '"updates"' in capsys.readouterr().out


def test_two_rank_sharded_replay(golden):
    """Config 5 over ranks: the library sharded over two processes that the
    replay launches itself (one GPU box: both on device 0 with the host key
    reducer; RCCL on a multi-GPU node), pose cells replicated; rank 0's outputs
    equal the reference's."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK'):
        env.pop(k, None)
    cmd = [sys.executable, '-m', 'pyratslam_amd.replay', '--synthetic', str(int(golden['n'])),
           '--gpus', '2', '--host-reduce', '--device', '0']
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=150)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(lines[-1])
    assert out['ranks'] == 2
    assert np.array_equal(np.array(out['pc_max']), golden['pc_max'])
    assert np.array_equal(np.array(out['template_index']), golden['template_index'])
    assert np.array_equal(np.array(out['em_points']), golden['em_points'])
