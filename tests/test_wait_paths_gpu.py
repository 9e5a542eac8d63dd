"""The library's host waits, both ways: by default a call returns once its results have
landed in pinned host memory (the pose-cell records and result words, the volume
writers' per-block flags, the matcher's keys, a small batch read in place by the plane
kernel); with RS_PC_HALO_POLL=0, RS_PC_HALO_FLAGS=0, RS_VT_POLL=0 and RS_VT_ZC=0 every
call synchronises its stream and copies its queries first.  The ROS node's loop (the
replay of a synthetic stream, with every update's volume read as the node publishes it)
must give identical peaks, template indices and volumes either way.  The switches are
read once per process, so the synchronising run is a child process."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
sys.path.insert(0, %(root)r)
from pyratslam_amd import replay, synthetic
events = synthetic.ros_stream(160, seed=5)
out = {}
for publish in (False, True):
    r = replay.RatslamReplay(device=0, publish=publish).replay_events(events)
    res = r.results()
    out[str(publish)] = {'pc_max': res['pc_max'].tolist(), 'template_index': res['template_index'].tolist(),
                         'volume': r.pcn.posecells.tolist()}
json.dump(out, open(%(path)r, 'w'))
'''


def _run(tmp_path, name, env_extra):
    path = str(tmp_path / (name + '.json'))
    env = dict(os.environ)
    env.update(env_extra)
    subprocess.run([sys.executable, '-c', CHILD % {'root': ROOT, 'path': path}], env=env, check=True,
                   timeout=300)
    return json.load(open(path))


def test_polled_and_synchronised_waits_agree(tmp_path):
    from pyratslam_amd import _build
    _build.build()
    polled = _run(tmp_path, 'polled', {})
    synced = _run(tmp_path, 'synced', {'RS_PC_HALO_POLL': '0', 'RS_PC_HALO_FLAGS': '0', 'RS_VT_POLL': '0',
                                       'RS_VT_ZC': '0'})
    for publish in ('False', 'True'):
        a, b = polled[publish], synced[publish]
        assert a['pc_max'] == b['pc_max'], publish
        assert a['template_index'] == b['template_index'], publish
        assert np.array_equal(np.array(a['volume']), np.array(b['volume'])), publish
    assert polled['False']['pc_max'] == polled['True']['pc_max']
    assert len(polled['False']['template_index']) > 0
