"""The ROS node's threading model on the GPU (ros_simulate.py:98-113 vs :134-145).

In the reference the rospy vision thread calls ``pcn.get_pc_max()`` and
``vts.match()`` while the main thread is inside ``pcn.update()`` and then reads
``pcn.posecells`` to publish it.  Here one thread steps the pose cells (update()
and a read of the whole volume per step, as the node publishes it) while another
matches camera frames against the template library, taking the peak of the pose
cells for each new template, and a third reads the volume.  Every result must
equal a sequential run on the same inputs: the per-handle locks make each call
atomic with respect to the others on its handle, and distinct handles run
concurrently on their own streams.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def mod():
    from pyratslam_amd import _build
    _build.build()
    import pyratslam_amd
    return pyratslam_amd


def _inputs(n_steps, n_frames):
    from pyratslam_amd import replay, synthetic
    od = synthetic.odometry(n_steps, seed=4, vtrans_max=0.3, vrot_max=0.12)
    frames = [ev[2] for ev in synthetic.ros_stream(n_frames, seed=5) if ev[0] == 'image']
    geo = dict(x_range=replay.X_RANGE, y_range=replay.Y_RANGE, x_step=replay.X_STEP,
               y_step=replay.Y_STEP, im_x=replay.IM_SIZE[0], im_y=replay.IM_SIZE[1],
               match_threshold=replay.MATCH_THRESHOLD)
    return od, frames, geo


@pytest.mark.parametrize('precision', ['float32', 'float64'])
def test_vision_thread_concurrent_with_updates(mod, precision):
    from pyratslam_amd import replay
    shape = replay.POSE_SIZE
    od, frames, geo = _inputs(300, 80)
    start = tuple(s // 2 for s in shape)

    # sequential reference: every update (and its published volume), then every frame
    seq = mod.PoseCellNetwork(shape, precision=precision)
    seq.inject(1, start)
    first_peak = seq.get_pc_max()
    seq_max, seq_vol = [], []
    for v in od:
        seq_max.append(seq.update(v))
        seq_vol.append(seq.posecells)
    vts_seq = mod.ViewTemplates(**geo)
    seq_idx = [vts_seq.match(f, 0, 0, 0).get_index() for f in frames]

    net = mod.PoseCellNetwork(shape, precision=precision)
    net.inject(1, start)
    vts = mod.ViewTemplates(**geo)
    go = threading.Barrier(3)
    got_max, got_vol, vis_idx, vis_peak, reads, errors = [], [], [], [], [], []

    def main_thread():                      # ros_simulate.py:152-162 -> update_posecells
        try:
            go.wait()
            for v in od:
                got_max.append(net.update(v))
                got_vol.append(net.posecells)
        except Exception as e:              # pragma: no cover - reported below
            errors.append(e)

    def vision_thread():                    # ros_simulate.py:98-113
        try:
            go.wait()
            for f in frames:
                peak = net.get_pc_max()
                vis_peak.append(peak)
                vis_idx.append(vts.match(f, *peak).get_index())
        except Exception as e:              # pragma: no cover
            errors.append(e)

    def viewer_thread():                    # a subscriber reading the published volume
        try:
            go.wait()
            for _ in range(60):
                reads.append(net.posecells)
        except Exception as e:              # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=f) for f in (main_thread, vision_thread, viewer_thread)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors
    # the stepping thread's results are the sequential ones, bit for bit
    assert got_max == seq_max
    for a, b in zip(got_vol, seq_vol):
        assert np.array_equal(a, b)
    # the template indices do not depend on the pose cells
    assert vis_idx == seq_idx
    # every peak the vision thread saw is the state before or after some step
    allowed = {first_peak} | set(seq_max)
    assert set(vis_peak) <= allowed, set(vis_peak) - allowed
    # every volume the viewer read is a whole state of the sequential run
    for r in reads:
        assert np.isfinite(r).all()
        assert any(np.array_equal(r, s) for s in seq_vol) or np.array_equal(r, _injected(shape, start)), \
            'a read saw a state that is not the state after any step'


def _injected(shape, loc):
    v = np.zeros(shape)
    v[loc] = 1.0
    return v


def test_two_networks_on_two_threads(mod):
    """Distinct handles are independent: two networks stepped concurrently from two
    threads give the results each gives alone (ratslam_abi.h: distinct handles may
    be used from different threads)."""
    od, _, _ = _inputs(400, 1)
    shapes = [(21, 21, 36), (64, 64, 36)]
    alone = []
    for shape in shapes:
        n = mod.PoseCellNetwork(shape)
        n.inject(1, tuple(s // 2 for s in shape))
        alone.append(([n.update(v) for v in od[:200]], n.run(od[200:]), n.posecells))
    nets = [mod.PoseCellNetwork(s) for s in shapes]
    for n, s in zip(nets, shapes):
        n.inject(1, tuple(x // 2 for x in s))
    res = [None, None]
    go = threading.Barrier(2)

    def work(i):
        go.wait()
        res[i] = ([nets[i].update(v) for v in od[:200]], nets[i].run(od[200:]), nets[i].posecells)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for (ma, ra, pa), (mb, rb, pb) in zip(alone, res):
        assert ma == mb and np.array_equal(ra, rb) and np.array_equal(pa, pb)
