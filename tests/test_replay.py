"""Config 5 (bag replay through the ROS node's logic) on the CPU: the bag reader
and writer, the experience map, and the replay loop with the oracle classes --
all against the golden replay made with the reference's own PoseCellNetwork,
ViewTemplates and ExperienceMap (tests/golden/gen_golden.py gen_ros_replay)."""
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import posecell as P
from oracle import view_templates as V
from pyratslam_amd import experience_map as EM
from pyratslam_amd import replay, rosbag, synthetic


class _OracleTemplate:
    def __init__(self, index, loc):
        self.index, self.loc = index, loc

    def get_index(self):
        return self.index

    def location(self):
        return self.loc


class OracleViewTemplates(V.ViewTemplatesOracle):
    """ViewTemplates API (match -> template object) over the NumPy oracle."""

    def match(self, input, pc_x=0, pc_y=0, pc_th=0):
        i, _, _ = super().match(input, pc_x, pc_y, pc_th)
        return _OracleTemplate(i, self.locations[i])


def oracle_replay(**kw):
    vts = OracleViewTemplates(replay.X_RANGE, replay.Y_RANGE, replay.X_STEP, replay.Y_STEP,
                              replay.IM_SIZE[0], replay.IM_SIZE[1], replay.MATCH_THRESHOLD)
    return replay.RatslamReplay(pcn=P.PoseCellOracle(replay.POSE_SIZE), vts=vts, **kw)


@pytest.fixture(scope='module')
def golden():
    return load_golden('ros_replay')


@pytest.fixture(scope='module')
def events(golden):
    return synthetic.ros_stream(int(golden['n']), seed=int(golden['seed']))


@pytest.mark.parametrize('compression', ['none', 'bz2'])
def test_bag_roundtrip(tmp_path, events, compression):
    path = synthetic.write_ros_bag(str(tmp_path / 'x.bag'), events[:40], compression=compression)
    msgs = rosbag.read_bag(path)
    assert len(msgs) == 40
    for ev, m in zip(events[:40], msgs):
        assert abs(m.time - ev[1]) < 1e-6
        if ev[0] == 'odom':
            assert m.topic == '/navbot/odom' and m.type == 'nav_msgs/Odometry'
            tw = rosbag.decode_odometry_twist(m.data)
            assert tw.linear == ev[2] and tw.angular == ev[3]
        else:
            assert m.type == 'sensor_msgs/Image'
            img = rosbag.decode_image(m.data)
            assert img.encoding == 'mono8' and (img.height, img.width) == ev[2].shape
            assert np.array_equal(rosbag.image_to_mono8(img), ev[2])
    only = rosbag.read_bag(path, topics={'navbot/odom'})
    assert len(only) == 20 and all(m.topic == '/navbot/odom' for m in only)


def test_bag_errors(tmp_path):
    bad = tmp_path / 'bad.bag'
    bad.write_bytes(b'not a bag')
    with pytest.raises(rosbag.BagError):
        rosbag.read_bag(str(bad))
    img = rosbag.decode_image(rosbag.encode_image(1.0, np.zeros((4, 4), np.uint16), encoding='mono16'))
    with pytest.raises(rosbag.BagError):
        rosbag.image_to_mono8(img)


def test_colour_frames_to_mono8():
    rgb = np.random.default_rng(0).integers(0, 256, (5, 7, 3), dtype=np.uint8)
    img = rosbag.decode_image(rosbag.encode_image(2.0, rgb, encoding='rgb8'))
    got = rosbag.image_to_mono8(img)
    # cv_bridge / OpenCV RGB2GRAY on 8-bit data: 14-bit fixed point, rounded
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    want = (4899 * r + 9617 * g + 1868 * b + 8192) >> 14
    assert np.array_equal(got, want.astype(np.uint8))
    bgr = rosbag.decode_image(rosbag.encode_image(2.0, rgb[..., ::-1], encoding='bgr8'))
    assert np.array_equal(rosbag.image_to_mono8(bgr), got)
    # OpenCV's known outputs for the primaries and white: 76, 150, 29, 255
    prim = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255]]], dtype=np.uint8)
    img = rosbag.decode_image(rosbag.encode_image(2.0, prim, encoding='rgb8'))
    assert rosbag.image_to_mono8(img).tolist() == [[76, 150, 29, 255]]


def test_clip_rad_180():
    # the reference's ceil-based wrap (experience_map.py:6-11), kept as is: congruent
    # mod 2 pi, within (-pi, pi] for |angle| < 2 pi (all the map ever feeds it: the
    # accumulated heading plus one step), but 3 pi -> -pi and 7.5 -> 7.5 - 4 pi
    for a in (0.0, 1.0, np.pi, -np.pi, 3 * np.pi, -3 * np.pi, 7.5, -7.5, 100.0):
        c = EM.clip_rad_180(a)
        assert np.isclose(np.cos(c), np.cos(a)) and np.isclose(np.sin(c), np.sin(a))
        if abs(a) < 2 * np.pi:
            assert -np.pi < c <= np.pi
    assert EM.clip_rad_180(3 * np.pi) == 3 * np.pi - 4 * np.pi
    assert EM.clip_rad_180(7.5) == 7.5 - 4 * np.pi
    assert EM.clip_rad_180(-np.pi) == np.pi


def test_oracle_replay_matches_reference(golden, events):
    """The replay loop with the oracle pose cells / templates and this package's
    experience map reproduces the reference's run exactly."""
    r = oracle_replay(batch=False).replay_events(events)
    res = r.results()
    assert np.array_equal(res['pc_max'], golden['pc_max'])
    assert np.array_equal(res['template_index'], golden['template_index'])
    assert res['templates'] == int(golden['templates'])
    assert np.array_equal(res['em_points'], golden['em_points'])   # same float ops: bit-exact


def test_bag_replay_equals_event_replay(tmp_path, golden, events):
    path = synthetic.write_ros_bag(str(tmp_path / 'r.bag'), events, compression='bz2')
    res = oracle_replay(batch=False).replay_bag(path).results()
    assert np.array_equal(res['pc_max'], golden['pc_max'])
    assert np.array_equal(res['template_index'], golden['template_index'])
    assert np.array_equal(res['em_points'], golden['em_points'])


def test_replay_cli_needs_a_source():
    with pytest.raises(SystemExit):
        replay.main([])
