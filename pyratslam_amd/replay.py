"""Bag replay of the reference's ROS node (config 5), headless.

``RatslamReplay`` is ``RatslamRos`` (``/root/reference/ratslam/ros_simulate.py:45-170``)
with the rospy plumbing replaced by a deterministic event loop over a recorded
bag: the same constants (POSE_SIZE, IM_SIZE, ranges, steps, MATCH_THRESHOLD,
ODOM_FREQ, :31-41), the same start (inject 1 at the grid midpoint, :56-57) and
the same callbacks:

* ``odom_callback`` (:125-129) queues a twist when |linear.x| or |angular.z|
  exceeds 0.001;
* ``update_posecells`` (:134-146) steps the network with (x / ODOM_FREQ,
  z / ODOM_FREQ), reads the peak cell and advances the experience map;
* ``vis_callback`` (:98-113) converts the frame to mono8, matches it against the
  view templates at the current peak cell and records the template index
  (optionally feeding the match back: the reference's commented-out
  ``pcn.inject(e, template.location())``, :107-108).

Interleaving: the ROS node drains the twist queue on its main thread while the
image callback runs on a subscriber thread; the replay fixes the order the node
takes when its main loop keeps up -- messages in bag order, every queued twist
applied before the next frame is matched.  Consecutive twists are applied with
one ``PoseCellNetwork.run`` (one host round trip), which gives the same states
and peaks as one ``update`` each.

Outputs (the node's published topics): ``pc_max`` per update, ``em_points``
(``navbot/experiencemap``, :142-146) and ``template_index`` per frame
(``navbot/templatematches``, :110-113).

``python -m pyratslam_amd.replay --bag FILE`` replays a bag;
``--synthetic N`` writes and replays a synthetic one (``synthetic.ros_stream``).
"""
import argparse
import json
import math
import sys
import time
from collections import deque

import numpy as np

from . import rosbag
from .experience_map import ExperienceMap

# ros_simulate.py:31-41
POSE_SIZE = (21, 21, 36)
IM_SIZE = (256, 256)
X_RANGE = (32, 96)
Y_RANGE = (32, 96)
X_STEP = 2
Y_STEP = 2
MATCH_THRESHOLD = 45000
ODOM_FREQ = 10
ODOM_TOPIC = 'navbot/odom'
IMAGE_TOPIC = 'navbot/camera/image'


class RatslamReplay:
    """``RatslamRos`` driven by recorded messages.

    ``pcn`` / ``vts`` / ``em``: objects with the reference's APIs; by default the
    MI355X ``PoseCellNetwork`` and ``ViewTemplates`` of this package (any other
    implementation with the same API -- the CPU oracle, the reference itself --
    can be dropped in, which is how parity is checked)."""

    def __init__(self, pose_size=POSE_SIZE, im_size=IM_SIZE, x_range=X_RANGE, y_range=Y_RANGE,
                 x_step=X_STEP, y_step=Y_STEP, match_threshold=MATCH_THRESHOLD,
                 odom_freq=ODOM_FREQ, feedback_energy=None, pcn=None, vts=None, em=None,
                 device=0, precision='float32', batch=True, publish=False):
        # publish: the node's per-step work in full -- every update reads the whole
        # .posecells volume, as ros_simulate.py:140-145 does to publish it -- so steps
        # go one by one (no batched run()) and the network exports eagerly
        self.publish = publish
        if pcn is None:
            from .posecell_network import PoseCellNetwork
            pcn = PoseCellNetwork(shape=pose_size, precision=precision, device=device,
                                  readback='eager' if publish else 'lazy')
        if vts is None:
            from .view_templates import ViewTemplates
            vts = ViewTemplates(x_range=x_range, y_range=y_range, x_step=x_step, y_step=y_step,
                                im_x=im_size[0], im_y=im_size[1], match_threshold=match_threshold,
                                device=device)
        self.pcn, self.vts = pcn, vts
        self.em = em if em is not None else ExperienceMap()
        self.odom_freq = odom_freq
        self.feedback_energy = feedback_energy
        self.batch = batch and hasattr(pcn, 'run') and not publish
        self.published = 0   # .posecells volumes read (publish=True)
        self.twist_data = deque()
        # ros_simulate.py:56-57 (Python-2 int / 2, then math.floor)
        self.pcn.inject(1, tuple(int(math.floor(s // 2)) for s in pose_size))
        self.pc_max, self.em_points, self.template_index = [], [], []

    # -- callbacks ---------------------------------------------------------------
    def odom_callback(self, twist):
        """ros_simulate.py:125-129."""
        if abs(twist.linear[0]) > 0.001 or abs(twist.angular[2]) > 0.001:
            self.twist_data.append(twist)

    def vis_callback(self, im):
        """ros_simulate.py:98-113 (after imgmsg_to_cv(data, "mono8"))."""
        pc_max = self.pcn.get_pc_max()
        template_match = self.vts.match(input=im, pc_x=pc_max[0], pc_y=pc_max[1], pc_th=pc_max[2])
        self.template_index.append(int(template_match.get_index()))
        if self.feedback_energy:
            self.pcn.inject(self.feedback_energy, tuple(template_match.location()))

    def update_posecells(self, vtrans, vrot):
        """ros_simulate.py:134-146 (publishing reduced to recording; with publish=True
        the volume is read as the node reads it to publish, :140)."""
        self.pcn.update((vtrans, vrot))
        self._record(vtrans, vrot, self.pcn.get_pc_max())
        if self.publish:
            pc = self.pcn.posecells
            self.published += pc.size

    def _record(self, vtrans, vrot, pc_max):
        pc_max = tuple(int(v) for v in pc_max)
        self.em.update(vtrans, vrot, pc_max)
        self.pc_max.append(pc_max)
        self.em_points.append(tuple(float(v) for v in self.em.get_current_point()))

    def drain(self):
        """The main loop's queue drain (ros_simulate.py:156-162)."""
        if not self.twist_data:
            return
        steps = []
        while self.twist_data:
            twist = self.twist_data.popleft()
            steps.append((twist.linear[0] / self.odom_freq, twist.angular[2] / self.odom_freq))
        if self.batch:
            maxes = self.pcn.run(np.array(steps, dtype=np.float64))
            for (vt, vr), m in zip(steps, maxes):
                self._record(vt, vr, m)
        else:
            for vt, vr in steps:
                self.update_posecells(vt, vr)

    # -- drivers -----------------------------------------------------------------
    def replay_events(self, events):
        """``synthetic.ros_stream`` events (already decoded)."""
        for ev in events:
            if ev[0] == 'odom':
                self.odom_callback(rosbag.Twist(ev[2], ev[3]))
            else:
                self.drain()
                self.vis_callback(ev[2])
        self.drain()
        return self

    def replay_bag(self, path, odom_topic=ODOM_TOPIC, image_topic=IMAGE_TOPIC):
        """Messages of a bag in order; odometry from nav_msgs/Odometry (or a bare
        geometry_msgs/Twist), frames from sensor_msgs/Image."""
        o, i = odom_topic.lstrip('/'), image_topic.lstrip('/')
        for m in rosbag.read_bag(path, topics={o, i}):
            if m.topic.lstrip('/') == o:
                tw = rosbag.decode_twist(m.data) if m.type == 'geometry_msgs/Twist' else \
                    rosbag.decode_odometry_twist(m.data)
                self.odom_callback(tw)
            else:
                self.drain()
                self.vis_callback(rosbag.image_to_mono8(rosbag.decode_image(m.data)))
        self.drain()
        return self

    def results(self):
        return {'pc_max': np.array(self.pc_max, dtype=np.int64).reshape(-1, 3),
                'em_points': np.array(self.em_points, dtype=np.float64).reshape(-1, 2),
                'template_index': np.array(self.template_index, dtype=np.int64),
                'templates': len(self.vts.templates)}


def sharded_templates(d, device, host_reduce=False, x_range=X_RANGE, y_range=Y_RANGE, x_step=X_STEP,
                      y_step=Y_STEP, im_size=IM_SIZE, match_threshold=MATCH_THRESHOLD):
    """The view-template library sharded over the ranks of ``d`` (a dist.Dist):
    template g on rank g % N, one RCCL allreduce(min) per match (or the host
    reducer of the control plane with ``host_reduce``, for several ranks on one
    GPU)."""
    from .view_templates import ShardedViewTemplates
    if host_reduce:
        return ShardedViewTemplates(x_range, y_range, x_step, y_step, im_size[0], im_size[1],
                                    match_threshold, d.rank, d.world, reducer=d.min_keys, device=device)
    uid = d.bcast_bytes(ShardedViewTemplates.unique_id() if d.rank == 0 else None)
    return ShardedViewTemplates(x_range, y_range, x_step, y_step, im_size[0], im_size[1],
                                match_threshold, d.rank, d.world, reducer='rccl', unique_id=uid,
                                device=device)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument('--bag', help='ROS 1 bag with navbot/odom and navbot/camera/image')
    src.add_argument('--synthetic', type=int, metavar='N', help='replay N synthetic odometry+frame pairs')
    ap.add_argument('--device', type=int, default=None, help='default: LOCAL_RANK')
    ap.add_argument('--precision', default='float32')
    ap.add_argument('--feedback', type=float, default=None,
                    help='inject this energy at each matched template (ros_simulate.py:107-108)')
    ap.add_argument('--gpus', type=int, default=1,
                    help='ranks (launched here, or by torch.distributed.run): the template '
                         'library is sharded over them, the pose cells are replicated')
    ap.add_argument('--host-reduce', action='store_true',
                    help='combine the ranks\' keys on the host (several ranks on one GPU)')
    args = ap.parse_args(argv)
    from . import launch
    if args.gpus > 1 and not launch.under_launcher():
        return launch.spawn(args.gpus, ['-m', 'pyratslam_amd.replay'] + list(
            sys.argv[1:] if argv is None else argv))
    from .dist import Dist
    d = Dist(args.gpus)
    dev = d.local if args.device is None else args.device
    vts = sharded_templates(d, dev, args.host_reduce) if d.world > 1 else None
    r = RatslamReplay(device=dev, precision=args.precision, feedback_energy=args.feedback, vts=vts)
    d.barrier()
    t0 = time.perf_counter()
    if args.bag:
        r.replay_bag(args.bag)
    else:
        from . import synthetic
        r.replay_events(synthetic.ros_stream(args.synthetic))
    dt = d.max(time.perf_counter() - t0)
    res = r.results()
    if d.rank == 0:
        print(json.dumps({'ranks': d.world, 'updates': len(res['pc_max']),
                          'frames': len(res['template_index']), 'templates': res['templates'],
                          'seconds': dt, 'pc_max': res['pc_max'].tolist(),
                          'template_index': res['template_index'].tolist(),
                          'em_points': res['em_points'].tolist()}))
    d.close()
    return 0


if __name__ == '__main__':
    sys.exit(main())
