"""Headless equivalent of the reference's offline driver
(``/root/reference/ratslam/simulate.py:13-67``) on the MI355X pose-cell network.

``RatSLAM(data, shape).step()`` advances the network by one odometry row, as the
reference does; ``scenario()`` is its ``main`` input (40 steps, vtrans = 3,
vrot = pi/4 on steps 4..8).  Plotting is left out (matplotlib is a viewer
concern); ``python -m pyratslam_amd.simulate`` prints the peak cell per step.
"""
import math
import sys

import numpy as np

from .posecell_network import PoseCellNetwork

POSE_SIZE = (50, 50, 10)   # simulate.py:9


def scenario(steps=40):
    """simulate.py:38-40."""
    data = np.zeros((steps, 2))
    data[:, 0] = 3
    data[4:9, 1] = np.pi / 4
    return data


class RatSLAM:
    """simulate.py:13-34."""

    def __init__(self, data=np.zeros((20, 2)), shape=POSE_SIZE, **pcn_kwargs):
        self.cur_step = 0
        self.pcn = self.init_pcn(shape, **pcn_kwargs)
        self.data = data

    def init_pcn(self, shape, **pcn_kwargs):
        pcn = PoseCellNetwork(shape, **pcn_kwargs)
        midpoint = tuple(int(math.floor(s / 2)) for s in shape)   # all energy in the centre
        pcn.inject(1, midpoint)
        self.current_pose_cell = midpoint
        return pcn

    def step(self):
        self.current_pose_cell = self.pcn.update(self.data[self.cur_step, :])
        self.cur_step += 1


def main(steps=40, out=sys.stdout):
    sim = RatSLAM(data=scenario(steps), shape=POSE_SIZE)
    for s in range(steps):
        sim.step()
        pc = sim.pcn.posecells
        print('step %2d  max_pc %s  cells>0.002: %d' % (s, sim.current_pose_cell,
                                                       int((pc > .002).sum())), file=out)
    return sim


if __name__ == '__main__':
    main()
