"""Experience map of the ROS node (host side, O(1) per step).

Out of the GPU path by design (dead reckoning, one point
per pose-cell step), kept here because it is the observable the reference's
config-5 replay publishes (``ros_simulate.py:137,143``).  Same API and
arithmetic as ``/root/reference/ratslam/experience_map.py``:

* ``clip_rad_180``: wrap an angle into (-pi, pi] with the reference's ceil-based
  correction (:6-11);
* ``ExperienceMap.update(vtrans, vrot, pc_loc)``: heading first, then the
  position along the new heading, then a new experience at the accumulated
  point (:52-60) -- linking and view templates are TODO in the reference too;
* ``get_points`` / ``get_current_point`` (:62-70).
"""
import numpy as np


def clip_rad_180(angle):
    """experience_map.py:6-11."""
    two_pi = 2 * np.pi
    if angle > np.pi:
        return angle - np.ceil(angle / two_pi) * two_pi
    if angle <= -np.pi:
        return angle + np.ceil(abs(angle) / two_pi) * two_pi
    return angle


class Experience:
    """experience_map.py:13-29: the pose cell it was created at, its view
    template (unused) and its point on the map."""

    def __init__(self, pc_loc, em_loc, vt=None):
        self.pc_x, self.pc_y, self.pc_th = pc_loc[0], pc_loc[1], pc_loc[2]
        self.vt = vt
        self.m_x, self.m_y = em_loc[0], em_loc[1]

    def get_point(self):
        return (self.m_x, self.m_y)


class ExperienceMap:
    """experience_map.py:31-70."""

    def __init__(self):
        self.accum_delta_x = 0
        self.accum_delta_y = 0
        self.accum_delta_th = 0
        self.experiences = []
        self.current_exp = None

    def create(self, pc_loc, vt=None):
        exp = Experience(pc_loc, (self.accum_delta_x, self.accum_delta_y), vt)
        self.experiences.append(exp)
        self.current_exp = exp

    def update(self, vtrans, vrot, pc_loc, vt=None):
        self.accum_delta_th = clip_rad_180(self.accum_delta_th + vrot)
        self.accum_delta_x += vtrans * np.cos(self.accum_delta_th)
        self.accum_delta_y += vtrans * np.sin(self.accum_delta_th)
        self.create(pc_loc)

    def get_points(self):
        return [e.get_point() for e in self.experiences]

    def get_current_point(self):
        return self.current_exp.get_point()
