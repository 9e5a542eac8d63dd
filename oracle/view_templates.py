"""NumPy restatement of the view-template matcher (TEST INFRASTRUCTURE ONLY).

Restates ``/root/reference/ratslam/view_templates.py`` with Python-2 semantics
(integer ``/`` in ``ViewTemplates.__init__``).  With ``uint8`` inputs -- the
ROS camera path, ``ros_simulate.py:100-101`` -- NumPy's ``a - b`` wraps mod 256
and ``abs`` is the identity, so a compare is ``sum((a - b) & 0xFF)`` as
``uint64``; other dtypes get NumPy's ordinary ``|a - b|``.
"""
import numpy as np

MAX_OFFSET = 8  # view_templates.py:14


def vt_score(template, query, max_offset=MAX_OFFSET):
    """``ViewTemplate.match`` (view_templates.py:16-28).

    min over o in [-(m-1), m-1] of sum |T[m+o : H-m+o, :] - Q[m : H-m, :]|
    (rows shift along axis 0 only).
    """
    h = template.shape[0]
    q = query[max_offset:h - max_offset]
    best = np.inf
    for o in range(-max_offset + 1, max_offset):
        d = np.sum(np.abs(template[max_offset + o:h - max_offset + o] - q))
        if d < best:
            best = d
    return best


def vt_scores_library(library, query, max_offset=MAX_OFFSET):
    """Vectorised ``vt_score`` of one query against a (T, H, W) uint8 library.

    Returns uint64[T]; wraps mod 256 exactly like the scalar form.
    """
    lib = np.asarray(library)
    t, h, _ = lib.shape
    if t == 0:
        return np.zeros(0, dtype=np.uint64)
    q = np.asarray(query)[max_offset:h - max_offset]
    best = None
    for o in range(-max_offset + 1, max_offset):
        d = (lib[:, max_offset + o:h - max_offset + o, :] - q[None]).sum(axis=(1, 2), dtype=np.uint64)
        best = d if best is None else np.minimum(best, d)
    return best


def py2_mask(x_range, y_range, x_step, y_step, im_x, im_y):
    """Subsampling mask and template shape of ``ViewTemplates.__init__``
    (view_templates.py:42-57) with Python-2 floor division."""
    base = np.arange(im_x * im_y)
    row = base // im_x
    col = base % im_x
    mask = (row > y_range[0]) & (row < y_range[1]) & (col > x_range[0]) & (col < x_range[1]) & \
           ((row - y_range[0]) % y_step != 0) & ((col - x_range[0]) % x_step != 0)
    shape = ((x_range[1] - x_range[0]) // x_step, (y_range[1] - y_range[0]) // y_step)
    return mask.reshape((im_x, im_y)), shape


class ViewTemplatesOracle:
    """``ViewTemplates`` (view_templates.py:40-75): linear scan, first argmin,
    strict threshold, append-on-miss with index ``len(templates)``."""

    def __init__(self, x_range, y_range, x_step, y_step, im_x, im_y, match_threshold):
        self.mask, self.shape = py2_mask(x_range, y_range, x_step, y_step, im_x, im_y)
        self.match_threshold = match_threshold
        self.templates = []   # list of (H, W) arrays
        self.locations = []

    def subsample(self, image):
        return np.asarray(image)[self.mask].reshape(self.shape)

    def match_template(self, template, pc_x=0, pc_y=0, pc_th=0):
        """Returns (index, is_new, best_score_or_None)."""
        if self.templates:
            scores = vt_scores_library(np.stack(self.templates), template)
            best = scores.min()
            if not best > self.match_threshold:
                return int(np.argmin(scores)), False, int(best)
        else:
            best = None
        self.templates.append(np.array(template))
        self.locations.append((pc_x, pc_y, pc_th))
        return len(self.templates) - 1, True, (None if best is None else int(best))

    def match(self, image, pc_x=0, pc_y=0, pc_th=0):
        return self.match_template(self.subsample(image), pc_x, pc_y, pc_th)


def synthetic_library(t, h=64, w=32, seed=1):
    """(T, H, W) uint8 ~ U[0, 255] from default_rng(1)."""
    return np.random.default_rng(seed).integers(0, 256, size=(t, h, w), dtype=np.uint8)


def synthetic_queries(library, q, seed=2, hit_frac=0.9, max_shift=7, noise=3):
    """SURVEY.md section 8(d) queries: ``hit_frac`` of them are a stored template
    rolled by o ~ U{-7..7} on axis 0 minus one-sided noise in [0, noise]
    (clipped at 0, so no byte wraps); the rest are fresh random images.
    Returns (queries uint8 (Q,H,W), source index or -1)."""
    rng = np.random.default_rng(seed)
    t, h, w = library.shape
    out = np.empty((q, h, w), dtype=np.uint8)
    src = np.full(q, -1, dtype=np.int64)
    for i in range(q):
        if t > 0 and rng.random() < hit_frac:
            j = int(rng.integers(0, t))
            o = int(rng.integers(-max_shift, max_shift + 1))
            base = np.roll(library[j], o, axis=0).astype(np.int16)
            n = rng.integers(0, noise + 1, size=(h, w))
            out[i] = np.clip(base - n, 0, 255).astype(np.uint8)
            src[i] = j
        else:
            out[i] = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    return out, src
