"""NumPy restatement of the pose-cell network step (TEST INFRASTRUCTURE ONLY).

Restates ``/root/reference/ratslam/posecell_network.py`` and the three OpenCL
kernels ``conv`` / ``conv_xy_origin_filters`` / ``conv_z`` of
``/root/reference/ratslam/convolution.py`` in float64.  Semantics follow the
reference as it runs under Python 2 (its only runnable interpreter, see
``convolution.py:25``): integer ``/`` in the 2-D filter LUT builder.

Bit-exactness: every correlation accumulates its taps in the reference kernel's
loop order (x outer, then y, then z) as separate multiply and add (the golden
vectors are produced with ``gcc -ffp-contract=off``), and all host-side
arithmetic uses the same NumPy/SciPy calls on the same operand values.
"""
import math

import numpy as np
from scipy.special import cbrt

# posecell_network.py:10-16
PC_E_SIGMA = 1
PC_I_SIGMA = 2
PC_E_DIM = 7
PC_I_DIM = 5
PC_GLOBAL_INHIB = 0.2
PC_CELL_X_SIZE = 0.2
FILTER_LEN = 7          # convolution.py:40 (max(fil.shape) of the 7x7x7 kernel)
HALF = FILTER_LEN // 2  # convolution.py:41


class LutKeyError(KeyError):
    """Raised where the reference raises ``KeyError`` (posecell_network.py:249)."""


# ----------------------------------------------------------------------------
# Filters
# ----------------------------------------------------------------------------
def dog_kernel_3d(dim_e=PC_E_DIM, dim_i=PC_I_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA):
    """3-D difference-of-Gaussians excitation kernel (posecell_network.py:97-113).

    The window masks of :105/:108 are always 1 for dim 7 (centre 3 +/- 5 or 7
    covers every index), so every tap carries both Gaussians.  Evaluated with
    scalar ``math.exp`` per tap like the reference, then normalised by
    ``|numpy.sum|``.
    """
    dim = max(dim_e, dim_i)
    c = dim // 2
    coef_e = 1.0 / (sigma_e * math.sqrt(2 * math.pi)) ** 3
    coef_i = 1.0 / (sigma_i * math.sqrt(2 * math.pi)) ** 3
    k = np.empty((dim, dim, dim))
    for idx in np.ndindex(dim, dim, dim):
        num = -sum((v - c) ** 2 for v in idx)
        inside_e = max(idx) <= c + dim_e and min(idx) >= c - dim_e
        inside_i = max(idx) <= c + dim_i and min(idx) >= c - dim_i
        k[idx] = (inside_e * coef_e) * math.exp(num / (2 * sigma_e ** 2)) - \
                 (inside_i * coef_i) * math.exp(num / (2 * sigma_i ** 2))
    k /= abs(np.sum(k.ravel()))
    return k


def gauss_1d_factors(dim=PC_E_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA):
    """1-D factors g_e, g_i with K = (g_e x g_e x g_e - g_i x g_i x g_i) / |sum K|.

    Used by the HIP path's rank-2 separable form of the 3-D kernel; returned
    here so tests can confirm the factorisation against ``dog_kernel_3d``.
    """
    c = dim // 2
    x = np.arange(dim) - c
    ge = np.exp(-(x ** 2) / (2.0 * sigma_e ** 2)) / (sigma_e * math.sqrt(2 * math.pi))
    gi = np.exp(-(x ** 2) / (2.0 * sigma_i ** 2)) / (sigma_i * math.sqrt(2 * math.pi))
    full = np.einsum('i,j,k->ijk', ge, ge, ge) - np.einsum('i,j,k->ijk', gi, gi, gi)
    return ge, gi, abs(full.sum())


def dog_offset_2d(origin, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA, shape=(7, 7)):
    """Shifted 2-D DoG, cube-rooted (posecell_network.py:210-222).

    Built on ``meshgrid`` ('xy' indexing: the first origin component shifts the
    column axis), normalised by ``|sum|`` then ``scipy.special.cbrt``.
    """
    cx, cy = shape[0] // 2, shape[1] // 2
    gx, gy = np.meshgrid(np.arange(shape[0]) - origin[0], np.arange(shape[1]) - origin[1])
    r2 = -(gx - cx) ** 2 - (gy - cy) ** 2
    f = 1.0 / (2 * sigma_e ** 2 * np.pi) * np.exp(r2 / (2 * sigma_e ** 2)) - \
        1.0 / (2 * sigma_i ** 2 * np.pi) * np.exp(r2 / (2 * sigma_i ** 2))
    f /= abs(np.sum(f.ravel()))
    return cbrt(f)


def dog_offset_1d(origin, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA, size=7):
    """Shifted 1-D DoG, cube-rooted (posecell_network.py:224-235)."""
    d = np.arange(size) - origin - size // 2
    f = 1.0 / (sigma_e * math.sqrt(2 * np.pi)) * np.exp(-np.square(d) / (2 * sigma_e ** 2)) - \
        1.0 / (sigma_i * math.sqrt(2 * np.pi)) * np.exp(-np.square(d) / (2 * sigma_i ** 2))
    f /= abs(np.sum(f.ravel()))
    return cbrt(f)


def lut_2d(precision=1):
    """The 100-entry filter LUT (posecell_network.py:50-59), Python-2 semantics.

    Under Python 2 ``x / (precision*10)`` is floor division on ints, so each
    key's filter origin is (x // 10, y // 10) in {-1, 0}^2.
    """
    span = range(-5 * precision, 5 * precision)
    return {(x, y): dog_offset_2d((x // (precision * 10), y // (precision * 10)))
            for x in span for y in span}


# ----------------------------------------------------------------------------
# Per-step control (host scalars of path_integration, posecell_network.py:252-308)
# ----------------------------------------------------------------------------
def step_control(vtrans, vrot, shape, lut, lut_precision=10):
    """Return the per-step control the reference derives on the host.

    ``ox, oy``   integer shifts per theta layer (:262-265, ``around`` = half-even)
    ``keys``     LUT keys per layer; note both components come from the x
                 residual (:249) and ``int`` truncates
    ``filters``  (7, 7, TH) per-layer 2-D filters looked up in ``lut``
    ``radius``   ``ceil(|vtrans|)`` in cells (:273)
    ``z_origin`` ``floor(vrot + .5)`` in layers (:304) and ``zf`` its 1-D filter
    Raises ``LutKeyError`` exactly where the reference raises ``KeyError``.
    """
    th = shape[2]
    vrot_scale = 2.0 * np.pi / th
    vt = vtrans / PC_CELL_X_SIZE
    vr = vrot / vrot_scale
    mid = th // 2
    ang = (np.arange(th).reshape((1, th)) - mid) * vrot_scale
    with np.errstate(invalid='ignore', over='ignore'):   # non-finite vtrans: NaN residuals, as numpy gives
        exact = np.concatenate((vt * np.cos(ang), vt * np.sin(ang)), axis=0)
        rounded = np.concatenate((np.around(vt * np.cos(ang)), np.around(vt * np.sin(ang))), axis=0)
        resid = exact - rounded
    keys = []
    filters = np.empty((7, 7, th))
    for z in range(th):
        k = int(resid[0, z] * lut_precision)
        keys.append(k)
        try:
            filters[:, :, z] = lut[(k, k)]
        except KeyError as e:
            raise LutKeyError((k, k)) from e
    # Python 2: math.floor returns a NaN / infinite argument unchanged, and the 1-D
    # filter built on it is all NaN (exp(NaN), or 0/0 in its normalisation) -- the
    # reference runs on with a NaN volume; Python 3's floor would raise instead
    z_origin = math.floor(vr + .5) if math.isfinite(vr + .5) else vr + .5
    return {
        'ox': rounded[0].astype(np.int32),
        'oy': rounded[1].astype(np.int32),
        'keys': np.asarray(keys, dtype=np.int32),
        'filters': filters,
        'radius': int(np.ceil(abs(vt))),
        'z_origin': z_origin,
        'zf': dog_offset_1d(z_origin) if math.isfinite(z_origin) else np.full(7, np.nan),
    }


# ----------------------------------------------------------------------------
# The three device kernels (convolution.py), reference tap order
# ----------------------------------------------------------------------------
def conv3d_wrap(p, k3):
    """Kernel ``conv`` (convolution.py:228-246): 343-tap periodic correlation."""
    n = k3.shape[0]
    h = n // 2
    pp = np.pad(p, h, mode='wrap')
    X, Y, Z = p.shape
    acc = np.zeros_like(p)
    for x in range(n):
        for y in range(n):
            for z in range(n):
                acc += pp[x:x + X, y:y + Y, z:z + Z] * k3[x, y, z]
    return acc


def conv_xy_shift(p, ox, oy, filters):
    """Kernel ``conv_xy_origin_filters`` (convolution.py:320-340).

    out[i,j,k] = sum_{x,y} P[(i+x-3+ox[k]) % X, (j+y-3+oy[k]) % Y, k] * F[x,y,k]
    The reference's halo is only valid while 3 + radius <= X, Y
    (convolution.py:671-675); this restatement is the periodic meaning of it.
    """
    X, Y, TH = p.shape
    n = filters.shape[0]
    h = n // 2
    ii = np.arange(X)[:, None, None]
    jj = np.arange(Y)[None, :, None]
    kk = np.arange(TH)[None, None, :]
    ox = np.asarray(ox)[None, None, :]
    oy = np.asarray(oy)[None, None, :]
    acc = np.zeros_like(p)
    for x in range(n):
        for y in range(n):
            tap = p[(ii + x - h + ox) % X, (jj + y - h + oy) % Y, kk]
            acc += tap * filters[x, y, :][None, None, :]
    return acc


def conv_z_wrap(p, zf):
    """Kernel ``conv_z`` (convolution.py:344-359): 7-tap periodic along theta."""
    n = len(zf)
    h = n // 2
    Z = p.shape[2]
    pp = np.pad(p, ((0, 0), (0, 0), (h, h)), mode='wrap')
    acc = np.zeros_like(p)
    for z in range(n):
        acc += pp[:, :, z:z + Z] * zf[z]
    return acc


# ----------------------------------------------------------------------------
# Network
# ----------------------------------------------------------------------------
class PoseCellOracle:
    """Float64 restatement of ``PoseCellNetwork`` (posecell_network.py:22-353)."""

    def __init__(self, shape):
        self.shape = tuple(int(s) for s in shape)
        self.posecells = np.zeros(self.shape)
        self.kernel_3d = dog_kernel_3d()
        self.lut = lut_2d()
        self.global_inhibition = PC_GLOBAL_INHIB
        self.max_pc = None

    def inject(self, energy, loc):  # posecell_network.py:322-324
        self.posecells[tuple(int(v) for v in loc)] += energy

    def get_pc_max(self):  # posecell_network.py:317-319
        return tuple(int(v) for v in np.unravel_index(self.posecells.argmax(), self.shape))

    def excite_inhibit_normalise(self):
        """Steps 1-4 of update (posecell_network.py:336-345)."""
        p = conv3d_wrap(self.posecells, self.kernel_3d)
        p[p < self.global_inhibition] = 0
        p[p >= self.global_inhibition] -= self.global_inhibition
        total = np.sum(p.ravel())
        if total != 0:
            p /= total
        self.posecells = p
        return total

    def path_integration(self, vtrans, vrot):  # posecell_network.py:252-314
        ctl = step_control(vtrans, vrot, self.shape, self.lut)
        p = conv_xy_shift(self.posecells, ctl['ox'], ctl['oy'], ctl['filters'])
        p[p < 0] = 0
        p = conv_z_wrap(p, ctl['zf'])
        p[p < 0] = 0
        self.posecells = p
        return ctl

    def update(self, v=(0.0, 0.0)):  # posecell_network.py:326-353
        vtrans, vrot = v[0], v[1]
        self.excite_inhibit_normalise()
        self.path_integration(vtrans, vrot)
        self.max_pc = self.get_pc_max()
        return self.max_pc


def synthetic_odometry(n, seed=0, vtrans_max=0.6, vrot_max=0.15):
    """SURVEY.md section 8(d) odometry: vtrans ~ U(0, 0.6) m, vrot ~ U(-0.15, 0.15) rad."""
    rng = np.random.default_rng(seed)
    vt = rng.uniform(0.0, vtrans_max, n)
    vr = rng.uniform(-vrot_max, vrot_max, n)
    return np.stack([vt, vr], axis=1)
