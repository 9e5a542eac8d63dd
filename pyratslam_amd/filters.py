"""Host-side filter construction and per-step control of the pose-cell network.

These are the small host computations the reference performs in NumPy around
its device kernels (``/root/reference/ratslam/posecell_network.py``).  They stay
on the host, in NumPy/SciPy, so every control value handed to the GPU is
bit-identical to the reference's: filter taps (``exp``/``cbrt`` on the same
operands), the half-even ``around`` of the shifts, ``int`` truncation of the LUT
key and ``floor(vrot + .5)``.  The GPU does all volume work.

Semantics follow Python 2, the only interpreter the reference runs on
(``convolution.py:25``): the LUT origins use integer division (:58).
"""
import math

import numpy as np
from scipy.special import cbrt

# posecell_network.py:10-17
PC_E_SIGMA = 1
PC_I_SIGMA = 2
PC_E_DIM = 7
PC_I_DIM = 5
PC_GLOBAL_INHIB = 0.2
PC_CELL_X_SIZE = 0.2
FILTER_LEN = 7
LUT_PRECISION = 10          # filter_dict_2d_precision (:48)
LUT_KEYS = range(-5, 5)     # xrange(-5*precision, 5*precision), precision = 1 (:55-56)

_SQRT_2PI = math.sqrt(2 * math.pi)


def _gauss_coef(sigma, order):
    return 1.0 / (sigma * _SQRT_2PI) ** order


def kernel_3d(dim_e=PC_E_DIM, dim_i=PC_I_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA):
    """diff_gaussian(order=3) (posecell_network.py:97-113), bit-identical.

    Every tap depends only on the integer squared radius d2 = dx^2+dy^2+dz^2, so
    the 28 distinct values are evaluated with scalar ``math.exp`` (as the
    reference does per tap) and scattered; the window masks are always 1 here.
    """
    dim = max(dim_e, dim_i)
    c = dim // 2
    d = np.arange(dim) - c
    d2 = (d[:, None, None] ** 2 + d[None, :, None] ** 2 + d[None, None, :] ** 2)
    ce, ci = _gauss_coef(sigma_e, 3), _gauss_coef(sigma_i, 3)
    table = np.array([ce * math.exp(-r / (2 * sigma_e ** 2)) - ci * math.exp(-r / (2 * sigma_i ** 2))
                      for r in range(int(d2.max()) + 1)])
    k = table[d2]
    k /= abs(np.sum(k.ravel()))
    return k


def diff_gaussian(dim_e=PC_E_DIM, dim_i=PC_I_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA, order=3):
    """diff_gaussian(order=1, 2 or 3) (posecell_network.py:97-142): a DoG over a cube,
    square or line of max(dim_e, dim_i) taps with the reference's window masks and
    per-order coefficients -- 1/(s*sqrt(2pi))^3, 1/(s*s*2*pi), 1/(s*sqrt(2pi)) -- each
    tap one scalar ``math.exp`` per Gaussian, then divided by |sum| (numpy's sum).
    Order 3 is ``kernel_3d`` (the network's excitation kernel); the reference keeps
    orders 2 and 1 as attributes it never uses (:30-31).  Other orders return None,
    as the reference's fall-through does."""
    if order == 3:
        return kernel_3d(dim_e, dim_i, sigma_e, sigma_i)
    if order not in (1, 2):
        return None
    dim = max(dim_e, dim_i)
    c = dim // 2
    if order == 2:
        ce, ci = 1.0 / (sigma_e * sigma_e * 2 * math.pi), 1.0 / (sigma_i * sigma_i * 2 * math.pi)
    else:
        ce, ci = _gauss_coef(sigma_e, 1), _gauss_coef(sigma_i, 1)
    f = np.empty((dim,) * order)
    for idx in np.ndindex(*f.shape):
        hi, lo = max(idx), min(idx)
        r = sum((v - c) ** 2 for v in idx)
        me = 1 if hi <= c + dim_e and lo >= c - dim_e else 0
        mi = 1 if hi <= c + dim_i and lo >= c - dim_i else 0
        f[idx] = me * ce * math.exp(-r / (2 * sigma_e ** 2)) - mi * ci * math.exp(-r / (2 * sigma_i ** 2))
    f /= abs(np.sum(f.ravel()))
    return f


def diff_gaussian_separable(dim_e=PC_E_DIM, dim_i=PC_I_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA):
    """diff_gaussian_separable (posecell_network.py:192-208): the order-1 DoG, cube
    rooted (the reference's own FIXME: a DoG is not separable; kept as the attribute
    ``kernel_1d_sep``, unused)."""
    return cbrt(diff_gaussian(dim_e, dim_i, sigma_e, sigma_i, order=1))


def separable_factors(dim=PC_E_DIM, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA):
    """(ge, gi, scale) with kernel_3d == (ge x ge x ge - gi x gi x gi) * scale.

    exp(-(dx^2+dy^2+dz^2)/2s^2)/(s*sqrt(2pi))^3 factorises exactly per axis, so the
    343-tap kernel is rank 2 (agreement with kernel_3d ~2e-16).
    """
    d = np.arange(dim) - dim // 2
    ge = np.exp(-(d ** 2) / (2.0 * sigma_e ** 2)) * _gauss_coef(sigma_e, 1)
    gi = np.exp(-(d ** 2) / (2.0 * sigma_i ** 2)) * _gauss_coef(sigma_i, 1)
    full = np.einsum('i,j,k->ijk', ge, ge, ge) - np.einsum('i,j,k->ijk', gi, gi, gi)
    return ge, gi, 1.0 / abs(full.sum())


def filter_2d(origin, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA, shape=(7, 7)):
    """diff_gaussian_offset_2d (posecell_network.py:210-222), bit-identical.

    'xy' meshgrid: the first origin component shifts the second array axis.
    """
    cols = np.arange(shape[0]) - origin[0] - shape[0] // 2
    rows = np.arange(shape[1]) - origin[1] - shape[1] // 2
    gx, gy = np.meshgrid(cols, rows)
    neg_r2 = -gx ** 2 - gy ** 2
    f = (1.0 / (2 * sigma_e ** 2 * np.pi)) * np.exp(neg_r2 / (2 * sigma_e ** 2)) - \
        (1.0 / (2 * sigma_i ** 2 * np.pi)) * np.exp(neg_r2 / (2 * sigma_i ** 2))
    f /= abs(np.sum(f.ravel()))
    return cbrt(f)


_F1D_CACHE = {}


def filter_1d(origin, sigma_e=PC_E_SIGMA, sigma_i=PC_I_SIGMA, size=7):
    """diff_gaussian_offset_1d (posecell_network.py:224-235), bit-identical, memoised
    per integer origin."""
    key = (int(origin), sigma_e, sigma_i, size)
    f = _F1D_CACHE.get(key)
    if f is None:
        sq = np.square(np.arange(size) - int(origin) - size // 2)
        f = _gauss_coef(sigma_e, 1) * np.exp(-sq / (2 * sigma_e ** 2)) - \
            _gauss_coef(sigma_i, 1) * np.exp(-sq / (2 * sigma_i ** 2))
        f /= abs(np.sum(f.ravel()))
        f = cbrt(f)
        f.setflags(write=False)
        _F1D_CACHE[key] = f
    return f


def lut_origin(key):
    """Python-2 origin of LUT entry ``key`` (posecell_network.py:58): key // 10."""
    return key // LUT_PRECISION


class FilterTable:
    """The 100-entry LUT ``filter_dict_2d`` (posecell_network.py:47,50-59) and the
    table of its distinct filters uploaded to the device once."""

    def __init__(self):
        origins = sorted({(lut_origin(x), lut_origin(y)) for x in LUT_KEYS for y in LUT_KEYS})
        self.origins = origins
        self.index = {o: i for i, o in enumerate(origins)}
        self.filters = np.stack([filter_2d(o) for o in origins])          # (nf, 7, 7)
        self.dict = {(x, y): self.filters[self.index[(lut_origin(x), lut_origin(y))]]
                     for x in LUT_KEYS for y in LUT_KEYS}
        # key k (both components from the x residual, :249) -> table row, for k in [-5, 4]
        self._key_to_row = np.array([self.index[(lut_origin(k), lut_origin(k))] for k in LUT_KEYS],
                                    dtype=np.int32)

    def rows_for_keys(self, keys):
        """Table rows for per-layer keys; raises KeyError like posecell_network.py:249."""
        idx = np.asarray(keys) - LUT_KEYS.start
        if idx.min() < 0 or idx.max() >= len(LUT_KEYS):
            bad = (idx < 0) | (idx >= len(LUT_KEYS))
            k = int(idx[np.argmax(bad)]) + LUT_KEYS.start
            raise KeyError((k, k))
        return self._key_to_row[idx]


_TRIG = {}


def layer_trig(th):
    """(cos, sin) of each layer's heading (dir - mid) * 2pi/TH (posecell_network.py:257-265).

    They do not depend on the odometry, so they are evaluated once per TH with the
    same NumPy calls; vtrans * cos(...) then has the reference's exact bits.
    """
    t = _TRIG.get(th)
    if t is None:
        ang = (np.arange(th) - th // 2) * (2.0 * np.pi / th)
        t = (np.cos(ang), np.sin(ang))
        for a in t:
            a.setflags(write=False)
        _TRIG[th] = t
    return t


def _layer_key_error(resid):
    """The exception the reference's per-layer LUT lookup raises first, in layer order
    (posecell_network.py:244-250: ``filter_dict_2d[(int(r * prec), int(r * prec))]``), or
    None: ``int`` of a NaN residual raises ValueError, of an infinite one OverflowError
    (Python 2 and 3 alike), a finite key outside the table KeyError((k, k)).  A NaN
    residual is what a non-finite vtrans gives: ``inf - around(inf)`` is NaN."""
    for r in resid:
        if math.isnan(r):
            return ValueError('cannot convert float NaN to integer')
        if math.isinf(r):
            return OverflowError('cannot convert float infinity to integer')
        k = int(r)
        if not (LUT_KEYS.start <= k < LUT_KEYS.stop):
            return KeyError((k, k))
    return None


NAN_FILTER_1D = np.full(FILTER_LEN, np.nan)
NAN_FILTER_1D.setflags(write=False)


def theta_filter(vr):
    """diff_gaussian_offset_1d(origin=floor(vr + .5)) (posecell_network.py:304-308).  Under
    Python 2 ``math.floor`` of a NaN or infinite argument returns it as a float, and the
    filter built on it is all NaN (``exp`` of NaN, or 0/0 in the normalisation): the
    reference runs on with a NaN volume instead of raising."""
    zo = vr + .5
    if not math.isfinite(zo):
        return NAN_FILTER_1D
    return filter_1d(math.floor(zo))


def step_control(vtrans, vrot, th, table):
    """Per-step control of path_integration (posecell_network.py:252-308).

    Returns (ox, oy, rows, zf, radius) with ox/oy/rows int32[th], zf float64[7].
    Same NumPy operations on the same operands as the reference, so bit-identical.
    Raises what the reference raises at its LUT lookup (:249): KeyError((k, k)) for a
    key outside the table, ValueError for a non-finite vtrans.
    """
    vrot_scale = 2.0 * np.pi / th
    vt = vtrans / PC_CELL_X_SIZE
    vr = vrot / vrot_scale
    cos_a, sin_a = layer_trig(th)
    with np.errstate(invalid='ignore', over='ignore'):
        ex = vt * cos_a
        ey = vt * sin_a
        rx = np.around(ex)
        ry = np.around(ey)
        resid = (ex - rx) * LUT_PRECISION
    if not np.isfinite(resid).all() or resid.min() < LUT_KEYS.start or resid.max() >= LUT_KEYS.stop:
        err = _layer_key_error(resid)
        if err is not None:
            raise err
    keys = np.trunc(resid).astype(np.int64)   # int() truncates
    rows = table.rows_for_keys(keys)
    zf = theta_filter(vr)
    radius = int(np.ceil(abs(vt)))
    # shifts beyond int32 (|vtrans| above ~4e8 m per step) saturate instead of wrapping
    # through a cast warning; the reference would fail allocating a halo of that radius
    lim = np.iinfo(np.int32)
    return (np.clip(rx, lim.min, lim.max).astype(np.int32), np.clip(ry, lim.min, lim.max).astype(np.int32),
            rows, zf, radius)


def batch_control(odometry, th, table):
    """step_control for n steps at once (vectorised over steps).

    Returns (ox, oy, rows, zf) shaped (n, th), (n, th), (n, th), (n, 7) and the
    index of the first step whose LUT lookup raises (or None): steps before it
    are valid, matching the point where the reference would raise.
    """
    od = np.asarray(odometry, dtype=np.float64).reshape(-1, 2)
    n = od.shape[0]
    vrot_scale = 2.0 * np.pi / th
    vt = od[:, 0] / PC_CELL_X_SIZE
    vr = od[:, 1] / vrot_scale
    cos_a, sin_a = layer_trig(th)
    with np.errstate(invalid='ignore', over='ignore'):
        ex = vt[:, None] * cos_a[None, :]
        ey = vt[:, None] * sin_a[None, :]
        rx = np.around(ex)
        ry = np.around(ey)
        resid = (ex - rx) * LUT_PRECISION
    bad = (~np.isfinite(resid)).any(axis=1)
    keys = np.trunc(np.where(np.isfinite(resid), resid, 0.0)).astype(np.int64)
    bad |= ((keys < LUT_KEYS.start) | (keys >= LUT_KEYS.stop)).any(axis=1)
    first_bad = int(np.argmax(bad)) if bad.any() else None
    keys = np.clip(keys, LUT_KEYS.start, LUT_KEYS.stop - 1)
    rows = table._key_to_row[keys - LUT_KEYS.start]
    zf = np.empty((n, FILTER_LEN))
    zo = vr + .5
    fin = np.isfinite(zo)
    zf[~fin] = np.nan
    zorig = np.floor(np.where(fin, zo, 0.0)).astype(np.int64)
    for o in np.unique(zorig[fin]):
        zf[fin & (zorig == o)] = filter_1d(int(o))
    lim = np.iinfo(np.int32)
    ox = np.clip(np.where(np.isfinite(rx), rx, 0), lim.min, lim.max).astype(np.int32)
    oy = np.clip(np.where(np.isfinite(ry), ry, 0), lim.min, lim.max).astype(np.int32)
    return (ox, oy, rows.astype(np.int32), zf, first_bad)


ZORIG_MARGIN = 8


def odometry_tables(th, table, margin=ZORIG_MARGIN):
    """Tables of the library-side control (rs_pc_set_odometry_tables,
    rs_pc_odom_control): every transcendental of path_integration evaluated by
    NumPy exactly as step_control evaluates it, so the library applies only
    correctly rounded IEEE operations to them.  Theta-filter origins cover
    |origin| <= th // 2 + margin (|vrot| up to about pi + margin layers per step)."""
    cos_a, sin_a = layer_trig(th)
    zmin = -(th // 2 + margin)
    nz = 2 * (th // 2 + margin) + 1
    return dict(vtrans_scale=PC_CELL_X_SIZE, vrot_scale=2.0 * np.pi / th,
                cos_a=np.ascontiguousarray(cos_a, dtype=np.float64),
                sin_a=np.ascontiguousarray(sin_a, dtype=np.float64),
                key_min=LUT_KEYS.start, nkeys=len(LUT_KEYS),
                key_rows=np.ascontiguousarray(table._key_to_row, dtype=np.int32),
                zorig_min=zmin, nz=nz,
                zf_table=np.ascontiguousarray(
                    np.stack([filter_1d(o) for o in range(zmin, zmin + nz)]), dtype=np.float64))


def table_args(t):
    """rs_pc_set_odometry_tables / rs_pc_odom_control table arguments as ctypes values."""
    import ctypes
    f64 = ctypes.POINTER(ctypes.c_double)
    return (t['vtrans_scale'], t['vrot_scale'], t['cos_a'].ctypes.data_as(f64),
            t['sin_a'].ctypes.data_as(f64), t['key_min'], t['nkeys'],
            t['key_rows'].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), t['zorig_min'], t['nz'],
            t['zf_table'].ctypes.data_as(f64))
