"""Host-side control plane of the drop-in (pyratslam_amd.filters, view mask):
every value handed to the GPU must be bit-identical to the reference's."""
import math

import numpy as np
import pytest

from conftest import load_golden
from oracle import posecell as P
from oracle import view_templates as V
from pyratslam_amd import filters as F
from pyratslam_amd.view_templates import py2_mask


def test_kernel_3d_matches_reference_bits():
    assert np.array_equal(F.kernel_3d(), load_golden('kernels')['kernel_3d'])


def test_unused_reference_kernels_match_reference_bits():
    """kernel_2d, kernel_1d and kernel_1d_sep (posecell_network.py:30-32), kept by the
    reference as attributes it never uses: bit-identical to the reference-made golden
    values (diff_gaussian orders 2 and 1, diff_gaussian_separable); order 3 is kernel_3d,
    any other order None, as the reference's fall-through."""
    g = load_golden('kernels')
    assert np.array_equal(F.diff_gaussian(order=2), g['kernel_2d'])
    assert np.array_equal(F.diff_gaussian(order=1), g['kernel_1d'])
    assert np.array_equal(F.diff_gaussian_separable(), g['kernel_1d_sep'])
    assert np.array_equal(F.diff_gaussian(order=3), g['kernel_3d'])
    assert F.diff_gaussian(order=4) is None


def test_separable_factors_reconstruct_kernel():
    ge, gi, scale = F.separable_factors()
    k = (np.einsum('i,j,k->ijk', ge, ge, ge) - np.einsum('i,j,k->ijk', gi, gi, gi)) * scale
    assert np.abs(k - load_golden('kernels')['kernel_3d']).max() < 2e-16 * 8


def test_filter_table_matches_lut():
    g = load_golden('kernels')
    t = F.FilterTable()
    assert t.filters.shape == (4, 7, 7)   # Py2: origins in {-1, 0}^2
    for key, f in zip(g['lut_keys'], g['lut_filters']):
        assert np.array_equal(t.dict[tuple(int(v) for v in key)], f)


def test_filter_1d_bits_and_cache():
    g = load_golden('kernels')
    for o, f in zip(g['f1d_origins'], g['f1d']):
        assert np.array_equal(F.filter_1d(int(o)), f)
        assert F.filter_1d(int(o)) is F.filter_1d(int(o))


def _odometry(n, seed):
    r = np.random.default_rng(seed)
    return np.stack([r.uniform(0, 0.6, n), r.uniform(-0.15, 0.15, n)], axis=1)


@pytest.mark.parametrize('th', [10, 18, 36, 72])
def test_step_control_matches_oracle(th):
    table = F.FilterTable()
    lut = P.lut_2d()
    od = np.concatenate([_odometry(200, th), [[3.0, np.pi / 4], [3.0, 0.0], [0.0, 0.0]]])
    for vt, vr in od:
        try:
            ref = P.step_control(vt, vr, (8, 8, th), lut)
        except KeyError:
            with pytest.raises(KeyError):
                F.step_control(vt, vr, th, table)
            continue
        ox, oy, rows, zf, radius = F.step_control(vt, vr, th, table)
        assert np.array_equal(ox, ref['ox']) and np.array_equal(oy, ref['oy'])
        assert np.array_equal(zf, ref['zf'])
        assert radius == ref['radius']
        assert np.array_equal(table.filters[rows], np.moveaxis(ref['filters'], -1, 0))


def test_batch_control_equals_step_control():
    table = F.FilterTable()
    od = _odometry(300, 7)
    ox, oy, rows, zf, bad = F.batch_control(od, 36, table)
    assert bad is None
    for s in range(len(od)):
        a = F.step_control(od[s, 0], od[s, 1], 36, table)
        assert np.array_equal(ox[s], a[0]) and np.array_equal(oy[s], a[1])
        assert np.array_equal(rows[s], a[2]) and np.array_equal(zf[s], a[3])


def test_keyerror_at_half_cell():
    # vtrans = 0.1 m = 0.5 cell: around(0.5) = 0 -> residual 0.5 -> key 5 (posecell_network.py:249)
    table = F.FilterTable()
    with pytest.raises(KeyError) as e:
        F.step_control(0.1, 0.0, 18, table)
    assert e.value.args[0] == (5, 5)
    od = np.array([[0.2, 0.0], [0.3, 0.01], [0.1, 0.0], [0.2, 0.0]])
    *_, bad = F.batch_control(od, 18, table)
    assert bad == 2


def test_simulate_scenario_half_boundaries():
    # simulate.py: vtrans 3 m -> 15 cells; 15*cos(60 deg) sits on a .5 rounding edge
    table = F.FilterTable()
    lut = P.lut_2d()
    for th in (10, 36):
        ref = P.step_control(3.0, np.pi / 4, (8, 8, th), lut)
        ox, oy, rows, zf, _ = F.step_control(3.0, np.pi / 4, th, table)
        assert np.array_equal(ox, ref['ox']) and np.array_equal(oy, ref['oy'])
        assert math.floor((np.pi / 4) / (2 * np.pi / th) + .5) == ref['z_origin']


@pytest.mark.parametrize('name', ['vt_trace_ros', 'vt_trace_64x32'])
def test_view_mask_matches_reference(name):
    d = load_golden(name)
    p = d['params']
    mask, shape = py2_mask((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7])
    assert np.array_equal(mask, d['mask'])
    assert shape == tuple(d['shape'])
    m2, s2 = V.py2_mask((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7])
    assert np.array_equal(mask, m2) and shape == s2


def _library_control(th, od):
    """rs_pc_odom_control (host-only entry of libratslam_hip.so) over odometry od (n, 2)."""
    import ctypes
    from pyratslam_amd import _lib
    lib = _lib.load()
    t = F.odometry_tables(th, F.FilterTable())
    od = np.ascontiguousarray(od, dtype=np.float64)
    n = od.shape[0]
    ox = np.empty((n, th), np.int32)
    oy = np.empty((n, th), np.int32)
    rows = np.empty((n, th), np.int32)
    zf = np.empty((n, 7))
    st = np.empty(n, np.int32)
    _lib.check(lib.rs_pc_odom_control(th, *F.table_args(t), n, _lib.ptr(od, ctypes.c_double),
                                      _lib.ptr(ox, ctypes.c_int32), _lib.ptr(oy, ctypes.c_int32),
                                      _lib.ptr(rows, ctypes.c_int32), _lib.ptr(zf, ctypes.c_double),
                                      _lib.ptr(st, ctypes.c_int32)))
    return ox, oy, rows, zf, st


def _edge_odometry(th, n, seed):
    """Odometry whose per-layer residuals sit on the LUT key boundaries: vtrans chosen
    so that vtrans/0.2 * cos(layer) lands within a few ulps of k/10 and of x.5."""
    rng = np.random.default_rng(seed)
    cos_a, _ = F.layer_trig(th)
    layer = rng.integers(0, th, n)
    c = cos_a[layer]
    c[np.abs(c) < 1e-3] = 1.0
    target = rng.integers(-30, 30, n) + rng.integers(-5, 6, n) / 10.0
    vt = target / c * 0.2
    vt += rng.integers(-4, 5, n) * np.spacing(np.abs(vt) + 1e-300)
    vrot = (rng.integers(-th, th, n) + 0.5) * (2.0 * np.pi / th)
    vrot += rng.integers(-2, 3, n) * np.spacing(np.abs(vrot))
    return np.stack([vt, vrot], axis=1)


@pytest.mark.parametrize('th', [18, 36, 72])
def test_library_control_bit_identical_to_numpy(th):
    """The library-side control (rs_pc_update_odom / rs_pc_run_odom) equals
    filters.step_control bit for bit, including on key and rounding boundaries,
    and reports the reference's KeyError (:249) / out-of-table origins."""
    table = F.FilterTable()
    rng = np.random.default_rng(th)
    live = np.stack([rng.uniform(0, 0.6, 3000), rng.uniform(-0.15, 0.15, 3000)], axis=1)
    wide = np.stack([rng.uniform(-3, 3, 3000), rng.uniform(-7, 7, 3000)], axis=1)
    od = np.concatenate([live, wide, _edge_odometry(th, 6000, th),
                         [[0.0, 0.0], [-0.0, -0.0], [np.nan, 0.0], [0.1, np.nan], [1e300, 0.0],
                          [np.inf, 0.0], [-np.inf, 0.1], [0.3, np.nan], [0.3, np.inf], [0.25, -np.inf]]])
    ox, oy, rows, zf, st = _library_control(th, od)
    from pyratslam_amd import _lib
    n_ok = n_key = n_range = 0
    for i, (vt, vr) in enumerate(od):
        try:
            rx, ry, rr, zz, _ = F.step_control(float(vt), float(vr), th, table)
        except (KeyError, ValueError, OverflowError):
            # KeyError((k, k)) for a key outside the LUT, ValueError for the NaN residual
            # of a non-finite vtrans: the library reports both at the same layer as
            # RS_ERR_LUT_KEY, and the wrapper re-raises the host's exception
            assert st[i] == _lib.RS_ERR_LUT_KEY, (i, vt, vr, st[i])
            n_key += 1
            continue
        if st[i] == _lib.RS_ERR_CTL_RANGE:
            n_range += 1
            o = math.floor(float(vr) / (2.0 * np.pi / th) + .5)
            assert abs(o) > th // 2 + F.ZORIG_MARGIN or abs(float(vt)) / 0.2 >= 2 ** 30
            continue
        assert st[i] == _lib.RS_OK, (i, vt, vr, st[i])
        n_ok += 1
        assert np.array_equal(ox[i], rx) and np.array_equal(oy[i], ry), (i, vt, vr)
        assert np.array_equal(rows[i], rr), (i, vt, vr)
        assert zf[i].tobytes() == zz.tobytes(), (i, vt, vr)
    assert n_ok > 5000 and n_key > 100 and n_range > 0


def test_pinned_pool_reuses_and_caps_blocks():
    """_PinnedArrays (the .posecells readback pool) with a host stand-in for
    rs_host_alloc: freed arrays' blocks are reused, at most CAP exist at once (then
    array() returns None and the caller copies into pageable memory), and close()
    frees the free list and later releases."""
    import ctypes
    import gc
    from pyratslam_amd import _lib
    from pyratslam_amd.posecell_network import _PinnedArrays

    class FakeLib:
        def __init__(self):
            self.live = {}

        def rs_host_alloc(self, nbytes, out):
            buf = ctypes.create_string_buffer(nbytes)
            out._obj.value = ctypes.addressof(buf)
            self.live[ctypes.addressof(buf)] = buf
            return _lib.RS_OK

        def rs_host_free(self, ptr):
            del self.live[ptr.value]
            return _lib.RS_OK

    lib = FakeLib()
    pool = _PinnedArrays(lib, 6, cap=3)
    a, pa = pool.array((2, 3))
    b, pb = pool.array((2, 3))
    assert a.shape == (2, 3) and pa != pb and len(lib.live) == 2
    a[:] = 1.0
    del a
    gc.collect()
    c, pc = pool.array((2, 3))
    assert pc == pa and len(lib.live) == 2        # reused, not a new block
    d, pd = pool.array((2, 3))
    e, pe = pool.array((2, 3))
    assert d is not None and e is None and pe is None and pool._blocks == 3
    del c
    gc.collect()
    pool.close()
    assert len(lib.live) == 2                     # the free block went at close
    del b, d
    gc.collect()
    assert lib.live == {}                         # released after close: freed


@pytest.mark.parametrize('th', [18, 36])
def test_nonfinite_odometry_like_reference(th):
    """posecell_network.py:244-308 under Python 2, the reference's interpreter: a
    non-finite vtrans gives NaN residuals (inf - around(inf) is NaN) and int(NaN)
    raises ValueError at the first layer; a non-finite vrot makes math.floor return
    it unchanged and the theta filter all NaN, with no exception.  No cast warnings."""
    import warnings
    table = F.FilterTable()
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        for vt in (np.nan, np.inf, -np.inf, 1e308):    # 1e308 / 0.2 overflows to inf
            with pytest.raises(ValueError, match='NaN'):
                F.step_control(vt, 0.0, th, table)
            with pytest.raises(ValueError):
                P.step_control(vt, 0.0, (8, 8, th), P.lut_2d())
        with pytest.raises(KeyError) as e:              # a LUT miss at an earlier layer wins
            F.step_control(0.1, np.nan, th, table)
        assert e.value.args[0] == (5, 5)
        for vr in (np.nan, np.inf, -np.inf):
            ox, oy, rows, zf, _ = F.step_control(0.3, vr, th, table)
            assert np.isnan(zf).all() and zf.shape == (7,)
            ref = P.step_control(0.3, vr, (8, 8, th), P.lut_2d())
            assert np.isnan(ref['zf']).all()
            assert np.array_equal(ox, ref['ox']) and np.array_equal(oy, ref['oy'])
        od = np.array([[0.2, 0.0], [0.3, np.nan], [np.inf, 0.0], [0.1, 0.0]])
        ox, oy, rows, zf, first_bad = F.batch_control(od, th, table)
        assert first_bad == 2
        assert np.isnan(zf[1]).all() and np.isfinite(zf[0]).all()
        assert F.batch_control(od[[0, 3]], th, table)[4] == 1          # KeyError step
        assert F.batch_control(od[:2], th, table)[4] is None
        F.step_control(1e12, 0.0, th, table)            # huge finite shifts: no cast warning
