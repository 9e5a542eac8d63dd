"""Pose-cell network on the GPU vs the reference (golden trajectories) and the
oracle.  Tolerance (BASELINE.json north_star): float32 activations within 1e-5
of the float64 reference, argmax identical; float64 path within 1e-12."""
import ctypes

import numpy as np
import pytest

from conftest import dense_state, load_golden
from oracle import posecell as P

pytestmark = pytest.mark.gpu

F32_TOL = 1e-5
F64_TOL = 1e-12
CASES = ['pc32_s0', 'pc32_s1', 'pc32_s2', 'pc_ros21', 'pc_simulate', 'pc_ragged', 'pc64_s0']


@pytest.fixture(scope='module')
def pcn():
    from pyratslam_amd import _build
    _build.build()
    from pyratslam_amd import PoseCellNetwork
    return PoseCellNetwork


def odometry(n, seed, vmax=0.6, rmax=0.15):
    r = np.random.default_rng(seed)
    return np.stack([r.uniform(0, vmax, n), r.uniform(-rmax, rmax, n)], axis=1)


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
@pytest.mark.parametrize('name', CASES)
def test_golden_trajectory(pcn, name, precision, tol):
    case = load_golden(name)
    net = pcn(tuple(case['shape']), precision=precision)
    net.inject(1, tuple(case['inject']))
    worst = 0.0
    for s, v in enumerate(case['odom']):
        m = net.update(v)
        assert m == tuple(case['max_pc'][s]), (name, s)
        assert net.max_pc == m
        worst = max(worst, np.abs(net.posecells - dense_state(case, s)).max())
    assert worst < tol, worst


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
@pytest.mark.parametrize('form', ['rows', 'cols', 'stream', 'tiles'])
@pytest.mark.parametrize('name', ['pc_death64', 'pc_death32'])
def test_network_death_vs_reference(pcn, monkeypatch, name, form, precision, tol):
    """Golden fixture made by the reference (gen_golden.py --only death): a
    rotation beyond the theta window kills the network, the dead steps take the
    total == 0 branch (posecell_network.py:343-345) and must stay exactly zero
    (no NaN from a 0/0), the peak of the all-zero volume is (0, 0, 0) from
    update() and get_pc_max(), and a second inject revives it.  update() per
    step, and run() in two batches around the second inject."""
    monkeypatch.setenv('RS_PC_FORM', form)
    case = load_golden(name)
    shape = tuple(int(s) for s in case['shape'])
    kill, revive = int(case['kill_step']), int(case['revive_step'])
    odom = case['odom']
    net = pcn(shape, precision=precision)
    assert net.step_form() == form
    net.inject(1, tuple(case['inject']))
    for s, v in enumerate(odom):
        if s == revive:
            net.inject(1, tuple(int(c) for c in case['revive']))
        m = net.update(v)
        assert m == tuple(case['max_pc'][s]), (s, m)
        assert net.get_pc_max() == tuple(case['get_pc_max'][s])
        p = net.posecells
        if kill <= s < revive:
            assert not p.any(), s          # exactly zero, not NaN
            net._max_valid = False
            assert net.get_pc_max() == (0, 0, 0)   # argmax of the volume itself
        assert np.abs(p - dense_state(case, s)).max() < tol, s
    b = pcn(shape, precision=precision)
    b.inject(1, tuple(case['inject']))
    m1 = b.run(odom[:revive])
    b.inject(1, tuple(int(c) for c in case['revive']))
    m2 = b.run(odom[revive:])
    assert np.array_equal(np.concatenate([m1, m2]), case['max_pc'])
    assert np.abs(b.posecells - dense_state(case, len(odom) - 1)).max() < tol


def test_reference_attributes(pcn):
    """The reference's public attributes (posecell_network.py:24-48): shape, the zero
    state, the four kernels (three of them unused by the reference too), the scales,
    the 2-D filter LUT and its key precision, bit-identical to the reference-made golden
    values."""
    g = load_golden('kernels')
    net = pcn((21, 21, 36))
    assert net.shape == (21, 21, 36) and (net.posecells == 0).all() and net.max_pc is None
    for name in ('kernel_3d', 'kernel_2d', 'kernel_1d', 'kernel_1d_sep'):
        assert np.array_equal(getattr(net, name), g[name]), name
    assert np.array_equal(net.diff_gaussian(7, 5, 1, 2, order=2), g['kernel_2d'])
    assert np.array_equal(net.diff_gaussian_separable(7, 5, 1, 2), g['kernel_1d_sep'])
    assert net.global_inhibition == 0.2 and net.pc_vtrans_scale == 0.2
    assert net.pc_vrot_scale == 2.0 * np.pi / 36 and net.filter_dict_2d_precision == 10
    keys = [tuple(k) for k in g['lut_keys']]
    assert sorted(net.filter_dict_2d.keys()) == keys
    assert all(np.array_equal(net.filter_dict_2d[k], f) for k, f in zip(keys, g['lut_filters']))
    net.close()


def test_run_equals_repeated_update(pcn):
    # 4,200 steps in one run(): more results than one pass of the export kernel's
    # grid (64 blocks x 64 steps), so its grid-stride loop is exercised
    od = odometry(4200, 11)
    a = pcn((32, 32, 18))
    b = pcn((32, 32, 18))
    a.inject(1, (16, 16, 9))
    b.inject(1, (16, 16, 9))
    maxes = a.run(od)
    for s, v in enumerate(od):
        assert b.update(v) == tuple(maxes[s])
    assert np.array_equal(a.posecells, b.posecells)   # same kernels, deterministic


@pytest.mark.parametrize('shape,steps', [((64, 64, 36), 30), ((48, 40, 20), 30)])
def test_random_odometry_vs_oracle(pcn, shape, steps):
    od = odometry(steps, 5)
    net = pcn(shape)
    ref = P.PoseCellOracle(shape)
    loc = tuple(s // 2 for s in shape)
    net.inject(1, loc)
    ref.inject(1, loc)
    got = net.run(od)
    for s in range(steps):
        assert tuple(got[s]) == ref.update(od[s])
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
def test_mixed_shift_widths_vs_oracle(pcn, precision, tol):
    """Slow steps (|ox| <= 4) mixed with fast ones (vtrans up to 2 m, shifts up
    to 10 cells, beyond the 7-tap window): the path kernel's shifted window
    must follow the oracle step for step."""
    r = np.random.default_rng(21)
    od = np.stack([np.where(r.random(24) < 0.5, r.uniform(0, 0.8, 24), r.uniform(0.9, 2.0, 24)),
                   r.uniform(-0.15, 0.15, 24)], axis=1)
    for shape in ((64, 64, 36), (40, 100, 20)):
        net = pcn(shape, precision=precision)
        ref = P.PoseCellOracle(shape)
        loc = tuple(s // 2 for s in shape)
        net.inject(1, loc)
        ref.inject(1, loc)
        got = net.run(od)
        for s in range(len(od)):
            assert tuple(got[s]) == ref.update(od[s]), (shape, s)
        assert np.abs(net.posecells - ref.posecells).max() < tol


def _own_argmax(net):
    p = net.posecells
    return tuple(int(v) for v in np.unravel_index(np.argmax(p), p.shape)), p


def test_large_grid_full_rollout_vs_c_oracle(pcn):
    """128x128x72 (BASELINE configs[3]): 40 steps of update() against the C/OpenMP
    oracle (float64, the reference's kernels restated), float32 and float64
    handles.  At every step the returned peak equals the oracle's AND the
    argmax of the handle's own state (this separates the fused argmax-key path
    from the state path), the state is finite and non-negative, and the state
    stays within the north_star tolerance of the oracle's."""
    from oracle import c_oracle as C
    shape = (128, 128, 72)
    od = odometry(40, 9)
    a, b = pcn(shape), pcn(shape, precision='float64')
    assert a.step_form() == 'cols'
    ref = C.PoseCellC(shape)
    for n in (a, b, ref):
        n.inject(1, (64, 64, 36))
    for s in range(len(od)):
        m = ref.update(od[s])
        for net, tol in ((a, F32_TOL), (b, F64_TOL)):
            got = net.update(od[s])
            own, p = _own_argmax(net)
            assert got == own, (net.precision, s, got, own)
            assert got == m, (net.precision, s, got, m)
            assert np.isfinite(p).all() and (p >= 0).all()
            err = np.abs(p - ref.posecells).max()
            assert err < tol, (net.precision, s, err)
    # batched form: the same trajectory through run() on fresh handles
    c = pcn(shape)
    c.inject(1, (64, 64, 36))
    ref2 = C.PoseCellC(shape)
    ref2.inject(1, (64, 64, 36))
    mc = c.run(od)
    assert [tuple(r) for r in mc] == [ref2.update(v) for v in od]
    assert np.abs(c.posecells - ref2.posecells).max() < F32_TOL


# every step form on a fresh handle whose scratch is poisoned (rs_pc_debug): a
# step that read an excited cell, a partial sum or an argmax slot it had not
# written in that step would give NaN state or a wrong peak, every time
POISON_CASES = [((128, 128, 72), 'cols'), ((128, 128, 100), 'cols'), ((64, 64, 36), 'rows'),
                ((40, 44, 20), 'tiles'), ((128, 130, 72), 'stream')]


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
@pytest.mark.parametrize('shape,form', POISON_CASES)
def test_poisoned_scratch_first_updates_vs_c_oracle(pcn, monkeypatch, shape, form, precision, tol):
    from oracle import c_oracle as C
    from pyratslam_amd import _lib
    monkeypatch.setenv('RS_PC_FORM', form)
    od = odometry(4, 31)
    loc = tuple(s // 2 for s in shape)
    ref = C.PoseCellC(shape)
    ref.inject(1, loc)
    want = [ref.update(v) for v in od]
    for batched in (False, True):
        net = pcn(shape, precision=precision)
        assert net.step_form() == form
        _lib.check(net._lib.rs_pc_debug(net._h, _lib.RS_PC_DBG_POISON))
        net.inject(1, loc)
        got = [tuple(r) for r in net.run(od)] if batched else [net.update(v) for v in od]
        assert got == want, (shape, form, precision, batched)
        p = net.posecells
        assert np.isfinite(p).all()
        assert np.abs(p - ref.posecells).max() < tol
        net.close()


def test_result_export_sentinel(pcn):
    """A step whose argmax key never reaches the host result word fails loudly
    (rs_pc_debug(RS_PC_DBG_SKIP_EXPORT) withholds the export once); the next
    update is correct."""
    from pyratslam_amd import _lib
    shape = (32, 32, 18)
    net = pcn(shape)
    ref = P.PoseCellOracle(shape)
    for n in (net, ref):
        n.inject(1, (16, 16, 9))
    od = odometry(3, 2)
    _lib.check(net._lib.rs_pc_debug(net._h, _lib.RS_PC_DBG_SKIP_EXPORT))
    with pytest.raises(_lib.HipLibraryError, match='did not reach'):
        net.update(od[0])
    ref.update(od[0])                  # the step itself ran
    assert net.update(od[1]) == ref.update(od[1])
    assert net.run(od[2:]).tolist() == [list(ref.update(od[2]))]
    with pytest.raises(ValueError):
        _lib.check(net._lib.rs_pc_debug(net._h, 99))


@pytest.mark.parametrize('form', ['', 'cols'])   # cols: P theta-fastest, Q layer-major
def test_keyerror_leaves_reference_state(pcn, monkeypatch, form):
    monkeypatch.setenv('RS_PC_FORM', form)
    case = load_golden('pc_keyerror')
    shape = tuple(case['shape'])
    net = pcn(shape, precision='float64')
    assert not form or net.step_form() == form
    net.inject(1, (16, 16, 9))
    with pytest.raises(KeyError) as e:
        net.update(case['odom'][0])
    assert e.value.args[0] == (5, 5)
    ref = P.PoseCellOracle(shape)
    ref.inject(1, (16, 16, 9))
    ref.excite_inhibit_normalise()
    assert np.abs(net.posecells - ref.posecells).max() < F64_TOL
    # batched: steps before the bad one run, then steps 1-4 of it, then KeyError
    net2 = pcn(shape, precision='float64')
    net2.inject(1, (16, 16, 9))
    with pytest.raises(KeyError):
        net2.run([[0.2, 0.0], [0.1, 0.0]])
    ref2 = P.PoseCellOracle(shape)
    ref2.inject(1, (16, 16, 9))
    ref2.update((0.2, 0.0))
    ref2.excite_inhibit_normalise()
    assert np.abs(net2.posecells - ref2.posecells).max() < F64_TOL


def test_keyerror_late_in_a_long_batch(pcn):
    """A batch of 3,000 steps forms its control on several host threads (rs_pc_run_odom,
    one contiguous range of steps each); the LUT KeyError of step 2,500 (pc_keyerror's
    odometry) must stop the batch exactly as in order: steps 0 .. 2,499 run, then steps
    1-4 of the bad one, then KeyError -- the same state as the steps taken one by one."""
    case = load_golden('pc_keyerror')
    shape = tuple(case['shape'])
    od = odometry(3000, 5)
    od[2500] = case['odom'][0]
    a = pcn(shape, precision='float64')
    b = pcn(shape, precision='float64')
    for n in (a, b):
        n.inject(1, (16, 16, 9))
    with pytest.raises(KeyError):
        a.run(od)
    mb = b.run(od[:2500])
    with pytest.raises(KeyError):
        b.update(od[2500])
    assert tuple(mb[-1]) == a.max_pc
    assert np.array_equal(a.posecells, b.posecells)


# the default form at 21x21x36, and the column form (P theta-fastest) at a ragged
# grid whose theta extent is not a multiple of the 16-byte groups
@pytest.mark.parametrize('form,shape', [('', (21, 21, 36)), ('cols', (24, 40, 13)), ('cols', (32, 32, 20))])
def test_state_roundtrip_inject_and_argmax(pcn, monkeypatch, form, shape):
    monkeypatch.setenv('RS_PC_FORM', form)
    rng = np.random.default_rng(3)
    for precision in ('float32', 'float64'):
        net = pcn(shape, precision=precision)
        assert not form or net.step_form() == form
        assert (net.posecells == 0).all()
        assert net.get_pc_max() == (0, 0, 0)          # argmax of zeros = first cell
        v = rng.random(shape)
        net.posecells = v
        back = net.posecells
        if precision == 'float64':
            assert np.array_equal(back, v)
        else:
            assert np.array_equal(back, v.astype(np.float32).astype(np.float64))
        assert net.get_pc_max() == tuple(np.unravel_index(np.argmax(back), shape))
        net.inject(5.0, (3, 4, 5))
        assert net.get_pc_max() == (3, 4, 5)
        assert abs(net.total() - back.sum() - 5.0) < 1e-6 * back.size
        net.inject(1.0, (-1, -1, -1))                 # numpy negative indexing
        assert net.posecells[-1, -1, -1] == pytest.approx(back[-1, -1, -1] + 1.0, rel=1e-6)


def test_argmax_first_maximum_tie_break(pcn):
    shape = (8, 8, 8)
    net = pcn(shape, precision='float64')
    v = np.zeros(shape)
    v[5, 1, 2] = v[2, 7, 7] = v[2, 7, 1] = 1.0
    net.posecells = v
    assert net.get_pc_max() == (2, 7, 1)


def test_bad_inputs_raise(pcn):
    with pytest.raises(ValueError):
        pcn((2, 8, 8))
    net = pcn((8, 8, 8))
    with pytest.raises(TypeError):
        net.posecells = np.zeros((8, 8, 7))
    with pytest.raises(TypeError):
        net.inject(1, [1, 2, 3])
    with pytest.raises(IndexError):
        net.inject(1, (8, 0, 0))


def test_simulate_driver(pcn):
    """simulate.py:36-41 scenario through the headless driver."""
    from pyratslam_amd.simulate import RatSLAM, scenario
    case = load_golden('pc_simulate')
    sim = RatSLAM(data=scenario(), shape=(50, 50, 10))
    for s in range(40):
        sim.step()
        assert sim.current_pose_cell == tuple(case['max_pc'][s])


# every step-kernel form (RS_PC_FORM) against the oracle: the row-tiled and 3-D
# tiled single-pass forms, the column form and the layer-streaming form at several tile shapes
# (rows per wave, row groups, layers per block), incl. ragged tiles and grids
# whose theta extent is not a multiple of the chunk
FORMS = {'float32': ['rows', 'tiles', 'cols', 'cols:5', 'cols:12', 'stream:1,8,1,2', 'stream:1,8,1,5',
                     'stream:2,8,1,3', 'stream:2,8,1,6'],
         'float64': ['rows', 'tiles', 'cols', 'cols:7', 'stream:1,8,1,2', 'stream:1,8,1,5']}


def cols_fit(shape, precision, form='cols'):
    """The column form's limits (posecell.hip pc_cols_fit / pc_cols_set): 16-byte
    row vectors (Y a multiple of 4 cells at float32, 2 at float64), single-wrap
    halos, and the window layers in LDS (whole extent, or KC + 6 per chunk)."""
    X, Y, TH = shape
    vec, whole, chunk = (4, 76, 43) if precision == 'float32' else (2, 40, 21)
    kc = int(form.split(':')[1]) if ':' in form else (TH if TH <= whole else 0)
    if not (X >= 14 and Y >= 18 and Y % vec == 0 and TH >= 10):
        return False
    if kc == 0:
        return True                     # chunked automatically
    kc = min(kc, TH) if ':' not in form else kc
    return kc <= TH and (kc + 6 <= chunk if kc < TH else TH <= whole)


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
def test_step_forms_agree_with_oracle(pcn, monkeypatch, precision, tol):
    od = odometry(10, 17)
    for shape in ((64, 64, 36), (21, 21, 36), (24, 40, 13), (70, 100, 20)):
        loc = tuple(s // 2 for s in shape)
        ref = P.PoseCellOracle(shape)
        ref.inject(1, loc)
        maxes = [ref.update(v) for v in od]
        want = ref.posecells
        for form in FORMS[precision]:
            monkeypatch.setenv('RS_PC_FORM', form)
            if form.startswith('cols') and not cols_fit(shape, precision, form):
                with pytest.raises(ValueError):
                    pcn(shape, precision=precision)
                continue
            net = pcn(shape, precision=precision)
            assert net.step_form() == form.split(':')[0], form
            net.inject(1, loc)
            got = net.run(od)
            assert [tuple(m) for m in got] == maxes, (shape, form)
            assert np.abs(net.posecells - want).max() < tol, (shape, form)
            net.close()


def test_default_form_by_grid_size(pcn, monkeypatch):
    monkeypatch.delenv('RS_PC_FORM', raising=False)
    assert pcn((64, 64, 36)).step_form() == 'halo'       # float32, TH = 36, <= 256 tiles
    assert pcn((21, 21, 36)).step_form() == 'halo'
    assert pcn((64, 64, 36), precision='float64').step_form() == 'rows'
    assert pcn((68, 64, 36)).step_form() == 'rows'       # 17 x 16 tiles: more than one per CU
    assert pcn((32, 32, 18)).step_form() == 'halo'       # configs[0]'s grid: TH = 18
    assert pcn((50, 50, 10)).step_form() == 'halo'       # simulate.py's grid: TH = 10
    assert pcn((21, 21, 18)).step_form() != 'halo'       # X * Y * TH not a multiple of 4
    assert pcn((32, 32, 20)).step_form() != 'halo'       # no halo instance for TH = 20
    assert pcn((128, 128, 72)).step_form() == 'cols'
    assert pcn((128, 130, 72)).step_form() == 'stream'    # Y not a multiple of 4: no cols
    assert pcn((128, 128, 100)).step_form() == 'cols'     # theta extent beyond one block: chunked
    monkeypatch.setenv('RS_PC_FORM', 'stream:3,8,1')
    with pytest.raises(ValueError):
        pcn((64, 64, 36))
    monkeypatch.setenv('RS_PC_FORM', 'stream:2,8,1,3')   # spills at float64: refused
    with pytest.raises(ValueError):
        pcn((64, 64, 36), precision='float64')


@pytest.mark.parametrize('shape', [(32, 32, 18), (64, 64, 36)])
def test_library_control_matches_host_control(pcn, shape):
    """update()/run() take the odometry through rs_pc_update_odom / rs_pc_run_odom;
    the state must be bit-identical to the NumPy-control path (rs_pc_update /
    rs_pc_run), including odometry outside the library's tables (host fallback)."""
    od = odometry(60, 11, vmax=1.2, rmax=0.4)
    od[20] = (0.3, 6.0)      # theta origin outside the tables -> host control
    od[40] = (0.25, -6.5)
    a, b, c, d = (pcn(shape) for _ in range(4))
    for n in (a, b, c, d):
        n.inject(1, (shape[0] // 2, shape[1] // 2, shape[2] // 2))
    ma = [a.update(v) for v in od]
    mb = [b._update_host_control(float(v[0]), float(v[1])) for v in od]
    mc = c.run(od)
    md = d._run_host_control(np.ascontiguousarray(od))
    assert ma == mb
    assert np.array_equal(mc, md) and [tuple(r) for r in mc] == ma
    pa = a.posecells
    for n in (b, c, d):
        assert n.posecells.tobytes() == pa.tobytes()
    # a batch that needs the host fallback as a whole (step 20 is outside the tables)
    e, f = pcn(shape), pcn(shape)
    for n in (e, f):
        n.inject(1, (shape[0] // 2, shape[1] // 2, shape[2] // 2))
    assert np.array_equal(e.run(od[15:25]), f._run_host_control(np.ascontiguousarray(od[15:25])))
    assert e.posecells.tobytes() == f.posecells.tobytes()
    assert e.run(np.zeros((0, 2))).shape == (0, 3)


@pytest.mark.parametrize('precision', ['float32', 'float64'])
def test_posecells_pinned_readback_arrays_are_independent(pcn, precision):
    """.posecells is written by the GPU straight into a pinned host array
    (rs_pc_read_pinned): each read returns its own array, equal to the copying
    readback (rs_pc_read), unchanged by later steps and reads, across pool reuse
    and an odd cell count."""
    import ctypes
    from pyratslam_amd import _lib
    for shape in ((32, 32, 18), (13, 11, 7)):
        net = pcn(shape, precision=precision)
        ref = P.PoseCellOracle(shape)
        loc = tuple(s // 2 for s in shape)
        net.inject(1, loc)
        ref.inject(1, loc)
        od = odometry(12, 7)
        kept = []
        for s, v in enumerate(od):
            net.update(v)
            ref.update(v)
            a = net.posecells
            b = np.empty(shape, dtype=np.float64)
            _lib.check(net._lib.rs_pc_read(net._h, _lib.ptr(b, ctypes.c_double)))
            assert a.dtype == np.float64 and a.shape == shape and a.flags.c_contiguous
            assert np.array_equal(a, b)
            tol = F32_TOL if precision == 'float32' else F64_TOL
            assert np.abs(a - ref.posecells).max() < tol
            if s % 3 == 0:
                kept.append((a, a.copy()))      # held across later steps
            del a                               # the others go back to the pool
        for a, snap in kept:
            assert np.array_equal(a, snap)
        net.close()
        for a, snap in kept:                    # arrays outlive their network
            assert np.array_equal(a, snap)


@pytest.mark.parametrize('readback', ['lazy', 'eager'])
def test_posecells_kept_history_bounds_pinned_pool(pcn, readback):
    """A caller that keeps every volume (a history list) holds the pinned pool's
    blocks; past _PinnedArrays.CAP reads fall back to pageable copies and stay
    correct, and pinned host memory stays bounded."""
    from pyratslam_amd.posecell_network import _PinnedArrays
    shape = (32, 32, 18)
    net = pcn(shape, readback=readback)
    ref = P.PoseCellOracle(shape)
    net.inject(1, (16, 16, 9))
    ref.inject(1, (16, 16, 9))
    hist, want = [], []
    for v in odometry(3 * _PinnedArrays.CAP, 11):
        net.update(v)
        ref.update(v)
        hist.append(net.posecells)
        want.append(ref.posecells.copy())
    assert net._pinned._blocks <= _PinnedArrays.CAP
    for a, b in zip(hist, want):
        assert np.abs(a - b).max() < F32_TOL
    assert len({a.ctypes.data for a in hist}) == len(hist)
    del hist
    v = odometry(1, 12)[0]
    net.update(v)
    ref.update(v)
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL
    net.close()


def test_eager_readback_equals_lazy(pcn):
    """readback='eager': update() exports the new volume before its one sync and the
    next .posecells returns it; identical to the lazy readback after every update,
    after inject (the export is invalidated), after run() and with repeated reads."""
    shape = (32, 32, 18)
    a, b = pcn(shape), pcn(shape, readback='eager')
    for n in (a, b):
        n.inject(1, (16, 16, 9))
    od = odometry(20, 13)
    for s, v in enumerate(od[:12]):
        assert a.update(v) == b.update(v)
        pb = b.posecells
        assert np.array_equal(a.posecells, pb)
        assert np.array_equal(b.posecells, pb)        # a second read: a fresh export
        if s == 5:
            for n in (a, b):
                n.inject(0.5, (3, 4, 5))
            assert np.array_equal(a.posecells, b.posecells)
    b.update(od[12])
    a.update(od[12])
    assert np.array_equal(a.run(od[13:]), b.run(od[13:]))
    assert np.array_equal(a.posecells, b.posecells)  # run() invalidated the export
    with pytest.raises(ValueError):
        pcn(shape, readback='sometimes')


@pytest.mark.parametrize('shape,precision', [((21, 21, 35), 'float32'), ((21, 21, 35), 'float64'),
                                             ((50, 50, 10), 'float32'), ((128, 128, 72), 'float32')])
def test_volume_reads_vs_c_oracle(pcn, shape, precision):
    """Every way the volume reaches the host -- the pinned read (`.posecells`), the
    copying rs_pc_read and the eager readback -- against the C oracle, on an odd-sized
    volume (the export's lone last cell), the simulate grid and the column form's
    128x128x72 (a capped export grid: several 16-byte pieces per thread).  The export
    kernel's blocks' flags are polled by the host (pc_read_volume)."""
    from oracle import c_oracle as C
    from pyratslam_amd import _lib
    tol = F32_TOL if precision == 'float32' else F64_TOL
    a, b = pcn(shape, precision=precision), pcn(shape, precision=precision, readback='eager')
    ref = C.PoseCellC(shape)
    loc = tuple(x // 2 for x in shape)
    for n in (a, b, ref):
        n.inject(1, loc)
    buf = np.empty(shape)
    for v in odometry(4, 31):
        want = ref.update(v)
        assert a.update(v) == want and b.update(v) == want
        assert np.abs(b.posecells - ref.posecells).max() < tol
        assert np.abs(a.posecells - ref.posecells).max() < tol
        _lib.check(a._lib.rs_pc_read(a._h, _lib.ptr(buf, ctypes.c_double)))
        assert np.array_equal(buf, a.posecells)
    a.close()
    b.close()


@pytest.mark.parametrize('precision,tol', [('float32', F32_TOL), ('float64', F64_TOL)])
def test_large_grid_wide_shifts_vs_c_oracle(pcn, precision, tol):
    """128x128x72 (the column form's TH = 72 instances): steps whose shifted windows'
    union fits the LDS-DMA image (|shift| <= 3) mixed with fast ones (vtrans up to
    2 m: shifts up to 10 cells, the per-layer-window fallback), and a step that
    turns the heading by more than a layer, against the C oracle step by step."""
    from oracle import c_oracle as C
    shape = (128, 128, 72)
    r = np.random.default_rng(23)
    n = 12
    od = np.stack([np.where(r.random(n) < 0.5, r.uniform(0, 0.6, n), r.uniform(0.9, 2.0, n)),
                   r.uniform(-0.15, 0.15, n)], axis=1)
    od[5, 1] = 0.2
    net = pcn(shape, precision=precision)
    assert net.step_form() == 'cols'
    ref = C.PoseCellC(shape)
    for x in (net, ref):
        x.inject(1, (64, 64, 36))
    for s, v in enumerate(od):
        m = ref.update(v)
        assert net.update(v) == m, (s, v)
    assert np.abs(net.posecells - ref.posecells).max() < tol


@pytest.mark.parametrize('form,precision', [('', 'float32'), ('', 'float64'), ('cols', 'float32')])
def test_nonfinite_odometry_vs_reference_fixture(pcn, monkeypatch, form, precision):
    """pc_nonfinite, made by the reference itself (tests/golden/gen_golden.py): NaN / -inf
    vrot leaves an all-NaN volume for good, peak (0, 0, 0) per step; NaN / inf vtrans
    raises ValueError after steps 1-4, whose state matches the reference's (32 x 32 x 18:
    the halo form by default since round 6, rows at float64, the column form)."""
    from conftest import nonfinite_state
    monkeypatch.setenv('RS_PC_FORM', form)
    case = load_golden('pc_nonfinite')
    shape, loc = tuple(int(x) for x in case['shape']), tuple(int(x) for x in case['inject'])
    tol = F32_TOL if precision == 'float32' else F64_TOL
    for i, vr in enumerate(case['vrot']):
        net = pcn(shape, precision=precision)
        assert not form or net.step_form() == form
        net.inject(1, loc)
        for st, v in enumerate(case['vrot_odom_other']):
            m = net.update((v[0], vr) if st == 1 else tuple(v))
            assert m == tuple(case['vrot_max_pc'][i][st]), (i, st)
            assert bool(np.isnan(net.posecells).all()) == bool(case['vrot_all_nan'][i][st]), (i, st)
    for i, vt in enumerate(case['vtrans']):
        net = pcn(shape, precision=precision)
        net.inject(1, loc)
        assert net.update((0.2, 0.01)) == tuple(case['vtrans_pre_max_pc'][i])
        with pytest.raises(ValueError):
            net.update((vt, 0.0))
        assert np.abs(net.posecells - nonfinite_state(case, i)).max() < tol, i


@pytest.mark.parametrize('form,precision', [('', 'float32'), ('', 'float64'), ('halo', 'float32'),
                                            ('cols', 'float32')])
def test_nonfinite_odometry_like_reference(pcn, monkeypatch, form, precision):
    """posecell_network.py:244-310 under Python 2: a NaN or infinite vtrans raises
    ValueError at the LUT lookup (int() of the NaN residual inf - around(inf)) after
    steps 1-4 ran, per call and at the first bad step of run(); a NaN or infinite vrot
    raises nothing (Python 2's math.floor returns it) and the all-NaN theta filter
    leaves a NaN volume whose peak, numpy's first NaN, is (0, 0, 0), for good."""
    monkeypatch.setenv('RS_PC_FORM', form)
    shape = (64, 64, 36)
    tol = F32_TOL if precision == 'float32' else F64_TOL
    loc = (32, 32, 18)
    for vt in (np.nan, np.inf):
        net, ref = pcn(shape, precision=precision), P.PoseCellOracle(shape)
        assert not form or net.step_form() == form
        for x in (net, ref):
            x.inject(1, loc)
        assert net.update((0.2, 0.01)) == ref.update((0.2, 0.01))
        with pytest.raises(ValueError):
            net.update((vt, 0.0))
        ref.excite_inhibit_normalise()
        assert np.abs(net.posecells - ref.posecells).max() < tol
        b, rb = pcn(shape, precision=precision), P.PoseCellOracle(shape)
        for x in (b, rb):
            x.inject(1, loc)
        with pytest.raises(ValueError):
            b.run([[0.2, 0.01], [0.3, 0.0], [vt, 0.0], [0.2, 0.0]])
        rb.update((0.2, 0.01))
        rb.update((0.3, 0.0))
        rb.excite_inhibit_normalise()
        assert np.abs(b.posecells - rb.posecells).max() < tol
    for vr in (np.nan, -np.inf):
        net, ref = pcn(shape, precision=precision), P.PoseCellOracle(shape)
        for x in (net, ref):
            x.inject(1, loc)
        assert net.update((0.3, vr)) == ref.update((0.3, vr)) == (0, 0, 0)
        assert np.isnan(net.posecells).all() and np.isnan(ref.posecells).all()
        assert net.get_pc_max() == (0, 0, 0)
        assert [tuple(m) for m in net.run([[0.2, 0.0], [0.25, 0.3]])] == [(0, 0, 0)] * 2
        assert np.isnan(net.posecells).all()
