"""The halo form (RS_PC_FORM=halo): one launch per pose-cell step, the excitation
recomputed on each tile's halo and the state carried unnormalised between the
launches of a call (posecell.hip, pc_step_halo / pc_halo_finish).  Checked against
the reference-made golden trajectories and the float64 oracle: float32 activations
within 1e-5 (BASELINE.json north_star), argmax identical at every step, and the
peak returned always the argmax of the handle's own state."""
import ctypes

import numpy as np
import pytest

from conftest import dense_state, load_golden
from oracle import posecell as P

pytestmark = pytest.mark.gpu

F32_TOL = 1e-5


@pytest.fixture(scope='module')
def pcn():
    from pyratslam_amd import _build
    _build.build()
    from pyratslam_amd import PoseCellNetwork
    return PoseCellNetwork


@pytest.fixture
def halo(monkeypatch, pcn):
    monkeypatch.setenv('RS_PC_FORM', 'halo')

    def make(shape, **kw):
        net = pcn(shape, **kw)
        assert net.step_form() == 'halo'
        return net
    return make


def odometry(n, seed, vmax=0.6, rmax=0.15):
    r = np.random.default_rng(seed)
    return np.stack([r.uniform(0, vmax, n), r.uniform(-rmax, rmax, n)], axis=1)


def own_argmax(net):
    p = net.posecells
    return tuple(int(v) for v in np.unravel_index(np.argmax(p), p.shape)), p


@pytest.mark.parametrize('name', ['pc64_s0', 'pc_ros21', 'pc32_s0', 'pc32_s1', 'pc32_s2', 'pc_simulate'])
def test_golden_trajectory_per_step_and_batched(halo, name):
    # (pc32_*: configs[0]'s 32 x 32 x 18; pc_simulate: simulate.py's 50 x 50 x 10 -- the
    # instances whose theta columns are not whole 16-byte pieces)
    case = load_golden(name)
    shape = tuple(int(s) for s in case['shape'])
    net = halo(shape)
    net.inject(1, tuple(case['inject']))
    for s, v in enumerate(case['odom']):
        m = net.update(v)
        assert m == tuple(case['max_pc'][s]), (name, s)
        own, p = own_argmax(net)
        assert own == m, (name, s)
        assert np.abs(p - dense_state(case, s)).max() < F32_TOL, (name, s)
    b = halo(shape)
    b.inject(1, tuple(case['inject']))
    n = len(case['odom'])
    got = np.concatenate([b.run(case['odom'][:n // 3]), b.run(case['odom'][n // 3:])])
    assert np.array_equal(got, case['max_pc'])
    assert np.abs(b.posecells - dense_state(case, n - 1)).max() < F32_TOL


@pytest.mark.parametrize('name', ['pc_death64', 'pc_death32'])
def test_network_death_vs_reference(halo, name):
    """pc_death64 / pc_death32 (made by the reference): the dead steps take the total == 0
    branch and stay exactly zero, the peak of the all-zero volume is (0, 0, 0), a
    second inject revives it; per step and batched around the inject."""
    case = load_golden(name)
    shape = tuple(int(s) for s in case['shape'])
    kill, revive = int(case['kill_step']), int(case['revive_step'])
    odom = case['odom']
    net = halo(shape)
    net.inject(1, tuple(case['inject']))
    for s, v in enumerate(odom):
        if s == revive:
            net.inject(1, tuple(int(c) for c in case['revive']))
        m = net.update(v)
        assert m == tuple(case['max_pc'][s]), (s, m)
        assert net.get_pc_max() == tuple(case['get_pc_max'][s])
        p = net.posecells
        if kill <= s < revive:
            assert not p.any(), s
        assert np.abs(p - dense_state(case, s)).max() < F32_TOL, s
    b = halo(shape)
    b.inject(1, tuple(case['inject']))
    m1 = b.run(odom[:revive])
    b.inject(1, tuple(int(c) for c in case['revive']))
    m2 = b.run(odom[revive:])
    assert np.array_equal(np.concatenate([m1, m2]), case['max_pc'])
    assert np.abs(b.posecells - dense_state(case, len(odom) - 1)).max() < F32_TOL


@pytest.mark.parametrize('shape', [(64, 64, 36), (21, 21, 36), (17, 30, 36), (16, 16, 36), (128, 72, 36),
                                   (32, 32, 18), (50, 50, 10), (18, 30, 18), (17, 28, 10)])
def test_random_and_fast_odometry_vs_oracle(halo, shape):
    """Bench odometry mixed with fast steps (vtrans up to 2 m: shifts up to 10 cells,
    unions beyond the LDS-DMA image, which take the direct-load path), ragged tiles
    (17 x 30), a grid of exactly one window (16 x 16) and one of 576 tiles (more than
    one block per CU and per argmax slot, RS_PC_FORM=halo beyond the default's range);
    run() in batches of 7 so every batch starts from a normalised state and ends in
    pc_halo_finish."""
    r = np.random.default_rng(41)
    n = 28
    od = np.stack([np.where(r.random(n) < 0.6, r.uniform(0, 0.6, n), r.uniform(0.9, 2.0, n)),
                   r.uniform(-0.15, 0.15, n)], axis=1)
    net = halo(shape)
    ref = P.PoseCellOracle(shape)
    loc = tuple(s // 2 for s in shape)
    net.inject(1, loc)
    ref.inject(1, loc)
    got = np.concatenate([net.run(od[i:i + 7]) for i in range(0, n, 7)])
    for s in range(n):
        assert tuple(got[s]) == ref.update(od[s]), (shape, s)
    own, p = own_argmax(net)
    assert own == tuple(got[-1])
    assert np.abs(p - ref.posecells).max() < F32_TOL


def _oracle_step_with_control(ref, ox, oy, rows, zf, table):
    ref.excite_inhibit_normalise()
    filters = np.moveaxis(table[rows], 0, -1)
    p = P.conv_xy_shift(ref.posecells, ox, oy, filters)
    p[p < 0] = 0
    p = P.conv_z_wrap(p, zf)
    p[p < 0] = 0
    ref.posecells = p
    return ref.get_pc_max()


def test_uniform_large_shift_own_tile_outside_union(halo):
    """Every layer shifted by the same 9 cells (explicit control through
    rs_pc_update): the union of the step's windows no longer holds a tile's own
    cells, whose argmax keys then come from memory."""
    shape = (64, 64, 36)
    net = halo(shape)
    ref = P.PoseCellOracle(shape)
    for x in (net, ref):
        x.inject(1, (32, 32, 18))
    table = net._table
    zf = np.ascontiguousarray(P.dog_offset_1d(0), dtype=np.float64)
    for s, (sx, sy) in enumerate([(9, 9), (-9, 5), (9, -12), (0, 0)]):
        ox = np.full(36, sx, dtype=np.int32)
        oy = np.full(36, sy, dtype=np.int32)
        rows = np.full(36, net.filter_table.index[(0, 0)], dtype=np.int32)
        want = _oracle_step_with_control(ref, ox, oy, rows, zf, table)
        st = net._update(net._h, ox.ctypes.data, oy.ctypes.data, rows.ctypes.data, zf.ctypes.data,
                         net._out3_addr)
        assert st == 0
        assert tuple(int(v) for v in net._out3) == want, s
    # the next update() re-reads the state the uniform steps left
    v = (0.3, 0.05)
    assert net.update(v) == ref.update(v)
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


def test_wrapped_union_per_layer_shifts(halo):
    """Per-layer shifts whose spread makes the union span a whole period (16 + spread
    > 21): the 36-layer theta pass then maps window cells to union cells modulo the
    period.  Shifts change from layer to layer (each change reloads a column) and
    wrap in x only, in y only and in both."""
    shape = (21, 21, 36)
    net = halo(shape)
    ref = P.PoseCellOracle(shape)
    for x in (net, ref):
        x.inject(1, (10, 10, 18))
    table = net._table
    zf = np.ascontiguousarray(P.dog_offset_1d(0), dtype=np.float64)
    j = np.arange(36)
    cases = [((j % 7) - 3, 3 - (j * 5) % 9),        # both
             ((j // 4) % 7 - 3, np.full(36, 1)),     # x only
             (np.zeros(36, int), (j * 3) % 8 - 4),   # y only
             ((j % 2) * 8 - 4, (j % 3) * 4 - 4)]     # every layer a new shift
    for s, (sx, sy) in enumerate(cases * 2):
        ox = np.ascontiguousarray(sx, dtype=np.int32)
        oy = np.ascontiguousarray(sy, dtype=np.int32)
        rows = np.full(36, net.filter_table.index[(0, 0)], dtype=np.int32)
        want = _oracle_step_with_control(ref, ox, oy, rows, zf, table)
        st = net._update(net._h, ox.ctypes.data, oy.ctypes.data, rows.ctypes.data, zf.ctypes.data,
                         net._out3_addr)
        assert st == 0
        assert tuple(int(v) for v in net._out3) == want, s
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


def test_poisoned_scratch_first_updates_vs_c_oracle(halo):
    from oracle import c_oracle as C
    from pyratslam_amd import _lib
    shape = (64, 64, 36)
    od = odometry(4, 31)
    ref = C.PoseCellC(shape)
    ref.inject(1, (32, 32, 18))
    want = [ref.update(v) for v in od]
    for batched in (False, True):
        net = halo(shape)
        _lib.check(net._lib.rs_pc_debug(net._h, _lib.RS_PC_DBG_POISON))
        net.inject(1, (32, 32, 18))
        got = [tuple(r) for r in net.run(od)] if batched else [net.update(v) for v in od]
        assert got == want, batched
        p = net.posecells
        assert np.isfinite(p).all()
        assert np.abs(p - ref.posecells).max() < F32_TOL
        net.close()


@pytest.mark.parametrize('shape', [(64, 64, 36), (32, 32, 18), (50, 50, 10)])
def test_keyerror_leaves_reference_state(halo, shape):
    """vtrans 0.1 m = half a cell: the layer at heading 0 has residual +0.5, key 5,
    the reference's KeyError((5, 5)) after steps 1-4 (posecell_network.py:249); the
    excitation-only instance of each theta extent."""
    net = halo(shape)
    loc = tuple(x // 2 for x in shape)
    net.inject(1, loc)
    with pytest.raises(KeyError) as e:
        net.update((0.1, 0.0))
    ref = P.PoseCellOracle(shape)
    ref.inject(1, loc)
    with pytest.raises(KeyError) as e_ref:
        P.PoseCellOracle(shape).update((0.1, 0.0))
    assert e.value.args[0] == e_ref.value.args[0]
    if shape[2] == 36:
        assert e.value.args[0] == (5, 5)
    ref.excite_inhibit_normalise()
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL
    net2 = halo(shape)
    net2.inject(1, loc)
    with pytest.raises(KeyError):
        net2.run([[0.2, 0.0], [0.3, 0.01], [0.1, 0.0]])
    ref2 = P.PoseCellOracle(shape)
    ref2.inject(1, loc)
    ref2.update((0.2, 0.0))
    ref2.update((0.3, 0.01))
    ref2.excite_inhibit_normalise()
    assert np.abs(net2.posecells - ref2.posecells).max() < F32_TOL


def test_long_run_export_and_eager_readback(halo, pcn, monkeypatch):
    """A run() longer than pc_halo_finish exports itself (the separate export kernel
    then returns the keys) equals update() per step, and equals the rows form; the
    eager readback (the float64 volume written by pc_halo_finish) equals the lazy
    one; the export sentinel still fails a step whose key never arrived."""
    from pyratslam_amd import _lib
    shape = (64, 64, 36)
    od = odometry(150, 12)
    a, b = halo(shape), halo(shape, readback='eager')
    for n in (a, b):
        n.inject(1, (32, 32, 18))
    ma = a.run(od)
    for s, v in enumerate(od):
        assert b.update(v) == tuple(ma[s]), s
        if s % 25 == 0:
            assert np.array_equal(b.posecells, b.posecells.copy())
    pa = a.posecells
    assert np.array_equal(b.posecells, pa)
    monkeypatch.setenv('RS_PC_FORM', 'rows')
    c = pcn(shape)
    assert c.step_form() == 'rows'
    c.inject(1, (32, 32, 18))
    assert np.array_equal(c.run(od), ma)
    assert np.abs(c.posecells - pa).max() < 1e-6
    _lib.check(a._lib.rs_pc_debug(a._h, _lib.RS_PC_DBG_SKIP_EXPORT))
    with pytest.raises(_lib.HipLibraryError, match='did not reach'):
        a.update(od[0])
    assert a.update(od[1]) == own_argmax(a)[0]


def test_state_roundtrip_inject_argmax_total(halo):
    shape = (21, 21, 36)
    rng = np.random.default_rng(3)
    net = halo(shape)
    assert (net.posecells == 0).all()
    assert net.get_pc_max() == (0, 0, 0)
    v = rng.random(shape)
    net.posecells = v
    back = net.posecells
    assert np.array_equal(back, v.astype(np.float32).astype(np.float64))
    assert net.get_pc_max() == tuple(np.unravel_index(np.argmax(back), shape))
    net.inject(5.0, (3, 4, 5))
    assert net.get_pc_max() == (3, 4, 5)
    assert abs(net.total() - back.sum() - 5.0) < 1e-6 * back.size
    buf = np.empty(shape)
    from pyratslam_amd import _lib
    _lib.check(net._lib.rs_pc_read(net._h, _lib.ptr(buf, ctypes.c_double)))
    assert buf[3, 4, 5] == pytest.approx(back[3, 4, 5] + 5.0, rel=1e-6)


def test_entry_points_between_updates(halo):
    """inject, get_pc_max, total, the volume read, write and the next update() between
    update() calls see the normalised state the reference's update() leaves."""
    shape = (64, 64, 36)
    od = odometry(6, 8)
    net = halo(shape)
    ref = P.PoseCellOracle(shape)
    for x in (net, ref):
        x.inject(1, (20, 40, 7))
    for v in od[:2]:
        assert net.update(v) == ref.update(v)
    net.inject(0.3, (50, 10, 30))                 # inject into a pending state
    ref.inject(0.3, (50, 10, 30))
    assert net.get_pc_max() == ref.get_pc_max()
    assert abs(net.total() - ref.posecells.sum()) < 1e-4
    for v in od[2:4]:
        assert net.update(v) == ref.update(v)
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL
    v0 = ref.posecells.copy()
    assert net.update(od[4]) == ref.update(od[4])
    net.posecells = v0                            # a write replaces the pending volume
    ref.posecells = v0.copy()
    assert net.update(od[5]) == ref.update(od[5])
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


@pytest.mark.parametrize('case', ['six_layers', 'twins'])
def test_argmax_exact_ties(halo, case):
    """Exact ties in the new state: six identical packets 6 layers apart in one cell
    (without translation the step keeps the 6-fold symmetry: six tied cells in one tile)
    and two identical packets 32 cells apart (ties across blocks); the lowest index
    wins, as numpy's argmax, per call and batched, against the C oracle."""
    from oracle import c_oracle as C
    shape = (64, 64, 36)
    v = np.zeros(shape)
    if case == 'six_layers':
        v[10, 20, 0::6] = 1.0
        od = [(0.0, 0.0), (0.0, 0.1), (0.0, 0.0)]
    else:
        v[10, 20, 5] = v[42, 20, 5] = 1.0
        od = [(0.0, 0.0), (0.4, 0.0), (0.4, 0.0), (0.2, 0.1)]
    ref = C.PoseCellC(shape)
    ref.posecells = v.copy()
    want = [ref.update(o) for o in od]
    for batched in (False, True):
        net = halo(shape)
        net.posecells = v
        got = [tuple(r) for r in net.run(od)] if batched else [net.update(o) for o in od]
        assert got == want, (case, batched, got, want)
        # the tied peaks are within HF_NEAR of each other: each call's last step was
        # keyed by the finishing pass, not from the per-block records
        assert ambig_calls(net) == (1 if batched else len(od)), (case, batched)
        own, p = own_argmax(net)
        assert own == want[-1]
        assert np.abs(p - ref.posecells).max() < F32_TOL


def ambig_calls(net):
    from pyratslam_amd import _lib
    v = ctypes.c_int64(-1)
    _lib.check(net._lib.rs_pc_debug_value(net._h, _lib.RS_PC_DBG_HALO_AMBIG, ctypes.byref(v)))
    return v.value


@pytest.mark.parametrize('shape', [(64, 64, 36), (21, 21, 36), (32, 32, 18), (50, 50, 10)])
def test_unnormalised_call_end_equals_settled(halo, shape):
    """A call leaves the state unnormalised and returns the last step's peak from the
    per-block records of U (pc_halo_export); the next call scales it on load.  Against a
    handle that settles every call (RS_PC_DBG_HALO_SETTLE, the finishing pass): the same
    peaks, bit-identical states (read at every 7th call, which settles), per call and in
    batches of 1..5 steps, and no call needed the finishing pass to break a near-tie."""
    from pyratslam_amd import _lib
    od = odometry(90, 41)
    a, b = halo(shape), halo(shape)
    _lib.check(b._lib.rs_pc_debug(b._h, _lib.RS_PC_DBG_HALO_SETTLE))
    loc = tuple(x // 2 for x in shape)
    for n in (a, b):
        n.inject(1, loc)
    i, k = 0, 0
    while i < len(od):
        m = 1 + k % 5 if k % 2 else 1
        chunk = od[i:i + m]
        if len(chunk) == 1:
            assert a.update(chunk[0]) == b.update(chunk[0]), i
        else:
            assert np.array_equal(a.run(chunk), b.run(chunk)), i
        if k % 7 == 0:
            assert np.array_equal(a.posecells, b.posecells), i
        i += len(chunk)
        k += 1
    assert np.array_equal(a.posecells, b.posecells)
    assert a.get_pc_max() == own_argmax(a)[0]
    assert ambig_calls(a) == 0 and ambig_calls(b) == 0


@pytest.mark.parametrize('shape', [(64, 64, 36), (21, 21, 36), (32, 32, 18), (50, 50, 10)])
def test_read_of_pending_state_settles_in_one_pass(halo, shape):
    """The ROS node's step: update() then a read of the volume.  The read of a state a
    call left unnormalised normalises it and writes the float64 volume in one pass
    (pc_halo_settle_read: the finishing kernel with the volume, its blocks' flags
    polled).  Against a handle that settles every call: bit-identical volumes through
    the pinned read (`.posecells`) and the copying read (rs_pc_read); a second read of
    the now settled state (the export kernel) gives the same bytes; the next update(),
    inject and get_pc_max continue from the settled state."""
    from pyratslam_amd import _lib
    od = odometry(24, 77)
    a, b = halo(shape), halo(shape)
    _lib.check(b._lib.rs_pc_debug(b._h, _lib.RS_PC_DBG_HALO_SETTLE))
    loc = tuple(x // 3 for x in shape)
    for n in (a, b):
        n.inject(1, loc)
    buf = np.empty(shape)
    for i, v in enumerate(od):
        assert a.update(v) == b.update(v), i
        want = b.posecells
        if i % 3 == 2:
            _lib.check(a._lib.rs_pc_read(a._h, _lib.ptr(buf, ctypes.c_double)))
            got = buf.copy()
        else:
            got = a.posecells
        assert np.array_equal(got, want), i
        assert np.array_equal(a.posecells, got), i      # settled: the export kernel
        if i == 10:
            for n in (a, b):
                n.inject(0.25, (1, 2, 3))
            assert a.get_pc_max() == b.get_pc_max()
    assert a.get_pc_max() == own_argmax(a)[0] == own_argmax(b)[0]
    assert ambig_calls(a) == 0


def test_halo_refused_beyond_16bit_union_fields(pcn, monkeypatch):
    """The union's origin and extent travel to the kernel as 16-bit fields
    (make_ctl_halo / hf_pack): a grid with X or Y beyond 32767 is refused by the halo
    form (a silent truncation would load the wrong cells), and the default form for
    such a grid is another one."""
    monkeypatch.setenv('RS_PC_FORM', 'halo')
    for shape in ((32768, 16, 36), (16, 32768, 36)):
        with pytest.raises(ValueError, match='32767'):
            pcn(shape)
    monkeypatch.delenv('RS_PC_FORM')
    assert pcn((16, 32768, 36)).step_form() != 'halo'
