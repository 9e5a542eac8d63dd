"""The theta-chunked column form (RS_PC_FORM=tc:G,NW; posecell.hip pc_excite_tc /
pc_path_tc) against the oracles: the reference-made golden fixtures, the NumPy oracle
and the C/OpenMP oracle (the reference's kernels restated).  Float32 activations within
the north_star 1e-5 of the float64 reference, argmax identical at every step."""
import numpy as np
import pytest

from conftest import dense_state, load_golden
from oracle import posecell as P

pytestmark = pytest.mark.gpu

F32_TOL = 1e-5
VARIANTS = ['tc:12,4', 'tc:24,4', 'tc:24,8', 'tc:36,4', 'tc:36,8', 'tc:24,4,1', 'tc:36,8,1']


@pytest.fixture(scope='module')
def pcn():
    from pyratslam_amd import _build
    _build.build()
    from pyratslam_amd import PoseCellNetwork
    return PoseCellNetwork


def odometry(n, seed, vmax=0.6, rmax=0.15):
    r = np.random.default_rng(seed)
    return np.stack([r.uniform(0, vmax, n), r.uniform(-rmax, rmax, n)], axis=1)


def fits(shape, form):
    X, Y, TH = shape
    parts = [int(p) for p in form.split(':')[1].split(',')]
    G = parts[0]
    cols_exc = len(parts) > 2 and parts[2] == 1        # the cols excitation: TH == 72 only
    return (X % 8 == 0 and Y % 8 == 0 and X >= 20 and Y >= 20 and TH % G == 0 and TH // G <= 18 and
            (not cols_exc or TH == 72))


@pytest.mark.parametrize('form', VARIANTS)
def test_golden_64(pcn, monkeypatch, form):
    """The reference's own 64x64x36 trajectory (gen_golden.py), per call."""
    monkeypatch.setenv('RS_PC_FORM', form)
    case = load_golden('pc64_s0')
    shape = tuple(case['shape'])
    if not fits(shape, form):
        with pytest.raises(ValueError):
            pcn(shape)
        return
    net = pcn(shape)
    assert net.step_form() == 'tc'
    net.inject(1, tuple(case['inject']))
    worst = 0.0
    for s, v in enumerate(case['odom']):
        assert net.update(v) == tuple(case['max_pc'][s]), (form, s)
        worst = max(worst, np.abs(net.posecells - dense_state(case, s)).max())
    assert worst < F32_TOL, worst


@pytest.mark.parametrize('name', ['pc_death64'])
def test_network_death_vs_reference(pcn, monkeypatch, name):
    """Reference-made death fixture: the dead steps take the total == 0 branch and
    stay exactly zero, the peak of the zero volume is (0, 0, 0), a second inject
    revives it; per call and batched."""
    monkeypatch.setenv('RS_PC_FORM', 'tc:12,4')
    case = load_golden(name)
    shape = tuple(int(s) for s in case['shape'])
    kill, revive = int(case['kill_step']), int(case['revive_step'])
    odom = case['odom']
    net = pcn(shape)
    assert net.step_form() == 'tc'
    net.inject(1, tuple(case['inject']))
    for s, v in enumerate(odom):
        if s == revive:
            net.inject(1, tuple(int(c) for c in case['revive']))
        assert net.update(v) == tuple(case['max_pc'][s]), s
        p = net.posecells
        if kill <= s < revive:
            assert not p.any(), s
        assert np.abs(p - dense_state(case, s)).max() < F32_TOL, s
    b = pcn(shape)
    b.inject(1, tuple(case['inject']))
    m1 = b.run(odom[:revive])
    b.inject(1, tuple(int(c) for c in case['revive']))
    m2 = b.run(odom[revive:])
    assert np.array_equal(np.concatenate([m1, m2]), case['max_pc'])


@pytest.mark.parametrize('form', VARIANTS)
def test_large_grid_rollout_vs_c_oracle(pcn, monkeypatch, form):
    """BASELINE configs[3], 128x128x72: 24 steps per call against the C oracle, the
    returned peak equal to the oracle's and to the argmax of the handle's own state
    at every step; then the same trajectory batched on a fresh handle."""
    from oracle import c_oracle as C
    monkeypatch.setenv('RS_PC_FORM', form)
    shape = (128, 128, 72)
    od = odometry(24, 9)
    net = pcn(shape)
    assert net.step_form() == 'tc'
    ref = C.PoseCellC(shape)
    for n in (net, ref):
        n.inject(1, (64, 64, 36))
    for s in range(len(od)):
        m = ref.update(od[s])
        got = net.update(od[s])
        p = net.posecells
        own = tuple(int(v) for v in np.unravel_index(np.argmax(p), p.shape))
        assert got == own == m, (form, s, got, own, m)
        assert np.isfinite(p).all() and (p >= 0).all()
        assert np.abs(p - ref.posecells).max() < F32_TOL, (form, s)
    c = pcn(shape)
    c.inject(1, (64, 64, 36))
    ref2 = C.PoseCellC(shape)
    ref2.inject(1, (64, 64, 36))
    mc = c.run(od)
    assert [tuple(r) for r in mc] == [ref2.update(v) for v in od]
    assert np.abs(c.posecells - ref2.posecells).max() < F32_TOL


@pytest.mark.parametrize('shape', [(40, 48, 36), (24, 32, 24), (64, 40, 72)])
def test_shapes_vs_oracle(pcn, monkeypatch, shape):
    """Non-square grids, several chunk counts (TH / G = 1 .. 6), batched."""
    od = odometry(12, 17)
    loc = tuple(s // 2 for s in shape)
    ref = P.PoseCellOracle(shape)
    ref.inject(1, loc)
    want = [ref.update(v) for v in od]
    for form in VARIANTS:
        monkeypatch.setenv('RS_PC_FORM', form)
        if not fits(shape, form):
            with pytest.raises(ValueError):
                pcn(shape)
            continue
        net = pcn(shape)
        net.inject(1, loc)
        got = net.run(od)
        assert [tuple(m) for m in got] == want, (shape, form)
        assert np.abs(net.posecells - ref.posecells).max() < F32_TOL, (shape, form)
        net.close()


@pytest.mark.parametrize('form', ['tc:12,4', 'tc:24,8'])
def test_wide_shifts_fallback_vs_c_oracle(pcn, monkeypatch, form):
    """Fast translations (vtrans up to 2.4 m = 12 cells per step): chunks whose layers'
    shifts spread beyond the LDS union (6 cells) read their windows from memory."""
    from oracle import c_oracle as C
    monkeypatch.setenv('RS_PC_FORM', form)
    shape = (128, 128, 72)
    r = np.random.default_rng(23)
    od = np.stack([np.where(r.random(12) < 0.5, r.uniform(0, 0.6, 12), r.uniform(1.2, 2.4, 12)),
                   r.uniform(-0.15, 0.15, 12)], axis=1)
    net = pcn(shape)
    ref = C.PoseCellC(shape)
    for n in (net, ref):
        n.inject(1, (64, 64, 36))
    got = net.run(od)
    assert [tuple(m) for m in got] == [ref.update(v) for v in od]
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


def test_poisoned_scratch_and_keyerror(pcn, monkeypatch):
    """Scratch filled with all-ones bits before the first steps (a read of anything a
    step did not write gives NaN or a wrong peak); then the KeyError path, which runs
    the excitation-only step as the reference does before raising."""
    from oracle import c_oracle as C
    from pyratslam_amd import _lib
    monkeypatch.setenv('RS_PC_FORM', 'tc:24,4')
    shape = (128, 128, 72)
    od = odometry(4, 31)
    ref = C.PoseCellC(shape)
    ref.inject(1, (64, 64, 36))
    want = [ref.update(v) for v in od]
    for batched in (False, True):
        net = pcn(shape)
        _lib.check(net._lib.rs_pc_debug(net._h, _lib.RS_PC_DBG_POISON))
        net.inject(1, (64, 64, 36))
        got = [tuple(r) for r in net.run(od)] if batched else [net.update(v) for v in od]
        assert got == want, batched
        assert np.abs(net.posecells - ref.posecells).max() < F32_TOL
        net.close()
    net = pcn((64, 64, 72))
    ref = P.PoseCellOracle((64, 64, 72))
    for n in (net, ref):
        n.inject(1, (16, 16, 9))
    # a +0.5-cell residual on layer 0: vtrans = 0.5 cell * 0.2 m
    with pytest.raises(KeyError):
        net.update((0.1, 0.0))
    ref.excite_inhibit_normalise()
    assert np.abs(net.posecells - ref.posecells).max() < F32_TOL


def test_roundtrip_inject_argmax(pcn, monkeypatch):
    monkeypatch.setenv('RS_PC_FORM', 'tc:24,4')
    shape = (32, 40, 48)
    net = pcn(shape)
    rng = np.random.default_rng(5)
    v = rng.random(shape)
    net.posecells = v
    back = net.posecells
    assert np.array_equal(back, v.astype(np.float32).astype(np.float64))
    assert net.get_pc_max() == tuple(np.unravel_index(np.argmax(back), shape))
    net.inject(5.0, (3, 4, 5))
    assert net.get_pc_max() == (3, 4, 5)
