"""Pin the CPU oracle to the reference: every golden vector produced by running
the reference itself (tests/golden/gen_golden.py) must be reproduced exactly."""
import numpy as np
import pytest

from conftest import dense_state, load_golden, nonfinite_state
from oracle import posecell as P
from oracle import view_templates as V

PC_CASES = ['pc32_s0', 'pc32_s1', 'pc32_s2', 'pc_ros21', 'pc_simulate', 'pc_ragged', 'pc64_s0']


def test_kernel_3d_bit_exact():
    k = load_golden('kernels')
    assert np.array_equal(P.dog_kernel_3d(), k['kernel_3d'])
    # posecell_network.py:97-113 known answer
    assert k['kernel_3d'][3, 3, 3] == 0.2610825802870828


def test_kernel_3d_is_rank2_separable():
    ge, gi, s = P.gauss_1d_factors()
    sep = (np.einsum('i,j,k->ijk', ge, ge, ge) - np.einsum('i,j,k->ijk', gi, gi, gi)) / s
    assert np.abs(sep - load_golden('kernels')['kernel_3d']).max() < 1e-15


def test_lut_py2_bit_exact():
    k = load_golden('kernels')
    lut = P.lut_2d()
    assert len(lut) == len(k['lut_keys']) == 100
    for key, f in zip(k['lut_keys'], k['lut_filters']):
        assert np.array_equal(lut[tuple(int(v) for v in key)], f)


def test_filter_1d_bit_exact():
    k = load_golden('kernels')
    for o, f in zip(k['f1d_origins'], k['f1d']):
        assert np.array_equal(P.dog_offset_1d(int(o)), f)
    assert np.array_equal(P.dog_offset_2d((0, 0)), k['f2d_origin0'])


@pytest.mark.parametrize('name', PC_CASES)
def test_posecell_trajectory_bit_exact(name):
    case = load_golden(name)
    net = P.PoseCellOracle(tuple(case['shape']))
    net.inject(1, tuple(case['inject']))
    steps = len(case['odom']) if name != 'pc64_s0' else 4
    for s in range(steps):
        m = net.update(case['odom'][s])
        assert m == tuple(case['max_pc'][s])
        assert np.array_equal(net.posecells, dense_state(case, s)), (name, s)


@pytest.mark.parametrize('name', ['pc_death64', 'pc_death32'])
def test_network_death_bit_exact(name):
    """The reference's network-death regime (posecell_network.py:304-308,343-345):
    a rotation beyond the 7-tap theta window zeroes the volume, the dead steps
    skip the normalisation (total == 0), get_pc_max of zeros is (0, 0, 0), and a
    second inject revives the network."""
    case = load_golden(name)
    net = P.PoseCellOracle(tuple(case['shape']))
    net.inject(1, tuple(case['inject']))
    kill, revive = int(case['kill_step']), int(case['revive_step'])
    for s, v in enumerate(case['odom']):
        if s == revive:
            net.inject(1, tuple(case['revive']))
        m = net.update(v)
        assert m == tuple(case['max_pc'][s]) == tuple(case['get_pc_max'][s]) == net.get_pc_max()
        assert np.array_equal(net.posecells, dense_state(case, s)), (name, s)
        if kill <= s < revive:
            assert not net.posecells.any() and m == (0, 0, 0)


def test_nonfinite_odometry_bit_exact():
    """pc_nonfinite (made by the reference, with Python 2's floor of a non-finite theta
    origin, tests/golden/gen_golden.py): a NaN or -inf vrot leaves an all-NaN volume for
    good with peak (0, 0, 0); a NaN or inf vtrans raises ValueError after steps 1-4 of
    its update, whose state the oracle reproduces bit for bit."""
    case = load_golden('pc_nonfinite')
    shape, loc = tuple(case['shape']), tuple(case['inject'])
    for i, vr in enumerate(case['vrot']):
        net = P.PoseCellOracle(shape)
        net.inject(1, loc)
        for s, v in enumerate(case['vrot_odom_other']):
            m = net.update((v[0], vr) if s == 1 else tuple(v))
            assert m == tuple(case['vrot_max_pc'][i][s]), (i, s)
            assert bool(np.isnan(net.posecells).all()) == bool(case['vrot_all_nan'][i][s]), (i, s)
    for i, vt in enumerate(case['vtrans']):
        net = P.PoseCellOracle(shape)
        net.inject(1, loc)
        assert net.update((0.2, 0.01)) == tuple(case['vtrans_pre_max_pc'][i])
        assert str(case['vtrans_raised'][i]) == 'ValueError'
        with pytest.raises(ValueError):
            net.update((vt, 0.0))
        assert np.array_equal(net.posecells, nonfinite_state(case, i)), i


def test_keyerror_parity():
    case = load_golden('pc_keyerror')
    assert str(case['raised']) == '(5, 5)'
    net = P.PoseCellOracle(tuple(case['shape']))
    net.inject(1, (16, 16, 9))
    with pytest.raises(KeyError) as e:
        net.update(case['odom'][0])
    assert e.value.args[0] == (5, 5)


@pytest.mark.parametrize('i', [0, 1, 2])
def test_vt_pair_scores_bit_exact(i):
    d = load_golden('vt_pairs')
    a, b, s = d[f'u8_{i}_a'], d[f'u8_{i}_b'], d[f'u8_{i}_score']
    for j in range(len(a)):
        assert V.vt_score(a[j], b[j]) == s[j]
        assert V.vt_scores_library(a[j:j + 1], b[j])[0] == s[j]
        assert V.vt_score(a[j].astype(np.float64), b[j].astype(np.float64)) == d[f'f64_{i}_score'][j]


def test_vt_wraps_uint8():
    # wrapped sum 188,233 vs float SAD 124,981 for rng(1) pairs
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (64, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (64, 32), dtype=np.uint8)
    wrapped = V.vt_score(a, b)
    sad = V.vt_score(a.astype(np.int64), b.astype(np.int64))
    assert wrapped != sad and wrapped > sad


@pytest.mark.parametrize('name', ['vt_trace_ros', 'vt_trace_64x32'])
def test_vt_trace_bit_exact(name):
    d = load_golden(name)
    p = d['params']
    o = V.ViewTemplatesOracle((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    assert np.array_equal(o.mask, d['mask'])
    assert o.shape == tuple(d['shape'])
    idx = [o.match_template(q, *pc)[0] for q, pc in zip(d['queries'], d['pcs'])]
    assert np.array_equal(idx, d['index'])
    assert np.array_equal(np.stack(o.templates), d['templates'])
    assert np.array_equal(np.array(o.locations), d['locations'])


def test_c_oracle_matches_reference():
    """The C/OpenMP restatement (oracle/c) is a second checker and the CPU baseline."""
    from oracle import c_oracle as C
    for name in ('pc32_s1', 'pc_ragged', 'pc_simulate'):
        case = load_golden(name)
        net = C.PoseCellC(tuple(case['shape']))
        net.inject(1, tuple(case['inject']))
        for s, v in enumerate(case['odom']):
            assert net.update(v) == tuple(case['max_pc'][s])
            assert np.abs(net.posecells - dense_state(case, s)).max() < 1e-12
    lib = V.synthetic_library(300, seed=3)
    qs, _ = V.synthetic_queries(lib, 40, seed=4)
    sc, ix = C.vt_best(lib, qs)
    for i, q in enumerate(qs):
        ref = V.vt_scores_library(lib, q)
        assert sc[i] == ref.min() and ix[i] == np.argmin(ref)


@pytest.mark.parametrize('tag', ['f64', 'f32'])
@pytest.mark.parametrize('i', [0, 1, 2])
def test_vt_float_pair_scores_bit_exact(tag, i):
    """Float frames (view_templates.py:16-28 without the uint8 wrap): the reference's
    own scores on non-integer float64 / float32 data (tests/golden: float_pairs)."""
    d = load_golden('vt_pairs_float')
    a, b, s = d[f'{tag}_{i}_a'], d[f'{tag}_{i}_b'], d[f'{tag}_{i}_score']
    assert s.dtype == a.dtype
    for j in range(len(a)):
        got = V.vt_score(a[j], b[j])
        assert got == s[j] and np.asarray(got).dtype == s.dtype


def test_vt_float_trace_bit_exact():
    """ViewTemplates.match with float64 frames through the reference's rule (builtin
    min against the threshold, numpy argmin): the oracle replays the golden trace."""
    d = load_golden('vt_pairs_float')
    thr = float(d['trace_threshold'])
    lib = []
    for q, want in zip(d['trace_queries'], d['trace_index']):
        vals = [V.vt_score(t, q) for t in lib]
        if not vals or min(vals) > thr:
            lib.append(q)
            got = len(lib) - 1
        else:
            got = int(np.argmin(vals))
        assert got == want
    assert np.array_equal(np.stack(lib), d['trace_templates'])
