"""View-template matcher on the GPU: bit-exact scores and template indices vs the
reference's golden vectors and the oracle (integer work -> exact equality)."""
import functools

import numpy as np
import pytest

from conftest import load_golden
from oracle import view_templates as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def vtmod():
    from pyratslam_amd import _build
    _build.build()
    import pyratslam_amd.view_templates as m
    return m


def image_from_template(mask, template):
    im = np.zeros(mask.shape, dtype=np.uint8)
    im[mask] = template.ravel()
    return im


@pytest.mark.parametrize('i', [0, 1, 2])
def test_pair_scores_bit_exact(vtmod, i):
    d = load_golden('vt_pairs')
    a, b, s = d[f'u8_{i}_a'], d[f'u8_{i}_b'], d[f'u8_{i}_score']
    lib = vtmod.ViewTemplates._from_shape(a.shape[1:], 45000)
    lib.add(a)
    sc = lib.scores(b)                        # (query, template)
    assert np.array_equal(np.diagonal(sc), s)
    # ViewTemplate.match on owned templates
    assert lib.templates[3].match(b[3]) == s[3]


@pytest.mark.parametrize('name', ['vt_trace_ros', 'vt_trace_64x32'])
def test_trace_via_match(vtmod, name):
    d = load_golden(name)
    p = [int(v) for v in d['params']]
    vts = vtmod.ViewTemplates((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    assert np.array_equal(vts.mask, d['mask'])
    for q, pc, idx, cnt in zip(d['queries'], d['pcs'], d['index'], d['count']):
        t = vts.match(image_from_template(vts.mask, q), *pc)
        assert t.get_index() == idx
        assert len(vts.templates) == cnt
    assert np.array_equal(np.stack([t.template for t in vts.templates]), d['templates'])
    assert np.array_equal(np.array([t.location() for t in vts.templates]), d['locations'])


@pytest.mark.parametrize('name', ['vt_trace_ros', 'vt_trace_64x32'])
def test_trace_via_match_batch(vtmod, name):
    d = load_golden(name)
    p = [int(v) for v in d['params']]
    vts = vtmod.ViewTemplates((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    half = len(d['queries']) // 2
    idx1, _, _ = vts.match_templates(d['queries'][:half], d['pcs'][:half])
    idx2, _, _ = vts.match_templates(d['queries'][half:], d['pcs'][half:])
    assert np.array_equal(np.concatenate([idx1, idx2]), d['index'])
    assert np.array_equal(np.stack([t.template for t in vts.templates]), d['templates'])
    for i in (0, len(vts.templates) - 1):
        assert vts.templates[i].location() == tuple(d['locations'][i])


@pytest.mark.parametrize('t,q,h,w', [(1000, 256, 64, 32), (130, 40, 32, 32), (3000, 7, 64, 32),
                                     (200, 33, 24, 20), (70, 9, 17, 5)])
def test_frozen_scan_vs_oracle(vtmod, t, q, h, w):
    lib_np = V.synthetic_library(t, h, w, seed=t)
    queries, src = V.synthetic_queries(lib_np, q, seed=q)
    lib = vtmod.ViewTemplates._from_shape((h, w), 45000)
    lib.add(lib_np)
    idx, score, new = lib.match_templates(queries, mode=0)
    assert not new.any()
    for i in range(q):
        ref = V.vt_scores_library(lib_np, queries[i])
        assert score[i] == ref.min(), i
        assert idx[i] == int(np.argmin(ref)), i
    assert len(lib.templates) == t


@pytest.mark.parametrize('scan', ['plane', 'carry'])
@pytest.mark.parametrize('h', [64, 32])
def test_scan_variants_vs_oracle(vtmod, monkeypatch, scan, h):
    """Both scan forms (RS_VT_SCAN; 'plane' is the default bit-plane scan) give
    the oracle's scores on the same inputs, including all-0 / all-255 extremes."""
    monkeypatch.setenv('RS_VT_SCAN', scan)
    rng = np.random.default_rng(h)
    lib_np = V.synthetic_library(300, h, 32, seed=h + 1)
    lib_np[5] = 0
    lib_np[6] = 255
    lib_np[7] = np.where(rng.random((h, 32)) < 0.5, 0, 255)
    queries, _ = V.synthetic_queries(lib_np, 37, seed=h + 2)
    queries[0] = 255
    queries[1] = 0
    lib = vtmod.ViewTemplates._from_shape((h, 32), 45000)
    lib.add(lib_np)
    ref = np.stack([V.vt_scores_library(lib_np, q) for q in queries])
    assert np.array_equal(lib.scores(queries), ref)
    idx, score, _ = lib.match_templates(queries, mode=0)
    assert np.array_equal(score, ref.min(axis=1))
    assert np.array_equal(idx, ref.argmin(axis=1))


@functools.lru_cache(maxsize=1)
def _split_case():
    lib_np = V.synthetic_library(700, 64, 32, seed=11)
    queries, _ = V.synthetic_queries(lib_np, 240, seed=12)
    return lib_np, queries, np.stack([V.vt_scores_library(lib_np, q) for q in queries])


@pytest.mark.parametrize('nqc', ['1', '3', '8', '24', '64', '512'])
def test_plane_scan_work_splits(vtmod, monkeypatch, nqc):
    """The plane scan gives the oracle's first argmin whatever the number of
    blocks per template block (RS_VT_NQC): one block of all queries, split
    without XCD query groups (3), with them (8, 24, 64), and more blocks than
    query batches (512, capped at the batch count); the library spans several rounds of resident blocks at
    the large splits, and a second launch reuses the batch counters."""
    monkeypatch.setenv('RS_VT_NQC', nqc)
    lib_np, queries, ref = _split_case()
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    lib.add(lib_np)
    for _ in range(2):
        idx, score, _ = lib.match_templates(queries, mode=0)
        assert np.array_equal(score, ref.min(axis=1))
        assert np.array_equal(idx, ref.argmin(axis=1))


def test_all_pair_scores_vs_oracle(vtmod):
    lib_np = V.synthetic_library(150, 64, 32, seed=4)
    queries, _ = V.synthetic_queries(lib_np, 20, seed=5)
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    lib.add(lib_np)
    sc = lib.scores(queries)
    ref = np.stack([V.vt_scores_library(lib_np, q) for q in queries])
    assert np.array_equal(sc, ref)


def test_sequential_batch_equals_oracle_sequence(vtmod):
    """Exact ViewTemplates.match semantics inside one batch: later queries may hit
    templates appended earlier in the same batch, first argmin wins."""
    base = V.synthetic_library(40, 64, 32, seed=8)
    rng = np.random.default_rng(9)
    qs = []
    for i in range(300):
        b = base[int(rng.integers(0, 40))]
        n = rng.integers(0, 3 if rng.random() < 0.8 else 60, b.shape)
        qs.append(np.clip(np.roll(b, int(rng.integers(-6, 7)), axis=0).astype(int) - n, 0, 255))
    qs = np.array(qs, dtype=np.uint8)
    ref = V.ViewTemplatesOracle((0, 128), (0, 64), 2, 2, 8, 8, 45000)
    ref.shape = (64, 32)
    expect = [ref.match_template(q)[0] for q in qs]
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    got = np.concatenate([lib.match_templates(qs[i:i + 64])[0] for i in range(0, 300, 64)])
    assert np.array_equal(got, expect)
    assert np.array_equal(np.stack([t.template for t in lib.templates]), np.stack(ref.templates))


def test_add_from_pinned_or_device_memory_then_overwrite(vtmod):
    """rs_vt_add from pinned host memory (rs_host_alloc) and from device memory: the DMA
    engine reads those sources directly, so the call waits for its copy before returning;
    the caller overwrites or frees the array at once and the stored templates are still
    the bytes it passed (every pair score against the oracle, and the bytes read back)."""
    import ctypes
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(192, 64, 32, seed=31)
    ll = _lib.require_device()
    p = ctypes.c_void_p()
    _lib.check(ll.rs_host_alloc(lib_np.nbytes, ctypes.byref(p)))
    try:
        pinned = np.frombuffer((ctypes.c_uint8 * lib_np.nbytes).from_address(p.value),
                               dtype=np.uint8).reshape(lib_np.shape)
        lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
        for i in range(0, 128, 32):
            pinned[:32] = lib_np[i:i + 32]
            lib.add(pinned[:32])
            pinned[:32] = 0xA5          # overwritten the moment add() returns
        pinned[:] = 0x5A
    finally:
        _lib.check(ll.rs_host_free(p))
    hip = ctypes.CDLL('libamdhip64.so')   # device memory as a caller might hold it
    src = np.ascontiguousarray(lib_np[128:])
    dev = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(src.nbytes)) == 0
    try:
        assert hip.hipMemcpy(dev, src.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(src.nbytes), 1) == 0
        first = ctypes.c_int64()
        with lib._mutex:
            _lib.check(lib._lib.rs_vt_add(lib._h, 64, ctypes.cast(dev, ctypes.POINTER(ctypes.c_uint8)),
                                          ctypes.byref(first)))
        assert hip.hipMemset(dev, 0x3C, ctypes.c_size_t(src.nbytes)) == 0
        assert hip.hipDeviceSynchronize() == 0
    finally:
        hip.hipFree(dev)
    assert first.value == 128
    queries, _ = V.synthetic_queries(lib_np, 24, seed=32)
    ref = np.stack([V.vt_scores_library(lib_np, q) for q in queries])
    assert np.array_equal(lib.scores(queries), ref)
    out = np.empty((64, 32), dtype=np.uint8)
    for t in (0, 31, 100, 130, 191):
        _lib.check(lib._lib.rs_vt_read(lib._h, t, _lib.ptr(out, ctypes.c_uint8)))
        assert np.array_equal(out, lib_np[t]), t


def test_small_batches_in_place_and_back_to_back_adds(vtmod):
    """Batches of at most 64 queries are read by the plane kernel straight from the
    pinned staging array (which also leaves their bytes on the device for the template
    stores); larger ones are copied first.  Templates added in small chunks back to back
    (each rs_vt_add returns with its copy from the staging array queued; the next one
    waits for it before overwriting the array), then single queries, 64 and 65 queries
    against the oracle, every pair score of the device library, and single-query
    sequential matching (a query that becomes a template is stored from the device copy
    the plane kernel made) against the reference's match sequence."""
    lib_np = V.synthetic_library(200, 64, 32, seed=21)
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    i, k = 0, 0
    while i < len(lib_np):
        n = 1 + k % 4
        lib.add(lib_np[i:i + n])
        i += n
        k += 1
    queries, _ = V.synthetic_queries(lib_np, 150, seed=22)
    ref = np.stack([V.vt_scores_library(lib_np, q) for q in queries])
    for j in range(12):
        idx, score, _ = lib.match_templates(queries[j:j + 1], mode=0)
        assert idx[0] == ref[j].argmin() and score[0] == ref[j].min(), j
    for a, b in ((12, 76), (76, 141)):           # 64 queries in place, 65 copied
        idx, score, _ = lib.match_templates(queries[a:b], mode=0)
        assert np.array_equal(idx, ref[a:b].argmin(axis=1)) and np.array_equal(score, ref[a:b].min(axis=1))
    assert np.array_equal(lib.scores(queries[:9]), ref[:9])
    base = V.synthetic_library(30, 64, 32, seed=23)
    rng = np.random.default_rng(24)
    qs = np.array([np.clip(np.roll(base[int(rng.integers(0, 30))], int(rng.integers(-6, 7)), axis=0).astype(int)
                           - rng.integers(0, 3 if rng.random() < 0.7 else 60, (64, 32)), 0, 255)
                   for _ in range(120)], dtype=np.uint8)
    oracle = V.ViewTemplatesOracle((0, 128), (0, 64), 2, 2, 8, 8, 45000)
    oracle.shape = (64, 32)
    expect = [oracle.match_template(q)[0] for q in qs]
    seq = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    got = [int(seq.match_templates(q[None])[0][0]) for q in qs]
    assert got == expect
    assert np.array_equal(np.stack([t.template for t in seq.templates]), np.stack(oracle.templates))
    assert np.array_equal(seq.scores(qs[:5]), np.stack([V.vt_scores_library(np.stack(oracle.templates), q)
                                                         for q in qs[:5]]))


def test_zero_sized_calls(vtmod):
    """Empty inputs at every entry point return empty results and leave the library as
    it was: no queries (match_templates, match_batch, match_stream with nb = 0 or
    nq = 0, host and HBM-resident), no templates added, scores against an empty
    library, and an ordinary match afterwards."""
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(70, 64, 32, seed=31)
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    assert lib.scores(lib_np[:2]).shape == (2, 0)
    lib.add(lib_np[:0])
    assert lib.count() == 0
    lib.add(lib_np)
    idx, score, new = lib.match_templates(np.empty((0, 64, 32), np.uint8), mode=0)
    assert idx.shape == score.shape == new.shape == (0,)
    idx, score, new = lib.match_templates(np.empty((0, 64, 32), np.uint8))
    assert idx.shape == (0,) and lib.count() == 70
    for shape in ((0, 5, 64, 32), (3, 0, 64, 32)):
        i, sc = lib.match_stream(np.empty(shape, np.uint8))
        assert i.shape == sc.shape == shape[:2]
    buf = _lib.DeviceBuffer(64 * 32 * 4)
    i, sc = lib.match_stream((0, 4, buf))
    assert i.shape == (0, 4)
    buf.close()
    q, src = V.synthetic_queries(lib_np, 5, seed=32)
    ref = np.stack([V.vt_scores_library(lib_np, x) for x in q])
    idx, score, _ = lib.match_templates(q, mode=0)
    assert np.array_equal(idx, ref.argmin(axis=1)) and np.array_equal(score, ref.min(axis=1))
    assert lib.count() == 70
    ros = vtmod.ViewTemplates((32, 96), (32, 96), 2, 2, 256, 256, 45000)
    assert ros.match_batch([], []) == [] and len(ros.templates) == 0


def test_ties_pick_first_index(vtmod):
    t = V.synthetic_library(5, 64, 32, seed=2)
    lib_np = np.concatenate([t, t, t])                       # indices 0..4 repeated
    lib = vtmod.ViewTemplates._from_shape((64, 32), 10 ** 9)
    lib.add(lib_np)
    idx, score, _ = lib.match_templates(t, mode=0)
    assert np.array_equal(idx, np.arange(5)) and (score == 0).all()


def test_empty_library_appends(vtmod):
    lib = vtmod.ViewTemplates._from_shape((32, 32), 0)
    q = V.synthetic_library(3, 32, 32, seed=1)
    idx, score, new = lib.match_templates(q)
    assert list(idx) == [0, 1, 2] and new.all()
    assert score[0] == np.iinfo(np.uint64).max           # nothing to compare against
    idx, _, new = lib.match_templates(q)                   # exact copies: score 0 > 0 is False
    assert list(idx) == [0, 1, 2] and not new.any()


@pytest.mark.parametrize('nranks', [2, 3, 4])
def test_sharded_ranks_simulated_on_one_gpu(vtmod, nranks):
    """nranks handles on one GPU, each owning templates g % nranks == rank; the
    elementwise min over their local keys plays the RCCL allreduce(min)."""
    base = V.synthetic_library(60, 64, 32, seed=21)
    queries, _ = V.synthetic_queries(base, 200, seed=22, hit_frac=0.7)
    import ctypes
    from pyratslam_amd import _lib
    shards = [vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, r, nranks, reducer=lambda k: k)
              for r in range(nranks)]
    pending = {}
    single = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    for s in shards:
        s.add(base[:30])
    single.add(base[:30])
    for lo in range(0, 200, 50):
        batch = queries[lo:lo + 50]
        # scan on every rank first (collective order), then resolve everywhere
        for r, s in enumerate(shards):
            local = np.empty(len(batch), dtype=np.uint64)
            _lib.check(s._lib.rs_vt_scan_local(s._h, len(batch), _lib.ptr(batch, ctypes.c_uint8),
                                               _lib.ptr(local, ctypes.c_uint64)))
            pending[r] = local
        glob = np.minimum.reduce([pending[r] for r in range(nranks)])
        results = []
        for s in shards:
            idx = np.empty(len(batch), dtype=np.int64)
            new = np.empty(len(batch), dtype=np.uint8)
            _lib.check(s._lib.rs_vt_resolve(s._h, len(batch), _lib.ptr(glob, ctypes.c_uint64), 1,
                                            None, _lib.ptr(idx, ctypes.c_int64),
                                            _lib.ptr(new, ctypes.c_uint8)))
            results.append(idx)
        ref_idx, _, _ = single.match_templates(batch)
        for idx in results:
            assert np.array_equal(idx, ref_idx)
    total = single.count()
    assert all(s.count() == total for s in shards)
    # every template readable on exactly its owner
    for g in range(total):
        s = shards[g % nranks]
        out = np.empty((64, 32), dtype=np.uint8)
        _lib.check(s._lib.rs_vt_read(s._h, g, _lib.ptr(out, ctypes.c_uint8)))
        ref = np.empty((64, 32), dtype=np.uint8)
        _lib.check(single._lib.rs_vt_read(single._h, g, _lib.ptr(ref, ctypes.c_uint8)))
        assert np.array_equal(out, ref)


def test_sharded_python_reducer_path(vtmod):
    """ShardedViewTemplates with a callable reducer, one rank (reduce = identity)."""
    base = V.synthetic_library(30, 64, 32, seed=31)
    queries, _ = V.synthetic_queries(base, 64, seed=32)
    s = vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, 0, 1, reducer=lambda k: k)
    s.add(base)
    single = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    single.add(base)
    assert np.array_equal(s.match_templates(queries)[0], single.match_templates(queries)[0])


def test_type_and_shape_errors(vtmod):
    vts = vtmod.ViewTemplates((32, 96), (32, 96), 2, 2, 256, 256, 45000)
    with pytest.raises(TypeError):
        vts.match(np.zeros((256, 256), dtype=np.int16), 0, 0, 0)
    with pytest.raises(ValueError):
        vts.match(np.zeros((128, 128), dtype=np.uint8), 0, 0, 0)
    with pytest.raises(TypeError):
        vtmod.sad_scores(np.zeros((1, 32, 32), np.int32), np.zeros((1, 32, 32), np.int32))


@pytest.mark.parametrize('thr', [-1, -0.5, float('inf'), float('nan'), 2 ** 70, 0, 0.999, 5])
def test_threshold_rule_like_numpy(vtmod, thr):
    """`min(match_val) > match_threshold` (view_templates.py:67) for any Python number,
    compared as numpy compares the uint64 score: a negative threshold always appends,
    inf / NaN / huge never do, an exact copy (score 0) is a hit for any threshold >= 0."""
    t = V.synthetic_library(4, 32, 32, seed=3)
    lib = vtmod.ViewTemplates._from_shape((32, 32), thr)
    lib.add(t)
    idx, score, new = lib.match_templates(t)      # exact copies, score 0
    assert (score == 0).all()
    expect = bool(np.uint64(0) > thr)
    assert list(new) == [expect] * 4
    if not expect:
        assert list(idx) == [0, 1, 2, 3]
    q = V.synthetic_library(1, 32, 32, seed=99)   # unrelated frame: a large score
    _, sc, new = lib.match_templates(q)
    assert bool(new[0]) == bool(np.uint64(sc[0]) > thr)


def test_pair_score_of_one_template_scans_only_its_block(vtmod):
    """ViewTemplate.match on an owned template scores [t0, t0 + 1) only (no whole-
    library scan): right score for templates in every 64-slot block, and the staged
    match batch is not mistaken for the scored query."""
    import ctypes
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(300, 64, 32, seed=51)
    q, _ = V.synthetic_queries(lib_np, 3, seed=52)
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    lib.add(lib_np)
    lib.match_templates(q, mode=0)                 # stages q
    for t in (0, 63, 64, 200, 299):
        assert lib.templates[t].match(q[1]) == V.vt_score(lib_np[t], q[1])
    sc = lib.scores(q, 130, 7)
    assert np.array_equal(sc, np.stack([V.vt_scores_library(lib_np[130:137], x) for x in q]))
    with pytest.raises(RuntimeError):             # the staged batch was replaced by scores()
        _lib.check(lib._lib.rs_vt_resolve(lib._h, 3, _lib.ptr(np.zeros(3, np.uint64), ctypes.c_uint64),
                                          1, None, None, None))


def test_template_bytes_on_another_rank_raise(vtmod):
    t = vtmod.ViewTemplate(0, 0, 0, 5, None, _owner=vtmod.ShardedViewTemplates.from_shape(
        (32, 32), 45000, 0, 2, reducer=lambda k: k))
    with pytest.raises(ValueError, match='rank 1'):
        t.match(np.zeros((32, 32), np.uint8))


@pytest.mark.parametrize('tag', ['f64', 'f32'])
@pytest.mark.parametrize('i', [0, 1, 2])
def test_float_pair_scores_bit_exact(vtmod, tag, i):
    """Float ViewTemplate.match on the GPU (rs_sad_scores: true SAD in the arrays'
    dtype, numpy's pairwise summation order) equals the reference's scores bit for
    bit on non-integer float64 / float32 data."""
    d = load_golden('vt_pairs_float')
    a, b, s = d[f'{tag}_{i}_a'], d[f'{tag}_{i}_b'], d[f'{tag}_{i}_score']
    sc = vtmod.sad_scores(a, b)                   # (query, template)
    assert sc.dtype == s.dtype
    assert np.array_equal(np.diagonal(sc), s)
    for j in (0, 9):
        got = vtmod.ViewTemplate(0, 0, 0, j, a[j]).match(b[j])
        assert got == s[j] and np.asarray(got).dtype == s.dtype


@pytest.mark.parametrize('i', [0, 1, 2])
def test_integer_valued_float_pairs(vtmod, i):
    """uint8 pairs cast to float64 (the golden f64 scores): true SAD, no wrap."""
    d = load_golden('vt_pairs')
    a, b = d[f'u8_{i}_a'].astype(np.float64), d[f'u8_{i}_b'].astype(np.float64)
    assert np.array_equal(np.diagonal(vtmod.sad_scores(a, b)), d[f'f64_{i}_score'])
    mixed = vtmod.ViewTemplate(0, 0, 0, 0, d[f'u8_{i}_a'][4]).match(b[4])   # uint8 x float64
    assert mixed == d[f'f64_{i}_score'][4]


def test_float_frames_trace(vtmod):
    """ViewTemplates.match with float64 frames reproduces the reference's trace."""
    d = load_golden('vt_pairs_float')
    vts = vtmod.ViewTemplates((32, 96), (32, 96), 2, 2, 256, 256, float(d['trace_threshold']))
    for k, q in enumerate(d['trace_queries']):
        t = vts.match(_float_frame(vts.mask, q), k % 21, (3 * k) % 21, (5 * k) % 36)
        assert t.get_index() == d['trace_index'][k]
    assert np.array_equal(np.stack([t.template for t in vts.templates]), d['trace_templates'])
    # the device library no longer mirrors the template list: its calls refuse
    u8 = np.zeros((1,) + vts.shape, dtype=np.uint8)
    for call in (lambda: vts.add(u8), lambda: vts.scores(u8), lambda: vts.match_templates(u8),
                 lambda: vts.match_stream(u8[None])):
        with pytest.raises(TypeError, match='float frames'):
            call()


def _float_frame(mask, template):
    im = np.zeros(mask.shape, dtype=np.float64)
    im[mask] = template.ravel()
    return im


def test_library_growth(vtmod):
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000, capacity=64)
    data = V.synthetic_library(700, 64, 32, seed=41)
    for lo in range(0, 700, 100):
        lib.add(data[lo:lo + 100])
    idx, score, _ = lib.match_templates(data[::37], mode=0)
    assert np.array_equal(idx, np.arange(0, 700, 37)) and (score == 0).all()


def noisy_frame(mask, template, rng):
    """A frame whose masked pixels carry the template and every other pixel noise,
    so only a gather through exactly the mask's offsets reproduces the template."""
    im = rng.integers(0, 256, mask.shape, dtype=np.uint8)
    im[mask] = template.ravel()
    return im


@pytest.mark.parametrize('name', ['vt_trace_ros', 'vt_trace_64x32'])
def test_trace_via_match_frames(vtmod, name):
    """On-device subsampling (view_templates.py:64 as a GPU gather) + matching of
    whole frames reproduces the reference's library-evolution trace."""
    d = load_golden(name)
    p = [int(v) for v in d['params']]
    vts = vtmod.ViewTemplates((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    rng = np.random.default_rng(5)
    frames = np.stack([noisy_frame(vts.mask, q, rng) for q in d['queries']])
    third = len(frames) // 3
    got = []
    for lo, hi in ((0, third), (third, 2 * third), (2 * third, len(frames))):
        idx, _, _ = vts.match_frames(frames[lo:hi], d['pcs'][lo:hi])
        got.append(idx)
    assert np.array_equal(np.concatenate(got), d['index'])
    assert np.array_equal(np.stack([t.template for t in vts.templates]), d['templates'])
    assert np.array_equal(np.array([t.location() for t in vts.templates]), d['locations'])


def test_match_frames_device_resident(vtmod):
    """Frames already in HBM (rs_dev_malloc) are gathered in place and give the
    same answers as host frames."""
    from pyratslam_amd import _lib
    d = load_golden('vt_trace_ros')
    p = [int(v) for v in d['params']]
    a = vtmod.ViewTemplates((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    b = vtmod.ViewTemplates((p[0], p[1]), (p[2], p[3]), p[4], p[5], p[6], p[7], p[8])
    rng = np.random.default_rng(6)
    frames = np.stack([noisy_frame(a.mask, q, rng) for q in d['queries'][:120]])
    ia, sa, na = a.match_frames(frames, d['pcs'][:120])
    buf = _lib.DeviceBuffer(frames.nbytes).upload(frames)
    ib, sb, nb = b.match_frames((len(frames), buf), d['pcs'][:120])
    assert np.array_equal(ia, ib) and np.array_equal(sa, sb) and np.array_equal(na, nb)
    assert np.array_equal(ia, d['index'][:120])
    assert np.array_equal(np.stack([t.template for t in b.templates]),
                          np.stack([t.template for t in a.templates]))


def test_match_frames_errors(vtmod):
    vts = vtmod.ViewTemplates((32, 96), (32, 96), 2, 2, 256, 256, 45000)
    with pytest.raises(TypeError):
        vts.match_frames(np.zeros((2, 256, 256), dtype=np.float32), None)
    with pytest.raises(ValueError):
        vts.match_frames(np.zeros((2, 128, 256), dtype=np.uint8), None)
    lone = vtmod.ViewTemplates._from_shape((32, 32), 45000)
    with pytest.raises(ValueError):
        lone.match_frames(np.zeros((1, 256, 256), dtype=np.uint8), None)


def test_untimed_scans(vtmod):
    """rs_vt_set_timing(0) drops the scan's HIP events: same results, no time."""
    lib_np, queries, ref = _split_case()
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    lib.add(lib_np)
    lib.set_timing(False)
    idx, score, _ = lib.match_templates(queries, mode=0)
    assert np.array_equal(idx, ref.argmin(axis=1)) and np.array_equal(score, ref.min(axis=1))
    assert lib.device_ms() == -1.0
    lib.set_timing(True)
    idx, _, _ = lib.match_templates(queries[:50], mode=0)
    assert np.array_equal(idx, ref[:50].argmin(axis=1))
    assert lib.device_ms() > 0.0


@pytest.mark.parametrize('t,nb,q', [(1000, 4, 256), (70, 3, 33), (0, 2, 5), (200, 37, 20)])
def test_match_stream_equals_frozen_batches(vtmod, t, nb, q):
    """rs_vt_match_stream (nb batches, one host sync) == nb rs_vt_match_batch(FROZEN)
    calls, from host memory and from batches resident in HBM; the oracle pins scores."""
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(max(t, 1), 64, 32, seed=t + 5)[:t]
    batches = np.stack([V.synthetic_queries(V.synthetic_library(max(t, 8), 64, 32, seed=t + 5),
                                            q, seed=100 + b)[0] for b in range(nb)])
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    if t:
        lib.add(lib_np)
    idx_h, score_h = lib.match_stream(batches)
    buf = _lib.DeviceBuffer(batches.nbytes).upload(batches)
    idx_d, score_d = lib.match_stream((nb, q, buf))
    buf.close()
    assert np.array_equal(idx_h, idx_d) and np.array_equal(score_h, score_d)
    # the staged batch is gone after a stream (its forms came from elsewhere)
    with pytest.raises(RuntimeError):
        _lib.check(lib._lib.rs_vt_match_batch(lib._h, q, None, 0, None, None, None))
    for b in range(nb):
        idx, score, new = lib.match_templates(batches[b], mode=0)
        assert not new.any()
        assert np.array_equal(idx_h[b], idx) and np.array_equal(score_h[b], score)
        for i in range(0, q, max(1, q // 8)):
            if t == 0:
                assert idx_h[b, i] == -1 and score_h[b, i] == np.iinfo(np.uint64).max
                continue
            ref = V.vt_scores_library(lib_np, batches[b, i])
            assert score_h[b, i] == ref.min() and idx_h[b, i] == int(np.argmin(ref))
    assert lib.count() == t


def test_match_stream_host_groups_reuse_and_grow(vtmod):
    """Host batches go up in groups of 16 through two device buffers (the group
    before last's buffer is reused only after its planes were built): calls of 1, 16,
    17, 40 and again 3 batches of growing and shrinking size on one handle, each equal
    to the same batches from HBM."""
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(300, 64, 32, seed=9)
    lib = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    lib.add(lib_np)
    for nb, q in ((1, 64), (16, 8), (17, 64), (40, 30), (3, 100)):
        batches = np.stack([V.synthetic_queries(lib_np, q, seed=1000 * nb + b)[0] for b in range(nb)])
        idx_h, score_h = lib.match_stream(batches)
        buf = _lib.DeviceBuffer(batches.nbytes).upload(batches)
        idx_d, score_d = lib.match_stream((nb, q, buf))
        buf.close()
        assert np.array_equal(idx_h, idx_d) and np.array_equal(score_h, score_d), (nb, q)
        ref = V.vt_scores_library(lib_np, batches[-1, -1])
        assert score_h[-1, -1] == ref.min() and idx_h[-1, -1] == int(np.argmin(ref))


def test_match_stream_refuses_host_reduced_shards(vtmod):
    s = vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, 0, 2, reducer=lambda k: k)
    s.add(V.synthetic_library(10, 64, 32, seed=3))
    with pytest.raises(RuntimeError):
        s.match_stream(np.zeros((1, 4, 64, 32), np.uint8))


def test_match_stream_collective_path_one_rank(vtmod):
    """A 1-rank RCCL communicator runs rs_vt_match_stream's collective path on one
    GPU (each batch's allreduce on the second stream, overlapped with the next
    batch, then joined): results equal the plain frozen matching."""
    lib_np = V.synthetic_library(700, 64, 32, seed=9)
    batches = np.stack([V.synthetic_queries(lib_np, 300, seed=40 + b)[0] for b in range(6)])
    uid = vtmod.ShardedViewTemplates.unique_id()
    s = vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, 0, 1, reducer='rccl', unique_id=uid)
    plain = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    s.add(lib_np)
    plain.add(lib_np)
    for _ in range(2):   # twice: the streams and events are reused
        idx, score = s.match_stream(batches)
        ref_idx, ref_score = plain.match_stream(batches)
        assert np.array_equal(idx, ref_idx) and np.array_equal(score, ref_score)
    for b in range(6):
        i, sc, _ = plain.match_templates(batches[b], mode=0)
        assert np.array_equal(idx[b], i) and np.array_equal(score[b], sc)
    s.close()
    plain.close()


def test_match_stream_device_batches_collective_one_rank(vtmod):
    """HBM-resident batches through a 1-rank RCCL communicator: one fused scan of all
    batches, one collective over every row; equal to the per-batch frozen matching."""
    from pyratslam_amd import _lib
    lib_np = V.synthetic_library(900, 64, 32, seed=19)
    batches = np.stack([V.synthetic_queries(lib_np, 200, seed=60 + b)[0] for b in range(5)])
    uid = vtmod.ShardedViewTemplates.unique_id()
    s = vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, 0, 1, reducer='rccl', unique_id=uid)
    plain = vtmod.ViewTemplates._from_shape((64, 32), 45000)
    s.add(lib_np)
    plain.add(lib_np)
    buf = _lib.DeviceBuffer(batches.nbytes).upload(batches)
    for _ in range(2):
        idx, score = s.match_stream((5, 200, buf))
        for b in range(5):
            i, sc, _ = plain.match_templates(batches[b], mode=0)
            assert np.array_equal(idx[b], i) and np.array_equal(score[b], sc)
    buf.close()
    s.close()
    plain.close()
