"""Parity at BASELINE.json's full library sizes (configs[2] and configs[3]).

* configs[2]: 100,000 stored 64x32 templates.  A frozen scan of 64 queries is
  checked against the C/OpenMP oracle (oracle/c, the reference's
  ViewTemplate.match restated: first argmin, wrapped uint8 scores); the same
  library split over 8 ShardedViewTemplates handles on one GPU (template g on
  rank g % 8, the elementwise min of the per-rank keys playing the RCCL
  allreduce(min)) equals the unsharded result, frozen and sequential; the
  bench's rs_vt_match_stream path equals per-batch matching at this size.
* configs[3]: 10,000 stored templates, 256 queries vs the oracle.

Queries are drawn from the whole library (known answers spread over all 64-slot
blocks), plus fresh frames that miss.
"""
import ctypes
import functools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def vtmod():
    from pyratslam_amd import _build
    _build.build()
    import pyratslam_amd.view_templates as m
    return m


@functools.lru_cache(maxsize=2)
def _library(t):
    from pyratslam_amd import synthetic
    return synthetic.library(t, seed=1)


def _oracle_best(lib, queries):
    from oracle import c_oracle as C
    return C.vt_best(lib, queries)


def _loaded(vtmod, lib, **kw):
    vts = vtmod.ViewTemplates._from_shape((64, 32), 45000, capacity=len(lib), **kw)
    for lo in range(0, len(lib), 16384):
        vts.add(lib[lo:lo + 16384])
    return vts


@pytest.mark.parametrize('t,nq', [(100000, 64), (10000, 256)])
def test_full_size_frozen_scan_vs_c_oracle(vtmod, t, nq):
    from pyratslam_amd import _lib, synthetic
    lib = _library(t)
    qs, src = synthetic.queries_fast(lib, nq, seed=7)
    qs[0] = 0                      # extremes: all-0 and all-255 frames
    qs[1] = 255
    vts = _loaded(vtmod, lib)
    idx, score, new = vts.match_templates(qs, mode=_lib.RS_VT_FROZEN)
    ref_score, ref_idx = _oracle_best(lib, qs)
    assert not new.any()
    assert np.array_equal(score, ref_score)
    assert np.array_equal(idx, ref_idx)
    hits = src[2:] >= 0
    assert np.array_equal(idx[2:][hits], src[2:][hits])      # known answers
    vts.close()


def test_configs2_eight_shards_equal_unsharded(vtmod):
    """configs[2]'s protocol at its size: 8 ranks (handles) on one GPU."""
    from pyratslam_amd import _lib, synthetic
    lib = _library(100000)
    nranks = 8
    single = _loaded(vtmod, lib)
    shards = []
    for r in range(nranks):
        s = vtmod.ShardedViewTemplates.from_shape((64, 32), 45000, r, nranks, reducer=lambda k: k,
                                                  capacity=len(lib) // nranks + 64)
        for lo in range(0, len(lib), 16384):
            s.add(lib[lo:lo + 16384])
        shards.append(s)

    def sharded(batch, mode):
        locs = []
        for s in shards:           # every rank scans first (collective order), then resolves
            loc = np.empty(len(batch), dtype=np.uint64)
            _lib.check(s._lib.rs_vt_scan_local(s._h, len(batch), _lib.ptr(batch, ctypes.c_uint8),
                                               _lib.ptr(loc, ctypes.c_uint64)))
            locs.append(loc)
        glob = np.minimum.reduce(locs)
        outs = []
        for s in shards:
            idx = np.empty(len(batch), dtype=np.int64)
            sc = np.empty(len(batch), dtype=np.uint64)
            new = np.empty(len(batch), dtype=np.uint8)
            _lib.check(s._lib.rs_vt_resolve(s._h, len(batch), _lib.ptr(glob, ctypes.c_uint64), mode,
                                            _lib.ptr(sc, ctypes.c_uint64), _lib.ptr(idx, ctypes.c_int64),
                                            _lib.ptr(new, ctypes.c_uint8)))
            outs.append((idx, sc, new))
        return outs

    qs, _ = synthetic.queries_fast(lib, 256, seed=9)
    ri, rs_, _ = single.match_templates(qs, mode=_lib.RS_VT_FROZEN)
    for idx, sc, new in sharded(qs, _lib.RS_VT_FROZEN):
        assert np.array_equal(idx, ri) and np.array_equal(sc, rs_) and not new.any()
    # sequential: half the queries miss and grow the library on their owner ranks
    q2, _ = synthetic.queries_fast(lib, 96, seed=10, hit_frac=0.5)
    r2i, r2s, r2n = single.match_templates(q2, mode=_lib.RS_VT_SEQUENTIAL)
    assert r2n.any()
    for idx, sc, new in sharded(q2, _lib.RS_VT_SEQUENTIAL):
        assert np.array_equal(idx, r2i) and np.array_equal(sc, r2s) and np.array_equal(new, r2n)
    assert all(s.count() == single.count() for s in shards)
    # the appended templates live on their owners only
    g = int(r2i[np.flatnonzero(r2n)[0]])
    out = np.empty((64, 32), dtype=np.uint8)
    owner = shards[g % nranks]
    _lib.check(owner._lib.rs_vt_read(owner._h, g, _lib.ptr(out, ctypes.c_uint8)))
    assert np.array_equal(out, q2[np.flatnonzero(r2n)[0]])
    for s in shards:
        s.close()
    single.close()


def test_configs2_stream_path_equals_batches(vtmod):
    """The bench's rs_vt_match_stream over HBM-resident batches at 100k templates
    equals per-batch frozen matching (and the known answers)."""
    from pyratslam_amd import _lib, synthetic
    lib = _library(100000)
    vts = _loaded(vtmod, lib)
    batches = np.stack([synthetic.queries_fast(lib, 512, seed=20 + b)[0] for b in range(3)])
    buf = _lib.DeviceBuffer(batches.nbytes).upload(batches)
    si, ss = vts.match_stream((3, 512, buf))
    buf.close()
    for b in range(3):
        i, s, _ = vts.match_templates(batches[b], mode=_lib.RS_VT_FROZEN)
        assert np.array_equal(si[b], i) and np.array_equal(ss[b], s)
    ref_score, ref_idx = _oracle_best(lib, batches[0][:32])
    assert np.array_equal(si[0][:32], ref_idx) and np.array_equal(ss[0][:32], ref_score)
    vts.close()
