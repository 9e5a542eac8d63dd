#!/usr/bin/env python3
"""Benchmark of the pyratslam hot path on MI355X (BASELINE.json metric).

One JSON line on rank 0:
  value        template compares/s of the whole job (all ranks).  A step is one
               ``rs_vt_match_stream`` call over `--batches-per-step` distinct
               batches of `--queries` subsampled 64x32 uint8 views, resident in
               HBM, matched against the whole library (`--templates-per-gpu` per
               rank, sharded round-robin, first argmin combined by one RCCL
               allreduce(min, uint64) per batch); results reach the host inside
               the step.  Weak scaling: the library grows with the GPUs.
  library_sharded  configs[2]: a fixed 100k-template library sharded over the
               ranks (strong scaling), same batches and allreduce.
  pose_cell    64x64x36 pose-cell network steps/s (the other half of the
               metric): batched `run()` and the per-call `update()` drop-in
               rate; replicated per GPU (one network, nothing to shard).
  pose_cell_stress  configs[3]: the 128x128x72 grid plus its 10k-template scan.
  roofline     dominant kernel = the template scan, which is bound by VALU issue
               (each template is read once per launch and reused from registers
               by every query): PMC VALU wave-instructions per launch / the scan
               kernel's live HIP-event duration / the wave64 issue peak, with the
               measured HBM bytes beside it (profiles/pmc_traffic.json).
  cpu_baseline the oracle (C/OpenMP restatement of the reference) on this
               host's cores, bounded sample, rank 0 at N=1.

Usage: python bench.py [--gpus N --steps K --warmup W].  N > 1 launches its own
N rank processes (pyratslam_amd.launch) unless a launcher such as
torch.distributed.run already set RANK / WORLD_SIZE; the control plane is
pyratslam_amd.dist (TCP, no PyTorch), the data path RCCL.
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pyratslam_amd import launch  # noqa: E402
from pyratslam_amd.dist import Dist  # noqa: E402,F401  (tests import bench.Dist)

# wave64 VALU issue peak: one wave-instruction per 2 cycles per SIMD, 1,024 SIMDs,
# 2.4 GHz (MI355X_MICROARCH.md chip table)
VALU_PEAK_GINSTS = 1024 * 2.4 * 0.5
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_COMPARE = 64 * 32  # one stored 64x32 u8 template
SCAN_KERNELS = {'plane': 'vt_scan_plane_kernel', 'carry': 'vt_scan_carry_kernel',
                'generic': 'vt_scan_generic_kernel'}
METRIC = 'pose-cell steps/sec (64×64×36) + template-compares/sec at 1/2/4/8 GPU'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20, help='timed steps (template match calls)')
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--clock-warmup-ms', type=float, default=200.0,
                    help='untimed matching before the warm-up steps of the headline leg, so the '
                         'timed steps run at the GPU\'s steady clock (0 = off)')
    ap.add_argument('--batches-per-step', type=int, default=10,
                    help='query batches matched per step (one rs_vt_match_stream call)')
    ap.add_argument('--queries', type=int, default=1024, help='queries per batch (one scan launch)')
    ap.add_argument('--templates-per-gpu', type=int, default=1000)
    ap.add_argument('--library-total', type=int, default=100000,
                    help='configs[2]: fixed library sharded over the ranks (strong scaling); 0 = off')
    ap.add_argument('--library-steps', type=int, default=4)
    ap.add_argument('--stress-templates', type=int, default=10000,
                    help='configs[3]: templates per GPU scanned beside the stress grid; 0 = off')
    ap.add_argument('--pc-shape', default='64,64,36')
    ap.add_argument('--pc-steps', type=int, default=10000,
                    help='timed pose-cell steps (SURVEY.md 8(d): >= 10,000)')
    ap.add_argument('--pc-warmup', type=int, default=200)
    ap.add_argument('--pc-calls', type=int, default=10000, help='timed per-call update()s')
    ap.add_argument('--node-calls', type=int, default=2000,
                    help='timed update() + .posecells read pairs (the ROS node step)')
    ap.add_argument('--pc-stress-shape', default='128,128,72',
                    help='configs[3] stencil-stress grid, reported beside the headline grid')
    ap.add_argument('--pc-stress-steps', type=int, default=10000)
    ap.add_argument('--no-pc-stress', action='store_true')
    ap.add_argument('--replay-messages', type=int, default=600,
                    help='configs[4] replay: odometry messages (each followed by a frame)')
    ap.add_argument('--no-replay', action='store_true')
    ap.add_argument('--same-device', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--cpu-seconds', type=float, default=6.0, help='CPU baseline budget per leg')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'profiles', 'pmc_traffic.json'))
    return ap.parse_args()


def _sharded_library(args, d, T):
    """(view-template handle with room for T local templates, reduce kind)."""
    from pyratslam_amd.view_templates import ShardedViewTemplates, ViewTemplates
    n = d.world
    if n == 1:
        return ViewTemplates._from_shape((64, 32), 45000, device=d.dev, capacity=T), 'none'
    if args.same_device:  # RCCL refuses two ranks on one GPU: host reducer
        return (ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer=d.min_keys,
                                                device=d.dev, capacity=T), 'host-tcp-min')
    uid = d.bcast_bytes(ShardedViewTemplates.unique_id() if d.rank == 0 else None)
    try:
        return (ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer='rccl',
                                                unique_id=uid, device=d.dev, capacity=T),
                'rccl-allreduce-min-u64')
    except Exception as e:  # pragma: no cover - recorded in the output, not hidden
        print('rank %d: RCCL attach failed (%s); host reduction' % (d.rank, e), file=sys.stderr)
        return (ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer=d.min_keys,
                                                device=d.dev, capacity=T), 'host-tcp-min')


def bench_templates(args, d, per_gpu=None, total=None, steps=None, warmup=None, bps=None):
    """Frozen-library template matching.  ``per_gpu`` templates on every rank
    (weak scaling), or a fixed library of ``total`` sharded over the ranks
    (strong scaling).  A step = one rs_vt_match_stream call over ``bps``
    distinct HBM-resident batches of ``args.queries`` queries."""
    import ctypes

    from pyratslam_amd import _lib, synthetic
    Q, n = args.queries, d.world
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    bps = args.batches_per_step if bps is None else bps
    if total is None:
        T, total = per_gpu, per_gpu * n
    else:
        T = (total + n - 1) // n             # rank r holds templates g % n == r
    vts, reduce_kind = _sharded_library(args, d, T)
    # every rank adds the whole global library; rank r keeps templates g % n == r
    for lo in range(0, total, 8192):
        vts.add(synthetic.library(min(8192, total - lo), seed=1, first=lo))
    qlib = synthetic.library(min(total, 4096), seed=1)
    queries, src = synthetic.queries(qlib, Q, seed=2)
    lib = vts._lib
    idx = np.empty(Q, dtype=np.int64)
    score = np.empty(Q, dtype=np.uint64)
    new = np.empty(Q, dtype=np.uint8)
    p_score, p_idx, p_new = (_lib.ptr(score, ctypes.c_uint64), _lib.ptr(idx, ctypes.c_int64),
                             _lib.ptr(new, ctypes.c_uint8))
    p_queries = _lib.ptr(queries, ctypes.c_uint8)

    def match(staged):
        """one batch through rs_vt_match_batch (or scan_local + host reduce + resolve)"""
        qp = None if staged else p_queries
        if vts.nranks > 1 and vts.reducer != 'rccl':
            local = np.empty(Q, dtype=np.uint64)
            _lib.check(lib.rs_vt_scan_local(vts._h, Q, qp, _lib.ptr(local, ctypes.c_uint64)))
            glob = np.ascontiguousarray(vts.reducer(local))
            _lib.check(lib.rs_vt_resolve(vts._h, Q, _lib.ptr(glob, ctypes.c_uint64), 0,
                                         p_score, p_idx, p_new))
        else:
            _lib.check(lib.rs_vt_match_batch(vts._h, Q, qp, _lib.RS_VT_FROZEN, p_score, p_idx, p_new))

    match(staged=False)                      # stage one batch (+ correctness probe)
    hits = src >= 0
    correct = bool(np.all(idx[hits] == src[hits]))

    # Distinct batches resident in HBM before the timed region (at most 400; longer
    # runs cycle through them).  Handles reduced on the host (--same-device) run the
    # per-batch loop instead of the stream.
    pipeline = 'stream' if (vts.nranks == 1 or vts.reducer == 'rccl') else 'per-batch'
    nres = max(1, min(steps * bps, 400))
    nres -= nres % bps if nres >= bps else 0
    bufs, srcs = None, None
    if pipeline == 'stream':
        qs, srcs = [queries], [src]
        for b in range(1, nres):
            q_, s_ = synthetic.queries_fast(qlib, Q, seed=2 + 1000 * b)
            qs.append(q_)
            srcs.append(s_)
        bufs = _lib.DeviceBuffer(Q * queries[0].nbytes * nres, device=d.dev).upload(np.stack(qs))
        first_step = np.ascontiguousarray(np.concatenate(qs[:min(bps, nres)]))
        del qs
        nchunk = max(1, nres // bps)
        bpc = min(bps, nres)

        def step(i):
            c = i % nchunk
            dev_ptr = bufs.offset(c * bpc * Q * queries[0].nbytes)
            return vts.match_stream((bpc, Q, dev_ptr)), c
        try:
            # The GPU's clocks ramp up over the first tens of ms of load after idle
            # (rocprof: the same scan launch 1,757 -> 1,499 us over its first 21
            # launches, profiles/r2_v4_kernel_summary.md's trace): bring it to its
            # steady clock with untimed steps before the W warm-up steps.
            # Every rank runs the same number of them (each step may hold a collective).
            if args.clock_warmup_ms > 0:
                step(0)                               # sizes the stream's buffers
                c0 = time.perf_counter()
                step(1)
                per = d.max(time.perf_counter() - c0)
                for i in range(int(np.ceil(args.clock_warmup_ms * 1e-3 / max(per, 1e-4)))):
                    step(i)
            for i in range(max(1, warmup)):          # the first sizes the stream's buffers
                (sidx, _), c = step(i)
                correct = correct and all(bool(np.all(sidx[b][srcs[c * bpc + b] >= 0] ==
                                                      srcs[c * bpc + b][srcs[c * bpc + b] >= 0]))
                                          for b in range(bpc))
        except Exception as e:  # pragma: no cover - recorded, not hidden
            print('rank %d: rs_vt_match_stream failed (%s); per-batch loop' % (d.rank, e),
                  file=sys.stderr)
            pipeline = 'per-batch'
            bufs.close()
            bufs = None
            match(staged=False)
    if pipeline == 'per-batch':
        bpc = 1
        for _ in range(warmup):
            match(staged=True)
    # The scan kernel's duration is taken live in the timed steps: with timing on, a
    # step's one scan launch (all bpc x Q queries of its HBM-resident batches) is
    # bracketed by two HIP events on the stream it runs on.
    vts.set_timing(True)
    kernel_ms = []
    d.barrier()
    t0 = time.perf_counter()
    results = []
    for i in range(steps):
        if pipeline == 'stream':
            results.append(step(i))
        else:
            match(staged=True)
        kernel_ms.append(vts.device_ms())
    t1 = time.perf_counter()
    d.barrier()
    dt = d.max(t1 - t0)
    # The same K steps again on the library's default path (scan timing off): the call
    # polls its keys in pinned host memory and the scan's last block exports them, with
    # no HIP events around the scan -- what a caller of match_stream gets.  Reported
    # beside the value, which carries the live kernel timing the roofline needs.
    vts.set_timing(False)
    d.barrier()
    u0 = time.perf_counter()
    for i in range(steps):
        if pipeline == 'stream':
            results.append(step(i))
        else:
            match(staged=True)
    u1 = time.perf_counter()
    d.barrier()
    dt_default = d.max(u1 - u0)
    if pipeline == 'stream':
        for (sidx, _), c in results:
            for b in range(bpc):
                s_ = srcs[c * bpc + b]
                correct = correct and bool(np.all(sidx[b][s_ >= 0] == s_[s_ >= 0]))
        bufs.close()
        match(staged=False)                  # stage one batch again for the PCIe-inclusive rate
    kernel_ms = [m for m in kernel_ms if m is not None and m >= 0]
    compares = float(total) * Q
    # PCIe-inclusive rates (queries uploaded from host memory), not the value: the
    # stream call over a step's batches from a pageable host array (uploaded in groups
    # behind the scan, rs_vt_match_stream), and one batch per rs_vt_match_batch call
    pcie_stream = None
    if pipeline == 'stream':
        hq = first_step.reshape((bpc, Q) + queries.shape[1:])
        for _ in range(3):
            vts.match_stream(hq)                  # sizes the upload buffers
        d.barrier()
        p0 = time.perf_counter()
        ncall = max(2, min(2 * steps, 40))        # (10 calls, about 18 ms, before round 6)
        for _ in range(ncall):
            hidx, _ = vts.match_stream(hq)
        p1 = time.perf_counter()
        d.barrier()
        pcie_stream = compares * bpc * ncall / d.max(p1 - p0)
        correct = correct and all(bool(np.all(hidx[b][srcs[b] >= 0] == srcs[b][srcs[b] >= 0]))
                                  for b in range(bpc))
    d.barrier()
    p0 = time.perf_counter()
    npcie = max(3, min(steps * bpc // 4, 50))
    for _ in range(npcie):
        match(staged=False)
    p1 = time.perf_counter()
    d.barrier()
    dtp = d.max(p1 - p0)
    res = {
        'value': compares * steps * bpc / dt,
        'ms_per_step': 1e3 * dt / steps,
        'default_path_value': compares * steps * bpc / dt_default,
        'default_path_ms_per_step': 1e3 * dt_default / steps,
        'batches_per_step': bpc,
        'timed_batches': steps * bpc,
        'timed_region_s': dt,
        'pcie_inclusive_value': pcie_stream if pcie_stream is not None else compares * npcie / dtp,
        'pcie_inclusive_per_batch_value': compares * npcie / dtp,
        'scan_ms': float(np.mean(kernel_ms)) if kernel_ms else float('nan'),
        'scan_ms_min': float(np.min(kernel_ms)) if kernel_ms else float('nan'),
        'kernel': SCAN_KERNELS.get(vts.scan_form(), vts.scan_form()),
        'compares_per_launch': float(len(range(d.rank, total, n))) * Q * bpc,
        'queries_per_launch': Q * bpc,
        'templates_per_launch': len(range(d.rank, total, n)),
        'reduce': reduce_kind,
        'pipeline': pipeline,
        'hits_correct': correct,
        'templates_total': total,
    }
    vts.close()
    return res


def _traffic():
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        return json.load(open(p))
    except (OSError, ValueError):
        return {}


def scan_roofline(tv, tj, key):
    """Roofline of one template-scan configuration: VALU-issue bound.  ``tj[key]``
    holds the PMC VALU wave-instructions and HBM bytes per launch of the same
    configuration (templates per launch, queries), from profiles/."""
    rec = (tj.get('scans') or {}).get(key) or {}
    same = (rec.get('templates_per_launch') == tv['templates_per_launch']
            and rec.get('queries') == tv['queries_per_launch']
            # the 64x32-template instantiation the bench launches (the profile's
            # clock warm-up runs another one, vt_scan_plane_kernel<32, ...>)
            and rec.get('kernel', '').startswith(tv['kernel'] + '<64'))
    scan_s = tv['scan_ms'] * 1e-3
    roof = {'bound': 'valu', 'unit': 'G wave-instructions/s', 'peak': VALU_PEAK_GINSTS,
            'achieved': None, 'frac': None, 'traffic': None,
            'kernel_ms': tv['scan_ms'], 'kernel_time_source': 'HIP events around the scan launch of every timed step'}
    if same and rec.get('valu_insts_per_launch'):
        vi = rec['valu_insts_per_launch']
        roof['achieved'] = vi / scan_s / 1e9
        roof['frac'] = roof['achieved'] / VALU_PEAK_GINSTS
        roof['valu_insts_per_launch'] = vi
        roof['traffic'] = rec.get('hbm_bytes_per_launch')
        roof['source'] = 'profiles/' + rec.get('source', '')
        if roof['traffic']:
            roof['hbm_achieved_GBs'] = roof['traffic'] / scan_s / 1e9
            roof['hbm_frac'] = roof['hbm_achieved_GBs'] / HBM_PEAK_GBS
    # unique bytes a launch must move: the stored templates (bytes + planes + sums)
    # once, the queries' planes once
    uniq = tv['templates_per_launch'] * (2048 + 4096 + 64) + tv['queries_per_launch'] * (4 * 51 * 32 + 4)
    roof['unique_bytes_per_launch'] = uniq
    if roof['traffic']:
        roof['traffic_over_unique'] = roof['traffic'] / uniq
    roof['hbm_equivalent_GBs'] = BYTES_PER_COMPARE * tv['compares_per_launch'] / scan_s / 1e9
    roof['note'] = ('frac = VALU issue rate / wave64 peak; hbm_equivalent_GBs = SURVEY 8(d) 2,048 '
                    'B per compare / scan time, an equivalence (each template is reused by every '
                    'query of the batch), not traffic')
    return roof


def pc_roofline(ncell, us_per_step, traffic=None):
    """24 algorithmic B per cell per step over the measured wall
    time per batched step (>= the kernels' time, so frac is a lower bound)."""
    alg = 24.0 * ncell
    ach = alg / (us_per_step * 1e-6) / 1e9
    return {'bound': 'hbm', 'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': ach / HBM_PEAK_GBS, 'traffic': traffic,
            'algorithmic_bytes_per_step': alg,
            'note': '24 B/cell/step algorithmic (SURVEY 8(d)) / wall time per batched step'}


def pc_kernel_rooflines(shape, kus, rec):
    """Per-kernel HBM rates from a profile record: each step kernel reads one float32
    volume and writes one (8 algorithmic B per cell) in its rocprof trace median; with
    the PMC bytes of that kernel (FETCH doubled per MI355X_MICROARCH.md + WRITE) where
    the record holds them."""
    ncell = shape[0] * shape[1] * shape[2]
    pmc = rec.get('hbm_bytes_per_kernel') or {}
    out = {}
    for name, us in kus.items():
        if us < 0.1:   # a once-per-call kernel amortised over the batch
            continue
        k = {'us_rocprof_median': us, 'algorithmic_bytes': 8.0 * ncell,
             'algorithmic_GBs': 8.0 * ncell / (us * 1e-6) / 1e9}
        k['algorithmic_frac'] = k['algorithmic_GBs'] / HBM_PEAK_GBS
        if name in pmc:
            k['pmc_bytes'] = pmc[name]
            k['pmc_GBs'] = pmc[name] / (us * 1e-6) / 1e9
        out[name] = k
    return out


def bench_posecell_stress(args, d):
    """configs[3]: the 128x128x72 grid, batched run() steps/s and kernel roofline."""
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in args.pc_stress_shape.split(','))
    net = PoseCellNetwork(shape, device=d.dev)
    net.inject(1, tuple(s // 2 for s in shape))
    n = args.pc_stress_steps
    od = synthetic.odometry(n + 50, seed=0)
    net.run(od[:50])
    net.run(od[50:50 + n])   # a batch of the timed size, untimed
    d.barrier()
    t0 = time.perf_counter()
    net.run(od[50:50 + n])
    t1 = time.perf_counter()
    d.barrier()
    dt = d.max(t1 - t0)
    dev_us = _device_us_per_step(net, od, 50, n)
    finite = bool(np.isfinite(net.posecells).all())
    form = net.step_form()
    net.close()
    ncell = shape[0] * shape[1] * shape[2]
    return {'shape': list(shape), 'steps_per_s': n / dt, 'us_per_step': 1e6 * dt / n,
            'device_us_per_step': dev_us,
            'step_form': form, 'finite': finite,
            'roofline': pc_roofline(ncell, 1e6 * dt / n)}


def _near_tie_calls(net):
    """Halo form: how many calls so far had their last step keyed by the finishing pass
    (a cell within 2^-20 of the peak, RS_PC_DBG_HALO_AMBIG); None for other forms."""
    if net.step_form() != 'halo':
        return None
    from pyratslam_amd import _lib
    v = ctypes.c_int64(-1)
    _lib.check(net._lib.rs_pc_debug_value(net._h, _lib.RS_PC_DBG_HALO_AMBIG, ctypes.byref(v)))
    return int(v.value)


def _device_us_per_step(net, od, start, n):
    """Device time per batched step: two HIP events around one whole run() of the n
    steps od[start:start + n] (no event between the launches, so nothing is added
    between the kernels), after the same warm run: at most the wall time per step
    beside it."""
    steps = od[start:start + n]
    assert start >= 0 and len(steps) == n, (start, n, len(od))
    net.set_profiling(True, per_kernel=False)
    net.run(steps)
    ms = net.device_ms()
    net.set_profiling(False)
    return 1e3 * ms / len(steps)


def bench_posecells(args, d):
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in args.pc_shape.split(','))
    net = PoseCellNetwork(shape, device=d.dev)
    net.inject(1, tuple(s // 2 for s in shape))
    od = synthetic.odometry(args.pc_warmup + args.pc_steps + args.pc_calls + 64, seed=0)
    net.run(od[:args.pc_warmup])
    net.run(od[args.pc_warmup:args.pc_warmup + args.pc_steps])   # a batch of the timed size, untimed
    d.barrier()
    t0 = time.perf_counter()
    net.run(od[args.pc_warmup:args.pc_warmup + args.pc_steps])
    t1 = time.perf_counter()
    d.barrier()
    dt = d.max(t1 - t0)
    # per-call drop-in rate: PoseCellNetwork.update() through ctypes, one sync each
    base = args.pc_warmup + args.pc_steps
    for v in od[base:base + 16]:
        net.update(v)
    c0 = time.perf_counter()
    for v in od[base + 16:base + 16 + args.pc_calls]:
        net.update(v)
    c1 = time.perf_counter()
    near_ties = _near_tie_calls(net)
    dev_us = _device_us_per_step(net, od, args.pc_warmup, args.pc_steps)
    ncell = shape[0] * shape[1] * shape[2]
    finite = bool(np.isfinite(net.posecells).all())
    form = net.step_form()
    net.close()
    roof = pc_roofline(ncell, 1e6 * dt / args.pc_steps)
    roof['note'] += ('; the 576 KiB volume is L2-resident and the step is launch/latency-bound at '
                     'this size (see pose_cell_stress for configs[3])')
    return {
        'shape': list(shape),
        'steps_per_s': args.pc_steps / dt,
        'update_calls_per_s': args.pc_calls / (c1 - c0),
        'update_near_tie_calls': near_ties,
        'us_per_step': 1e6 * dt / args.pc_steps,
        'device_us_per_step': dev_us,
        'replicas': d.world,
        'step_form': form,
        'finite': finite,
        'roofline': roof,
    }


def bench_other_grids(args, d):
    """Batched run() at the reference's other grids: configs[0]'s 32x32x18 and
    simulate.py's 50x50x10 (simulate.py:9), both one launch per step (the halo form's
    18- and 10-layer instances since round 6; two launches per step before)."""
    from pyratslam_amd import PoseCellNetwork, synthetic
    out = {}
    n = max(200, args.pc_steps // 5)
    for shape in ((32, 32, 18), (50, 50, 10)):
        net = PoseCellNetwork(shape, device=d.dev)
        net.inject(1, tuple(s // 2 for s in shape))
        od = synthetic.odometry(n + 200, seed=0)
        net.run(od[:200])
        net.run(od[200:200 + n])   # a batch of the timed size, untimed
        d.barrier()
        t0 = time.perf_counter()
        net.run(od[200:200 + n])
        t1 = time.perf_counter()
        d.barrier()
        dt = d.max(t1 - t0)
        out['x'.join(map(str, shape))] = {'steps_per_s': n / dt, 'us_per_step': 1e6 * dt / n,
                                          'steps': n, 'step_form': net.step_form(),
                                          'finite': bool(np.isfinite(net.posecells).all())}
        net.close()
    return out


def bench_node_step(args, d):
    """The ROS node's per-step drop-in cost (ros_simulate.py:134-145): update()
    and then a read of the whole ``.posecells`` volume (the node publishes it as a
    Float64MultiArray after every step), per call, at the node's grid (21x21x36,
    ros_simulate.py:31) and the headline grid."""
    from pyratslam_amd import PoseCellNetwork, synthetic
    out = {}
    for shape in ((21, 21, 36), tuple(int(s) for s in args.pc_shape.split(','))):
        net = PoseCellNetwork(shape, device=d.dev)
        net.inject(1, tuple(s // 2 for s in shape))
        n = args.node_calls
        od = synthetic.odometry(n + 32, seed=0)
        for v in od[:32]:
            net.update(v)
            net.posecells
        t0 = time.perf_counter()
        for v in od[32:32 + n]:
            net.update(v)
        t1 = time.perf_counter()
        for v in od[32:32 + n]:
            net.update(v)
            p = net.posecells
        t2 = time.perf_counter()
        r0 = time.perf_counter()
        for _ in range(n):
            p = net.posecells
        r1 = time.perf_counter()
        assert p.shape == shape
        net.close()
        # readback='eager': update() exports the new volume before its one sync
        eg = PoseCellNetwork(shape, device=d.dev, readback='eager')
        eg.inject(1, tuple(s // 2 for s in shape))
        for v in od[:32]:
            eg.update(v)
            eg.posecells
        e0 = time.perf_counter()
        for v in od[32:32 + n]:
            eg.update(v)
            p = eg.posecells
        e1 = time.perf_counter()
        eg.close()
        out['x'.join(map(str, shape))] = {
            'update_us': 1e6 * (t1 - t0) / n, 'update_plus_read_us': 1e6 * (t2 - t1) / n,
            'read_us': 1e6 * (r1 - r0) / n, 'node_steps_per_s': n / (t2 - t1),
            'update_plus_read_eager_us': 1e6 * (e1 - e0) / n, 'node_steps_per_s_eager': n / (e1 - e0),
            'read_bytes': 8 * shape[0] * shape[1] * shape[2]}
    out['note'] = ('update() then `.posecells` (float64, C order, a fresh array per read, written '
                   'by the GPU straight into pinned host memory) per step, as ros_simulate.py:134-145 '
                   'does; _eager: PoseCellNetwork(readback="eager"), the export queued inside '
                   'update() before its one host sync')
    return out


def host_info():
    model = platform.processor() or ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    aff = None
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    return {'cpu_model': model, 'os_cpu_count': os.cpu_count(), 'affinity_cpus': aff,
            'omp_num_threads': os.environ.get('OMP_NUM_THREADS'),
            'cores_policy': 'OpenMP threads = OMP_NUM_THREADS as the GPU pool sets it (16, the host '
                            'CPU share of one GPU on this pool); os_cpu_count and the affinity mask '
                            'show the whole machine, which this job does not own'}


def cpu_baseline(args):
    """The oracle on this host, bounded samples: the C/OpenMP restatement on all
    OpenMP threads (the reported baseline) and the NumPy restatement (1 thread)."""
    from oracle import c_oracle as C
    from oracle import posecell as P
    from oracle import view_templates as V
    from pyratslam_amd import synthetic
    T = args.templates_per_gpu
    lib = synthetic.library(T, seed=1)
    qs, _ = synthetic.queries(lib, 4096, seed=2)
    budget = args.cpu_seconds
    host = host_info()
    # thread count: OMP_NUM_THREADS as the pool sets it (its CPU share of one GPU)
    # and the affinity mask's size (all host cores) are both tried on a
    # short sample; the faster one runs the baseline (a mask wider than the job's
    # CPU quota oversubscribes it)
    cands = sorted({c for c in (C.threads(), host['affinity_cpus'] or 0) if c > 0})
    # (4 queries per call: the oracle parallelises each query over the templates, and
    # an oversubscribed mask runs a few queries per second, so a larger call would
    # hold the probe for many seconds past its time limit)
    probe = {}
    for c in cands:
        C.set_threads(c)
        span = min(1.0, budget / 4)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < span:       # thread pool up (its first calls run slow)
            C.vt_best(lib, qs[:4])
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < span:
            C.vt_best(lib, qs[n % 4096:n % 4096 + 4])
            n += 4
        probe[c] = n / (time.perf_counter() - t0)
    best = max(probe, key=probe.get)
    C.set_threads(best)
    host = dict(host, thread_probe_queries_per_s={str(k): round(v, 1) for k, v in probe.items()},
                cores_policy='OpenMP threads: the faster of OMP_NUM_THREADS and the affinity '
                              'mask size on a short probe (thread_probe_queries_per_s)')
    # C / OpenMP: template compares
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget:     # cycles through the 4,096 queries
        lo = n % len(qs)
        C.vt_best(lib, qs[lo:lo + 64])
        n += 64
    dt = time.perf_counter() - t0
    threads = C.threads()
    vt = {'value': T * n / dt, 'unit': 'compares/s', 'cores': threads, 'kind': 'port',
          'sample': '%d queries x %d stored 64x32 u8 templates in %.1f s, oracle/c (C restatement '
                    'of view_templates.py, OpenMP %d threads)' % (n, T, dt, threads), **host}
    # NumPy, single thread
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget / 2:
        V.vt_scores_library(lib, qs[n % len(qs)])
        n += 1
    dt = time.perf_counter() - t0
    vt_np = {'value': T * n / dt, 'unit': 'compares/s', 'cores': 1, 'kind': 'port',
             'sample': '%d queries in %.1f s, oracle/view_templates.py (NumPy)' % (n, dt)}
    shape = tuple(int(s) for s in args.pc_shape.split(','))
    od = synthetic.odometry(100000, seed=0)
    res = {}
    for name, cls, share in (('c', C.PoseCellC, 1.0), ('numpy', P.PoseCellOracle, 0.5)):
        net = cls(shape)
        net.inject(1, tuple(s // 2 for s in shape))
        k = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget * share:
            net.update(od[k])
            k += 1
        res[name] = (k, time.perf_counter() - t0)
    k, dt = res['c']
    pc = {'value': k / dt, 'unit': 'steps/s', 'cores': threads, 'kind': 'port',
          'sample': '%d updates of a %s grid in %.1f s, oracle/c (C restatement of the three '
                    'OpenCL kernels in float64, 343-tap direct correlation, OpenMP %d threads; '
                    'host control in NumPy)' % (k, shape, dt, threads), **host}
    k, dt = res['numpy']
    pc_np = {'value': k / dt, 'unit': 'steps/s', 'cores': 1, 'kind': 'port',
             'sample': '%d updates in %.1f s, oracle/posecell.py (NumPy float64)' % (k, dt)}
    return vt, vt_np, pc, pc_np


def bench_replay(args, d):
    """configs[4]: the ROS node's loop (ros_simulate.py:98-162) over a synthetic
    10 Hz odometry + 256x256 mono8 camera stream (the reference's bag is absent),
    ROS geometry (21x21x36 pose cells, 32x32 templates); the library is sharded
    over the ranks (template g on rank g % N), pose cells replicated."""
    from pyratslam_amd import replay, synthetic
    events = synthetic.ros_stream(args.replay_messages, seed=0)
    replay.RatslamReplay(device=d.dev).replay_events(events[:40])   # warm-up: kernels, allocations
    vts, reduce_kind = None, 'none'
    if d.world > 1 and args.same_device:
        vts, reduce_kind = replay.sharded_templates(d, d.dev, host_reduce=True), 'host-tcp-min'
    elif d.world > 1:
        try:
            vts, reduce_kind = replay.sharded_templates(d, d.dev), 'rccl-allreduce-min-u64'
        except Exception as e:  # pragma: no cover - recorded, not hidden
            print('rank %d: RCCL attach failed (%s); host reduction' % (d.rank, e), file=sys.stderr)
            vts, reduce_kind = replay.sharded_templates(d, d.dev, host_reduce=True), 'host-tcp-min'
    r = replay.RatslamReplay(device=d.dev, vts=vts)
    d.barrier()
    t0 = time.perf_counter()
    r.replay_events(events)
    dt = d.max(time.perf_counter() - t0)
    res = r.results()
    # the node's per-step work in full: every update also reads the whole .posecells
    # volume (ros_simulate.py:140-145 publishes it), steps one by one
    # (one rank: the pose cells are replicated, so each rank's node work is this)
    publish = None
    if d.world == 1:
        rp = replay.RatslamReplay(device=d.dev, publish=True)
        p0 = time.perf_counter()
        rp.replay_events(events)
        dtp = time.perf_counter() - p0
        resp = rp.results()
        assert [tuple(m) for m in resp['pc_max']] == [tuple(m) for m in res['pc_max']]
        publish = {'messages_per_s': len(events) / dtp, 'seconds': dtp,
                   'posecells_values_read_per_update': rp.published // max(1, len(resp['pc_max'])),
                   'note': 'per update also the .posecells read the node publishes '
                           '(PoseCellNetwork readback="eager"), steps one by one'}
    return {'publish': publish,
            'messages': len(events), 'updates': int(len(res['pc_max'])), 'reduce': reduce_kind,
            'frames': int(len(res['template_index'])), 'templates': int(res['templates']),
            'seconds': dt, 'messages_per_s': len(events) / dt,
            'updates_per_s': len(res['pc_max']) / dt, 'frames_per_s': len(res['template_index']) / dt,
            'note': 'per message: one pose-cell step or one frame match, each a host round trip '
                    '(the node publishes after every step); synthetic stand-in for dataset_10Hz.bag'}


def main():
    args = parse()
    if args.gpus > 1 and not launch.under_launcher():
        # our own N ranks, started before this process touches the GPU
        sys.exit(launch.spawn(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    d = Dist(args.gpus)
    # the GPU of this rank; --same-device puts every rank on GPU 0 (a test aid for
    # 1-GPU boxes: RCCL refuses two ranks on one GPU, so the host reducer is used)
    d.dev = 0 if args.same_device else d.local
    tv = bench_templates(args, d, per_gpu=args.templates_per_gpu)
    lib100 = None
    if args.library_total > 0:
        lib100 = bench_templates(args, d, total=args.library_total, steps=args.library_steps,
                                 warmup=1, bps=2)
    pc = bench_posecells(args, d)
    pc['node_step'] = bench_node_step(args, d)
    pc['other_grids'] = bench_other_grids(args, d)
    pcs, st = None, None
    if not args.no_pc_stress:
        pcs = bench_posecell_stress(args, d)
        if args.stress_templates > 0:
            st = bench_templates(args, d, per_gpu=args.stress_templates, steps=4, warmup=1, bps=5)
    rp = None if args.no_replay else bench_replay(args, d)
    if d.rank != 0:
        d.close()
        return
    tj = _traffic()
    roof = scan_roofline(tv, tj, 'headline')
    tj_pc = tj.get('pose_cell', {})
    for leg in (pc, pcs):
        if leg and leg['step_form'] in tj_pc:
            rec = tj_pc[leg['step_form']]
            if rec.get('shape') in (None, leg['shape']):
                leg['roofline']['traffic'] = rec.get('hbm_bytes_per_step')
                leg['roofline']['traffic_kernels'] = rec.get('kernels')
                # the profiles' per-kernel trace medians, with the record they come from
                # and whether their sum exceeds the wall time per step beside them (a
                # profiled run's kernels need not be the timed steps' kernels)
                kus = rec.get('kernel_us_rocprof')
                if kus:
                    leg['kernel_us_per_step_rocprof'] = kus
                    leg['kernel_us_rocprof_source'] = rec.get('kernel_us_source')
                    leg['kernel_us_rocprof_exceeds_wall'] = sum(kus.values()) > leg['us_per_step']
                    leg['roofline']['kernels'] = pc_kernel_rooflines(leg['shape'], kus, rec)
    out = {
        'metric': METRIC,
        'value': tv['value'],
        'unit': 'compares/s',
        'n_gpus': d.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': tv['ms_per_step'],
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'u8',
        'data': 'synthetic (SURVEY.md 8(d): uniform u8 library, shifted+noised queries, '
                'U(0,0.6) m / U(-0.15,0.15) rad odometry)',
        'config': {
            'workload': 'configs[1]: 64x64x36 pose-cell grid + %d stored 64x32 u8 templates per '
                        'GPU; a step matches %d batches of %d queries resident in HBM'
                        % (args.templates_per_gpu, tv['batches_per_step'], args.queries),
            'templates_per_gpu': args.templates_per_gpu,
            'templates_total': tv['templates_total'],
            'queries_per_batch': args.queries,
            'batches_per_step': tv['batches_per_step'],
            'timed_batches': tv['timed_batches'],
            'timed_region_s': tv['timed_region_s'],
            'template_shape': [64, 32],
            'pose_cell_grid': pc['shape'],
            'parallelism': 'library sharded over %d GPU(s), %s; pose cells replicated'
                           % (d.world, tv['reduce']),
        },
        'roofline': roof,
        'library_sharded': None if lib100 is None else {
            'workload': 'configs[2]: %d stored 64x32 u8 templates in total, sharded round-robin '
                        'over %d GPU(s), %d-query batches resident in HBM' % (
                            lib100['templates_total'], d.world, args.queries),
            'scaling': 'strong', 'compares_per_s': lib100['value'],
            'ms_per_step': lib100['ms_per_step'], 'steps': args.library_steps,
            'batches_per_step': lib100['batches_per_step'],
            'scan_ms_per_launch': lib100['scan_ms'], 'kernel': lib100['kernel'],
            'compares_per_launch_per_gpu': lib100['compares_per_launch'],
            'reduce': lib100['reduce'], 'pipeline': lib100['pipeline'],
            'known_answer_hits_correct': lib100['hits_correct'],
            'pcie_inclusive_compares_per_s': lib100['pcie_inclusive_value'],
            'roofline': scan_roofline(lib100, tj, 'library') if d.world == 1 else None},
        'pose_cell': pc,
        'pose_cell_stress': pcs,
        'replay': rp,
        'template_scan': {'kernel': tv['kernel'], 'kernel_ms_per_launch': tv['scan_ms'],
                          'kernel_ms_per_launch_min': tv['scan_ms_min'],
                          'pipeline': tv['pipeline'],
                          'default_path_compares_per_s': tv['default_path_value'],
                          'default_path_ms_per_step': tv['default_path_ms_per_step'],
                          'default_path_note': 'the same timed steps with scan timing off (the '
                                               'library default: keys polled in pinned memory, exported '
                                               'by the scan\'s last block, no events); value carries the '
                                               'HIP events the roofline needs',
                          'pcie_inclusive_compares_per_s': tv['pcie_inclusive_value'],
                          'pcie_inclusive_note': 'since round 5: a step\'s batches from a pageable host '
                                                 'array through one rs_vt_match_stream call (uploaded in '
                                                 'groups behind the scan; since round 6 timed over up '
                                                 'to 40 calls after 3 untimed ones, 10 calls before); '
                                                 'rounds 1-4 quoted the per-batch figure, kept below',
                          'pcie_inclusive_per_batch_compares_per_s': tv['pcie_inclusive_per_batch_value'],
                          'known_answer_hits_correct': tv['hits_correct']},
    }
    if pcs is not None and st is not None:
        pcs['templates'] = {
            'workload': 'configs[3]: %d stored 64x32 u8 templates per GPU, %d-query batches '
                        'resident in HBM' % (args.stress_templates, args.queries),
            'compares_per_s': st['value'], 'ms_per_step': st['ms_per_step'],
            'batches_per_step': st['batches_per_step'], 'scan_ms_per_launch': st['scan_ms'],
            'kernel': st['kernel'], 'known_answer_hits_correct': st['hits_correct'],
            'roofline': scan_roofline(st, tj, 'stress')}
    if d.world == 1 and not args.no_cpu_baseline:
        vt_cpu, vt_np, pc_cpu, pc_np = cpu_baseline(args)
        out['cpu_baseline'] = vt_cpu
        out['cpu_baseline_numpy'] = vt_np
        out['pose_cell']['cpu_baseline'] = pc_cpu
        out['pose_cell']['cpu_baseline_numpy'] = pc_np
    print(json.dumps(out), flush=True)
    d.close()


if __name__ == '__main__':
    main()
