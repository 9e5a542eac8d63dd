#!/usr/bin/env python3
"""Benchmark of the pyratslam hot path on MI355X (BASELINE.json metric).

One JSON line on rank 0:
  value        template compares/s of the whole job (all ranks): each step
               matches a batch of `--queries` subsampled 64x32 uint8 views,
               resident in HBM, against the whole library (`--templates-per-gpu`
               per rank, sharded round-robin, first-argmin combined by one RCCL
               allreduce(min, uint64) per batch).  Weak scaling: the library
               grows with the number of GPUs.
  library_sharded  configs[2]: a fixed 100k-template library sharded over the
               ranks (strong scaling), same query batches and allreduce.
  pose_cell    64x64x36 pose-cell network steps/s (the other half of the
               metric): batched `run()` (per-step control uploaded with the
               odometry) and the per-call `update()` drop-in rate; replicated
               per GPU (one network, nothing to shard).
  roofline     dominant kernel = the template scan: SURVEY.md section 8(d)'s
               2,048 algorithmic bytes per compare x compares per launch / the
               scan kernel's average HIP-event duration; the pose-cell kernels'
               roofline is in pose_cell.roofline (24 bytes per cell per step).
  cpu_baseline the oracle (NumPy restatement of the reference) on this host's
               cores, bounded sample, rank 0 at N=1.

Usage: python bench.py [--gpus N --steps K --warmup W]; N>1 under
torch.distributed.run (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE env).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

VALU_PEAK_GINSTS = 1024 * 2.4 * 0.5
SCAN_KERNELS = {'plane': 'vt_scan_plane_kernel', 'carry': 'vt_scan_carry_kernel',
                'sad': 'vt_scan_lane_kernel', 'rb2': 'vt_scan_rb_kernel', 'rb3': 'vt_scan_rb_kernel',
                'generic': 'vt_scan_generic_kernel'}
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_COMPARE = 64 * 32  # one stored 64x32 u8 template
from pyratslam_amd.dist import Dist  # noqa: E402

METRIC = 'pose-cell steps/sec (64×64×36) + template-compares/sec at 1/2/4/8 GPU'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20, help='timed template batches')
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--queries', type=int, default=1024)
    ap.add_argument('--templates-per-gpu', type=int, default=1000)
    ap.add_argument('--library-total', type=int, default=100000,
                    help='configs[2]: fixed library sharded over the ranks (strong scaling); 0 = off')
    ap.add_argument('--library-steps', type=int, default=5)
    ap.add_argument('--pc-shape', default='64,64,36')
    ap.add_argument('--pc-steps', type=int, default=10000,
                    help='timed pose-cell steps (SURVEY.md 8(d): >= 10,000)')
    ap.add_argument('--pc-warmup', type=int, default=200)
    ap.add_argument('--pc-calls', type=int, default=10000, help='timed per-call update()s')
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


def bench_templates(args, d, total=None, steps=None, warmup=None):
    """Frozen-library template matching.  Default (configs[1]): `--templates-per-gpu`
    templates on every rank (weak scaling).  With `total` (configs[2]): a fixed
    library of `total` templates sharded over the ranks (strong scaling)."""
    from pyratslam_amd import _lib, synthetic
    from pyratslam_amd.view_templates import ShardedViewTemplates, ViewTemplates
    Q, n = args.queries, d.world
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    if total is None:
        T, total = args.templates_per_gpu, args.templates_per_gpu * n
    else:
        T = (total + n - 1) // n             # rank r holds templates g % n == r
    reduce_kind = 'none'
    if n == 1:
        vts = ViewTemplates._from_shape((64, 32), 45000, device=d.dev, capacity=T)
    elif args.same_device:  # RCCL refuses two ranks on one GPU: host reducer
        vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer=d.min_keys,
                                              device=d.dev, capacity=T)
        reduce_kind = 'gloo-host-min'
    else:
        uid = d.bcast_bytes(ShardedViewTemplates.unique_id() if d.rank == 0 else None)
        try:
            vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer='rccl',
                                                  unique_id=uid, device=d.dev, capacity=T)
            reduce_kind = 'rccl-allreduce-min-u64'
        except Exception as e:  # pragma: no cover - recorded, not hidden
            print('rank %d: RCCL attach failed (%s); host gloo reduction' % (d.rank, e),
                  file=sys.stderr)
            vts = ShardedViewTemplates.from_shape((64, 32), 45000, d.rank, n, reducer=d.min_keys,
                                                  device=d.dev, capacity=T)
            reduce_kind = 'gloo-host-min'
    # every rank adds the whole global library; rank r keeps templates g % n == r
    for lo in range(0, total, 8192):
        vts.add(synthetic.library(min(8192, total - lo), seed=1, first=lo))
    qlib = synthetic.library(min(total, 4096), seed=1)
    queries, src = synthetic.queries(qlib, Q, seed=2)
    lib = vts._lib
    import ctypes
    idx = np.empty(Q, dtype=np.int64)
    score = np.empty(Q, dtype=np.uint64)
    new = np.empty(Q, dtype=np.uint8)

    # result pointers converted once (the arrays are reused every batch)
    p_score, p_idx, p_new = (_lib.ptr(score, ctypes.c_uint64), _lib.ptr(idx, ctypes.c_int64),
                             _lib.ptr(new, ctypes.c_uint8))
    p_queries = _lib.ptr(queries, ctypes.c_uint8)

    def match(staged):
        qp = None if staged else p_queries
        if vts.nranks > 1 and vts.reducer != 'rccl':
            local = np.empty(Q, dtype=np.uint64)
            _lib.check(lib.rs_vt_scan_local(vts._h, Q, qp, _lib.ptr(local, ctypes.c_uint64)))
            glob = np.ascontiguousarray(vts.reducer(local))
            _lib.check(lib.rs_vt_resolve(vts._h, Q, _lib.ptr(glob, ctypes.c_uint64), 0,
                                         p_score, p_idx, p_new))
        else:
            _lib.check(lib.rs_vt_match_batch(vts._h, Q, qp, _lib.RS_VT_FROZEN, p_score, p_idx, p_new))

    match(staged=False)                      # stage the batch in HBM (+ correctness probe)
    hits = src >= 0
    correct = bool(np.all(idx[hits] == src[hits]))

    # Timed region: `steps` distinct query batches, resident in HBM before it starts,
    # matched by one rs_vt_match_stream call (per batch: query forms, scan, RCCL
    # min-allreduce when sharded, key export; one host sync at the end).  Handles
    # reduced on the host (--same-device) run the per-batch loop instead.
    pipeline = 'stream' if (vts.nranks == 1 or vts.reducer == 'rccl') else 'per-batch'
    sbufs, srcs = None, None
    if pipeline == 'stream':
        qs = [queries] + [synthetic.queries(qlib, Q, seed=2 + 1000 * b)[0] for b in range(1, steps)]
        srcs = [src] + [synthetic.queries(qlib, Q, seed=2 + 1000 * b)[1] for b in range(1, steps)]
        sbufs = _lib.DeviceBuffer(Q * queries[0].nbytes * steps, device=d.dev).upload(np.stack(qs))
        del qs
        try:
            # warm-up: untimed passes over the same batches (the first sizes the
            # stream's key buffers, which must not be allocated in the timed region)
            for _ in range(max(1, (warmup + steps - 1) // steps)):
                sidx, _ = vts.match_stream((steps, Q, sbufs))
            correct = correct and bool(np.all(sidx[0][hits] == src[hits]))
        except Exception as e:  # pragma: no cover - recorded, not hidden
            print('rank %d: rs_vt_match_stream failed (%s); per-batch loop' % (d.rank, e),
                  file=sys.stderr)
            pipeline = 'per-batch'
            sbufs.close()
            sbufs = None
            match(staged=False)
    if pipeline == 'per-batch':
        for _ in range(warmup):
            match(staged=True)
    # the timed batches run without the scan's timing events (two stream markers per
    # batch); the scan kernel's duration for the roofline comes from a separate timed pass
    vts.set_timing(False)
    d.barrier()
    t0 = time.perf_counter()
    if pipeline == 'stream':
        sidx, _ = vts.match_stream((steps, Q, sbufs))
    else:
        for _ in range(steps):
            match(staged=True)
    t1 = time.perf_counter()
    d.barrier()
    dt = d.max(t1 - t0)
    if pipeline == 'stream':
        for b in range(steps):
            h = srcs[b] >= 0
            correct = correct and bool(np.all(sidx[b][h] == srcs[b][h]))
        sbufs.close()
        match(staged=False)                  # re-stage one batch for the timed-scan pass
    vts.set_timing(True)
    kernel_ms = []
    for _ in range(steps):
        match(staged=True)
        kernel_ms.append(vts.device_ms())
    # PCIe-inclusive rate (queries uploaded from host memory every batch), not the value
    d.barrier()
    p0 = time.perf_counter()
    npcie = max(3, steps // 4)
    for _ in range(npcie):
        match(staged=False)
    p1 = time.perf_counter()
    d.barrier()
    dtp = d.max(p1 - p0)
    compares = float(total) * Q
    scan_ms = float(np.mean(kernel_ms))
    res = {
        'value': compares * steps / dt,
        'ms_per_step': 1e3 * dt / steps,
        'pcie_inclusive_value': compares * npcie / dtp,
        'scan_ms': scan_ms,
        'kernel': SCAN_KERNELS[vts.scan_form()],
        'compares_per_launch': float(len(range(d.rank, total, n))) * Q,
        'reduce': reduce_kind,
        'pipeline': pipeline,
        'hits_correct': correct,
        'templates_total': total,
    }
    vts.close()
    return res


def pc_roofline(ncell, per_step_kernel_ms):
    alg = 24.0 * ncell            # 3 stencil passes x (read + write) x 4 B
    ach = alg / (per_step_kernel_ms * 1e-3) / 1e9
    return {'bound': 'hbm', 'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': ach / HBM_PEAK_GBS, 'traffic': None,
            'note': '24 B/cell/step algorithmic over the two kernels\' summed HIP-event time'}


def bench_posecell_stress(args, d):
    """configs[3]: the 128x128x72 grid, batched run() steps/s and kernel roofline."""
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in args.pc_stress_shape.split(','))
    net = PoseCellNetwork(shape, device=d.dev)
    net.inject(1, tuple(s // 2 for s in shape))
    n = args.pc_stress_steps
    od = synthetic.odometry(n + 50, seed=0)
    net.run(od[:50])
    d.barrier()
    t0 = time.perf_counter()
    net.run(od[50:50 + n])
    t1 = time.perf_counter()
    d.barrier()
    dt = d.max(t1 - t0)
    nprof = min(n, 200)
    net.set_profiling(True)
    net.run(od[:nprof])
    ex_ms, pi_ms = net.kernel_ms()
    net.set_profiling(False)
    finite = bool(np.isfinite(net.posecells).all())
    form = net.step_form()
    net.close()
    ncell = shape[0] * shape[1] * shape[2]
    return {'shape': list(shape), 'steps_per_s': n / dt, 'us_per_step': 1e6 * dt / n,
            'kernel_us_per_step': {'excite': 1e3 * ex_ms / nprof, 'path': 1e3 * pi_ms / nprof},
            'step_form': form, 'finite': finite,
            'roofline': pc_roofline(ncell, (ex_ms + pi_ms) / nprof)}


def bench_posecells(args, d):
    from pyratslam_amd import PoseCellNetwork, synthetic
    shape = tuple(int(s) for s in args.pc_shape.split(','))
    net = PoseCellNetwork(shape, device=d.dev)
    net.inject(1, tuple(s // 2 for s in shape))
    od = synthetic.odometry(args.pc_warmup + args.pc_steps + args.pc_calls + 64, seed=0)
    net.run(od[:args.pc_warmup])
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
    # kernel durations (HIP events around every launch) on a separate profiled run
    nprof = min(args.pc_steps, 500)
    net.set_profiling(True)
    net.run(od[:nprof])
    ex_ms, pi_ms = net.kernel_ms()
    net.set_profiling(False)
    per_step_kernel_ms = (ex_ms + pi_ms) / nprof
    ncell = shape[0] * shape[1] * shape[2]
    finite = bool(np.isfinite(net.posecells).all())
    form = net.step_form()
    net.close()
    roof = pc_roofline(ncell, per_step_kernel_ms)
    roof['note'] += ('; the 576 KiB volume is L2-resident and the step is launch/latency-bound '
                     'at this size (see pose_cell_stress for configs[3])')
    return {
        'shape': list(shape),
        'steps_per_s': args.pc_steps / dt,
        'update_calls_per_s': args.pc_calls / (c1 - c0),
        'us_per_step': 1e6 * dt / args.pc_steps,
        'kernel_us_per_step': {'excite': 1e3 * ex_ms / nprof, 'path': 1e3 * pi_ms / nprof},
        'replicas': d.world,
        'step_form': form,
        'finite': finite,
        'roofline': roof,
    }


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
    # C / OpenMP: template compares
    n = 0
    t0 = time.perf_counter()
    while n < len(qs) and time.perf_counter() - t0 < budget:
        C.vt_best(lib, qs[n:n + 16])
        n += 16
    dt = time.perf_counter() - t0
    threads = C.threads()
    vt = {'value': T * n / dt, 'unit': 'compares/s', 'cores': threads, 'kind': 'port',
          'sample': '%d queries x %d stored 64x32 u8 templates, oracle/c (C restatement of '
                    'view_templates.py, OpenMP %d threads)' % (n, T, threads)}
    # NumPy, single thread
    n = 0
    t0 = time.perf_counter()
    while n < len(qs) and time.perf_counter() - t0 < budget / 2:
        V.vt_scores_library(lib, qs[n])
        n += 1
    dt = time.perf_counter() - t0
    vt_np = {'value': T * n / dt, 'unit': 'compares/s', 'cores': 1, 'kind': 'port',
             'sample': '%d queries, oracle/view_templates.py (NumPy)' % n}
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
          'sample': '%d updates of a %s grid, oracle/c (C restatement of the three OpenCL '
                    'kernels in float64, 343-tap direct correlation, OpenMP %d threads; host '
                    'control in NumPy)' % (k, shape, threads)}
    k, dt = res['numpy']
    pc_np = {'value': k / dt, 'unit': 'steps/s', 'cores': 1, 'kind': 'port',
             'sample': '%d updates, oracle/posecell.py (NumPy float64)' % k}
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
        vts, reduce_kind = replay.sharded_templates(d, d.dev, gloo=True), 'gloo-host-min'
    elif d.world > 1:
        try:
            vts, reduce_kind = replay.sharded_templates(d, d.dev), 'rccl-allreduce-min-u64'
        except Exception as e:  # pragma: no cover - recorded, not hidden
            print('rank %d: RCCL attach failed (%s); host gloo reduction' % (d.rank, e), file=sys.stderr)
            vts, reduce_kind = replay.sharded_templates(d, d.dev, gloo=True), 'gloo-host-min'
    r = replay.RatslamReplay(device=d.dev, vts=vts)
    d.barrier()
    t0 = time.perf_counter()
    r.replay_events(events)
    dt = d.max(time.perf_counter() - t0)
    res = r.results()
    return {'messages': len(events), 'updates': int(len(res['pc_max'])), 'reduce': reduce_kind,
            'frames': int(len(res['template_index'])), 'templates': int(res['templates']),
            'seconds': dt, 'messages_per_s': len(events) / dt,
            'updates_per_s': len(res['pc_max']) / dt, 'frames_per_s': len(res['template_index']) / dt,
            'note': 'per message: one pose-cell step or one frame match, each a host round trip '
                    '(the node publishes after every step); synthetic stand-in for dataset_10Hz.bag'}


def main():
    args = parse()
    d = Dist(args.gpus)
    # the GPU of this rank; --same-device puts every rank on GPU 0 (a test aid for
    # 1-GPU boxes: RCCL refuses two ranks on one GPU, so the host reducer is used)
    d.dev = 0 if args.same_device else d.local
    tv = bench_templates(args, d)
    lib100 = None
    if args.library_total > 0:
        lib100 = bench_templates(args, d, total=args.library_total, steps=args.library_steps,
                                 warmup=1)
    pc = bench_posecells(args, d)
    pcs = None if args.no_pc_stress else bench_posecell_stress(args, d)
    rp = None if args.no_replay else bench_replay(args, d)
    if d.rank != 0:
        d.close()
        return
    roof = {
        'bound': 'hbm',
        'achieved': BYTES_PER_COMPARE * tv['compares_per_launch'] / (tv['scan_ms'] * 1e-3) / 1e9,
        'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'traffic': None,
    }
    roof['frac'] = roof['achieved'] / roof['peak']
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if (tj.get('templates_per_gpu') == args.templates_per_gpu and tj.get('queries') == args.queries
                    and tj.get('kernel', '').startswith(tv['kernel'])):
                roof['traffic'] = tj.get('hbm_bytes_per_launch')
                roof['traffic_source'] = os.path.relpath(args.traffic_json, ROOT)
                vi = tj.get('valu_insts_per_launch')
                if vi:
                    # the scan is VALU-bound: wave64 VALU issue peaks at one instruction per
                    # 2 cycles per SIMD (1024 SIMDs, 2.4 GHz)
                    ach = vi / (tv['scan_ms'] * 1e-3) / 1e9
                    roof['valu'] = {'insts_per_launch': vi, 'achieved': ach,
                                    'peak': VALU_PEAK_GINSTS, 'unit': 'G wave-instructions/s',
                                    'frac': ach / VALU_PEAK_GINSTS}
        except Exception:
            pass
    # measured HBM bytes of the pose-cell kernels (same PMC passes), per step form
    tj_pc = {}
    if os.path.exists(args.traffic_json):
        try:
            tj_pc = json.load(open(args.traffic_json)).get('pose_cell', {})
        except Exception:
            tj_pc = {}
    for leg in (pc, pcs):
        if leg and leg['step_form'] in tj_pc:
            leg['roofline']['traffic'] = tj_pc[leg['step_form']]['hbm_bytes_per_step']
            leg['roofline']['traffic_kernels'] = tj_pc[leg['step_form']]['kernels']
    roof['note'] = ('achieved = 2,048 algorithmic bytes per compare (SURVEY.md 8(d)) / scan time; '
                    'above the HBM peak because each template is read from HBM once per batch and '
                    'reused from registers by all queries (traffic = measured HBM bytes per launch); '
                    'the kernel is bound by VALU issue, see valu')
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
                        'GPU, %d-query batches resident in HBM' % (args.templates_per_gpu, args.queries),
            'templates_per_gpu': args.templates_per_gpu,
            'templates_total': tv['templates_total'],
            'queries_per_step': args.queries,
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
            'scan_ms_per_launch': lib100['scan_ms'], 'kernel': lib100['kernel'],
            'compares_per_launch_per_gpu': lib100['compares_per_launch'],
            'reduce': lib100['reduce'], 'pipeline': lib100['pipeline'],
            'known_answer_hits_correct': lib100['hits_correct'],
            'pcie_inclusive_compares_per_s': lib100['pcie_inclusive_value']},
        'pose_cell': pc,
        'pose_cell_stress': pcs,
        'replay': rp,
        'template_scan': {'kernel': tv['kernel'], 'kernel_ms_per_launch': tv['scan_ms'],
                          'pipeline': tv['pipeline'],
                          'pcie_inclusive_compares_per_s': tv['pcie_inclusive_value'],
                          'known_answer_hits_correct': tv['hits_correct']},
    }
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
