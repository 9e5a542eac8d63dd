#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE itself (build container only).

Runs ``/root/reference/ratslam/{posecell_network,convolution,view_templates,experience_map}.py``
under Python 3 with the minimum shims needed to reproduce their Python-2
behaviour, and with the reference's own OpenCL kernel text (rendered by its own
``Convolution.set_text``) compiled as host C by gcc (``-ffp-contract=off``) in
place of PyOpenCL.  Nothing from the reference is written to the repository:
only the resulting arrays, as ``tests/golden/*.npz``.

Shims (each is the smallest change that restores the Python-2 meaning):
  * ``builtins.xrange`` -> range yielding ``Py2Int`` (``/`` floors like Py2 ints),
    so ``build_diff_gaussian_set_2d`` (posecell_network.py:55-58) and
    ``ViewTemplates.__init__`` (view_templates.py:44-54) see integer division;
  * ``builtins.math``: numpy-1.x's ``from numpy import *`` exported ``math``;
  * module ``max``/``min`` reset to builtins (numpy-2's star export shadows
    them; numpy 1.x removed them from ``__all__``), posecell_network.py:98;
  * ``ceil`` in posecell_network returns ``int`` for scalars (Py2-era numpy
    accepted float buffer shapes, convolution.py:662-665);
  * ``raise E, msg`` -> ``raise E if 1 else msg`` in convolution.py (syntax only);
  * fake ``mako.template.Template`` (``${name}`` substitution) and fake
    ``pyopencl`` whose ``Program.build`` compiles the kernel text with gcc and
    runs each NDRange as a host triple loop.

Usage: python tests/golden/gen_golden.py [--out tests/golden]
"""
import argparse
import builtins
import ctypes
import hashlib
import math
import os
import re
import subprocess
import sys
import tempfile
import types

import numpy as np

REF = '/root/reference/ratslam'


# ----------------------------------------------------------------------------
# Python-2 integer semantics
# ----------------------------------------------------------------------------
class Py2Int(int):
    """int whose true division floors, like Python-2 int / int."""

    def __truediv__(self, other):
        if isinstance(other, int):
            return Py2Int(int(self) // int(other))
        return int(self) / other

    def __rtruediv__(self, other):
        if isinstance(other, int):
            return Py2Int(int(other) // int(self))
        return other / int(self)


class Py2IntArray(np.ndarray):
    """integer ndarray whose ``/`` floors (numpy under Python 2)."""

    def __truediv__(self, other):
        return np.floor_divide(self, other)


def py2_xrange(*args):
    return (Py2Int(v) for v in range(*args))


# ----------------------------------------------------------------------------
# Fake mako + pyopencl (kernel text compiled as host C)
# ----------------------------------------------------------------------------
class FakeTemplate:
    def __init__(self, text, output_encoding=None, **kw):
        self.text = text
        self.enc = output_encoding

    def render(self, **conf):
        out = re.sub(r'\$\{(\w+)\}', lambda m: str(conf[m.group(1)]), self.text)
        return out.encode(self.enc) if self.enc else out


_LIB_CACHE = {}
_BUILD_DIR = tempfile.mkdtemp(prefix='ratslam_ref_')
_SIG_RE = re.compile(r'__kernel\s+void\s+(\w+)\s*\(([^)]*)\)', re.S)


def _compile_kernels(text):
    if isinstance(text, bytes):
        text = text.decode()
    key = hashlib.sha1(text.encode()).hexdigest()
    if key in _LIB_CACHE:
        return _LIB_CACHE[key]
    body = text.replace('\\\n', ' ')
    wrappers = []
    kernels = {}
    for name, params in _SIG_RE.findall(body):
        plist = [p.strip() for p in params.replace('\n', ' ').split(',') if p.strip()]
        args, names, kinds = [], [], []
        for p in plist:
            p = p.replace('__global', '').strip()
            m = re.match(r'(.*?)(\w+)$', p)
            ctype_s, pname = m.group(1).strip(), m.group(2)
            args.append(f'{ctype_s} {pname}')
            names.append(pname)
            kinds.append('ptr' if '*' in ctype_s else 'int')
        wrappers.append(
            f'void run_{name}({", ".join(args)}, unsigned g0, unsigned g1, unsigned g2) {{\n'
            f'  for (unsigned a = 0; a < g0; a++) for (unsigned b = 0; b < g1; b++)\n'
            f'  for (unsigned c = 0; c < g2; c++) {{ __gid[0]=a; __gid[1]=b; __gid[2]=c;\n'
            f'    {name}({", ".join(names)}); }}\n}}\n')
        kernels[name] = kinds
    prelude = ('static unsigned __gid[3];\n#define __kernel static\n#define __global\n'
               '#define get_global_id(d) (__gid[d])\n')
    src = os.path.join(_BUILD_DIR, f'k_{key}.c')
    lib = os.path.join(_BUILD_DIR, f'k_{key}.so')
    with open(src, 'w') as f:
        f.write(prelude + body + '\n' + '\n'.join(wrappers))
    subprocess.check_call(['gcc', '-O2', '-ffp-contract=off', '-shared', '-fPIC', '-w',
                           '-o', lib, src])
    handle = ctypes.CDLL(lib)
    _LIB_CACHE[key] = (handle, kernels)
    return _LIB_CACHE[key]


class _Buffer:
    def __init__(self, ctx, flags, size=None, hostbuf=None):
        if hostbuf is not None:
            self.data = np.frombuffer(np.ascontiguousarray(hostbuf).tobytes(), dtype=np.uint8).copy()
        else:
            self.data = np.zeros(int(size), dtype=np.uint8)


class _Event:
    def wait(self):
        return None


class _Kernel:
    def __init__(self, fn, kinds):
        self.fn, self.kinds = fn, kinds

    def __call__(self, queue, gsize, lsize, *args):
        cargs = []
        for kind, a in zip(self.kinds, args):
            if kind == 'ptr':
                cargs.append(ctypes.c_void_p(a.data.ctypes.data))
            else:
                cargs.append(ctypes.c_int(int(a)))
        g = list(gsize) + [1] * (3 - len(gsize))
        self.fn(*cargs, ctypes.c_uint(g[0]), ctypes.c_uint(g[1]), ctypes.c_uint(g[2]))
        return _Event()


class _Program:
    def __init__(self, ctx, text):
        self.text = text

    def build(self):
        self.lib, self.kernels = _compile_kernels(self.text)
        return self

    def __getattr__(self, name):
        if name in ('lib', 'kernels', 'text'):
            raise AttributeError(name)
        return _Kernel(getattr(self.lib, 'run_' + name), self.kernels[name])


def _enqueue_read_buffer(queue, buf, out):
    flat = out.reshape(-1).view(np.uint8)
    flat[:] = buf.data[:flat.size]
    return _Event()


def install_fakes():
    cl = types.ModuleType('pyopencl')
    cl.create_some_context = lambda *a, **k: object()
    cl.CommandQueue = lambda ctx, *a, **k: object()
    cl.mem_flags = types.SimpleNamespace(READ_ONLY=1, WRITE_ONLY=2, READ_WRITE=4, COPY_HOST_PTR=8)
    cl.Buffer = _Buffer
    cl.Program = _Program
    cl.enqueue_read_buffer = _enqueue_read_buffer
    sys.modules['pyopencl'] = cl
    mako = types.ModuleType('mako')
    tmpl = types.ModuleType('mako.template')
    tmpl.Template = FakeTemplate
    mako.template = tmpl
    sys.modules['mako'] = mako
    sys.modules['mako.template'] = tmpl
    builtins.xrange = py2_xrange
    builtins.math = math


def load_reference():
    """Import the reference modules with the shims above."""
    install_fakes()
    src = open(os.path.join(REF, 'convolution.py')).read()
    src = re.sub(r'raise\s+(\w+)\s*,', r'raise \1 if 1 else ', src)
    conv = types.ModuleType('convolution')
    conv.__file__ = os.path.join(REF, 'convolution.py')
    exec(compile(src, conv.__file__, 'exec'), conv.__dict__)
    sys.modules['convolution'] = conv
    sys.path.insert(0, REF)
    import posecell_network as pn   # noqa: E402
    import view_templates as vt     # noqa: E402
    pn.max, pn.min = builtins.max, builtins.min
    vt.max, vt.min = builtins.max, builtins.min
    pn.ceil = lambda x: int(np.ceil(x)) if np.ndim(x) == 0 else np.ceil(x)
    vt.arange = lambda n: np.arange(n).view(Py2IntArray)
    return pn, vt


# ----------------------------------------------------------------------------
# Scenarios
# ----------------------------------------------------------------------------
def coo(p):
    idx = np.flatnonzero(p)
    return idx.astype(np.int64), p.ravel()[idx]


def run_posecell(pn, shape, odom, inject_loc=None):
    net = pn.PoseCellNetwork(shape)
    loc = inject_loc or tuple(int(math.floor(s / 2)) for s in shape)
    net.inject(1, loc)
    maxes, nnz, idxs, vals, totals = [], [], [], [], []
    for v in odom:
        net.update((float(v[0]), float(v[1])))
        maxes.append(net.max_pc)
        i, x = coo(net.posecells)
        nnz.append(len(i))
        idxs.append(i)
        vals.append(x)
    return {
        'shape': np.array(shape, dtype=np.int64),
        'inject': np.array(loc, dtype=np.int64),
        'odom': np.asarray(odom, dtype=np.float64),
        'max_pc': np.array(maxes, dtype=np.int64),
        'nnz': np.array(nnz, dtype=np.int64),
        'coo_idx': np.concatenate(idxs),
        'coo_val': np.concatenate(vals),
    }


def gen_kernels(pn, out):
    net = pn.PoseCellNetwork((16, 16, 8))
    lut = net.filter_dict_2d
    keys = sorted(lut.keys())
    one_d = {o: net.diff_gaussian_offset_1d(pn.PC_E_SIGMA, pn.PC_I_SIGMA, size=7, origin=o)
             for o in range(-4, 5)}
    np.savez_compressed(
        os.path.join(out, 'kernels.npz'),
        kernel_3d=net.kernel_3d,
        kernel_2d=net.kernel_2d,
        kernel_1d=net.kernel_1d,
        kernel_1d_sep=net.kernel_1d_sep,
        lut_keys=np.array(keys, dtype=np.int64),
        lut_filters=np.stack([lut[k] for k in keys]),
        f1d_origins=np.arange(-4, 5),
        f1d=np.stack([one_d[o] for o in range(-4, 5)]),
        f2d_origin0=net.diff_gaussian_offset_2d(pn.PC_E_SIGMA, pn.PC_I_SIGMA, shape=(7, 7), origin=(0, 0)),
    )


def gen_posecell(pn, out):
    rng = np.random.default_rng(0)
    cases = {}
    # synthetic odometry; seeds 0..2 at 32x32x18
    for seed in range(3):
        r = np.random.default_rng(seed)
        odom = np.stack([r.uniform(0, 0.6, 40), r.uniform(-0.15, 0.15, 40)], axis=1)
        cases[f'pc32_s{seed}'] = run_posecell(pn, (32, 32, 18), odom)
    r = np.random.default_rng(0)
    odom = np.stack([r.uniform(0, 0.6, 12), r.uniform(-0.15, 0.15, 12)], axis=1)
    cases['pc64_s0'] = run_posecell(pn, (64, 64, 36), odom)
    # the ROS node's grid (ros_simulate.py:31), odometry at 10 Hz-scaled magnitudes
    r = np.random.default_rng(3)
    odom = np.stack([r.uniform(0, 0.3, 30), r.uniform(-0.3, 0.3, 30)], axis=1)
    cases['pc_ros21'] = run_posecell(pn, (21, 21, 36), odom)
    # simulate.py:36-41 scenario (vtrans 3 m, vrot pi/4 on steps 4..8) on its grid
    data = np.zeros((40, 2))
    data[:, 0] = 3
    data[4:9, 1] = np.pi / 4
    cases['pc_simulate'] = run_posecell(pn, (50, 50, 10), data)
    # non-cubic grid, off-centre injection
    r = np.random.default_rng(4)
    odom = np.stack([r.uniform(0, 0.6, 20), r.uniform(-0.15, 0.15, 20)], axis=1)
    cases['pc_ragged'] = run_posecell(pn, (24, 40, 12), odom, inject_loc=(3, 37, 11))
    for name, c in cases.items():
        np.savez_compressed(os.path.join(out, f'{name}.npz'), **c)
    # the +0.5 LUT KeyError: vtrans = 0.1 m -> 0.5 cell
    net = pn.PoseCellNetwork((32, 32, 18))
    net.inject(1, (16, 16, 9))
    try:
        net.update((0.1, 0.0))
        raised = ''
    except KeyError as e:
        raised = repr(e.args[0])
    np.savez_compressed(os.path.join(out, 'pc_keyerror.npz'),
                        shape=np.array((32, 32, 18)), odom=np.array([[0.1, 0.0]]),
                        raised=np.array(raised))
    del rng


def gen_templates(vt, out):
    # per-pair scores: uint8 (wrapping) and float (true SAD), H in {32, 64}
    rng = np.random.default_rng(1)
    pairs_u8, pairs_f = [], []
    for h, w in ((64, 32), (32, 32), (24, 20)):
        a = rng.integers(0, 256, size=(40, h, w), dtype=np.uint8)
        b = rng.integers(0, 256, size=(40, h, w), dtype=np.uint8)
        # half of the pairs: b is a shifted, one-sided-noisy copy of a
        for i in range(20):
            sh = int(rng.integers(-7, 8))
            b[i] = np.clip(np.roll(a[i], sh, axis=0).astype(int) - rng.integers(0, 4, (h, w)), 0, 255)
        s = np.array([vt.ViewTemplate(0, 0, 0, 0, a[i]).match(b[i]) for i in range(40)])
        pairs_u8.append((a, b, s.astype(np.uint64)))
        af, bf = a.astype(np.float64), b.astype(np.float64)
        sf = np.array([vt.ViewTemplate(0, 0, 0, 0, af[i]).match(bf[i]) for i in range(40)])
        pairs_f.append((af, bf, sf))
    np.savez_compressed(
        os.path.join(out, 'vt_pairs.npz'),
        **{f'u8_{i}_a': p[0] for i, p in enumerate(pairs_u8)},
        **{f'u8_{i}_b': p[1] for i, p in enumerate(pairs_u8)},
        **{f'u8_{i}_score': p[2] for i, p in enumerate(pairs_u8)},
        **{f'f64_{i}_score': p[2] for i, p in enumerate(pairs_f)},
    )

    # library evolution through the unmodified ViewTemplates.match (:63-75)
    def trace(name, im, x_range, y_range, step, thr, n_queries, seed, max_shift):
        r = np.random.default_rng(seed)
        vts = vt.ViewTemplates(x_range=(x_range[0], x_range[1]), y_range=(y_range[0], y_range[1]),
                               x_step=Py2Int(step), y_step=Py2Int(step),
                               im_x=im, im_y=im, match_threshold=thr)
        vts.shape = tuple(int(s) for s in vts.shape)
        vts.mask = np.asarray(vts.mask, dtype=bool).view(np.ndarray)
        # first sight of a base is stored as-is; later sights are shifted copies
        # minus one-sided noise (no uint8 wrap at the true offset), some with
        # heavy noise so scores straddle the threshold; 25 % fresh frames miss
        bases = r.integers(0, 256, size=(max(4, n_queries // 6), im, im), dtype=np.uint8)
        seen = set()
        images = np.empty((n_queries, im, im), dtype=np.uint8)
        for i in range(n_queries):
            if r.random() < 0.75:
                b = int(r.integers(0, len(bases)))
                if b not in seen:
                    images[i] = bases[b]
                    seen.add(b)
                    continue
                sh = 2 * int(r.integers(-max_shift, max_shift + 1))  # even: keeps the subsample grid
                amp = 4 if r.random() < 0.7 else int(r.integers(40, 80))
                noisy = np.roll(bases[b], sh, axis=0).astype(int) - r.integers(0, amp, (im, im))
                images[i] = np.clip(noisy, 0, 255).astype(np.uint8)
            else:
                images[i] = r.integers(0, 256, size=(im, im), dtype=np.uint8)
        pcs = r.integers(0, 21, size=(n_queries, 3))
        idx, count = [], []
        for i in range(n_queries):
            m = vts.match(images[i], int(pcs[i, 0]), int(pcs[i, 1]), int(pcs[i, 2]))
            idx.append(m.get_index())
            count.append(len(vts.templates))
        np.savez_compressed(
            os.path.join(out, f'{name}.npz'),
            queries=np.stack([im_[vts.mask].reshape(vts.shape) for im_ in images]),
            pcs=pcs, index=np.array(idx), count=np.array(count),
            mask=vts.mask, shape=np.array(vts.shape),
            params=np.array([x_range[0], x_range[1], y_range[0], y_range[1], step, step, im, im, thr]),
            templates=np.stack([t.template for t in vts.templates]),
            locations=np.array([t.location() for t in vts.templates]))

    # ROS configuration (ros_simulate.py:32-40): 256x256 mono8, 32x32 templates
    trace('vt_trace_ros', 256, (32, 96), (32, 96), 2, 45000, 200, 5, 7)
    # bench geometry: 64x32 templates (x span 128, y span 64, step 2) from 160x160 frames
    trace('vt_trace_64x32', 160, (16, 144), (16, 80), 2, 45000, 300, 6, 3)


def gen_float_pairs(vt, out):
    """ViewTemplate.match / ViewTemplates.match on float frames (view_templates.py:
    16-28, 63-75): no uint8 wrap, numpy's own float arithmetic and summation order.
    Non-integer values, float64 and float32, H in {64, 32, 24}; plus a library
    trace through the unmodified ViewTemplates.match with float64 frames."""
    rng = np.random.default_rng(11)
    arrays = {}
    for i, (h, w) in enumerate(((64, 32), (32, 32), (24, 20))):
        for dt, tag in ((np.float64, 'f64'), (np.float32, 'f32')):
            a = (rng.random((16, h, w)) * 255).astype(dt)
            b = (rng.random((16, h, w)) * 255).astype(dt)
            for j in range(8):   # half: shifted noisy copies (scores near the minimum)
                sh = int(rng.integers(-7, 8))
                b[j] = (np.roll(a[j], sh, axis=0) + rng.normal(0, 3, (h, w))).astype(dt)
            s = np.array([vt.ViewTemplate(0, 0, 0, 0, a[j]).match(b[j]) for j in range(16)])
            assert s.dtype == dt, (s.dtype, dt)
            arrays.update({f'{tag}_{i}_a': a, f'{tag}_{i}_b': b, f'{tag}_{i}_score': s})
    # float64 frames normalised to [0, 1] (a camera pipeline that scales), ROS geometry
    r = np.random.default_rng(12)
    vts = vt.ViewTemplates(x_range=(32, 96), y_range=(32, 96), x_step=Py2Int(2), y_step=Py2Int(2),
                           im_x=256, im_y=256, match_threshold=45000 / 255.0)
    vts.shape = tuple(int(s) for s in vts.shape)
    vts.mask = np.asarray(vts.mask, dtype=bool).view(np.ndarray)
    bases = r.random((10, 256, 256))
    frames, idx = [], []
    for k in range(60):
        if r.random() < 0.75:
            f = np.roll(bases[int(r.integers(0, 10))], 2 * int(r.integers(-5, 6)), axis=0)
            f = f + r.normal(0, 0.01 if r.random() < 0.7 else 0.2, f.shape)
        else:
            f = r.random((256, 256))
        frames.append(f)
        idx.append(vts.match(f, k % 21, (3 * k) % 21, (5 * k) % 36).get_index())
    arrays.update(trace_queries=np.stack([f[vts.mask].reshape(vts.shape) for f in frames]),
                  trace_index=np.array(idx), trace_threshold=np.array(45000 / 255.0),
                  trace_templates=np.stack([t.template for t in vts.templates]))
    np.savez_compressed(os.path.join(out, 'vt_pairs_float.npz'), **arrays)
    print('float pairs: %d templates in the float trace' % len(vts.templates))


def gen_ros_replay(pn, vt, out, n=120, seed=0):
    """Config 5 end to end with the reference's own classes: PoseCellNetwork,
    ViewTemplates and ExperienceMap (experience_map.py, imported unmodified)
    driven through RatslamRos's callback logic (ros_simulate.py:98-162, restated
    in pyratslam_amd.replay because rospy/cv are absent) over the synthetic
    stand-in for the absent dataset_10Hz.bag (pyratslam_amd.synthetic.ros_stream)."""
    import experience_map as em_ref   # noqa: E402  (REF is on sys.path)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, root)
    from pyratslam_amd import replay, synthetic
    pcn = pn.PoseCellNetwork(replay.POSE_SIZE)
    vts = vt.ViewTemplates(x_range=replay.X_RANGE, y_range=replay.Y_RANGE, x_step=Py2Int(replay.X_STEP),
                           y_step=Py2Int(replay.Y_STEP), im_x=replay.IM_SIZE[0], im_y=replay.IM_SIZE[1],
                           match_threshold=replay.MATCH_THRESHOLD)
    vts.shape = tuple(int(s) for s in vts.shape)
    vts.mask = np.asarray(vts.mask, dtype=bool).view(np.ndarray)
    r = replay.RatslamReplay(pcn=pcn, vts=vts, em=em_ref.ExperienceMap(), batch=False)
    events = synthetic.ros_stream(n, seed=seed)
    r.replay_events(events)
    res = r.results()
    np.savez_compressed(os.path.join(out, 'ros_replay.npz'), n=np.array(n), seed=np.array(seed),
                        pc_max=res['pc_max'], em_points=res['em_points'],
                        template_index=res['template_index'], templates=np.array(res['templates']),
                        final_state_coo_idx=coo(pcn.posecells)[0], final_state_coo_val=coo(pcn.posecells)[1])
    print('ros_replay: %d updates, %d frames, %d templates' % (len(res['pc_max']),
                                                                len(res['template_index']), res['templates']))


def gen_death(pn, out):
    """Network death: a rotation whose theta origin lies
    beyond the 7-tap window (posecell_network.py:304-308; vrot = pi/4 at TH = 36
    is origin floor(4.5 + .5) = 5) zeroes the whole volume; the dead steps after it
    take the total == 0 branch (no normalisation, :343-345) and get_pc_max of an
    all-zero volume is the first cell (:317-319); a second inject revives it.
    Per grid: `live` normal steps, the killing step, `dead` normal steps, then
    inject(1, revive) and `after` more normal steps."""
    for name, shape, vrot_kill, revive in (('pc_death64', (64, 64, 36), np.pi / 4, (5, 60, 3)),
                                           ('pc_death32', (32, 32, 18), np.pi / 2, (30, 2, 17))):
        r = np.random.default_rng(7)
        live, dead, after = 6, 4, 6
        n = live + 1 + dead + after
        odom = np.stack([r.uniform(0, 0.6, n), r.uniform(-0.15, 0.15, n)], axis=1)
        odom[live] = (0.25, vrot_kill)
        net = pn.PoseCellNetwork(shape)
        loc = tuple(int(math.floor(s / 2)) for s in shape)
        net.inject(1, loc)
        revive_at = live + 1 + dead          # inject before this step
        maxes, nnz, idxs, vals, totals, getmax = [], [], [], [], [], []
        for s, v in enumerate(odom):
            if s == revive_at:
                net.inject(1, revive)
            net.update((float(v[0]), float(v[1])))
            maxes.append(net.max_pc)
            getmax.append(net.get_pc_max())
            i, x = coo(net.posecells)
            nnz.append(len(i))
            idxs.append(i)
            vals.append(x)
            totals.append(float(np.sum(net.posecells)))
        assert all(nnz[s] == 0 for s in range(live, revive_at)), nnz
        np.savez_compressed(os.path.join(out, f'{name}.npz'),
                            shape=np.array(shape, dtype=np.int64), inject=np.array(loc, dtype=np.int64),
                            odom=odom, max_pc=np.array(maxes, dtype=np.int64),
                            get_pc_max=np.array(getmax, dtype=np.int64), nnz=np.array(nnz, dtype=np.int64),
                            coo_idx=np.concatenate(idxs), coo_val=np.concatenate(vals),
                            totals=np.array(totals), kill_step=np.int64(live),
                            revive_step=np.int64(revive_at), revive=np.array(revive, dtype=np.int64))


class _Py2Math(types.ModuleType):
    """``math`` with Python 2's floor on non-finite arguments: Python 2's math.floor
    returned a float, so a NaN or infinite argument came back as it was, where
    Python 3's raises (posecell_network.py:304, the theta origin of a NaN or infinite
    vrot).  Finite arguments floor as before."""
    def __init__(self):
        super().__init__('math')
        for k in dir(math):
            if not k.startswith('__') and k != 'floor':
                setattr(self, k, getattr(math, k))

    @staticmethod
    def floor(x):
        if isinstance(x, (float, np.floating)) and not math.isfinite(x):
            return x
        return math.floor(x)


def gen_nonfinite(pn, out):
    """Non-finite odometry, run by the reference: a NaN or
    infinite vrot raises nothing and its all-NaN theta filter leaves a NaN volume for
    good (peak: numpy's first NaN, (0, 0, 0)); a NaN or infinite vtrans raises
    ValueError at the LUT lookup (int() of a NaN residual, :246-249) after steps 1-4,
    whose state is stored.  With the Python 2 floor of the theta origin above."""
    saved = builtins.math
    builtins.math = _Py2Math()
    try:
        shape, loc = (32, 32, 18), (16, 16, 9)
        arrays = {'shape': np.array(shape, dtype=np.int64), 'inject': np.array(loc, dtype=np.int64)}
        vr_cases = [float('nan'), float('-inf')]
        vr_max, vr_nan = [], []
        for vr in vr_cases:
            net = pn.PoseCellNetwork(shape)
            net.inject(1, loc)
            maxes, alln = [], []
            for v in ((0.2, 0.01), (0.3, vr), (0.2, 0.0), (0.25, 0.1)):
                net.update(v)
                maxes.append(net.max_pc)
                alln.append(bool(np.isnan(net.posecells).all()))
            vr_max.append(maxes)
            vr_nan.append(alln)
        arrays.update(vrot=np.array(vr_cases), vrot_odom_other=np.array([[0.2, 0.01], [0.3, 0.0], [0.2, 0.0],
                                                                           [0.25, 0.1]]),
                      vrot_max_pc=np.array(vr_max, dtype=np.int64), vrot_all_nan=np.array(vr_nan))
        vt_cases = [float('nan'), float('inf')]
        raised, idxs, vals, nnz, pre = [], [], [], [], []
        for vt in vt_cases:
            net = pn.PoseCellNetwork(shape)
            net.inject(1, loc)
            net.update((0.2, 0.01))
            pre.append(net.max_pc)
            try:
                net.update((vt, 0.0))
                raised.append('')
            except ValueError as e:
                raised.append(type(e).__name__)
            i, x = coo(net.posecells)
            idxs.append(i)
            vals.append(x)
            nnz.append(len(i))
        arrays.update(vtrans=np.array(vt_cases), vtrans_raised=np.array(raised),
                      vtrans_pre_max_pc=np.array(pre, dtype=np.int64), vtrans_nnz=np.array(nnz, dtype=np.int64),
                      vtrans_coo_idx=np.concatenate(idxs), vtrans_coo_val=np.concatenate(vals))
        np.savez_compressed(os.path.join(out, 'pc_nonfinite.npz'), **arrays)
    finally:
        builtins.math = saved


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument('--only', choices=['kernels', 'posecell', 'templates', 'float_pairs',
                                       'ros_replay', 'death', 'nonfinite'])
    args = ap.parse_args()
    pn, vt = load_reference()
    if args.only in (None, 'kernels'):
        gen_kernels(pn, args.out)
    if args.only in (None, 'posecell'):
        gen_posecell(pn, args.out)
    if args.only in (None, 'templates'):
        gen_templates(vt, args.out)
    if args.only in (None, 'float_pairs'):
        gen_float_pairs(vt, args.out)
    if args.only in (None, 'ros_replay'):
        gen_ros_replay(pn, vt, args.out)
    if args.only in (None, 'death'):
        gen_death(pn, args.out)
    if args.only in (None, 'nonfinite'):
        gen_nonfinite(pn, args.out)
    print('golden vectors written to', args.out)


if __name__ == '__main__':
    main()
