"""Build libratslam_hip.so in-tree with hipcc for gfx950 (no JIT cache, no pip).

``python -m pyratslam_amd._build`` or ``__graft_entry__.build()``.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
INCLUDE = os.path.join(ROOT, 'include')
LIB = os.path.join(HERE, 'libratslam_hip.so')
OBJDIR = os.path.join(HERE, 'build')
SOURCES = ['rs_common.cpp', 'posecell.hip', 'view_templates.hip']
# per-source flags: the plane scan's batch takes are single-lane atomics; the
# wave-aggregating atomic optimizer only adds a readfirstlane round trip to them.
# The pose-cell stencils keep scalar FMAs: SLP packing into v_pk_fma_f32 pairs the
# filter taps into register pairs and doubles the VGPRs of the conv_xy passes
# (pc_fused_rows 90 -> 220, pc_path_rows<128> 85 -> 146), halving occupancy.
EXTRA = {'view_templates.hip': ['-mllvm', '-amdgpu-atomic-optimizer-strategy=None'],
         # pc_step_halo's first 9 arguments (the union image's addresses, the partial sums) preloaded
         # into scalar registers (posecell.hip, before pc_step_halo)
         'posecell.hip': ['-fno-slp-vectorize', '-mllvm', '-amdgpu-kernarg-preload-count=9']}
HEADERS = [os.path.join(CSRC, 'rs_common.h'), os.path.join(INCLUDE, 'ratslam_abi.h')]
ARCH = os.environ.get('PYRATSLAM_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')


def _newer(src, dst):
    return not os.path.exists(dst) or os.path.getmtime(src) > os.path.getmtime(dst)


def build(verbose=False, force=False):
    """Compile every HIP/C++ source of the library and link it; returns the .so path."""
    os.makedirs(OBJDIR, exist_ok=True)
    hdr_mtime = max(os.path.getmtime(h) for h in HEADERS + [os.path.abspath(__file__)])
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJDIR, src.rsplit('.', 1)[0] + '.o')
        objs.append(obj)
        stale = force or _newer(path, obj) or (os.path.exists(obj) and os.path.getmtime(obj) < hdr_mtime)
        if not stale:
            continue
        lang = ['-x', 'hip'] if src.endswith('.hip') else []
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-Wall',
               '-Wno-unused-function', f'-I{INCLUDE}', f'-I{CSRC}', *lang, *EXTRA.get(src, []), '-c', path, '-o', obj]
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    if force or any(_newer(o, LIB) for o in objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB, *objs,
               '-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib']
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == '__main__':
    print(build(verbose=True, force='--force' in sys.argv))
