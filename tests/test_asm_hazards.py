"""Static regression guard for the class of bug behind round 1's illegal-address
fault: no vector-memory load's destination register may be
read or overwritten before an s_waitcnt retires the load.  Each HIP source is
compiled to gfx950 device assembly and checked with tools/asm_load_hazards.py.
CPU only (hipcc cross-compiles); skipped where hipcc is absent."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
sys.path.insert(0, os.path.join(ROOT, 'tools'))


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which('hipcc')), reason='hipcc absent')
@pytest.mark.parametrize('src', ['posecell.hip', 'view_templates.hip'])
def test_no_load_register_hazards(tmp_path, src):
    import asm_load_hazards as H
    out = tmp_path / (src + '.s')
    subprocess.check_call([HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC',
                           '-I' + os.path.join(ROOT, 'include'),
                           '-I' + os.path.join(ROOT, 'pyratslam_amd', 'csrc'), '-x', 'hip', '-S',
                           '--cuda-device-only', os.path.join(ROOT, 'pyratslam_amd', 'csrc', src),
                           '-o', str(out)], stderr=subprocess.DEVNULL)
    lines = out.read_text().splitlines()
    bad = {}
    for name, body in H.kernels(lines):
        hits = H.scan(name, body, asm_only=False)
        if hits:
            bad[name] = hits[:3]
    assert not bad, bad


def test_checker_flags_a_reused_load_destination():
    """Positive control, the round-1 pattern in miniature: an asm load into v89
    still in flight when v89 is rewritten as the high half of an address."""
    import asm_load_hazards as H
    listing = '''_Zkernel:
\t;;#ASMSTART
\tglobal_load_dword v89, v47, s[84:85]
\t;;#ASMEND
\tv_ashrrev_i32_e32 v89, 31, v88
\tv_lshl_add_u64 v[2:3], v[88:89], 2, s[36:37]
\ts_waitcnt vmcnt(0)
\tglobal_store_dword v[2:3], v5, off
\ts_endpgm
.Lfunc_end0:
'''.splitlines()
    (name, body), = list(H.kernels(listing))
    hits = H.scan(name, body, asm_only=True)
    kinds = sorted(k for _, k, _, _, _ in hits)
    assert kinds == ['read', 'write'], hits


def test_checker_lds_dma_has_no_register_destination():
    """global_load_lds reads its address VGPRs at issue and writes none, so they may
    be reused at once; it still counts in vmcnt for the loads issued before it."""
    import asm_load_hazards as H
    listing = '''_Zkernel:
\tglobal_load_dword v7, v[2:3], off
\tglobal_load_lds_dwordx4 v[80:81], off
\tv_min_i32_e32 v80, s50, v98
\ts_waitcnt vmcnt(1)
\tv_add_u32_e32 v9, v7, v7
\ts_endpgm
.Lfunc_end0:
'''.splitlines()
    (name, body), = list(H.kernels(listing))
    assert H.scan(name, body, asm_only=False) == []
    # with vmcnt(2) the plain load may still be in flight: its destination read is flagged
    body2 = [ln.replace('vmcnt(1)', 'vmcnt(2)') for ln in body]
    assert [k for _, k, _, _, _ in H.scan(name, body2, asm_only=False)] == ['read']
