"""The C-ABI library builds for gfx950, loads, and exports exactly what
include/ratslam_abi.h declares (no device calls: runs without a GPU)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT
from pyratslam_amd import _build, _lib

HEADER = os.path.join(ROOT, 'include', 'ratslam_abi.h')


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(rs_\w+)\s*\(', text)))


@pytest.fixture(scope='module')
def lib():
    _build.build()
    return _lib.load()


def test_header_declares_the_api():
    syms = declared_symbols()
    for s in ('rs_pc_create', 'rs_pc_update', 'rs_pc_run', 'rs_vt_create', 'rs_vt_match',
              'rs_vt_match_batch', 'rs_vt_attach_comm', 'rs_last_error'):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(['nm', '-D', '--defined-only', _lib.LIB_PATH], text=True)
    exported = set(re.findall(r' T (rs_\w+)$', out, flags=re.M))
    missing = set(declared_symbols()) - exported
    assert not missing, missing


def test_binding_covers_every_symbol(lib):
    assert set(_lib.SIGNATURES) == set(declared_symbols())
    for name in declared_symbols():
        assert getattr(lib, name) is not None


def test_library_is_gfx950_code_object(lib):
    out = subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-readelf', '--notes', _lib.LIB_PATH],
                                  text=True, stderr=subprocess.STDOUT)
    offload = subprocess.run(['/opt/rocm/bin/roc-obj-ls', _lib.LIB_PATH], capture_output=True,
                             text=True)
    assert 'gfx950' in (offload.stdout + out) or b'gfx950' in open(_lib.LIB_PATH, 'rb').read()


def test_version_and_error_state_without_gpu(lib):
    assert lib.rs_version() == 100
    assert isinstance(lib.rs_last_error(), bytes)
    assert lib.rs_device_count() >= 0


def test_no_cpu_fallback_without_device(lib):
    if lib.rs_device_count() > 0:
        pytest.skip('a GPU is visible')
    from pyratslam_amd import PoseCellNetwork, ViewTemplates
    with pytest.raises(_lib.HipLibraryError):
        PoseCellNetwork((16, 16, 8))
    with pytest.raises(_lib.HipLibraryError):
        ViewTemplates((0, 64), (0, 64), 2, 2, 64, 64, 45000)


def test_status_codes_map_to_reference_exceptions(lib):
    for code, exc in ((_lib.RS_ERR_ARG, ValueError), (_lib.RS_ERR_TYPE, TypeError),
                      (_lib.RS_ERR_LUT_KEY, KeyError), (_lib.RS_ERR_NOMEM, MemoryError),
                      (_lib.RS_ERR_HIP, RuntimeError)):
        with pytest.raises(exc):
            _lib.check(code)
