import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an AMD GPU (MI355X) and libratslam_hip.so')


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'))


def dense_state(case, step):
    """Reference state after `step` (0-based) of a golden pose-cell trajectory."""
    shape = tuple(int(s) for s in case['shape'])
    off = int(case['nnz'][:step].sum())
    n = int(case['nnz'][step])
    out = np.zeros(int(np.prod(shape)))
    out[case['coo_idx'][off:off + n]] = case['coo_val'][off:off + n]
    return out.reshape(shape)


@pytest.fixture(scope='session')
def golden():
    return load_golden


def nonfinite_state(case, i):
    """pc_nonfinite: the reference's state after the ValueError of vtrans case i."""
    shape = tuple(int(s) for s in case['shape'])
    off = int(case['vtrans_nnz'][:i].sum())
    n = int(case['vtrans_nnz'][i])
    out = np.zeros(int(np.prod(shape)))
    out[case['vtrans_coo_idx'][off:off + n]] = case['vtrans_coo_val'][off:off + n]
    return out.reshape(shape)
