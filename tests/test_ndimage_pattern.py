"""The reference's own oracle pattern (sandbox/opencl_test2.py:306-334): its
convolution kernels equal scipy.ndimage wrap-mode correlation -- the commented
CPU formulations in the model itself (posecell_network.py:335 for the 3-D
excitation, :290-291 for the per-layer xy filter, :311 for the theta filter).
Here the oracle's restatements of those kernels (oracle/posecell.py) are held to
the same pattern: exactly equal on integer-valued images with integer taps (as
opencl_test2.py:334 asserts with array_equal), and within float64 rounding with
the real DoG filters."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import posecell as P


def _int_image(shape, seed):
    return np.random.default_rng(seed).integers(0, 10, shape).astype(np.float64)


@pytest.mark.parametrize('shape', [(8, 9, 7), (12, 10, 18), (7, 7, 7)])
def test_conv3d_equals_ndimage_correlate_wrap(shape):
    img = _int_image(shape, 1)
    k_int = np.random.default_rng(2).integers(-3, 4, (7, 7, 7)).astype(np.float64)
    assert np.array_equal(P.conv3d_wrap(img, k_int), ndimage.correlate(img, k_int, mode='wrap'))
    k3 = P.dog_kernel_3d()
    a, b = P.conv3d_wrap(img, k3), ndimage.correlate(img, k3, mode='wrap')
    assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max()


@pytest.mark.parametrize('shape', [(9, 11, 5), (16, 16, 6)])
def test_conv_xy_equals_per_layer_ndimage_plus_shift(shape):
    X, Y, TH = shape
    img = _int_image(shape, 3)
    rng = np.random.default_rng(4)
    filters = rng.integers(-2, 3, (7, 7, TH)).astype(np.float64)
    ox = rng.integers(-4, 5, TH)
    oy = rng.integers(-4, 5, TH)
    got = P.conv_xy_shift(img, ox, oy, filters)
    for k in range(TH):
        # posecell_network.py:290-291 per layer, then the path-integration shift
        ref = ndimage.correlate(img[:, :, k], filters[:, :, k], mode='wrap')
        ref = np.roll(ref, (-int(ox[k]), -int(oy[k])), axis=(0, 1))
        assert np.array_equal(got[:, :, k], ref), k


@pytest.mark.parametrize('th', [7, 18, 36])
def test_conv_z_equals_correlate1d_wrap(th):
    img = _int_image((5, 6, th), 5)
    zf_int = np.arange(-3, 4, dtype=np.float64)
    assert np.array_equal(P.conv_z_wrap(img, zf_int),
                          ndimage.correlate1d(img, zf_int, axis=2, mode='wrap'))
    zf = P.dog_offset_1d(1)
    a, b = P.conv_z_wrap(img, zf), ndimage.correlate1d(img, zf, axis=2, mode='wrap')
    assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max()
