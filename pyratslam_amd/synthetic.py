"""Synthetic workloads of SURVEY.md section 8(d) (no datasets ship with the
reference: its ROS bag is absent, .MISSING_LARGE_BLOBS:1).

* odometry: vtrans ~ U(0, 0.6) m/step, vrot ~ U(-0.15, 0.15) rad/step -- keeps
  the activity packet alive and (almost surely) off the +0.5 LUT edge;
* template library: (T, H, W) uint8 ~ U[0, 255];
* queries: 90 % a stored template rolled by o ~ U{-7..7} rows minus one-sided
  noise in [0, 3] (known answer: that template), 10 % fresh random frames.
"""
import numpy as np


def odometry(n, seed=0, vtrans_max=0.6, vrot_max=0.15):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(0.0, vtrans_max, n), rng.uniform(-vrot_max, vrot_max, n)], axis=1)


def library(t, h=64, w=32, seed=1, first=0):
    """Templates [first, first + t) of the deterministic library stream `seed`
    (generated in blocks of 1024 so any slice is reproducible on its own)."""
    out = np.empty((t, h, w), dtype=np.uint8)
    blk = 1024
    i = first
    while i < first + t:
        b = i // blk
        rng = np.random.default_rng([seed, b])
        block = rng.integers(0, 256, size=(blk, h, w), dtype=np.uint8)
        lo = i - b * blk
        n = min(blk - lo, first + t - i)
        out[i - first:i - first + n] = block[lo:lo + n]
        i += n
    return out


def queries(lib, q, seed=2, hit_frac=0.9, max_shift=7, noise=3):
    """Returns (queries uint8 (q, H, W), source template index or -1)."""
    rng = np.random.default_rng(seed)
    t, h, w = lib.shape
    out = np.empty((q, h, w), dtype=np.uint8)
    src = np.full(q, -1, dtype=np.int64)
    for i in range(q):
        if t > 0 and rng.random() < hit_frac:
            j = int(rng.integers(0, t))
            o = int(rng.integers(-max_shift, max_shift + 1))
            base = np.roll(lib[j], o, axis=0).astype(np.int16)
            out[i] = np.clip(base - rng.integers(0, noise + 1, size=(h, w)), 0, 255).astype(np.uint8)
            src[i] = j
        else:
            out[i] = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    return out, src
