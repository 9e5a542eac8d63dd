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


def queries_fast(lib, q, seed=2, hit_frac=0.9, max_shift=7, noise=3):
    """``queries`` with the same statistics, vectorised (a different stream of
    draws): the bench's hundreds of distinct 1,024-query batches."""
    rng = np.random.default_rng(seed)
    t, h, w = lib.shape
    hit = rng.random(q) < hit_frac if t > 0 else np.zeros(q, dtype=bool)
    src = np.where(hit, rng.integers(0, max(t, 1), size=q), -1).astype(np.int64)
    shift = rng.integers(-max_shift, max_shift + 1, size=q)
    rows = (np.arange(h)[None, :] - shift[:, None]) % h          # np.roll(x, o, axis=0)
    base = lib[np.maximum(src, 0)[:, None], rows].astype(np.int16)
    base -= rng.integers(0, noise + 1, size=(q, h, w), dtype=np.int16)
    out = np.clip(base, 0, 255).astype(np.uint8)
    miss = ~hit
    out[miss] = rng.integers(0, 256, size=(int(miss.sum()), h, w), dtype=np.uint8)
    return out, src


def panorama(height=256, width=1024, seed=0):
    """A 360-degree scene: a sum of cosines periodic in the azimuth axis (up to 39
    cycles per turn, so a few degrees of heading change the view), scaled to uint8."""
    rng = np.random.default_rng(seed)
    y = np.arange(height)[:, None] / height
    x = np.arange(width)[None, :] / width
    img = np.zeros((height, width))
    for _ in range(24):
        kx = int(rng.integers(1, 40))
        ky = rng.uniform(0.5, 4.0)
        img += rng.uniform(0.3, 1.0) * np.cos(2 * np.pi * (kx * x + ky * y) + rng.uniform(0, 2 * np.pi))
    img = (img - img.min()) / (img.max() - img.min())
    return np.round(img * 255).astype(np.uint8)


def ros_stream(n, seed=0, im_size=(256, 256), odom_hz=10.0):
    """Stand-in for the reference's ``testdata/dataset_10Hz.bag`` (absent,
    .MISSING_LARGE_BLOBS:1): ``n`` odometry messages at ``odom_hz`` and one mono8
    camera frame after each (ros_scenario.py:12-25 publishes both at 10 Hz).

    Twist: linear.x ~ U(0.3, 3) m/s, angular.z ~ U(-1.2, 1.2) rad/s (vtrans <=
    0.3 m, |vrot| <= 0.12 rad per 10 Hz step, ros_simulate.py:159-160), with one
    message in 16 standing still (|v| below the 0.001 filter, :128).  Frames:
    the panorama column window at the integrated heading plus U{0..2} noise, so
    revisited headings give matching views.
    Returns a list of ('odom', t, (vx, vy, vz), (wx, wy, wz)) and
    ('image', t, frame uint8 (H, W)) events in time order.
    """
    rng = np.random.default_rng(seed)
    h, w = im_size
    pano = panorama(h, 4 * w, seed)
    events, heading, t = [], 0.0, 100.0
    for i in range(n):
        if i % 16 == 15:
            vx, wz = 0.0, 0.0005
        else:
            vx, wz = float(rng.uniform(0.3, 3.0)), float(rng.uniform(-1.2, 1.2))
        events.append(('odom', t, (vx, 0.0, 0.0), (0.0, 0.0, wz)))
        heading += wz / odom_hz
        off = int(np.floor((heading / (2 * np.pi)) % 1.0 * pano.shape[1]))
        cols = (off + np.arange(w)) % pano.shape[1]
        frame = pano[:, cols].astype(np.int16) + rng.integers(0, 3, size=(h, w))
        events.append(('image', t + 0.5 / odom_hz, np.clip(frame, 0, 255).astype(np.uint8)))
        t += 1.0 / odom_hz
    return events


def write_ros_bag(path, events, odom_topic='/navbot/odom', image_topic='/navbot/camera/image',
                  compression='none'):
    """Write ``ros_stream`` events as a ROS 1 bag (nav_msgs/Odometry, sensor_msgs/Image)."""
    from . import rosbag
    with rosbag.BagWriter(path, compression=compression) as w:
        for ev in events:
            if ev[0] == 'odom':
                w.write(odom_topic, 'nav_msgs/Odometry', ev[1], rosbag.encode_odometry(ev[1], ev[2], ev[3]))
            else:
                w.write(image_topic, 'sensor_msgs/Image', ev[1], rosbag.encode_image(ev[1], ev[2]))
    return path
