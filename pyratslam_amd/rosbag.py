"""Minimal ROS 1 bag (format 2.0) reader and writer, pure Python.

The reference's config 5 replays ``testdata/dataset_10Hz.bag`` through its ROS
node (``ros_simulate.py:82-83`` subscribes ``navbot/odom`` and
``navbot/camera/image``).  rospy/rosbag are not installed here and the bag is
absent (``.MISSING_LARGE_BLOBS:1``), so this module reads bags directly and
writes synthetic ones for the replay tests:

* records: ``<u32 header_len><header><u32 data_len><data>``; header fields are
  ``<u32 len>name=value``; ops 0x03 bag header (padded to 4096 bytes), 0x05
  chunk (``none`` or ``bz2``; ``lz4`` is reported, not decoded), 0x07
  connection, 0x02 message, 0x04 index, 0x06 chunk info;
* messages (ROS 1 serialisation, little endian): ``nav_msgs/Odometry``,
  ``geometry_msgs/Twist``, ``sensor_msgs/Image`` -- the types the node reads.
"""
import bz2
import io
import struct
from collections import namedtuple

import numpy as np

MAGIC = b'#ROSBAG V2.0\n'
OP_MSG, OP_BAG_HEADER, OP_INDEX, OP_CHUNK, OP_CHUNK_INFO, OP_CONNECTION = 2, 3, 4, 5, 6, 7

Message = namedtuple('Message', 'topic type time data')   # time: float seconds
Twist = namedtuple('Twist', 'linear angular')              # 3-tuples of float
Image = namedtuple('Image', 'stamp height width encoding is_bigendian step data')

# type -> (md5sum, message definition) written into connection headers
MSG_TYPES = {
    'nav_msgs/Odometry': ('cd5e73d190d741a2f92e81eda573aca7',
                          'Header header\nstring child_frame_id\n'
                          'geometry_msgs/PoseWithCovariance pose\n'
                          'geometry_msgs/TwistWithCovariance twist\n'),
    'geometry_msgs/Twist': ('9f195f881246fdfa2798d1d3eebca84a',
                            'Vector3  linear\nVector3  angular\n'),
    'sensor_msgs/Image': ('060021388200f6f0f447d0fcd9c64743',
                          'Header header\nuint32 height\nuint32 width\nstring encoding\n'
                          'uint8 is_bigendian\nuint32 step\nuint8[] data\n'),
}


class BagError(ValueError):
    pass


# ----------------------------------------------------------------------------
# record layer
# ----------------------------------------------------------------------------
def _fields(header):
    out, i = {}, 0
    while i < len(header):
        (n,) = struct.unpack_from('<I', header, i)
        name, _, value = header[i + 4:i + 4 + n].partition(b'=')
        out[name.decode()] = value
        i += 4 + n
    return out


def _header(**fields):
    parts = []
    for name, value in fields.items():
        if isinstance(value, str):
            value = value.encode()
        f = name.encode() + b'=' + value
        parts.append(struct.pack('<I', len(f)) + f)
    return b''.join(parts)


def _records(buf, pos=0, end=None):
    end = len(buf) if end is None else end
    while pos < end:
        if pos + 4 > end:
            raise BagError('truncated record at byte %d' % pos)
        (hl,) = struct.unpack_from('<I', buf, pos)
        h = _fields(buf[pos + 4:pos + 4 + hl])
        (dl,) = struct.unpack_from('<I', buf, pos + 4 + hl)
        d0 = pos + 8 + hl
        if d0 + dl > end:
            raise BagError('truncated record data at byte %d' % pos)
        yield pos, h, buf[d0:d0 + dl]
        pos = d0 + dl


def _time(b):
    sec, nsec = struct.unpack('<II', b)
    return sec + nsec * 1e-9


def _pack_time(t):
    sec = int(np.floor(t))
    nsec = int(round((t - sec) * 1e9))
    if nsec >= 1000000000:
        sec, nsec = sec + 1, nsec - 1000000000
    return struct.pack('<II', sec, nsec)


def read_bag(path, topics=None):
    """Messages of a bag in file order (chunk by chunk), as ``Message`` tuples with
    the raw serialised data.  ``topics``: optional set of topic names (a leading
    '/' is ignored when matching)."""
    with open(path, 'rb') as f:
        buf = f.read()
    if not buf.startswith(MAGIC):
        raise BagError('%s: not a ROS bag 2.0 file' % path)
    want = None if topics is None else {t.lstrip('/') for t in topics}
    conns = {}
    out = []

    def visit(h, d):
        op = h['op'][0]
        if op == OP_CONNECTION:
            c = _fields(d)
            conns[struct.unpack('<I', h['conn'])[0]] = (h['topic'].decode(), c['type'].decode())
        elif op == OP_MSG:
            topic, typ = conns[struct.unpack('<I', h['conn'])[0]]
            if want is None or topic.lstrip('/') in want:
                out.append(Message(topic, typ, _time(h['time']), d))

    for _, h, d in _records(buf, len(MAGIC)):
        if h['op'][0] == OP_CHUNK:
            comp = h['compression'].decode()
            if comp == 'bz2':
                d = bz2.decompress(d)
            elif comp != 'none':
                raise BagError('chunk compression %r is not supported (none, bz2)' % comp)
            for _, hh, dd in _records(d):
                visit(hh, dd)
        else:   # top-level connection records (index section); stray messages
            visit(h, d)
    return out


class BagWriter:
    """Writes a bag of one or more chunks (compression ``none`` or ``bz2``) with
    connection, index and chunk-info records, readable by rosbag."""

    def __init__(self, path, compression='none', chunk_messages=256):
        if compression not in ('none', 'bz2'):
            raise ValueError('compression must be none or bz2')
        self.path, self.compression, self.chunk_messages = path, compression, chunk_messages
        self.conns = {}          # topic -> (id, type)
        self.pending = []        # (conn, time, data)
        self.chunks = []         # (pos, start, end, {conn: count})
        self.f = open(path, 'wb')
        self.f.write(MAGIC)
        self.header_pos = self.f.tell()
        self._write_bag_header(0, 0, 0)

    def _write_record(self, f, header, data):
        f.write(struct.pack('<I', len(header)) + header + struct.pack('<I', len(data)) + data)

    def _write_bag_header(self, index_pos, conn_count, chunk_count):
        h = _header(op=bytes([OP_BAG_HEADER]), index_pos=struct.pack('<Q', index_pos),
                    conn_count=struct.pack('<I', conn_count), chunk_count=struct.pack('<I', chunk_count))
        pad = 4096 - (4 + len(h) + 4)
        self._write_record(self.f, h, b' ' * pad)

    def _conn_record(self, topic):
        cid, typ = self.conns[topic]
        md5, definition = MSG_TYPES.get(typ, ('*', ''))
        data = _header(topic=topic, type=typ, md5sum=md5, message_definition=definition)
        return _header(op=bytes([OP_CONNECTION]), conn=struct.pack('<I', cid), topic=topic), data

    def write(self, topic, typ, t, data):
        if topic not in self.conns:
            self.conns[topic] = (len(self.conns), typ)
        self.pending.append((topic, float(t), bytes(data)))
        if len(self.pending) >= self.chunk_messages:
            self._flush()

    def _flush(self):
        if not self.pending:
            return
        body = io.BytesIO()
        index = {}
        seen = set()
        for topic, t, data in self.pending:
            cid = self.conns[topic][0]
            if topic not in seen:
                seen.add(topic)
                self._write_record(body, *self._conn_record(topic))
            index.setdefault(cid, []).append((t, body.tell()))
            h = _header(op=bytes([OP_MSG]), conn=struct.pack('<I', cid), time=_pack_time(t))
            self._write_record(body, h, data)
        raw = body.getvalue()
        payload = bz2.compress(raw) if self.compression == 'bz2' else raw
        pos = self.f.tell()
        h = _header(op=bytes([OP_CHUNK]), compression=self.compression, size=struct.pack('<I', len(raw)))
        self._write_record(self.f, h, payload)
        for cid, entries in index.items():
            hi = _header(op=bytes([OP_INDEX]), ver=struct.pack('<I', 1), conn=struct.pack('<I', cid),
                         count=struct.pack('<I', len(entries)))
            self._write_record(self.f, hi, b''.join(_pack_time(t) + struct.pack('<I', o)
                                                    for t, o in entries))
        times = [t for _, t, _ in self.pending]
        self.chunks.append((pos, min(times), max(times), {c: len(e) for c, e in index.items()}))
        self.pending = []

    def close(self):
        self._flush()
        index_pos = self.f.tell()
        for topic in self.conns:
            self._write_record(self.f, *self._conn_record(topic))
        for pos, t0, t1, counts in self.chunks:
            h = _header(op=bytes([OP_CHUNK_INFO]), ver=struct.pack('<I', 1),
                        chunk_pos=struct.pack('<Q', pos), start_time=_pack_time(t0),
                        end_time=_pack_time(t1), count=struct.pack('<I', len(counts)))
            self._write_record(self.f, h, b''.join(struct.pack('<II', c, n) for c, n in counts.items()))
        self.f.seek(self.header_pos)
        self._write_bag_header(index_pos, len(self.conns), len(self.chunks))
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ----------------------------------------------------------------------------
# message layer (ROS 1 serialisation)
# ----------------------------------------------------------------------------
class _Reader:
    def __init__(self, b):
        self.b, self.i = b, 0

    def take(self, fmt):
        v = struct.unpack_from(fmt, self.b, self.i)
        self.i += struct.calcsize(fmt)
        return v

    def string(self):
        (n,) = self.take('<I')
        s = self.b[self.i:self.i + n]
        self.i += n
        return s

    def header(self):
        _seq, sec, nsec = self.take('<III')
        self.string()  # frame_id
        return sec + nsec * 1e-9


def _header_bytes(stamp, frame_id=b''):
    sec = int(np.floor(stamp))
    nsec = int(round((stamp - sec) * 1e9)) % 1000000000
    return struct.pack('<III', 0, sec, nsec) + struct.pack('<I', len(frame_id)) + frame_id


def decode_odometry_twist(data):
    """``nav_msgs/Odometry`` -> its ``twist.twist`` (what odom_callback reads,
    ros_simulate.py:125-126)."""
    r = _Reader(data)
    r.header()
    r.string()                       # child_frame_id
    r.take('<7d')                    # pose.pose: position, orientation
    r.take('<36d')                   # pose.covariance
    lin = r.take('<3d')
    ang = r.take('<3d')
    return Twist(lin, ang)


def encode_odometry(stamp, linear, angular, frame_id=b'odom', child=b'base_link'):
    body = _header_bytes(stamp, frame_id) + struct.pack('<I', len(child)) + child
    body += struct.pack('<7d', 0, 0, 0, 0, 0, 0, 1) + struct.pack('<36d', *([0.0] * 36))
    body += struct.pack('<3d', *linear) + struct.pack('<3d', *angular) + struct.pack('<36d', *([0.0] * 36))
    return body


def decode_twist(data):
    v = struct.unpack('<6d', data[:48])
    return Twist(v[:3], v[3:])


def decode_image(data):
    r = _Reader(data)
    stamp = r.header()
    height, width = r.take('<II')
    encoding = r.string().decode()
    (big,) = r.take('<B')
    (step,) = r.take('<I')
    pix = r.string()
    return Image(stamp, height, width, encoding, big, step, pix)


def encode_image(stamp, pixels, encoding='mono8', frame_id=b'camera'):
    a = np.ascontiguousarray(pixels)
    h, w = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    body = _header_bytes(stamp, frame_id) + struct.pack('<II', h, w)
    enc = encoding.encode()
    body += struct.pack('<I', len(enc)) + enc + struct.pack('<BI', 0, w * ch * a.itemsize)
    raw = a.tobytes()
    return body + struct.pack('<I', len(raw)) + raw


def image_to_mono8(img):
    """``bridge.imgmsg_to_cv(data, "mono8")`` then ``asarray`` (ros_simulate.py:100-101):
    (height, width) uint8.  mono8 passes through; 8-bit colour converts as
    cv_bridge does (OpenCV cvtColor RGB2GRAY on 8-bit data): the ITU-R 601 luma
    weights in 14-bit fixed point, (4899 R + 9617 G + 1868 B + 2^13) >> 14."""
    buf = np.frombuffer(img.data, dtype=np.uint8)
    if img.encoding in ('mono8', '8UC1'):
        rows = buf.reshape(img.height, img.step)[:, :img.width]
        return np.ascontiguousarray(rows)
    if img.encoding in ('rgb8', 'bgr8', 'rgba8', 'bgra8'):
        ch = 4 if img.encoding.endswith('a8') else 3
        px = buf.reshape(img.height, img.step)[:, :img.width * ch].reshape(img.height, img.width, ch)
        r, g, b = (px[..., 0], px[..., 1], px[..., 2]) if img.encoding.startswith('rgb') else \
                  (px[..., 2], px[..., 1], px[..., 0])
        y = (4899 * r.astype(np.uint32) + 9617 * g.astype(np.uint32) + 1868 * b.astype(np.uint32)
             + (1 << 13)) >> 14
        return y.astype(np.uint8)
    raise BagError('image encoding %r is not supported for mono8 conversion' % img.encoding)
