"""Process control plane of the multi-GPU paths (bench.py, the replay,
tools/rccl_check.py), with no PyTorch: one process per GPU, ranks from the
environment (RANK / LOCAL_RANK / WORLD_SIZE, as torch.distributed.run or
``launch.spawn`` set them), and a small TCP star through rank 0 for what the
control plane needs -- barriers, broadcasting the RCCL unique id, the
max-over-ranks time -- plus ``min_keys``, the host fallback reducer of the
sharded template library when RCCL cannot run (several ranks on one GPU).

Rendezvous: rank 0 listens on an ephemeral port of MASTER_ADDR (default
127.0.0.1) and publishes ``port token`` in a file every rank of the job can
name without talking to the others:
  * ``$RS_DIST_DIR/rendezvous`` when the launcher set RS_DIST_DIR (launch.spawn
    makes a fresh directory per job);
  * otherwise ``<tmp>/rs_dist_<MASTER_PORT>_<parent pid>`` -- the ranks of one
    torch.distributed.run job share their parent (the elastic agent).  The agent
    itself holds MASTER_PORT, so the star cannot bind it.
A client proves it read the current file by echoing the token; a stale file
from an earlier job fails the handshake and the client re-reads.  N = 1 opens
no socket at all.
"""
import os
import secrets
import socket
import struct
import tempfile
import time

import numpy as np

_HDR = struct.Struct('<Q')


def _send(sock, payload):
    sock.sendall(_HDR.pack(len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError('control-plane peer closed the connection')
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


def rendezvous_path(env=None):
    env = os.environ if env is None else env
    if env.get('RS_DIST_DIR'):
        return os.path.join(env['RS_DIST_DIR'], 'rendezvous')
    return os.path.join(tempfile.gettempdir(),
                        'rs_dist_%s_%d' % (env.get('MASTER_PORT', '0'), os.getppid()))


class Dist:
    """Control plane of one rank.  ``gpus`` (if given) must equal WORLD_SIZE."""

    def __init__(self, gpus=None, timeout=300.0):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', str(self.rank)))
        if gpus is not None and self.world != gpus:
            raise SystemExit('--gpus %d but WORLD_SIZE=%d: run `python bench.py --gpus N` (it '
                             'launches its own N ranks) or launch N ranks with WORLD_SIZE=N'
                             % (gpus, self.world))
        if not 0 <= self.rank < self.world:
            raise SystemExit('RANK=%d outside WORLD_SIZE=%d' % (self.rank, self.world))
        self.timeout = float(timeout)
        self._peers = {}      # rank 0: rank -> socket
        self._hub = None      # other ranks: socket to rank 0
        self._path = None
        if self.world > 1:
            if self.rank == 0:
                self._serve()
            else:
                self._connect()

    # -- rendezvous --------------------------------------------------------------
    def _serve(self):
        addr = os.environ.get('MASTER_ADDR', '127.0.0.1')
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((addr, 0))
        srv.listen(self.world)
        srv.settimeout(self.timeout)
        token = secrets.token_hex(16)
        self._path = rendezvous_path()
        tmp = self._path + '.%d.tmp' % os.getpid()
        # owner-only from creation: the file holds the job's auth token (a file left
        # world-readable in a shared tempdir would let another local user join)
        fd = os.open(tmp, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o600)
        with os.fdopen(fd, 'w') as f:
            f.write('%d %s\n' % (srv.getsockname()[1], token))
        os.replace(tmp, self._path)
        try:
            while len(self._peers) < self.world - 1:
                conn, _ = srv.accept()
                conn.settimeout(self.timeout)
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                try:
                    tok, rank = _recv(conn).decode().split()
                    rank = int(rank)
                except (ConnectionError, ValueError, OSError):
                    conn.close()
                    continue
                if tok != token or not 0 < rank < self.world or rank in self._peers:
                    conn.close()       # a client that read a stale file, or a duplicate
                    continue
                _send(conn, b'ok')
                self._peers[rank] = conn
        finally:
            srv.close()
            try:
                os.unlink(self._path)
            except OSError:
                pass

    def _connect(self):
        path = rendezvous_path()
        addr = os.environ.get('MASTER_ADDR', '127.0.0.1')
        t_end = time.monotonic() + self.timeout
        while True:
            if time.monotonic() > t_end:
                raise TimeoutError('rank %d: no rank-0 rendezvous at %s within %.0f s'
                                   % (self.rank, path, self.timeout))
            try:
                with open(path) as f:
                    port, token = f.read().split()
                s = socket.create_connection((addr, int(port)), timeout=5.0)
                s.settimeout(self.timeout)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                _send(s, ('%s %d' % (token, self.rank)).encode())
                if _recv(s) == b'ok':
                    self._hub = s
                    return
                s.close()
            except (OSError, ValueError, ConnectionError):
                pass
            time.sleep(0.05)

    # -- collectives over the star -------------------------------------------------
    def _gather(self, payload):
        """rank 0 gets [payload of rank 0, 1, ...]; other ranks get None."""
        if self.world == 1:
            return [payload]
        if self.rank != 0:
            _send(self._hub, payload)
            return None
        return [payload] + [_recv(self._peers[r]) for r in range(1, self.world)]

    def _bcast(self, payload):
        if self.world == 1:
            return payload
        if self.rank == 0:
            for r in range(1, self.world):
                _send(self._peers[r], payload)
            return payload
        return _recv(self._hub)

    def barrier(self):
        self._gather(b'')
        self._bcast(b'')

    def bcast_bytes(self, b):
        """rank 0's bytes on every rank."""
        return self._bcast(bytes(b) if self.rank == 0 else b'')

    def max(self, x):
        """max of a float over the ranks, on every rank."""
        got = self._gather(struct.pack('<d', float(x)))
        out = struct.pack('<d', max(struct.unpack('<d', g)[0] for g in got)) if got else b''
        return struct.unpack('<d', self._bcast(out))[0]

    def min_keys(self, keys):
        """Elementwise unsigned min of uint64 key vectors over the ranks (key =
        score << 32 | index, UINT64_MAX = no template): the host reducer of the
        sharded template library when RCCL is unavailable."""
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        got = self._gather(k.tobytes())
        if got is not None:
            m = np.frombuffer(got[0], dtype=np.uint64).copy()
            for g in got[1:]:
                np.minimum(m, np.frombuffer(g, dtype=np.uint64), out=m)
            out = m.tobytes()
        else:
            out = b''
        return np.frombuffer(self._bcast(out), dtype=np.uint64).copy()

    def close(self):
        for s in list(self._peers.values()) + ([self._hub] if self._hub else []):
            try:
                s.close()
            except OSError:
                pass
        self._peers, self._hub = {}, None


def _selftest():
    """``python -m pyratslam_amd.dist`` under a launcher: exercises every
    collective and prints one JSON line on rank 0 (tests/test_distributed_cpu.py)."""
    import json
    d = Dist()
    d.barrier()
    uid = d.bcast_bytes(b'unique-id-of-rank-0' if d.rank == 0 else None)
    mx = d.max(d.rank + 0.5)
    no_key = np.iinfo(np.uint64).max
    probe = np.array([no_key, 5 + d.rank, (1 << 63) + d.rank, (3 << 32) | (7 - d.rank)], dtype=np.uint64)
    mk = d.min_keys(probe)
    d.barrier()
    if d.rank == 0:
        print(json.dumps({'world': d.world, 'uid': uid.decode(), 'max': mx,
                          'min_keys': [int(v) for v in mk]}), flush=True)
    d.close()


if __name__ == '__main__':
    _selftest()
