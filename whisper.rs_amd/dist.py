"""Host-side rendezvous for one-process-per-GPU runs (torchrun-compatible env).

The data-path collective is RCCL (wmi_dist_gather_tokens over xGMI).  What
RCCL needs before it exists — every rank agreeing on one ncclUniqueId — and
the benchmark's host bookkeeping (barrier, max-over-ranks of a timing) go
through this small TCP star centred on rank 0, reading RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT as torch.distributed.run exports them.  No torch
import: the benchmark process must load exactly one HIP runtime (ours).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

_PORT_OFFSET = 23  # torchrun's own TCPStore holds MASTER_PORT itself
_PORT_TRIES = 8     # hub ports MASTER_PORT + 23 + 97 k, k < 8: the first one rank 0 can bind
_PORT_STRIDE = 97
_MAX_MSG = 1 << 24  # messages are ids, timings and small token lists
_MAGIC = b"wmi-rdv1"
_CONFIRM = b"wmi-rdv1-ok"
_HS_HUB = 10.0   # rank 0's handshake deadline per connection (hello + confirm together)
_HS_PEER = 15.0  # a peer's wait for rank 0's ack: longer than _HS_HUB


def _alive(sock) -> bool:
    """A registered peer's socket still open (a zero-timeout peek: EOF or an
    error means its process went away; no data pending means it waits)."""
    t = sock.gettimeout()
    try:
        sock.setblocking(False)
        return sock.recv(1, socket.MSG_PEEK) != b""
    except BlockingIOError:
        return True
    except OSError:
        return False
    finally:
        sock.settimeout(t)


def _recv_by(sock, deadline: float) -> bytes:
    sock.settimeout(max(0.01, deadline - time.time()))
    return _recv(sock)


def hub_ports(master_port: int):
    """Candidate ports of the rank-0 hub.  Rank 0 binds the first free one;
    peers try them in order and keep the one whose listener answers the
    rendezvous handshake (a foreign program on a candidate port is skipped)."""
    return [master_port + _PORT_OFFSET + _PORT_STRIDE * k for k in range(_PORT_TRIES)]


def _enc(obj) -> bytes:
    """JSON with bytes as {"b": hex}: the payloads are plain data (an RCCL
    unique id, floats, None, small int lists), so nothing a peer sends is ever
    executed (no pickle)."""
    def conv(o):
        if isinstance(o, (bytes, bytearray)):
            return {"b": bytes(o).hex()}
        if isinstance(o, (list, tuple)):
            return [conv(x) for x in o]
        if o is None or isinstance(o, (bool, int, float, str)):
            return o
        raise TypeError(f"dist: cannot send {type(o).__name__}")
    return json.dumps(conv(obj)).encode()


def _dec(data: bytes):
    def conv(o):
        if isinstance(o, dict):
            if set(o) != {"b"} or not isinstance(o["b"], str):
                raise ValueError("dist: malformed message")
            return bytes.fromhex(o["b"])
        if isinstance(o, list):
            return [conv(x) for x in o]
        return o
    return conv(json.loads(data.decode()))


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))


def _send(sock, data: bytes):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv(sock) -> bytes:
    hdr = b""
    while len(hdr) < 8:
        chunk = sock.recv(8 - len(hdr))
        if not chunk:
            raise ConnectionError("peer closed")
        hdr += chunk
    (n,) = struct.unpack("<Q", hdr)
    if n > _MAX_MSG:
        raise ConnectionError(f"dist: message of {n} bytes refused")
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


class Group:
    """All-gather of small plain-data objects over a TCP star (rank 0 hub)."""

    def __init__(self, rank: int, world: int, addr: str | None = None, port: int | None = None,
                 timeout: float = 300.0):
        """port: the hub's port, bound as given (tests); by default the first
        bindable port of hub_ports(MASTER_PORT).  Every socket operation and
        the whole rendezvous are bounded by `timeout` seconds."""
        self.rank, self.world = rank, world
        self.peers = []
        self.sock = None
        if world == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        ports = [port] if port else hub_ports(int(os.environ.get("MASTER_PORT", "29500")))
        hello = _MAGIC + struct.pack("<ii", world, ports[0])
        if rank == 0:
            srv = None
            for p in ports:  # bind check: the first free candidate
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                try:
                    s.bind((addr, p))
                except OSError:
                    s.close()
                    continue
                srv = s
                break
            if srv is None:
                raise OSError(f"dist: none of the hub ports {ports} can be bound on {addr}")
            srv.listen(world)
            deadline = time.time() + timeout
            peers = {}
            try:
                while len(peers) < world - 1:
                    left = deadline - time.time()
                    if left <= 0:
                        raise TimeoutError(f"dist: {world - 1 - len(peers)} rank(s) did not join within {timeout} s")
                    srv.settimeout(left)
                    c, _ = srv.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    # one deadline for the whole handshake of this connection
                    # (hello + confirm): rank 0 is held at most _HS_HUB by any
                    # one connection, less than a peer waits for its ack
                    hs = time.time() + min(timeout, _HS_HUB)
                    try:
                        msg = _recv_by(c, hs)
                        r = struct.unpack("<i", msg[-4:])[0] if len(msg) == len(hello) + 4 and msg[:-4] == hello \
                            else -1
                        if 1 <= r < world:
                            # ack, then the peer's confirmation: a connection
                            # its peer abandoned (it gave up waiting and
                            # reconnected) fails here instead of being kept
                            _send(c, hello)
                            if _recv_by(c, hs) != _CONFIRM:
                                r = -1
                    except (ConnectionError, OSError):
                        r = -1
                    if not 1 <= r < world:  # foreign, out of range or abandoned: not a peer
                        c.close()
                        continue
                    if r in peers:
                        # the same rank again: a reconnect replaces a peer whose
                        # socket is dead; a second live process claiming the
                        # rank (a misconfiguration) is refused, the first kept
                        if _alive(peers[r]):
                            c.close()
                            continue
                        peers[r].close()
                    c.settimeout(timeout)
                    peers[r] = c
            except BaseException:
                for c in peers.values():
                    c.close()
                raise
            finally:
                srv.close()
            self.peers = [peers[r] for r in range(1, world)]
        else:
            deadline = time.time() + timeout
            k = 0
            while True:
                p = ports[k % len(ports)]
                k += 1
                s = None
                try:
                    s = socket.create_connection((addr, p), timeout=5)
                    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    s.settimeout(_HS_PEER)  # (rank 0 may be busy with another connection for up to _HS_HUB)
                    _send(s, hello + struct.pack("<i", rank))
                    if _recv(s) == hello:
                        _send(s, _CONFIRM)
                        break
                    s.close()
                except OSError:  # (ConnectionError, socket.timeout are OSErrors)
                    if s is not None:
                        s.close()
                if time.time() > deadline:
                    raise TimeoutError(f"dist: rank {rank} found no rendezvous on {addr}:{ports} within {timeout} s")
                if k % len(ports) == 0:
                    time.sleep(0.2)
            s.settimeout(timeout)
            self.sock = s

    def all_gather(self, obj):
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            objs = [obj] + [_dec(_recv(p)) for p in self.peers]
            blob = _enc(objs)
            for p in self.peers:
                _send(p, blob)
            return _dec(blob)
        _send(self.sock, _enc(obj))
        return _dec(_recv(self.sock))

    def broadcast(self, obj, root: int = 0):
        return self.all_gather(obj if self.rank == root else None)[root]

    def barrier(self):
        self.all_gather(None)

    def max(self, x: float) -> float:
        return max(self.all_gather(x))

    def close(self):
        for p in self.peers:
            p.close()
        if self.sock:
            self.sock.close()
