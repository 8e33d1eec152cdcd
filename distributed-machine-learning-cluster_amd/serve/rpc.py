"""Minimal Python client for the node's RPC framing (csrc/control/rpc.cpp):
request = u32 length + u16 method + payload; response = u32 length + status
byte (0 ok, 1 handler error, 2 unknown method) + body. Used by tests to
talk to members and leaders directly (hostile-peer and fuzz tests)."""
from __future__ import annotations

import socket
import struct

# method ids (csrc/control/sdfs.h)
L_GET, L_GET_VERSIONS, L_PUT, L_DELETE, L_LS, L_TRAIN, L_PREDICT, L_JOBS, L_ALIVE, L_STATE = range(1, 11)
M_GET_LATEST_VERSION, M_RECEIVE, M_PREDICT, M_FETCH, M_READ_CHUNK, M_DELETE_FILE, M_LOAD_MODEL, M_INFO = range(20, 28)


def s(x: str | bytes) -> bytes:
    b = x.encode() if isinstance(x, str) else x
    return struct.pack("<I", len(b)) + b


def call(host: str, port: int, method: int, payload: bytes = b"", timeout: float = 10.0) -> tuple[int, bytes]:
    with socket.create_connection((host, port), timeout=timeout) as c:
        body = struct.pack("<H", method) + payload
        c.sendall(struct.pack("<I", len(body)) + body)
        hdr = _recv(c, 4)
        (n,) = struct.unpack("<I", hdr)
        resp = _recv(c, n)
    return resp[0], resp[1:]


def send_raw(host: str, port: int, frame: bytes, timeout: float = 2.0) -> bytes | None:
    """Send arbitrary bytes (a possibly malformed frame); return whatever comes back."""
    try:
        with socket.create_connection((host, port), timeout=timeout) as c:
            c.sendall(frame)
            c.shutdown(socket.SHUT_WR)
            out = b""
            while True:
                chunk = c.recv(65536)
                if not chunk:
                    return out
                out += chunk
    except OSError:
        return None


def _recv(c: socket.socket, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = c.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("connection closed")
        buf += chunk
    return buf
