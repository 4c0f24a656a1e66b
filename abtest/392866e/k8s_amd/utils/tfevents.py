"""Minimal TensorBoard event-file writer (no tensorflow / tensorboard package).

The TensorBoard sidecar the operator deploys (`/root/reference/pkg/trainer/
tensorboard.go:140-177`, `charts/tensorboard`) reads ``events.out.tfevents.*``
files from ``logDir``. This writes them byte-compatibly: TFRecord framing
(uint64 length, masked CRC32C of the length, payload, masked CRC32C of the
payload) around hand-encoded ``Event`` protos (wall_time, step, file_version
or ``Summary{Value{tag, simple_value}}``).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Optional

_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: Optional[str] = None,
                 scalars: Optional[Dict[str, float]] = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time)
    if step:
        ev += _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_field(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
            summ += _len_field(1, val)
        ev += _len_field(5, summ)
    return ev


def frame(record: bytes) -> bytes:
    n = struct.pack("<Q", len(record))
    return n + struct.pack("<I", masked_crc(n)) + record + struct.pack("<I", masked_crc(record))


def read_records(path: str):
    """Parse a TFRecord file back (verifying both CRCs); yields payloads."""
    with open(path, "rb") as f:
        while True:
            h = f.read(12)
            if len(h) < 12:
                return
            n, lc = struct.unpack("<QI", h)
            if masked_crc(h[:8]) != lc:
                raise ValueError("length crc mismatch")
            data = f.read(n)
            (dc,) = struct.unpack("<I", f.read(4))
            if masked_crc(data) != dc:
                raise ValueError("data crc mismatch")
            yield data


class EventWriter:
    def __init__(self, logdir: str, suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s%s" % (int(time.time()), socket.gethostname(), suffix)
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "ab")
        self.f.write(frame(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self.f.flush()

    def scalars(self, step: int, values: Dict[str, float]):
        self.f.write(frame(encode_event(time.time(), step, scalars=values)))

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()
