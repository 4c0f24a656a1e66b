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
    """Parse a TFRecord file back (verifying both CRCs); yields payloads. A record still being written (short
    read) ends the iteration."""
    with open(path, "rb") as f:
        while True:
            h = f.read(12)
            if len(h) < 12:
                return
            n, lc = struct.unpack("<QI", h)
            if masked_crc(h[:8]) != lc:
                raise ValueError("length crc mismatch")
            data = f.read(n)
            tail = f.read(4)
            if len(data) < n or len(tail) < 4:
                return
            (dc,) = struct.unpack("<I", tail)
            if masked_crc(data) != dc:
                raise ValueError("data crc mismatch")
            yield data


def _read_varint(b: bytes, i: int):
    n = shift = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        if not c & 0x80:
            return n, i
        shift += 7


def _fields(b: bytes):
    """(field number, wire type, value) of one protobuf message: varint -> int, fixed64/32 -> raw bytes,
    length-delimited -> bytes."""
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, w = key >> 3, key & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError("unsupported wire type %d" % w)
        yield f, w, v


def decode_event(data: bytes) -> dict:
    """Event{wall_time=1 double, step=2 int64, file_version=3 string, summary=5 Summary{value=1 repeated
    Value{tag=1 string, simple_value=2 float}}} -> {"wall_time", "step", "file_version"?, "scalars"}."""
    ev = {"wall_time": 0.0, "step": 0, "scalars": {}}
    for f, w, v in _fields(data):
        if f == 1 and w == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif f == 2 and w == 0:
            ev["step"] = v
        elif f == 3 and w == 2:
            ev["file_version"] = v.decode()
        elif f == 5 and w == 2:
            for sf, sw, sv in _fields(v):
                if sf != 1 or sw != 2:
                    continue
                tag, val = None, None
                for vf, vw, vv in _fields(sv):
                    if vf == 1 and vw == 2:
                        tag = vv.decode()
                    elif vf == 2 and vw == 5:
                        val = struct.unpack("<f", vv)[0]
                if tag is not None and val is not None:
                    ev["scalars"][tag] = val
    return ev


def read_events(path: str):
    """Decoded events of one file (CRC-checked); stops cleanly at a partially written tail record."""
    try:
        for rec in read_records(path):
            yield decode_event(rec)
    except (ValueError, struct.error):
        return


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
