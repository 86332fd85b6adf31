"""Minimal TensorBoard event writer (the ``tensorboard`` package is not
installed in this image) + a JSONL metrics log.

Reproduces what the reference writes through ``SummaryWriter("imagenet_FR")``
(``imagenet.py:362-363, 405-421``): ``add_scalars(main_tag, {k: v}, step)``
creates one sub-writer per key in ``<logdir>/<main_tag>_<key>`` holding the
scalar under tag ``main_tag`` ([torch] utils/tensorboard/writer.py:424-434),
``add_scalar`` writes into the root run.

File format: TFRecord framing (uint64 length, masked crc32c(length), payload,
masked crc32c(payload)) of hand-encoded ``Event`` protobufs
(wall_time=1:double, step=2:int64, file_version=3:string,
summary=5:Summary{value=1:Value{tag=1:string, simple_value=2:float}}).
"""

from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Dict, Optional

# ------------------------------------------------------------------ crc32c
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf
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
    hdr = struct.pack("<Q", len(record))
    return hdr + struct.pack("<I", masked_crc(hdr)) + record + struct.pack("<I", masked_crc(record))


def read_events(path: str):
    """Parse an event file back into (wall_time, step, {tag: value}) tuples (tests)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (hc,) = struct.unpack_from("<I", data, i + 8)
        assert hc == masked_crc(data[i:i + 8]), "header crc"
        rec = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack_from("<I", data, i + 12 + n)
        assert dc == masked_crc(rec), "data crc"
        out.append(_decode_event(rec))
        i += 12 + n + 4
    return out


def _read_varint(b: bytes, i: int):
    shift = val = 0
    while True:
        c = b[i]
        i += 1
        val |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return val, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(w)
        yield f, w, v


def _decode_event(rec: bytes):
    wt, step, sc = 0.0, 0, {}
    for f, w, v in _fields(rec):
        if f == 1:
            wt = struct.unpack("<d", v)[0]
        elif f == 2:
            step = v
        elif f == 5:
            for f2, _, val in _fields(v):
                if f2 == 1:
                    tag, sv = None, None
                    for f3, _, x in _fields(val):
                        if f3 == 1:
                            tag = x.decode()
                        elif f3 == 2:
                            sv = struct.unpack("<f", x)[0]
                    sc[tag] = sv
    return wt, step, sc


class _EventFile:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "ab")
        self.f.write(frame(encode_event(time.time(), file_version="brain.Event:2")))
        self.f.flush()

    def write(self, scalars: Dict[str, float], step: int):
        self.f.write(frame(encode_event(time.time(), step=step, scalars=scalars)))
        self.f.flush()

    def close(self):
        self.f.close()


class SummaryWriter:
    """``add_scalar`` / ``add_scalars`` with torch's on-disk layout."""

    def __init__(self, logdir: str = "runs", jsonl: Optional[str] = None):
        self.logdir = logdir
        self._root = _EventFile(logdir)
        self._subs: Dict[str, _EventFile] = {}
        self._jsonl = open(jsonl, "a") if jsonl else None

    def add_scalar(self, tag: str, value: float, global_step: int = 0):
        self._root.write({tag: value}, global_step)
        self._log(tag, value, global_step)

    def add_scalars(self, main_tag: str, tag_scalar_dict: Dict[str, float], global_step: int = 0):
        for k, v in tag_scalar_dict.items():
            d = os.path.join(self.logdir, f"{main_tag}_{k}")
            if d not in self._subs:
                self._subs[d] = _EventFile(d)
            self._subs[d].write({main_tag: v}, global_step)
            self._log(f"{main_tag}/{k}", v, global_step)

    def _log(self, tag, value, step):
        if self._jsonl:
            self._jsonl.write(json.dumps({"t": time.time(), "tag": tag, "value": float(value), "step": step}) + "\n")
            self._jsonl.flush()

    def flush(self):
        pass

    def close(self):
        self._root.close()
        for s in self._subs.values():
            s.close()
        if self._jsonl:
            self._jsonl.close()
