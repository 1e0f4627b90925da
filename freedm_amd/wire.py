"""VVC wire formats: the proto2 messages the Broker exchanges around the solve.

The line search's result leaves the master Broker as a `GradientMessage` (the
21 control set-points S2) inside `VoltVarMessage` inside `ModuleMessage`
(`Broker/src/vvc/VoltVarCtrl.cpp:1497-1510`, built by `VVCAgent::Gradient`
`:187-198`, wrapped by `PrepareForSending` `:201-208`); slaves unpack it into a
21x1 `arma::mat` and save it as `xx.mat` (`Broker_s1/src/vvc/VoltVarCtrl.cpp:141-154`).
Schemas: `Broker/src/messages/VoltVarCtrl.proto:12-35`, `ModuleMessage.proto`
(recipient_module = 1, volt_var_message = 6).

Hand-written proto2 encoder/decoder (no generated code, no protoc): fields in
field-number order, repeated scalars unpacked (proto2 default), which is what
the reference's C++ protobuf runtime emits for these messages.
"""
from __future__ import annotations

import datetime as _dt
import struct
from dataclasses import dataclass, field

import numpy as np

_VARINT, _I64, _LEN, _I32 = 0, 1, 2, 5


def _varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num: int, wt: int) -> bytes:
    return _varint((num << 3) | wt)


def _len_field(num: int, payload: bytes) -> bytes:
    return _key(num, _LEN) + _varint(len(payload)) + payload


def _read_varint(buf: bytes, pos: int) -> tuple[int, int]:
    v = shift = 0
    while True:
        if pos >= len(buf):
            raise ValueError("truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _fields(buf: bytes):
    """Yield (field number, wire type, value) over one message's bytes; LEN
    values are bytes, I64/I32 values raw little-endian bytes."""
    pos = 0
    while pos < len(buf):
        k, pos = _read_varint(buf, pos)
        num, wt = k >> 3, k & 7
        if wt == _VARINT:
            v, pos = _read_varint(buf, pos)
        elif wt == _I64:
            v, pos = buf[pos:pos + 8], pos + 8
        elif wt == _I32:
            v, pos = buf[pos:pos + 4], pos + 4
        elif wt == _LEN:
            n, pos = _read_varint(buf, pos)
            v, pos = buf[pos:pos + n], pos + n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        if pos > len(buf):
            raise ValueError("truncated field")
        yield num, wt, v


def _packed_or_single(wt: int, v, fmt: str) -> list:
    size = struct.calcsize(fmt)
    if wt == _LEN:      # a packed encoding is accepted on parse (proto2 parsers do)
        return list(struct.unpack(f"<{len(v) // size}{fmt}", v))
    return [struct.unpack(f"<{fmt}", v)[0]]


def simple_time_string(t: _dt.datetime | None = None) -> str:
    """boost::posix_time::to_simple_string(microsec_clock::universal_time()):
    'YYYY-Mon-DD HH:MM:SS.ffffff' (`VoltVarCtrl.cpp:196`)."""
    t = t or _dt.datetime.now(_dt.timezone.utc)
    return t.strftime("%Y-") + t.strftime("%b").capitalize() + t.strftime("-%d %H:%M:%S.%f")


@dataclass
class GradientMessage:
    """`GradientMessage { repeated double gradient_value = 1; required string
    gradient_capture_time = 2; }` (VoltVarCtrl.proto:25-29)."""
    gradient_value: list = field(default_factory=list)
    gradient_capture_time: str = ""

    def encode(self) -> bytes:
        out = b"".join(_key(1, _I64) + struct.pack("<d", float(x)) for x in self.gradient_value)
        return out + _len_field(2, self.gradient_capture_time.encode())

    @classmethod
    def decode(cls, buf: bytes) -> "GradientMessage":
        m, seen = cls(), False
        for num, wt, v in _fields(buf):
            if num == 1:
                m.gradient_value += _packed_or_single(wt, v, "d")
            elif num == 2:
                m.gradient_capture_time, seen = v.decode(), True
        if not seen:
            raise ValueError("GradientMessage: missing required gradient_capture_time")
        return m


@dataclass
class LineReadingsMessage:
    """`LineReadingsMessage { repeated float measurement = 1; required string
    capture_time = 2; }` (VoltVarCtrl.proto:19-23)."""
    measurement: list = field(default_factory=list)
    capture_time: str = ""

    def encode(self) -> bytes:
        out = b"".join(_key(1, _I32) + struct.pack("<f", float(x)) for x in self.measurement)
        return out + _len_field(2, self.capture_time.encode())

    @classmethod
    def decode(cls, buf: bytes) -> "LineReadingsMessage":
        m, seen = cls(), False
        for num, wt, v in _fields(buf):
            if num == 1:
                m.measurement += _packed_or_single(wt, v, "f")
            elif num == 2:
                m.capture_time, seen = v.decode(), True
        if not seen:
            raise ValueError("LineReadingsMessage: missing required capture_time")
        return m


@dataclass
class VoltageDeltaMessage:
    """`VoltageDeltaMessage { required uint32 control_factor = 1; required float
    phase_measurement = 2; optional string reading_location = 3; }`
    (VoltVarCtrl.proto:13-17)."""
    control_factor: int = 0
    phase_measurement: float = 0.0
    reading_location: str | None = None

    def encode(self) -> bytes:
        out = _key(1, _VARINT) + _varint(int(self.control_factor) & 0xFFFFFFFF)
        out += _key(2, _I32) + struct.pack("<f", float(self.phase_measurement))
        if self.reading_location is not None:
            out += _len_field(3, self.reading_location.encode())
        return out

    @classmethod
    def decode(cls, buf: bytes) -> "VoltageDeltaMessage":
        m, seen = cls(), set()
        for num, wt, v in _fields(buf):
            if num == 1:
                m.control_factor = v & 0xFFFFFFFF
            elif num == 2:
                m.phase_measurement = struct.unpack("<f", v)[0]
            elif num == 3:
                m.reading_location = v.decode()
            seen.add(num)
        if not {1, 2} <= seen:
            raise ValueError("VoltageDeltaMessage: missing a required field")
        return m


_VVM_KINDS = {1: VoltageDeltaMessage, 2: LineReadingsMessage, 3: GradientMessage}


def encode_module_message(sub, recipient: str = "vvc") -> bytes:
    """ModuleMessage{recipient_module = 1, volt_var_message = 6 {oneof-like
    optional sub-message 1|2|3}} -- `PrepareForSending` (`VoltVarCtrl.cpp:201-208`)."""
    num = {v: k for k, v in _VVM_KINDS.items()}[type(sub)]
    vvm = _len_field(num, sub.encode())
    return _len_field(1, recipient.encode()) + _len_field(6, vvm)


def decode_module_message(buf: bytes):
    """-> (recipient_module, sub-message or None).  Dispatch order of
    `HandleIncomingMessage` (`VoltVarCtrl.cpp:88-110`): voltage delta, then line
    readings, then gradient."""
    recipient, vvm = None, None
    for num, wt, v in _fields(buf):
        if num == 1:
            recipient = v.decode()
        elif num == 6:
            vvm = (vvm or b"") + v      # repeated embedded messages merge
    if recipient is None:
        raise ValueError("ModuleMessage: missing required recipient_module")
    if vvm is None:
        return recipient, None
    subs = {}
    for num, wt, v in _fields(vvm):
        if num in _VVM_KINDS:
            subs[num] = subs.get(num, b"") + v
    for num in (1, 2, 3):
        if num in subs:
            return recipient, _VVM_KINDS[num].decode(subs[num])
    return recipient, None


# Dl rows and Q columns whose set-points form S2 (`VoltVarCtrl.cpp:1504`):
# rows 1-4 and 6-8 (the load rows of the 9-row feeder) of Q1, Q2, Q3.
S2_ROWS = (1, 2, 3, 4, 6, 7, 8)
S2_COLS = (7, 9, 11)


def gradient_s2(Dl: np.ndarray) -> np.ndarray:
    """S2 = [Dl(r, c) for c in (7, 9, 11) for r in rows], a 21-vector, the
    phase-major order of the `<<` chain at `VoltVarCtrl.cpp:1504`."""
    Dl = np.asarray(Dl, dtype=np.float64)
    return np.array([Dl[r, c] for c in S2_COLS for r in S2_ROWS], dtype=np.float64)


def gradient_message(Dl: np.ndarray, when: _dt.datetime | None = None) -> bytes:
    """The master's message to each slave after a loss-reducing step."""
    return encode_module_message(GradientMessage(list(gradient_s2(Dl)), simple_time_string(when)))


def handle_gradient(buf: bytes, path: str | None = None) -> np.ndarray:
    """The slave side (`Broker_s1/src/vvc/VoltVarCtrl.cpp:141-154`): the gradient
    values as a (n x 1) matrix, saved as Armadillo binary when `path` is given
    (the reference writes `xx.mat`)."""
    _, sub = decode_module_message(buf)
    if not isinstance(sub, GradientMessage):
        raise ValueError("not a gradient message")
    xx = np.asarray(sub.gradient_value, dtype=np.float64).reshape(-1, 1)
    if path is not None:
        from .feeder import save_arma_bin
        save_arma_bin(path, xx)
    return xx
