"""LCM ingest of depth frames: the event log and `bot_core.pointcloud_t`.

The reference's tracking loop reads its depth frames from an LCM event log
(examples/irb_and_squishable.ipynb cells 9 and 12):

    log = PyLCM.pylcm[:EventLog]("../squishable/squishable_squish_out.lcm")
    for event in log
        if event[:channel] == "KINECT_POINTS_REDUCED"
            msg = bot_core[:pointcloud_t][:decode](event["data"])
            sensed_points = map(SVector{3, Float64}, msg[:points][1:200:end])
            gradient_descent!(state, model, sensed_points)

and the log was produced by convert_kinect_log_data.py:11-31, which re-encodes
every `kinect.pointcloud_t` of that channel as a `bot_core.pointcloud_t`
(utime, n_points, points, n_channels = 3, channel_names "r" "g" "b", channels)
and copies every other event unchanged. This module restates, without the lcm
Python package (absent here, like in the reference's own tree):

  * the LCM event-log file format (EventLog / write_log): per event a
    big-endian record {u32 sync 0xEDA1DA01, i64 event number, i64 timestamp
    (µs), i32 channel length, i32 data length, channel bytes, data bytes};
  * the LCM binary encoding of bot_core.pointcloud_t (decode_pointcloud /
    encode_pointcloud): an 8-byte type fingerprint, then the fields in
    declaration order, big-endian, strings as i32 length (incl. the NUL) +
    bytes + NUL, arrays sized by earlier fields;
  * the frame loop over a log (frames / track_log), with the [1:200:end]
    subsample and the warm start carried by flash.tracking.Tracker.

The pointcloud_t layout is the one of bot_core's published lcmtype
(libbot2 `lcmtypes/bot_core_pointcloud_t.lcm`):

    struct pointcloud_t {
        int64_t utime;
        int32_t seq;
        string  frame_id;
        int32_t n_points;
        float   points[n_points][3];
        int32_t n_channels;
        string  channel_names[n_channels];
        float   channels[n_channels][n_points];
    }

The .lcm file itself is not in the reference (BotCoreLCMTypes is an
un-vendored dependency, REQUIRE.dev), and the reference holds no encoded
message, so byte-level parity with a real log is UNPINNED: the tests pin the
encoder against the decoder, the fingerprint against lcm-gen's published
hash rule (computed here, not copied), and the conversion against
convert_kinect_log_data.py's field assignments.
"""
from __future__ import annotations

import io
import os
import struct
from dataclasses import dataclass, field

import numpy as np

LCM_SYNC = 0xEDA1DA01
_MASK = (1 << 64) - 1

# (member name, LCM type, dimensions as (mode, size)); mode 0 = const, 1 = variable
POINTCLOUD_T = (
    ("utime", "int64_t", ()),
    ("seq", "int32_t", ()),
    ("frame_id", "string", ()),
    ("n_points", "int32_t", ()),
    ("points", "float", ((1, "n_points"), (0, "3"))),
    ("n_channels", "int32_t", ()),
    ("channel_names", "string", ((1, "n_channels"),)),
    ("channels", "float", ((1, "n_channels"), (1, "n_points"))),
)
_PRIMITIVES = {"int8_t", "int16_t", "int32_t", "int64_t", "byte", "float", "double", "string", "boolean"}


def _s64(v: int) -> int:
    v &= _MASK
    return v - (1 << 64) if v >> 63 else v


def _hash_update(v: int, c: int) -> int:
    # lcm-gen: v = ((v << 8) ^ (v >> 55)) + c on int64_t (arithmetic shift)
    return _s64(((v << 8) ^ (v >> 55)) + c)


def _hash_string(v: int, s: str) -> int:
    v = _hash_update(v, len(s))
    for ch in s.encode():
        v = _hash_update(v, ch)
    return v


def struct_fingerprint(members=POINTCLOUD_T) -> int:
    """The 64-bit type fingerprint lcm-gen emits for a struct whose members
    are all primitive: base hash 0x12345678 updated with every member name,
    primitive type name, dimension count, and each dimension's mode and size
    string; then rotated left by one bit (_get_hash_recursive)."""
    v = 0x12345678
    for name, typ, dims in members:
        v = _hash_string(v, name)
        if typ in _PRIMITIVES:
            v = _hash_string(v, typ)
        v = _hash_update(v, len(dims))
        for mode, size in dims:
            v = _hash_update(v, mode)
            v = _hash_string(v, size)
    u = v & _MASK
    return ((u << 1) & _MASK) + (u >> 63)


POINTCLOUD_FINGERPRINT = struct_fingerprint()


@dataclass
class PointCloudMsg:
    """bot_core.pointcloud_t (points [n,3] float32, channels [c,n] float32)."""
    utime: int = 0
    seq: int = 0
    frame_id: str = ""
    points: np.ndarray = field(default_factory=lambda: np.zeros((0, 3), np.float32))
    channel_names: list = field(default_factory=list)
    channels: np.ndarray = field(default_factory=lambda: np.zeros((0, 0), np.float32))

    @property
    def n_points(self) -> int:
        return int(len(self.points))

    @property
    def n_channels(self) -> int:
        return len(self.channel_names)


def _pack_string(s: str) -> bytes:
    b = s.encode()
    return struct.pack(">i", len(b) + 1) + b + b"\0"


def _unpack_string(buf: memoryview, off: int):
    (n,) = struct.unpack_from(">i", buf, off)
    off += 4
    if n < 1 or off + n > len(buf) or buf[off + n - 1] != 0:
        raise ValueError("pointcloud_t: malformed string")
    return bytes(buf[off:off + n - 1]).decode(), off + n


def encode_pointcloud(msg: PointCloudMsg) -> bytes:
    """bot_core.pointcloud_t.encode()."""
    pts = np.ascontiguousarray(msg.points, np.float32).reshape(-1, 3)
    n = len(pts)
    ch = np.ascontiguousarray(msg.channels, np.float32).reshape(len(msg.channel_names), n)
    out = [struct.pack(">Q", POINTCLOUD_FINGERPRINT), struct.pack(">qi", int(msg.utime), int(msg.seq)),
           _pack_string(msg.frame_id), struct.pack(">i", n), pts.astype(">f4").tobytes(),
           struct.pack(">i", len(msg.channel_names))]
    out += [_pack_string(s) for s in msg.channel_names]
    out.append(ch.astype(">f4").tobytes())
    return b"".join(out)


def decode_pointcloud(data: bytes, check_fingerprint: bool = True) -> PointCloudMsg:
    """bot_core.pointcloud_t.decode(data) (the notebook's
    bot_core[:pointcloud_t][:decode](event["data"]))."""
    buf = memoryview(data)
    if len(buf) < 8 + 12:
        raise ValueError("pointcloud_t: message too short")
    (fp,) = struct.unpack_from(">Q", buf, 0)
    if check_fingerprint and fp != POINTCLOUD_FINGERPRINT:
        raise ValueError(f"pointcloud_t: fingerprint {fp:#018x} != {POINTCLOUD_FINGERPRINT:#018x}")
    utime, seq = struct.unpack_from(">qi", buf, 8)
    frame_id, off = _unpack_string(buf, 20)
    (n,) = struct.unpack_from(">i", buf, off)
    off += 4
    if n < 0 or off + 12 * n > len(buf):
        raise ValueError("pointcloud_t: bad n_points")
    pts = np.frombuffer(buf, ">f4", 3 * n, off).astype(np.float32).reshape(n, 3)
    off += 12 * n
    (nc,) = struct.unpack_from(">i", buf, off)
    off += 4
    if nc < 0:
        raise ValueError("pointcloud_t: bad n_channels")
    names = []
    for _ in range(nc):
        s, off = _unpack_string(buf, off)
        names.append(s)
    if off + 4 * nc * n > len(buf):
        raise ValueError("pointcloud_t: truncated channels")
    ch = np.frombuffer(buf, ">f4", nc * n, off).astype(np.float32).reshape(nc, n)
    return PointCloudMsg(int(utime), int(seq), frame_id, pts, names, ch)


def kinect_to_bot_core(x, y, z, num: int | None = None, utime: int = 0) -> PointCloudMsg:
    """convert_kinect_log_data.py:15-25: a kinect.pointcloud_t interleaves
    positions (even indices) and colours (odd indices) in x/y/z; the
    bot_core message holds n_points = num // 2 points and channels r, g, b."""
    from .depthdata import kinect_to_pointcloud
    d = kinect_to_pointcloud(x, y, z, num, utime)
    return PointCloudMsg(d["utime"], 0, "", d["points"], list(d["channel_names"]), d["channels"])


@dataclass
class Event:
    eventnum: int
    timestamp: int
    channel: str
    data: bytes


class EventLog:
    """Read-only LCM event log: iterating yields Event records in file order
    (lcm.EventLog(path) / PyLCM.pylcm[:EventLog]). Garbage between records is
    skipped by re-synchronising on the sync word, as the LCM reader does."""

    def __init__(self, source):
        if isinstance(source, (bytes, bytearray, memoryview)):
            self._f = io.BytesIO(bytes(source))
        elif isinstance(source, (str, os.PathLike)):
            self._f = open(source, "rb")
        else:
            self._f = source

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __iter__(self):
        f = self._f
        f.seek(0)
        blob = f.read()
        sync = struct.pack(">I", LCM_SYNC)
        off = 0
        while True:
            off = blob.find(sync, off)
            if off < 0 or off + 28 > len(blob):
                return
            num, ts, clen, dlen = struct.unpack_from(">qqii", blob, off + 4)
            start = off + 28
            if clen < 0 or dlen < 0 or start + clen + dlen > len(blob):
                off += 1  # not a record: resynchronise
                continue
            chan = blob[start:start + clen].decode(errors="replace")
            yield Event(num, ts, chan, blob[start + clen:start + clen + dlen])
            off = start + clen + dlen


def write_log(path_or_file, events) -> None:
    """lcm.EventLog(dest, "w").write_event(...) for (timestamp, channel,
    data) triples; event numbers count from 0."""
    own = isinstance(path_or_file, (str, os.PathLike))
    f = open(path_or_file, "wb") if own else path_or_file
    try:
        for i, (ts, chan, data) in enumerate(events):
            c = chan.encode()
            f.write(struct.pack(">Iqqii", LCM_SYNC, i, int(ts), len(c), len(data)) + c + bytes(data))
    finally:
        if own:
            f.close()


def frames(log, channel: str = "KINECT_POINTS_REDUCED", step: int = 200):
    """The notebook's loop body up to gradient_descent!: for each event on
    `channel`, decode the bot_core.pointcloud_t and yield
    msg.points[1:200:end] as [n,3] float64 (SVector{3,Float64} per point)."""
    own = not isinstance(log, EventLog)
    lg = EventLog(log) if own else log
    try:
        for ev in lg:
            if ev.channel == channel:
                msg = decode_pointcloud(ev.data)
                yield np.ascontiguousarray(msg.points[::step], np.float64)
    finally:
        if own:
            lg.close()


def track_log(manipulator, log, state=None, solver=None, channel: str = "KINECT_POINTS_REDUCED", step: int = 200,
              callback=None, device: int = 0, precision: int = 64):
    """examples/irb_and_squishable.ipynb cell 12 end to end: every frame of
    the log through gradient_descent! (flash.tracking.Tracker: resident
    context, warm start carried). Returns (solutions [F, n], Tracker)."""
    from .tracking import Tracker
    tr = Tracker(manipulator, state, solver, device, precision)
    xs = [tr.step(pts, callback) for pts in frames(log, channel, step)]
    return np.array(xs), tr
