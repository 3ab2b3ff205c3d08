"""LCM ingest (flash/lcmlog.py): event-log records and bot_core.pointcloud_t.

The lcmtypes and the lcm package are not in the reference, and no encoded
message is either, so byte parity with a real log is unpinned (module header);
these tests pin the codec against itself, the fingerprint against lcm-gen's
hash rule, and the conversion against convert_kinect_log_data.py:15-25."""
import io
import struct

import numpy as np
import pytest


def test_fingerprint_rule():
    from flash import lcmlog
    # no members: 0x12345678 rotated left by one bit
    assert lcmlog.struct_fingerprint(()) == 0x2468ACF0
    # one int32 member "a": base hash updated by the name, the type name, ndim 0
    v = 0x12345678
    for c in [1, ord("a"), 7] + [ord(ch) for ch in "int32_t"] + [0]:
        v = ((v << 8) ^ (v >> 55)) + c
        v &= (1 << 64) - 1
        v = v - (1 << 64) if v >> 63 else v
    u = v & ((1 << 64) - 1)
    assert lcmlog.struct_fingerprint((("a", "int32_t", ()),)) == ((u << 1) & ((1 << 64) - 1)) + (u >> 63)
    fp = lcmlog.POINTCLOUD_FINGERPRINT
    assert 0 <= fp < 1 << 64 and fp == lcmlog.struct_fingerprint()


def _msg(n=7, seed=0):
    from flash import lcmlog
    rng = np.random.default_rng(seed)
    return lcmlog.PointCloudMsg(utime=1234567890123, seq=5, frame_id="kinect", points=rng.normal(size=(n, 3)),
                                channel_names=["r", "g", "b"], channels=rng.uniform(size=(3, n)))


def test_pointcloud_roundtrip_and_layout():
    from flash import lcmlog
    m = _msg()
    b = lcmlog.encode_pointcloud(m)
    # fingerprint, utime, seq, "kinect\0", n_points, 7x3 f32, n_channels, 3 strings, 3x7 f32
    assert len(b) == 8 + 8 + 4 + (4 + 7) + 4 + 84 + 4 + 3 * (4 + 2) + 84
    assert struct.unpack_from(">Q", b)[0] == lcmlog.POINTCLOUD_FINGERPRINT
    assert struct.unpack_from(">qi", b, 8) == (1234567890123, 5)
    d = lcmlog.decode_pointcloud(b)
    assert (d.utime, d.seq, d.frame_id, d.n_points, d.n_channels) == (1234567890123, 5, "kinect", 7, 3)
    assert np.array_equal(d.points, m.points.astype(np.float32))
    assert np.array_equal(d.channels, m.channels.astype(np.float32))
    assert d.channel_names == ["r", "g", "b"]
    # big-endian float32 on the wire
    assert struct.unpack_from(">f", b, 8 + 12 + 11 + 4)[0] == np.float32(m.points[0, 0])


def test_pointcloud_decode_errors():
    from flash import lcmlog
    b = bytearray(lcmlog.encode_pointcloud(_msg()))
    with pytest.raises(ValueError):
        lcmlog.decode_pointcloud(bytes(b[:-5]))
    b[0] ^= 1
    with pytest.raises(ValueError, match="fingerprint"):
        lcmlog.decode_pointcloud(bytes(b))
    assert lcmlog.decode_pointcloud(bytes(b), check_fingerprint=False).n_points == 7
    empty = lcmlog.decode_pointcloud(lcmlog.encode_pointcloud(lcmlog.PointCloudMsg()))
    assert empty.n_points == 0 and empty.n_channels == 0


def test_kinect_conversion():
    """convert_kinect_log_data.py:15-25: even indices xyz, odd indices rgb."""
    from flash import lcmlog
    num = 10
    x, y, z = (np.arange(num, dtype=np.float32) + o for o in (0.0, 100.0, 200.0))
    m = lcmlog.decode_pointcloud(lcmlog.encode_pointcloud(lcmlog.kinect_to_bot_core(x, y, z, num, utime=42)))
    assert m.utime == 42 and m.n_points == 5 and m.channel_names == ["r", "g", "b"]
    assert np.array_equal(m.points[:, 0], x[0::2]) and np.array_equal(m.points[:, 2], z[0::2])
    assert np.array_equal(m.channels[1], y[1::2])


def test_event_log_roundtrip_and_frames(tmp_path):
    from flash import lcmlog
    msgs = [_msg(1000, s) for s in range(3)]
    events = [(10, "OTHER", b"xyz")]
    for i, m in enumerate(msgs):
        events += [(100 + i, "KINECT_POINTS_REDUCED", lcmlog.encode_pointcloud(m)), (101 + i, "OTHER", b"")]
    path = tmp_path / "frames.lcm"
    lcmlog.write_log(path, events)
    raw = path.read_bytes()
    assert struct.unpack_from(">I", raw)[0] == 0xEDA1DA01
    with lcmlog.EventLog(path) as lg:
        evs = list(lg)
    assert [(e.eventnum, e.timestamp, e.channel, e.data) for e in evs] == [(i, *ev) for i, ev in enumerate(events)]
    # garbage before and between records is skipped (resynchronisation)
    noisy = b"\x00\x01junk" + raw[:28 + 5 + 3] + b"\xed\xa1zz" + raw[28 + 5 + 3:]
    assert [e.channel for e in lcmlog.EventLog(noisy)] == [e[1] for e in events]
    fr = list(lcmlog.frames(str(path)))
    assert len(fr) == 3
    for f, m in zip(fr, msgs):  # msg[:points][1:200:end] as SVector{3,Float64}
        assert f.dtype == np.float64 and f.shape == (5, 3)
        assert np.array_equal(f, m.points.astype(np.float32)[::200].astype(np.float64))
