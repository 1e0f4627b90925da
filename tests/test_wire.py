"""VVC wire formats (freedm_amd/wire.py) against the protobuf runtime built from
the reference schemas (VoltVarCtrl.proto:12-35, ModuleMessage.proto), and the
slave's xx.mat against the reference's own Broker_s1/xx.mat (tests/golden/xx_s1.mat)."""
import datetime as dt
import os
import re

import numpy as np
import pytest

from freedm_amd import demo_feeder, load_arma_bin
from freedm_amd import wire as W

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _pb_classes():
    """The reference's proto2 schemas rebuilt as descriptors (no protoc here)."""
    pytest.importorskip("google.protobuf")
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="vvc_test.proto", package="freedm.broker", syntax="proto2")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
    R, O, Rep = F.LABEL_REQUIRED, F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("VoltageDeltaMessage", [("control_factor", 1, F.TYPE_UINT32, R, None),
                                ("phase_measurement", 2, F.TYPE_FLOAT, R, None),
                                ("reading_location", 3, F.TYPE_STRING, O, None)])
    msg("LineReadingsMessage", [("measurement", 1, F.TYPE_FLOAT, Rep, None),
                                ("capture_time", 2, F.TYPE_STRING, R, None)])
    msg("GradientMessage", [("gradient_value", 1, F.TYPE_DOUBLE, Rep, None),
                            ("gradient_capture_time", 2, F.TYPE_STRING, R, None)])
    msg("VoltVarMessage", [("voltage_delta_message", 1, F.TYPE_MESSAGE, O, ".freedm.broker.VoltageDeltaMessage"),
                           ("line_readings_message", 2, F.TYPE_MESSAGE, O, ".freedm.broker.LineReadingsMessage"),
                           ("gradient_message", 3, F.TYPE_MESSAGE, O, ".freedm.broker.GradientMessage")])
    msg("ModuleMessage", [("recipient_module", 1, F.TYPE_STRING, R, None),
                          ("volt_var_message", 6, F.TYPE_MESSAGE, O, ".freedm.broker.VoltVarMessage")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = getattr(message_factory, "GetMessageClass", None)
    return {n: (get(pool.FindMessageTypeByName(f"freedm.broker.{n}")) if get else
                message_factory.MessageFactory(pool).GetPrototype(pool.FindMessageTypeByName(f"freedm.broker.{n}")))
            for n in ("ModuleMessage",)}


def test_gradient_bytes_match_protobuf_runtime():
    MM = _pb_classes()["ModuleMessage"]
    Dl = demo_feeder().Dl
    when = dt.datetime(2026, 10, 16, 7, 8, 9, 123456)
    ours = W.gradient_message(Dl, when)
    m = MM()
    m.recipient_module = "vvc"
    g = m.volt_var_message.gradient_message
    g.gradient_value.extend(W.gradient_s2(Dl).tolist())
    g.gradient_capture_time = "2026-Oct-16 07:08:09.123456"
    assert ours == m.SerializeToString()
    back = MM.FromString(ours)
    assert list(back.volt_var_message.gradient_message.gradient_value) == W.gradient_s2(Dl).tolist()


def test_voltage_delta_and_line_readings_roundtrip():
    MM = _pb_classes()["ModuleMessage"]
    vd = W.VoltageDeltaMessage(2, 3.0, "NCSU")          # VoltVarCtrl.cpp:1500
    buf = W.encode_module_message(vd)
    m = MM.FromString(buf)
    assert m.volt_var_message.voltage_delta_message.control_factor == 2
    assert m.volt_var_message.voltage_delta_message.reading_location == "NCSU"
    assert m.SerializeToString() == buf
    lr = W.LineReadingsMessage([1.5, -2.25, 0.0], "t")
    buf = W.encode_module_message(lr, recipient="vvc")
    assert MM.FromString(buf).SerializeToString() == buf
    rec, back = W.decode_module_message(buf)
    assert rec == "vvc" and back == lr
    # a packed encoding from another runtime decodes too
    m2 = MM()
    m2.recipient_module = "vvc"
    m2.volt_var_message.gradient_message.gradient_value.extend([1.0, 2.0])
    m2.volt_var_message.gradient_message.gradient_capture_time = "x"
    assert W.decode_module_message(m2.SerializeToString())[1].gradient_value == [1.0, 2.0]


def test_required_fields_enforced():
    with pytest.raises(ValueError):
        W.GradientMessage.decode(W._key(1, W._I64) + b"\0" * 8)
    with pytest.raises(ValueError):
        W.decode_module_message(W._len_field(6, b""))
    with pytest.raises(ValueError):
        W.GradientMessage.decode(b"\x09\x00")            # truncated double


def test_simple_time_string_format():
    s = W.simple_time_string(dt.datetime(2026, 1, 2, 3, 4, 5, 6))
    assert s == "2026-Jan-02 03:04:05.000006"
    assert re.fullmatch(r"\d{4}-[A-Z][a-z]{2}-\d{2} \d{2}:\d{2}:\d{2}\.\d{6}", W.simple_time_string())


def test_s2_order_and_slave_xx_mat(tmp_path):
    Dl = demo_feeder().Dl
    s2 = W.gradient_s2(Dl)
    assert s2.shape == (21,)
    assert s2[0] == Dl[1, 7] and s2[7] == Dl[1, 9] and s2[20] == Dl[8, 11]
    # the slave's xx.mat: same bytes as the reference's own Broker_s1/xx.mat when
    # fed that file's values
    ref_path = os.path.join(GOLDEN, "xx_s1.mat")
    ref = load_arma_bin(ref_path)
    buf = W.encode_module_message(W.GradientMessage(ref[:, 0].tolist(), "t"))
    out = tmp_path / "xx.mat"
    xx = W.handle_gradient(buf, str(out))
    np.testing.assert_array_equal(xx, ref)
    assert out.read_bytes() == open(ref_path, "rb").read()
