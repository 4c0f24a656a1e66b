"""Byte-level parity of the formats other tools read: tfevents files (TensorBoard sidecar), and the default-PS
command line the operator generates (reference grpc_tensorflow_server.py CLI)."""
import struct

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from k8s_amd.ps_server.grpc_tensorflow_server import build_parser
from k8s_amd.utils import tfevents


def test_crc32c_known_answers():
    # RFC 3720 (iSCSI) appendix B.4 check value, and the all-zero / all-0xff 32-byte vectors
    assert tfevents.crc32c(b"123456789") == 0xE3069283
    assert tfevents.crc32c(bytes(32)) == 0x8A9136AA
    assert tfevents.crc32c(b"\xff" * 32) == 0x62A8AB43
    # TFRecord's mask: rotate right by 15, add 0xa282ead8
    c = tfevents.crc32c(b"abc")
    assert tfevents.masked_crc(b"abc") == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _event_classes():
    """Event / Summary / Summary.Value built from the field numbers of tensorflow/core/util/event.proto and
    tensorflow/core/framework/summary.proto (wall_time=1, step=2, file_version=3, summary=5; Summary.value=1;
    Value.tag=1, Value.simple_value=2): an independent decoder for what utils/tfevents.py encodes by hand."""
    f = descriptor_pb2.FileDescriptorProto(name="k8s_amd_test_event.proto", package="k8s_amd_test", syntax="proto3")
    summ = f.message_type.add(name="Summary")
    val = summ.nested_type.add(name="Value")
    val.field.add(name="tag", number=1, type=9, label=1)
    val.field.add(name="simple_value", number=2, type=2, label=1)
    summ.field.add(name="value", number=1, type=11, label=3, type_name=".k8s_amd_test.Summary.Value")
    ev = f.message_type.add(name="Event")
    ev.oneof_decl.add(name="what")
    ev.field.add(name="wall_time", number=1, type=1, label=1)
    ev.field.add(name="step", number=2, type=3, label=1)
    ev.field.add(name="file_version", number=3, type=9, label=1, oneof_index=0)
    ev.field.add(name="summary", number=5, type=11, label=1, type_name=".k8s_amd_test.Summary", oneof_index=0)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(f)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("k8s_amd_test.Event"))


def test_event_file_round_trip_through_protobuf(tmp_path):
    Event = _event_classes()
    w = tfevents.EventWriter(str(tmp_path))
    w.scalars(7, {"loss": 2.5, "images_per_sec": 9111.0})
    w.scalars(8, {"loss": 2.25})
    w.close()
    recs = list(tfevents.read_records(w.path))  # verifies both masked CRCs of every record
    assert len(recs) == 3
    first = Event.FromString(recs[0])
    assert first.file_version == "brain.Event:2" and first.wall_time > 1.6e9
    e1 = Event.FromString(recs[1])
    assert e1.step == 7 and e1.WhichOneof("what") == "summary"
    assert {v.tag: v.simple_value for v in e1.summary.value} == {"loss": 2.5, "images_per_sec": 9111.0}
    e2 = Event.FromString(recs[2])
    assert e2.step == 8 and [(v.tag, v.simple_value) for v in e2.summary.value] == [("loss", 2.25)]
    # and the protobuf encoder produces the same bytes as ours for a fixed event
    ref = Event(wall_time=1700000000.5, step=3)
    ref.summary.value.add(tag="x", simple_value=1.5)
    assert tfevents.encode_event(1700000000.5, 3, scalars={"x": 1.5}) == ref.SerializeToString()
    # record framing: little-endian u64 length + masked crc of it
    raw = open(w.path, "rb").read()
    n, = struct.unpack("<Q", raw[:8])
    assert n == len(recs[0])


def test_default_ps_verbose_flag_semantics():
    p = build_parser()
    base = ["--cluster_spec", "ps|localhost:2222", "--job_name", "ps", "--task_id", "0"]
    assert p.parse_args(base).verbose is False
    assert p.parse_args(base + ["--verbose"]).verbose is True
    assert p.parse_args(base + ["--verbose=true"]).verbose is True
    assert p.parse_args(base + ["--verbose", "True"]).verbose is True
    assert p.parse_args(base + ["--verbose", "False"]).verbose is False
    assert p.parse_args(base + ["--verbose=0"]).verbose is False
