"""Build protobuf message classes for rpc/llm.proto at import time.

A small proto3 reader (messages with scalar / message / repeated fields and
one service with unary and server-streaming rpcs -- exactly what the contract
uses) turns the .proto into a FileDescriptorProto; descriptor_pool +
message_factory then produce real protobuf classes, wire-compatible with the
reference's generated code (same package, names and field numbers)."""
from __future__ import annotations

import re
from pathlib import Path

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PROTO = Path(__file__).with_name("llm.proto")
F = descriptor_pb2.FieldDescriptorProto
SCALARS = {"string": F.TYPE_STRING, "int32": F.TYPE_INT32, "int64": F.TYPE_INT64,
           "bool": F.TYPE_BOOL, "double": F.TYPE_DOUBLE, "float": F.TYPE_FLOAT,
           "bytes": F.TYPE_BYTES, "uint32": F.TYPE_UINT32, "uint64": F.TYPE_UINT64}


def parse(text: str, name: str = "llm.proto") -> descriptor_pb2.FileDescriptorProto:
    text = re.sub(r"//[^\n]*", "", text)
    fd = descriptor_pb2.FileDescriptorProto(name=name, syntax="proto3")
    fd.package = re.search(r"package\s+([\w.]+)\s*;", text).group(1)
    for name, body in re.findall(r"message\s+(\w+)\s*\{([^}]*)\}", text):
        m = fd.message_type.add(name=name)
        for rep, typ, fname, num in re.findall(
                r"(repeated\s+)?([\w.]+)\s+(\w+)\s*=\s*(\d+)\s*;", body):
            f = m.field.add(name=fname, number=int(num), json_name=fname)
            f.label = F.LABEL_REPEATED if rep else F.LABEL_OPTIONAL
            if typ in SCALARS:
                f.type = SCALARS[typ]
            else:
                f.type = F.TYPE_MESSAGE
                f.type_name = f".{fd.package}.{typ}"
    for sname, body in re.findall(r"service\s+(\w+)\s*\{(.*?)\n\}", text, re.S):
        s = fd.service.add(name=sname)
        for mname, cstream, inp, stream, out in re.findall(
                r"rpc\s+(\w+)\s*\(\s*(stream\s+)?(\w+)\s*\)\s*returns\s*\(\s*(stream\s+)?(\w+)\s*\)",
                body):
            s.method.add(name=mname, input_type=f".{fd.package}.{inp}",
                         output_type=f".{fd.package}.{out}", server_streaming=bool(stream),
                         client_streaming=bool(cstream))
    return fd


FILE = parse(PROTO.read_text())
_pool = descriptor_pool.DescriptorPool()
_pool.Add(FILE)
PACKAGE = FILE.package
SERVICE = f"{PACKAGE}.{FILE.service[0].name}"
METHODS = {m.name: (m.input_type.rsplit(".", 1)[1], m.output_type.rsplit(".", 1)[1],
                    m.server_streaming) for m in FILE.service[0].method}
msgs = {m.name: message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{PACKAGE}.{m.name}"))
        for m in FILE.message_type}


# server reflection messages (separate pool: their own package)
REFLECTION_FILE = parse(PROTO.with_name("reflection.proto").read_text(), "reflection.proto")
_rpool = descriptor_pool.DescriptorPool()
_rpool.Add(REFLECTION_FILE)
REFLECTION_SERVICE = f"{REFLECTION_FILE.package}.{REFLECTION_FILE.service[0].name}"
reflection = {m.name: message_factory.GetMessageClass(
    _rpool.FindMessageTypeByName(f"{REFLECTION_FILE.package}.{m.name}"))
    for m in REFLECTION_FILE.message_type}


def __getattr__(name):  # pb.SubmitJobRequest etc.
    try:
        return msgs[name]
    except KeyError:
        raise AttributeError(name) from None
