"""Runtime protobuf descriptors + gRPC stubs/servicers built from schema.py.

Usage::

    from drtc_amd.protos import raft_pb, llm_pb, chat_pb, RAFT_SERVICE
    req = raft_pb.VoteRequest(term=3, candidate_id=1)
    stub = make_stub(channel, RAFT_SERVICE)      # stub.RequestVote(req, timeout=3)
    add_servicer(server, RAFT_SERVICE, node)     # node.RequestVote(request, context)

Messages are real protobuf classes (upb backend), so the bytes on the wire
are identical to those of protoc-generated code for the same contract.
"""
from __future__ import annotations

import inspect
import time
import types
from dataclasses import dataclass

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, timestamp_pb2

from . import schema

_SCALARS = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
}
_LABEL_OPT = descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL
_LABEL_REP = descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED
_TYPE_MSG = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE


def _camel(name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _set_type(f, pkg: str, t: str) -> None:
    if t in _SCALARS:
        f.type = _SCALARS[t]
    else:
        f.type = _TYPE_MSG
        f.type_name = t if t.startswith(".") else f".{pkg}.{t}"


def build_file(spec: dict) -> descriptor_pb2.FileDescriptorProto:
    pkg = spec["package"]
    fd = descriptor_pb2.FileDescriptorProto(name=spec["file"], package=pkg, syntax="proto3")
    fd.dependency.extend(spec["imports"])
    for mname, fields in spec["messages"].items():
        m = fd.message_type.add(name=mname)
        for fname, num, ftype in fields:
            f = m.field.add(name=fname, number=num, json_name=_json_name(fname))
            if ftype.startswith("map<"):
                kt, vt = ftype[4:-1].split(",")
                entry = m.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                k = entry.field.add(name="key", number=1, label=_LABEL_OPT, json_name="key")
                _set_type(k, pkg, kt.strip())
                v = entry.field.add(name="value", number=2, label=_LABEL_OPT, json_name="value")
                _set_type(v, pkg, vt.strip())
                f.label = _LABEL_REP
                f.type = _TYPE_MSG
                f.type_name = f".{pkg}.{mname}.{entry.name}"
            elif ftype.startswith("repeated "):
                f.label = _LABEL_REP
                _set_type(f, pkg, ftype[len("repeated "):])
            else:
                f.label = _LABEL_OPT
                _set_type(f, pkg, ftype)
    for sname, methods in spec["services"].items():
        s = fd.service.add(name=sname)
        for name, inp, out, stream in methods:
            s.method.add(name=name, input_type=f".{pkg}.{inp}", output_type=f".{pkg}.{out}",
                         server_streaming=stream)
    return fd


def _pool_with(specs) -> tuple[descriptor_pool.DescriptorPool, dict]:
    pool = descriptor_pool.DescriptorPool()
    pool.Add(descriptor_pb2.FileDescriptorProto.FromString(
        timestamp_pb2.DESCRIPTOR.serialized_pb))
    files = {}
    for spec in specs:
        fdp = build_file(spec)
        pool.Add(fdp)
        files[spec["file"]] = pool.FindFileByName(spec["file"])
    return pool, files


def _namespace(pool, spec) -> types.SimpleNamespace:
    ns = types.SimpleNamespace()
    fdesc = pool.FindFileByName(spec["file"])
    classes = message_factory.GetMessageClassesForFiles([spec["file"]], pool)
    for mname in spec["messages"]:
        setattr(ns, mname, classes[f"{spec['package']}.{mname}"])
    if spec["imports"]:
        ns.Timestamp = message_factory.GetMessageClass(
            pool.FindMessageTypeByName("google.protobuf.Timestamp"))
    ns.DESCRIPTOR = fdesc
    return ns


@dataclass(frozen=True)
class Method:
    name: str
    request: type
    response: type
    server_streaming: bool


@dataclass(frozen=True)
class Service:
    full_name: str
    methods: tuple

    def method(self, name: str) -> Method:
        for m in self.methods:
            if m.name == name:
                return m
        raise KeyError(name)


def _service(ns, spec, sname) -> Service:
    ms = tuple(Method(n, getattr(ns, i), getattr(ns, o), st) for n, i, o, st in spec["services"][sname])
    return Service(f"{spec['package']}.{sname}", ms)


_MAIN_POOL, _ = _pool_with([schema.RAFT, schema.RAFT_SNAPSHOT, schema.LLM, schema.CHAT])
_TOY_POOL, _ = _pool_with([schema.CHAT_TOY])

raft_pb = _namespace(_MAIN_POOL, schema.RAFT)
raft_snap_pb = _namespace(_MAIN_POOL, schema.RAFT_SNAPSHOT)
llm_pb = _namespace(_MAIN_POOL, schema.LLM)
chat_pb = _namespace(_MAIN_POOL, schema.CHAT)
chat_toy_pb = _namespace(_TOY_POOL, schema.CHAT_TOY)

RAFT_SERVICE = _service(raft_pb, schema.RAFT, "RaftNode")
RAFT_SNAPSHOT_SERVICE = _service(raft_snap_pb, schema.RAFT_SNAPSHOT, "RaftSnapshot")
LLM_SERVICE = _service(llm_pb, schema.LLM, "LLMService")
CHAT_SERVICE = _service(chat_pb, schema.CHAT, "ChatService")
CHAT_TOY_SERVICE = _service(chat_toy_pb, schema.CHAT_TOY, "ChatService")


# ---------------------------------------------------------------- gRPC glue
class _Stub:
    def __init__(self, channel: grpc.Channel, service: Service):
        self._service = service
        for m in service.methods:
            path = f"/{service.full_name}/{m.name}"
            factory = channel.unary_stream if m.server_streaming else channel.unary_unary
            setattr(self, m.name, factory(path, request_serializer=m.request.SerializeToString,
                                          response_deserializer=m.response.FromString))


def make_stub(channel: grpc.Channel, service: Service) -> _Stub:
    """Client stub with one callable per RPC (same call surface as protoc stubs)."""
    return _Stub(channel, service)


def _unimplemented(request, context):
    context.set_code(grpc.StatusCode.UNIMPLEMENTED)
    context.set_details("Method not implemented!")
    raise NotImplementedError("Method not implemented!")


def _instrumented(fn, label: str):
    """Per-RPC latency histogram + request counter + trace span."""
    from ..utils import tracing
    from ..utils.metrics import METRICS

    hist, cnt, span = f"rpc.{label}.latency_s", f"rpc.{label}.calls", f"rpc {label}"

    if inspect.iscoroutinefunction(fn):  # grpc.aio handler: coroutines of one loop thread
        # interleave, so no (thread-stacked) roctx range around the await
        async def ahandler(request, context):
            t = time.perf_counter()
            try:
                return await fn(request, context)
            finally:
                METRICS.observe(hist, time.perf_counter() - t)
                METRICS.inc(cnt)
        return ahandler

    def handler(request, context):
        t = time.perf_counter()
        try:
            with tracing.span(span):
                return fn(request, context)
        finally:
            METRICS.observe(hist, time.perf_counter() - t)
            METRICS.inc(cnt)
    return handler


def add_servicer(server: grpc.Server, service: Service, impl) -> None:
    """Register ``impl``'s methods (by RPC name) on ``server``; missing
    methods answer UNIMPLEMENTED like a protoc base servicer."""
    handlers = {}
    for m in service.methods:
        fn = getattr(impl, m.name, None) or _unimplemented
        if not m.server_streaming and fn is not _unimplemented:
            fn = _instrumented(fn, f"{service.full_name}/{m.name}")
        mk = grpc.unary_stream_rpc_method_handler if m.server_streaming else grpc.unary_unary_rpc_method_handler
        handlers[m.name] = mk(fn, request_deserializer=m.request.FromString,
                              response_serializer=m.response.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(service.full_name, handlers),))


def file_descriptor_protos() -> dict:
    return {spec["file"]: build_file(spec) for spec in schema.ALL}
