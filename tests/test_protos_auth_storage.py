"""Wire contract, auth and on-disk compatibility with the reference."""
import ast
import ctypes
import ctypes.util
import datetime as dt
import os
import pickle
import re

import pytest
from google.protobuf import descriptor_pb2

from drtc_amd.protos import chat_pb, file_descriptor_protos, llm_pb, raft_pb
from drtc_amd.raft.core import Entry
from drtc_amd.raft.state_machine import ChatState
from drtc_amd.raft.storage import NativeStorage, PickleStorage
from drtc_amd.utils import auth, pickle_compat

REF = "/root/reference"
have_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")


def _ref_fdp(name):
    src = open(f"{REF}/generated/{name}_pb2.py").read()
    m = re.search(r"AddSerializedFile\((b'.*?')\)", src, re.S)
    return descriptor_pb2.FileDescriptorProto.FromString(ast.literal_eval(m.group(1)))


def _norm(fd):
    msgs = {}
    for m in fd.message_type:
        msgs[m.name] = sorted((f.name, f.number, f.type, f.label, f.type_name) for f in m.field)
        for n in m.nested_type:
            msgs[m.name + "." + n.name] = sorted((f.name, f.number, f.type, f.label, f.type_name)
                                                 for f in n.field)
    svc = {s.name: [(x.name, x.input_type, x.output_type, x.server_streaming) for x in s.method]
           for s in fd.service}
    return fd.package, msgs, svc


@have_ref
@pytest.mark.parametrize("name", ["raft_node", "llm_service", "chat_service", "chat_client"])
def test_descriptors_match_reference(name):
    """Every reference message/field/RPC is present unchanged; the only extra
    fields are the documented additive ones (schema.ADDITIONS)."""
    from drtc_amd.protos.schema import ADDITIONS

    mine = file_descriptor_protos()[name + ".proto"]
    pkg, msgs, svc = _norm(mine)
    rpkg, rmsgs, rsvc = _norm(_ref_fdp(name))
    assert (pkg, svc) == (rpkg, rsvc)
    assert msgs.keys() == rmsgs.keys()
    extra = ADDITIONS.get(name + ".proto", {})
    for m, fields in rmsgs.items():
        added = [f for f in msgs[m] if f not in fields]
        assert set(fields) <= set(msgs[m]), m
        assert sorted(f[0] for f in added) == sorted(extra.get(m, [])), m


def test_wire_roundtrip():
    e = raft_pb.AppendEntriesRequest(term=3, leader_id=2, prev_log_index=-1, prev_log_term=0,
                                     entries=[raft_pb.LogEntry(term=3, command="SEND_MESSAGE", data=b'{"a": 1}')],
                                     leader_commit=-1)
    b = e.SerializeToString()
    assert raft_pb.AppendEntriesRequest.FromString(b) == e
    r = llm_pb.LLMRequest(request_id="x", query="q", context=["a", "b"], parameters={"k": "v"})
    assert llm_pb.LLMRequest.FromString(r.SerializeToString()).parameters["k"] == "v"
    u = chat_pb.UserInfo(username="a")
    u.last_seen.FromDatetime(dt.datetime(2025, 1, 1))
    assert chat_pb.UserInfo.FromString(u.SerializeToString()).last_seen.seconds == 1735689600


def test_jwt_pyjwt_byte_format():
    exp = dt.datetime(2030, 1, 1, tzinfo=dt.timezone.utc)
    tok = auth.jwt_encode({"user_id": "alice", "username": "alice", "exp": exp}, "raft-chat-secret-key")
    h, p, s = tok.split(".")
    assert h == "eyJhbGciOiJIUzI1NiIsInR5cCI6IkpXVCJ9"  # {"alg":"HS256","typ":"JWT"}
    import base64
    body = base64.urlsafe_b64decode(p + "=" * (-len(p) % 4))
    assert body == b'{"user_id":"alice","username":"alice","exp":1893456000}'
    assert "=" not in tok
    assert auth.jwt_decode(tok, "raft-chat-secret-key")["username"] == "alice"
    with pytest.raises(auth.InvalidTokenError):
        auth.jwt_decode(tok, "other-secret")
    with pytest.raises(auth.InvalidTokenError):
        auth.jwt_decode(tok[:-2] + "xx", "raft-chat-secret-key")
    old = auth.jwt_encode({"username": "a", "exp": 1000}, "k")
    with pytest.raises(auth.ExpiredSignatureError):
        auth.jwt_decode(old, "k")


def test_bcrypt_matches_libxcrypt():
    lib = ctypes.util.find_library("crypt")
    if not lib:
        pytest.skip("libcrypt not available")
    c = ctypes.CDLL(lib)
    c.crypt.restype = ctypes.c_char_p
    for pw in (b"alice123", b"", b"p\xc3\xa4ss", b"x" * 72, b"y" * 90):
        salt = auth.bcrypt_gensalt(4)
        assert auth.bcrypt_hashpw(pw, salt) == c.crypt(pw, salt)
        assert auth.bcrypt_checkpw(pw, auth.bcrypt_hashpw(pw, salt))


@have_ref
def test_bcrypt_verifies_reference_hashes():
    users = pickle_compat.safe_load(f"{REF}/server/server_data/users.pkl")["users"]
    assert auth.bcrypt_checkpw(b"admin123", users["admin"]["password"])
    assert auth.bcrypt_checkpw(b"user123", users["user1"]["password"])
    assert not auth.bcrypt_checkpw(b"nope", users["user2"]["password"])


def test_safe_unpickler_rejects_code():
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    with pytest.raises(pickle.UnpicklingError):
        pickle_compat.safe_loads(pickle.dumps(Evil()))
    ok = {"a": {1, 2}, "t": dt.datetime(2024, 1, 1, tzinfo=dt.timezone.utc), "b": b"x"}
    assert pickle_compat.safe_loads(pickle.dumps(ok, protocol=4)) == ok


@have_ref
def test_state_loads_legacy_reference_pickles(tmp_path):
    import shutil
    shutil.copy(f"{REF}/server/server_data/users.pkl", tmp_path / "users.pkl")
    shutil.copy(f"{REF}/server/server_data/channels.pkl", tmp_path / "channels.pkl")
    st = ChatState()
    st.load(str(tmp_path))
    assert "admin" in st.users and isinstance(st.users["admin"]["password"], bytes)
    assert {c["name"] for c in st.channels.values()} == {"general", "random", "development"}
    assert all(isinstance(c["members"], set) for c in st.channels.values())


def _apply_all(st):
    st.apply("CREATE_USER", {"user_id": "u1", "username": "dave", "password": "$2b$04$abc",
                             "email": "d@x.com", "display_name": "Dave", "is_admin": False})
    st.apply("CREATE_CHANNEL", {"channel_id": "c1", "name": "proj", "description": "d", "is_private": True,
                                "members": ["u1"], "admins": ["u1"]})
    st.apply("JOIN_CHANNEL", {"channel_id": "c1", "user_id": "alice"})
    st.apply("LEAVE_CHANNEL", {"channel_id": "c1", "user_id": "alice"})
    m = {"id": "m1", "sender_id": "u1", "sender_name": "dave", "channel_id": "c1", "content": "hi",
         "timestamp": 1}
    st.apply("SEND_MESSAGE", m)
    st.apply("SEND_MESSAGE", dict(m))  # duplicate id ignored
    d = {"id": "d1", "sender_id": "u1", "sender_name": "dave", "recipient_id": "alice",
         "recipient_name": "alice", "content": "yo", "timestamp": 2, "is_read": False}
    st.apply("SEND_DM", d)
    st.apply("SEND_DM", dict(d))
    st.apply("UPLOAD_FILE", {"file_id": "f1", "name": "a.txt", "data": b"abc".hex(), "size": 3,
                             "mime_type": "text/plain", "uploader_id": "u1", "uploader_name": "dave",
                             "channel_id": "c1", "recipient": None, "description": ""})
    st.apply("JOIN_CHANNEL", {"channel_id": "nope", "user_id": "u1"})  # Q13: dropped


def test_state_machine_semantics_and_pickle_roundtrip(tmp_path):
    st = ChatState()
    _apply_all(st)
    assert st.users["dave"]["password"] == b"$2b$04$abc"
    assert st.channels["c1"]["members"] == {"u1"}
    assert len(st.channel_messages["c1"]) == 1 and len(st.direct_messages) == 1
    assert st.files["f1"]["data"] == b"abc"
    assert st.conversation("alice", "dave")[0]["content"] == "yo"
    st.save_all(str(tmp_path))
    raw = open(tmp_path / "channels.pkl", "rb").read()
    assert raw[:2] == b"\x80\x04"  # pickle protocol 4
    ch = pickle_compat.safe_load(str(tmp_path / "channels.pkl"))
    assert isinstance(ch["c1"]["members"], list) and isinstance(ch["c1"]["created_at"], str)
    st2 = ChatState()
    st2.load(str(tmp_path))
    assert st2.channels["c1"]["members"] == {"u1"}
    assert st2.users == st.users and st2.channel_messages == st.channel_messages
    assert st2.conversation("dave", "alice") == st.conversation("dave", "alice")


def test_native_log_store_recovery(tmp_path):
    from drtc_amd import _native
    p = str(tmp_path / "log.seg")
    s = _native.LogStore(p, False)
    for i in range(10):
        s.append(i // 3, f"C{i}", bytes([i]) * i)
    s.truncate_from(7)
    s.close()
    with open(p, "ab") as f:  # torn tail of a crashed append
        f.write(b"TFAR\x10\x00\x00\x00garbage")
    s2 = _native.LogStore(p, False)
    assert s2.size() == 7
    assert s2.get(6) == (2, "C6", b"\x06" * 6)
    assert s2.term_at(3) == 1
    s2.append(5, "X", b"y")
    assert s2.size() == 8


def test_storage_formats_and_migration(tmp_path):
    d = str(tmp_path / "raft_node_1_data")
    ps = PickleStorage(d, 50051)
    ps.load()
    ps.append([Entry(1, "SEND_MESSAGE", b"{}"), Entry(1, "SEND_DM", b"{}")])
    ps.save_state({"current_term": 1, "voted_for": 2, "commit_index": 1, "last_applied": 1})
    log = pickle_compat.safe_load(os.path.join(d, "raft_log_port_50051.pkl"))
    assert log == [{"term": 1, "command": "SEND_MESSAGE", "data": b"{}"},
                   {"term": 1, "command": "SEND_DM", "data": b"{}"}]
    st = pickle_compat.safe_load(os.path.join(d, "raft_state_port_50051.pkl"))
    assert st == {"current_term": 1, "voted_for": 2, "commit_index": 1, "last_applied": 1}
    # a native store opened on the reference-format dir imports the log
    ns = NativeStorage(d, 50051)
    state, entries = ns.load()
    assert [e.command for e in entries] == ["SEND_MESSAGE", "SEND_DM"] and state["voted_for"] == 2
    ns.append([Entry(2, "NOOP", b"")])
    ns.export()
    assert len(pickle_compat.safe_load(os.path.join(d, "raft_log_port_50051.pkl"))) == 3
    ns.close()


def test_native_storage_compaction_and_crash_recovery(tmp_path):
    from drtc_amd.raft.core import Entry
    from drtc_amd.raft.storage import NativeStorage

    d = str(tmp_path / "n1")
    st = NativeStorage(d, 50051)
    st.load()
    ents = [Entry(1 + i // 4, "SEND_MESSAGE", f"{i}".encode()) for i in range(20)]
    st.append(ents)
    st.compact(9, ents[9].term, b"image@9")
    st.append([Entry(6, "SEND_MESSAGE", b"20")])
    st.truncate_from(20)  # absolute index
    st.append([Entry(6, "SEND_MESSAGE", b"20b")])
    st.save_state({"current_term": 6, "voted_for": None, "commit_index": 15, "last_applied": 15})
    st.close()
    st2 = NativeStorage(d, 50051)
    state, entries = st2.load()
    assert state["snap_index"] == 9 and state["snap_term"] == ents[9].term
    assert [e.data for e in entries] == [f"{i}".encode() for i in range(10, 20)] + [b"20b"]
    assert st2.latest_snapshot() == (9, ents[9].term, b"image@9")
    # crash after the snapshot file was written but before the log moved to
    # its new segment: the covered prefix is skipped and the move completed
    st2.snap.save(14, entries[4].term, b"image@14")
    st2.close()
    st3 = NativeStorage(d, 50051)
    state, entries = st3.load()
    assert state["snap_index"] == 14
    assert [e.data for e in entries] == [f"{i}".encode() for i in range(15, 20)] + [b"20b"]
    import os
    segs = sorted(f for f in os.listdir(d) if f.endswith(".seg"))
    assert segs == ["raft_log_port_50051.b15.seg"]
    st3.close()


def test_config_file_layer(tmp_path):
    import argparse

    import pytest as _pytest

    from drtc_amd.utils.config import parse_with_config

    def parser():
        ap = argparse.ArgumentParser()
        ap.add_argument("--node-id", type=int, required=True)
        ap.add_argument("--port", type=int, default=50051)
        ap.add_argument("--snapshot-every", type=int, default=0)
        return ap

    y = tmp_path / "n.yaml"
    y.write_text("node_id: 2\nport: 50052\nsnapshot_every: 100\n")
    a = parse_with_config(parser(), ["--config", str(y), "--port", "6000"])
    assert (a.node_id, a.port, a.snapshot_every) == (2, 6000, 100)  # CLI beats file
    j = tmp_path / "n.json"
    j.write_text('{"node_id": 3, "bogus": 1}')
    with _pytest.raises(SystemExit):
        parse_with_config(parser(), ["--config", str(j)])


def test_checked_in_proto_files_match_schema(tmp_path):
    """protos/*.proto (for protoc users / other languages) are generated from
    the same schema the runtime descriptors are built from - no drift."""
    import os

    from drtc_amd.protos import gen_proto

    here = os.path.dirname(gen_proto.__file__)
    for p in gen_proto.main(str(tmp_path)):
        name = os.path.basename(p)
        with open(p) as a, open(os.path.join(here, name)) as b:
            assert a.read() == b.read(), f"{name} is stale: run python -m drtc_amd.protos.gen_proto"
