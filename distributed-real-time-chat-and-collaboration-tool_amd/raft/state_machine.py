"""Replicated chat state machine (the apply side of the Raft log).

Log-entry commands and their JSON payloads are the reference's (SURVEY §2.7,
server/raft_node.py:1196-1397); in-memory records keep the reference's dict
schemas so the app-state pickles (users/channels/messages/direct_messages)
stay byte-compatible.  Differences, all deliberate:

* idempotency by id *sets* (O(1)) instead of linear scans (raft_node.py:1354,1376);
* secondary indexes for the read RPCs (DMs by user pair / by user id);
* JOIN_CHANNEL for an unknown channel is dropped instead of silently joining
  the first default channel found (survey quirk Q13);
* ``apply`` is deterministic given the entry - nothing node-local (sessions,
  presence) is touched, so every replica converges to the same state;
* CREATE_CHANNEL may carry ``created_at`` (ISO string, the proposing leader's
  clock; an additive key the reference's apply ignores) so the timestamp -
  and therefore channels.pkl - is identical on every replica;
* REVOKE_TOKEN (an additive command; a reference node logs "Unknown command"
  and skips it) replicates logout: {username, token_hash, exp, ts}; revoked
  hashes are dropped deterministically once the entry clock ``ts`` passes
  their ``exp``.
"""
from __future__ import annotations

import datetime as _dt
import logging
import os
import pickle
from collections import defaultdict

from ..utils import pickle_compat

log = logging.getLogger(__name__)

DEFAULT_USERS = (("alice", "alice123"), ("bob", "bob123"), ("charlie", "charlie123"))
DEFAULT_CHANNELS = ("general", "random", "tech")

COMMANDS = ("CREATE_USER", "LOGIN_USER", "CREATE_CHANNEL", "JOIN_CHANNEL", "LEAVE_CHANNEL",
            "SEND_MESSAGE", "SEND_DM", "UPLOAD_FILE", "REVOKE_TOKEN")
GENESIS_CREATED_AT = "2025-01-01T00:00:00+00:00"


def _utcnow() -> _dt.datetime:
    return _dt.datetime.now(_dt.timezone.utc)


class ChatState:
    def __init__(self):
        self.users: dict[str, dict] = {}
        self.users_by_id: dict[str, str] = {}
        self.channels: dict[str, dict] = {}
        self.channel_messages: dict[str, list] = {}
        self.direct_messages: list[dict] = []
        self.files: dict[str, dict] = {}
        self.online_users: set[str] = set()
        self.revoked_tokens: dict[str, int] = {}   # sha256(token) hex -> exp (epoch s)
        self._msg_ids: set[str] = set()
        self._dm_ids: set[str] = set()
        self._dm_pair: dict[tuple, list] = defaultdict(list)
        self._dm_user: dict[str, list] = defaultdict(list)
        self.dirty: set[str] = set()

    # --------------------------------------------------------------- apply
    def apply(self, command: str, data: dict) -> bool:
        """Apply one committed entry. Returns False for unknown commands."""
        fn = getattr(self, "_apply_" + command.lower(), None)
        if fn is None:
            log.warning("unknown command %s", command)
            return False
        fn(data)
        return True

    def _apply_create_user(self, d: dict) -> None:
        name = d["username"]
        if name in self.users:
            return
        self.users[name] = {
            "id": d["user_id"], "username": name,
            "password": d["password"].encode("latin1"),
            "email": d["email"], "display_name": d["display_name"],
            "is_admin": d["is_admin"], "status": "offline",
        }
        self.users_by_id[d["user_id"]] = name
        self.dirty.add("users")

    def _apply_login_user(self, d: dict) -> None:
        name = d["username"]
        if name in self.users:
            self.users[name]["status"] = "online"
            self.online_users.add(name)
            self.dirty.add("users")

    def _apply_create_channel(self, d: dict) -> None:
        cid = d["channel_id"]
        if cid in self.channels:
            return
        created = _utcnow()
        if isinstance(d.get("created_at"), str):
            try:
                created = _dt.datetime.fromisoformat(d["created_at"])
            except ValueError:
                pass
        self.channels[cid] = {
            "id": cid, "name": d["name"], "description": d["description"],
            "is_private": d["is_private"], "members": set(d["members"]),
            "admins": set(d["admins"]), "created_at": created,
        }
        self.channel_messages.setdefault(cid, [])
        self.dirty.add("channels")

    def _apply_join_channel(self, d: dict) -> None:
        ch = self.channels.get(d["channel_id"])
        if ch is None:
            log.info("JOIN_CHANNEL for unknown channel %s dropped", d["channel_id"])
            return
        ch["members"].add(d["user_id"])
        self.dirty.add("channels")

    def _apply_leave_channel(self, d: dict) -> None:
        ch = self.channels.get(d["channel_id"])
        if ch is not None:
            ch["members"].discard(d["user_id"])
            self.dirty.add("channels")

    def _apply_send_message(self, d: dict) -> None:
        mid = d.get("id")
        if mid in self._msg_ids:
            return
        self.channel_messages.setdefault(d["channel_id"], []).append(d)
        self._msg_ids.add(mid)
        self.dirty.add("messages")

    def _apply_send_dm(self, d: dict) -> None:
        did = d.get("id")
        if did and did in self._dm_ids:
            return
        self._index_dm(d)
        self.direct_messages.append(d)
        self.dirty.add("direct_messages")

    def _index_dm(self, d: dict) -> None:
        if d.get("id"):
            self._dm_ids.add(d["id"])
        self._dm_pair[tuple(sorted((d["sender_name"], d["recipient_name"])))].append(d)
        self._dm_user[d["sender_id"]].append(d)
        if d["recipient_id"] != d["sender_id"]:
            self._dm_user[d["recipient_id"]].append(d)

    def _apply_revoke_token(self, d: dict) -> None:
        ts = int(d.get("ts", 0))
        for h in [h for h, exp in self.revoked_tokens.items() if exp < ts]:
            del self.revoked_tokens[h]
        if int(d.get("exp", 0)) >= ts:
            self.revoked_tokens[d["token_hash"]] = int(d["exp"])
        self.dirty.add("revoked_tokens")

    def _apply_upload_file(self, d: dict) -> None:
        fid = d["file_id"]
        if fid in self.files:
            return
        rec = dict(d)
        if isinstance(rec.get("data"), str):
            rec["data"] = bytes.fromhex(rec["data"])
        self.files[fid] = rec

    # ------------------------------------------------------------- queries
    def channel_by_name(self, name: str) -> dict | None:
        for ch in self.channels.values():
            if ch["name"] == name:
                return ch
        return None

    def conversation(self, a: str, b: str) -> list:
        conv = list(self._dm_pair.get(tuple(sorted((a, b))), ()))
        # a DM entry without a timestamp (hand-built or foreign log) sorts
        # first instead of failing the read
        conv.sort(key=lambda m: m.get("timestamp") or "")
        return conv

    def dms_of_user(self, user_id: str) -> list:
        return self._dm_user.get(user_id, [])

    # ------------------------------------------------------------- seeding
    def genesis_entries(self, hash_password) -> list[tuple[str, dict]]:
        """The default users/channels as log entries (CREATE_USER /
        CREATE_CHANNEL) for whatever is still missing: proposed once by the
        first leader of a fresh cluster, so every replica applies the same
        bcrypt hashes and timestamps (byte-identical pickles).
        Ids are the names, as in the reference (server/raft_node.py:426-467)."""
        out = []
        ids = [name for name, _ in DEFAULT_USERS]
        for name, pw in DEFAULT_USERS:
            if name not in self.users:
                out.append(("CREATE_USER", {
                    "user_id": name, "username": name,
                    "password": hash_password(pw.encode()).decode("latin1"),
                    "email": f"{name}@chat.com", "display_name": name.title(), "is_admin": False}))
        for cname in DEFAULT_CHANNELS:
            if cname not in self.channels:
                out.append(("CREATE_CHANNEL", {
                    "channel_id": cname, "name": cname,
                    "description": f"Default {cname} channel (public)", "is_private": False,
                    "members": list(ids), "admins": list(ids),
                    "created_at": GENESIS_CREATED_AT}))
        return out

    def seed_defaults(self, hash_password) -> None:
        """Default users/channels with deterministic ids (username / channel
        name), identical on every node (server/raft_node.py:426-467)."""
        ids = []
        for name, pw in DEFAULT_USERS:
            self.users[name] = {
                "id": name, "username": name, "password": hash_password(pw.encode()),
                "email": f"{name}@chat.com", "display_name": name.title(),
                "is_admin": False, "status": "offline",
            }
            self.users_by_id[name] = name
            ids.append(name)
        for cname in DEFAULT_CHANNELS:
            self.channels[cname] = {
                "id": cname, "name": cname, "description": f"Default {cname} channel (public)",
                "is_private": False, "members": set(ids), "admins": set(ids),
                "created_at": _utcnow(),
            }
            self.channel_messages[cname] = []
        self.dirty.update(("users", "channels"))

    # --------------------------------------------------------- persistence
    FILES = {"users": "users.pkl", "channels": "channels.pkl", "messages": "messages.pkl",
             "direct_messages": "direct_messages.pkl",
             # not part of the reference layout: replicated logout revocations
             "revoked_tokens": "revoked_tokens.pkl"}

    def snapshot_obj(self, which: str):
        if which == "users":
            return {"users": self.users, "users_by_id": self.users_by_id}
        if which == "channels":
            out = {}
            for cid, ch in self.channels.items():
                c = dict(ch)
                c["members"] = list(ch["members"])
                c["admins"] = list(ch["admins"]) if isinstance(ch["admins"], set) else ch["admins"]
                if isinstance(c.get("created_at"), _dt.datetime):
                    c["created_at"] = c["created_at"].isoformat()
                out[cid] = c
            return out
        if which == "messages":
            return self.channel_messages
        if which == "direct_messages":
            return self.direct_messages
        if which == "revoked_tokens":
            return self.revoked_tokens
        raise KeyError(which)

    def save(self, data_dir: str, which=None, fsync: bool = False) -> None:
        for path, data in self.encode(data_dir, which):
            pickle_compat.write_bytes(data, path, fsync)

    def encode(self, data_dir: str, which=None) -> list[tuple[str, bytes]]:
        """Pickled images (reference layout) of the given or the dirty files, marked
        clean: the caller holds the state lock for this step only and writes the
        bytes after releasing it (``pickle_compat.write_bytes``)."""
        out = []
        for w in (which or list(self.dirty)):
            out.append((os.path.join(data_dir, self.FILES[w]),
                        pickle.dumps(self.snapshot_obj(w), protocol=pickle_compat.PROTOCOL)))
            self.dirty.discard(w)
        return out

    def save_all(self, data_dir: str, fsync: bool = False) -> None:
        self.save(data_dir, list(self.FILES), fsync)

    def load(self, data_dir: str) -> None:
        """Load app-state pickles (reference layout; also accepts the legacy
        server's users.pkl with naive datetimes and users_by_email)."""
        p = os.path.join(data_dir, "users.pkl")
        if os.path.exists(p):
            d = pickle_compat.safe_load(p)
            self.users = d.get("users", {})
            self.users_by_id = d.get("users_by_id", {})
        p = os.path.join(data_dir, "channels.pkl")
        if os.path.exists(p):
            for cid, ch in pickle_compat.safe_load(p).items():
                if isinstance(ch.get("members"), (list, tuple)):
                    ch["members"] = set(ch["members"])
                if isinstance(ch.get("admins"), (list, tuple)):
                    ch["admins"] = set(ch["admins"])
                if isinstance(ch.get("created_at"), str):
                    try:
                        ch["created_at"] = _dt.datetime.fromisoformat(ch["created_at"])
                    except ValueError:
                        ch["created_at"] = _utcnow()
                self.channels[cid] = ch
        p = os.path.join(data_dir, "messages.pkl")
        if os.path.exists(p):
            self.channel_messages = pickle_compat.safe_load(p)
        p = os.path.join(data_dir, "direct_messages.pkl")
        if os.path.exists(p):
            self.direct_messages = pickle_compat.safe_load(p)
        p = os.path.join(data_dir, "revoked_tokens.pkl")
        if os.path.exists(p):
            self.revoked_tokens = dict(pickle_compat.safe_load(p))
        self.reindex()

    # ------------------------------------------------- Raft snapshot image
    def image(self) -> bytes:
        """Whole replicated state as one blob for Raft snapshots (plain data,
        pickle protocol 4; read back with the code-free SafeUnpickler).  Files
        are included: the reference keeps uploads only in the log, so a
        compacted log would otherwise lose them."""
        return pickle.dumps({"users": self.users, "users_by_id": self.users_by_id,
                             "channels": self.channels, "messages": self.channel_messages,
                             "direct_messages": self.direct_messages, "files": self.files,
                             "revoked_tokens": self.revoked_tokens},
                            protocol=pickle_compat.PROTOCOL)

    def restore_image(self, data: bytes) -> None:
        d = pickle_compat.safe_loads(data)
        self.users, self.users_by_id = d["users"], d["users_by_id"]
        self.channels, self.channel_messages = d["channels"], d["messages"]
        self.direct_messages, self.files = d["direct_messages"], d["files"]
        self.revoked_tokens = dict(d.get("revoked_tokens", {}))
        self.reindex()
        self.dirty.update(self.FILES)

    def reindex(self) -> None:
        self._msg_ids = {m.get("id") for ms in self.channel_messages.values() for m in ms}
        self._dm_ids = set()
        self._dm_pair = defaultdict(list)
        self._dm_user = defaultdict(list)
        for d in self.direct_messages:
            self._index_dm(d)
