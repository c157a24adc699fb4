"""Legacy single-node ``chat.ChatService`` (no Raft) with real-time streaming.

Capabilities of the reference's server/app_server.py:
signup with validation (username 3-20 ``[A-Za-z0-9_]``, e-mail regex,
password 6-50 with a digit/special), login/logout, channels with admin
management (``ManageChannel`` add_user/remove_user), channel posts, DMs,
file sharing, paged history (offset honoured), presence, and the
server-streaming ``StreamMessages`` fed by a per-user bounded broker (events
dropped when a subscriber's 100-slot queue is full, like the reference).
The four RPCs the reference left UNIMPLEMENTED are implemented here:
LeaveChannel, UpdatePresence, ManageUser (admin: promote/demote/disable/
enable) and GetServerInfo (single node: always its own leader).

Persistence: ``server_data/users.pkl`` and ``channels.pkl`` in the
reference's layout (pickle protocol 4; safe loader).
"""
from __future__ import annotations

import argparse
import datetime as _dt
import logging
import mimetypes
import os
import queue
import re
import threading
import uuid
from concurrent import futures

import grpc

from ..protos import CHAT_SERVICE, SERVER_QUEUE_OPTS, add_servicer, chat_pb
from ..utils import auth, pickle_compat
from ..utils.config import parse_with_config
from ..utils.logging_utils import setup_logging

log = logging.getLogger(__name__)


def _now():
    return _dt.datetime.now(_dt.timezone.utc)


def _ts(dt) -> object:
    t = chat_pb.Timestamp()
    if isinstance(dt, _dt.datetime):
        if dt.tzinfo is None:
            dt = dt.replace(tzinfo=_dt.timezone.utc)
        t.FromDatetime(dt)
    return t


class MessageBroker:
    """Per-user bounded event queues (server/app_server.py:32-69)."""

    def __init__(self, maxsize: int = 100):
        self.maxsize = maxsize
        self.subs: dict[str, queue.Queue] = {}
        self.lock = threading.Lock()
        self.dropped = 0

    def subscribe(self, user_id: str) -> queue.Queue:
        with self.lock:
            q = queue.Queue(maxsize=self.maxsize)
            self.subs[user_id] = q
            return q

    def unsubscribe(self, user_id: str, q: queue.Queue | None = None) -> None:
        with self.lock:
            if user_id in self.subs and (q is None or self.subs[user_id] is q):
                del self.subs[user_id]

    def send_to_user(self, user_id: str, event) -> None:
        with self.lock:
            q = self.subs.get(user_id)
        if q is not None:
            try:
                q.put_nowait(event)
            except queue.Full:
                self.dropped += 1

    def broadcast(self, members, event, exclude: str | None = None) -> None:
        for uid in list(members):
            if uid != exclude:
                self.send_to_user(uid, event)


class LegacyChatServer:
    DEFAULT_CHANNELS = ("general", "random", "development")

    def __init__(self, data_dir: str = "server_data", jwt_secret: str = "your-secret-key-here",
                 bcrypt_rounds: int = 12, node_id: int = 1, port: int = 50050, seed: bool = True):
        self.dir = data_dir
        self.secret = jwt_secret
        self.rounds = bcrypt_rounds
        self.node_id, self.port = node_id, port
        self.lock = threading.RLock()
        self.users: dict = {}
        self.users_by_email: dict = {}
        self.users_by_id: dict = {}
        self.channels: dict = {}
        self.messages: dict = {}
        self.direct_messages: list = []
        self.files: dict = {}
        self.sessions: dict = {}
        self.online: set = set()
        self.disabled: set = set()
        self.broker = MessageBroker()
        os.makedirs(self.dir, exist_ok=True)
        self._load()
        if seed and not self.channels:
            self._seed_channels()
        if seed and not self.users:
            self._seed_users()

    # ----------------------------------------------------------- storage
    @property
    def users_file(self):
        return os.path.join(self.dir, "users.pkl")

    @property
    def channels_file(self):
        return os.path.join(self.dir, "channels.pkl")

    def _load(self):
        if os.path.exists(self.users_file):
            d = pickle_compat.safe_load(self.users_file)
            self.users = d.get("users", {})
            self.users_by_email = d.get("users_by_email", {})
            self.users_by_id = d.get("users_by_id", {})
        if os.path.exists(self.channels_file):
            self.channels = pickle_compat.safe_load(self.channels_file)
            for ch in self.channels.values():
                if isinstance(ch.get("members"), list):
                    ch["members"] = set(ch["members"])
                if isinstance(ch.get("admins"), list):
                    ch["admins"] = set(ch["admins"])
                self.messages.setdefault(ch["id"], [])

    def _save_users(self):
        pickle_compat.dump({"users": self.users, "users_by_email": self.users_by_email,
                            "users_by_id": self.users_by_id}, self.users_file)

    def _save_channels(self):
        out = {}
        for cid, ch in self.channels.items():
            c = dict(ch)
            c["members"] = list(ch["members"])
            out[cid] = c
        pickle_compat.dump(out, self.channels_file)

    def _seed_channels(self):
        for name in self.DEFAULT_CHANNELS:
            cid = str(uuid.uuid4())
            self.channels[cid] = {"id": cid, "name": name, "description": f"Default {name} channel",
                                  "is_private": False, "members": set(), "admins": {"system"},
                                  "created_at": _now(), "created_by": "system"}
            self.messages[cid] = []
        self._save_channels()

    def _seed_users(self):
        for name, pw, email, admin, disp in (("admin", "admin123", "admin@chat.com", True, "Administrator"),
                                             ("user1", "user123", "user1@chat.com", False, "User One"),
                                             ("user2", "user123", "user2@chat.com", False, "User Two")):
            self._add_user(name, pw, email, disp, admin)
        self._save_users()

    def _add_user(self, name, pw, email, display, admin=False):
        uid = str(uuid.uuid4())
        self.users[name] = {"id": uid, "username": name,
                            "password": auth.bcrypt_hashpw(pw.encode(), auth.bcrypt_gensalt(self.rounds)),
                            "email": email, "display_name": display, "is_admin": admin,
                            "created_at": _now(), "status": "offline", "last_seen": _now()}
        self.users_by_email[email] = name
        self.users_by_id[uid] = name
        return uid

    # ----------------------------------------------------------- auth
    def _token(self, uid, name):
        now = _now()
        return auth.jwt_encode({"user_id": uid, "username": name,
                                "exp": now + _dt.timedelta(hours=24), "iat": now}, self.secret)

    def _verify(self, token):
        try:
            p = auth.jwt_decode(token, self.secret)
        except auth.InvalidTokenError:
            return None
        if p.get("username") in self.disabled:
            return None
        return p

    @staticmethod
    def _valid_username(u):
        return bool(u) and 3 <= len(u) <= 20 and re.match(r"^[a-zA-Z0-9_]+$", u) is not None

    @staticmethod
    def _valid_email(e):
        return re.match(r"^[a-zA-Z0-9._%+-]+@[a-zA-Z0-9.-]+\.[a-zA-Z]{2,}$", e) is not None

    @staticmethod
    def _valid_password(p):
        if len(p) < 6:
            return False, "Password must be at least 6 characters long"
        if len(p) > 50:
            return False, "Password must be less than 50 characters"
        if not re.search(r'[0-9!@#$%^&*(),.?":{}|<>]', p):
            return False, "Password must contain at least one number or special character"
        return True, "Password is valid"

    def _user_info(self, name):
        u = self.users[name]
        return chat_pb.UserInfo(user_id=u["id"], username=name, is_admin=u.get("is_admin", False),
                                status=u.get("status", "offline"), last_seen=_ts(u.get("last_seen")),
                                display_name=u.get("display_name", name), email=u.get("email", ""))

    def Signup(self, request, context):
        name = request.username.strip()
        pw = request.password
        email = request.email.strip().lower()
        disp = request.display_name.strip() if request.display_name else name
        if not name or not pw or not email:
            return chat_pb.SignupResponse(success=False, code=400,
                                          message="Username, password, and email are required")
        if not self._valid_username(name):
            return chat_pb.SignupResponse(success=False, code=400,
                                          message="Username must be 3-20 characters, alphanumeric and underscore only")
        if not self._valid_email(email):
            return chat_pb.SignupResponse(success=False, code=400, message="Invalid email format")
        ok, msg = self._valid_password(pw)
        if not ok:
            return chat_pb.SignupResponse(success=False, code=400, message=msg)
        with self.lock:
            if name in self.users:
                return chat_pb.SignupResponse(success=False, code=409, message="Username already exists")
            if email in self.users_by_email:
                return chat_pb.SignupResponse(success=False, code=409, message="Email already registered")
            self._add_user(name, pw, email, disp)
            self._save_users()
            info = self._user_info(name)
        return chat_pb.SignupResponse(success=True, code=201, message="Account created successfully!",
                                      user_info=info)

    def Login(self, request, context):
        with self.lock:
            u = self.users.get(request.username)
        if u is None or request.username in self.disabled or \
                not auth.bcrypt_checkpw(request.password.encode("utf-8"), u["password"]):
            return chat_pb.LoginResponse(success=False, message="Invalid username or password")
        tok = self._token(u["id"], request.username)
        with self.lock:
            self.sessions[tok] = {"user_id": u["id"], "username": request.username, "login_time": _now()}
            u["status"], u["last_seen"] = "online", _now()
            self.online.add(request.username)
            self._save_users()
            for ch in self.channels.values():
                if ch["name"] == "general":
                    ch["members"].add(u["id"])
                    self._save_channels()
                    break
            info = self._user_info(request.username)
        return chat_pb.LoginResponse(success=True, token=tok, message="Login successful", user_info=info)

    def Logout(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            self.sessions.pop(request.token, None)
            u = self.users.get(p["username"])
            if u:
                u["status"], u["last_seen"] = "offline", _now()
                self.online.discard(p["username"])
                self._save_users()
        self.broker.unsubscribe(p["user_id"])
        return chat_pb.StatusResponse(success=True, message="Logout successful", code=200)

    # ----------------------------------------------------------- streaming
    def StreamMessages(self, request, context):
        p = self._verify(request.token)
        if not p:
            return
        q = self.broker.subscribe(p["user_id"])
        try:
            while context.is_active():
                try:
                    yield q.get(timeout=0.5)
                except queue.Empty:
                    continue
        finally:
            self.broker.unsubscribe(p["user_id"], q)

    # ----------------------------------------------------------- channels
    def CreateChannel(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        name = request.channel_name.strip()
        if len(name) < 3:
            return chat_pb.StatusResponse(success=False, code=400,
                                          message="Channel name must be at least 3 characters")
        with self.lock:
            if any(c["name"].lower() == name.lower() for c in self.channels.values()):
                return chat_pb.StatusResponse(success=False, message="Channel already exists", code=409)
            cid = str(uuid.uuid4())
            self.channels[cid] = {"id": cid, "name": name, "description": request.description or f"Channel {name}",
                                  "is_private": request.is_private, "members": {p["user_id"]},
                                  "admins": {p["user_id"]}, "created_at": _now(), "created_by": p["username"]}
            self.messages[cid] = []
            self._save_channels()
        return chat_pb.StatusResponse(success=True, code=200, message=f"Channel #{name} created! You are the admin.")

    def JoinChannel(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            ch = self.channels.get(request.channel_id)
            if ch is None:
                return chat_pb.StatusResponse(success=False, message="Channel not found", code=404)
            ch["members"].add(p["user_id"])
            self._save_channels()
        self.broker.broadcast(ch["members"], chat_pb.MessageEvent(
            event_type="user_joined", user=self._user_info(p["username"]), channel_id=ch["id"]),
            exclude=p["user_id"])
        return chat_pb.StatusResponse(success=True, message=f"Joined #{ch['name']}", code=200)

    def LeaveChannel(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            ch = self.channels.get(request.channel_id)
            if ch is None:
                return chat_pb.StatusResponse(success=False, message="Channel not found", code=404)
            if p["user_id"] not in ch["members"]:
                return chat_pb.StatusResponse(success=False, message="Not a member of this channel", code=400)
            if ch["admins"] == {p["user_id"]} and len(ch["members"]) > 1:
                return chat_pb.StatusResponse(success=False, code=403,
                                              message="Last admin cannot leave; promote another admin first")
            ch["members"].discard(p["user_id"])
            self._save_channels()
        self.broker.broadcast(ch["members"], chat_pb.MessageEvent(
            event_type="user_left", user=self._user_info(p["username"]), channel_id=ch["id"]))
        return chat_pb.StatusResponse(success=True, message=f"Left #{ch['name']}", code=200)

    def GetChannels(self, request, context):
        if not self._verify(request.token):
            return chat_pb.ChannelListResponse(success=False, channels=[])
        with self.lock:
            chans = [chat_pb.Channel(channel_id=cid, name=c["name"], description=c["description"],
                                     is_private=c["is_private"], member_count=len(c["members"]),
                                     created_at=_ts(c.get("created_at")))
                     for cid, c in self.channels.items()]
        return chat_pb.ChannelListResponse(success=True, channels=chans)

    def ManageChannel(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            ch = self.channels.get(request.channel_id)
            if ch is None:
                return chat_pb.StatusResponse(success=False, message="Channel not found", code=404)
            if p["user_id"] not in ch["admins"]:
                return chat_pb.StatusResponse(success=False, code=403,
                                              message="Only channel admins can manage members")
            target = request.parameters.get("username")
            if request.action not in ("add_user", "remove_user"):
                return chat_pb.StatusResponse(success=False, message="Invalid action", code=400)
            if not target or target not in self.users:
                return chat_pb.StatusResponse(success=False, message="User not found", code=404)
            tid = self.users[target]["id"]
            if request.action == "add_user":
                ch["members"].add(tid)
                self._save_channels()
                return chat_pb.StatusResponse(success=True, message=f"Added {target} to channel", code=200)
            if tid in ch["admins"]:
                return chat_pb.StatusResponse(success=False, message="Cannot remove channel admin", code=403)
            ch["members"].discard(tid)
            self._save_channels()
            return chat_pb.StatusResponse(success=True, message=f"Removed {target} from channel", code=200)

    # ----------------------------------------------------------- messages
    def PostMessage(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            ch = self.channels.get(request.channel_id)
            if ch is None:
                return chat_pb.StatusResponse(success=False, message="Channel not found", code=404)
            if p["user_id"] not in ch["members"]:
                return chat_pb.StatusResponse(success=False, message="Not a member of this channel", code=403)
            m = {"id": str(uuid.uuid4()), "sender_id": p["user_id"], "sender_name": p["username"],
                 "channel_id": ch["id"], "content": request.content, "type": request.type or "text",
                 "timestamp": _now()}
            if request.file_data:
                fid = self._store_file(p, request.file_name or "attachment", request.file_data, "",
                                       ch["id"], None, "")
                m["file_url"] = f"file://{fid}"
            self.messages.setdefault(ch["id"], []).append(m)
            members = set(ch["members"])
        ev = chat_pb.MessageEvent(event_type="message", channel_id=ch["id"], message=self._msg_pb(m))
        self.broker.broadcast(members, ev, exclude=p["user_id"])
        return chat_pb.StatusResponse(success=True, message="Message sent", code=200)

    @staticmethod
    def _msg_pb(m):
        return chat_pb.Message(message_id=m["id"], sender_id=m["sender_id"], sender_name=m["sender_name"],
                               channel_id=m["channel_id"], content=m["content"], timestamp=_ts(m["timestamp"]),
                               type=m.get("type", ""), file_url=m.get("file_url", ""))

    def GetMessages(self, request, context):
        if not self._verify(request.token):
            return chat_pb.GetResponse(success=False, messages=[])
        limit = request.limit if request.limit > 0 else 50
        off = max(0, request.offset)
        with self.lock:
            allm = self.messages.get(request.channel_id, [])
            sl = allm[off:off + limit]
            nxt = str(off + limit) if off + limit < len(allm) else ""
            msgs = [self._msg_pb(m) for m in sl]
        return chat_pb.GetResponse(success=True, messages=msgs, next_cursor=nxt)

    def _dm_pb(self, d):
        return chat_pb.DirectMessage(message_id=d["id"], sender_id=d["sender_id"], sender_name=d["sender_name"],
                                     recipient_id=d["recipient_id"], recipient_name=d["recipient_name"],
                                     content=d["content"], timestamp=_ts(d["timestamp"]), is_read=d["is_read"],
                                     file_url=d.get("file_url", ""))

    def SendDirectMessage(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            r = self.users.get(request.recipient_username)
            if r is None:
                return chat_pb.StatusResponse(success=False, message="User not found", code=404)
            d = {"id": str(uuid.uuid4()), "sender_id": p["user_id"], "sender_name": p["username"],
                 "recipient_id": r["id"], "recipient_name": request.recipient_username,
                 "content": request.content, "timestamp": _now(), "is_read": False}
            if request.file_data:
                fid = self._store_file(p, request.file_name or "attachment", request.file_data, "", None,
                                       request.recipient_username, "")
                d["file_url"] = f"file://{fid}"
            self.direct_messages.append(d)
        self.broker.send_to_user(r["id"], chat_pb.MessageEvent(event_type="dm", direct_message=self._dm_pb(d)))
        return chat_pb.StatusResponse(success=True, message="DM sent", code=200)

    def GetDirectMessages(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.DirectMessageResponse(success=False, messages=[])
        with self.lock:
            o = self.users.get(request.other_username)
            if o is None:
                return chat_pb.DirectMessageResponse(success=False, messages=[])
            me, oid = p["user_id"], o["id"]
            conv = sorted((d for d in self.direct_messages
                           if {d["sender_id"], d["recipient_id"]} == {me, oid}),
                          key=lambda d: d["timestamp"])
            if request.offset > 0:
                conv = conv[: max(0, len(conv) - request.offset)]
            if request.limit > 0:
                conv = conv[-request.limit:]
            for d in conv:
                if d["recipient_id"] == me:
                    d["is_read"] = True
            msgs = [self._dm_pb(d) for d in conv]
        return chat_pb.DirectMessageResponse(success=True, messages=msgs)

    def ListConversations(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.ConversationsResponse(success=False, conversations=[])
        me = p["user_id"]
        with self.lock:
            last, unread = {}, {}
            for d in self.direct_messages:
                if me not in (d["sender_id"], d["recipient_id"]):
                    continue
                other = d["recipient_id"] if d["sender_id"] == me else d["sender_id"]
                last[other] = d
                if d["recipient_id"] == me and not d["is_read"]:
                    unread[other] = unread.get(other, 0) + 1
            convs = []
            for pid, d in last.items():
                name = self.users_by_id.get(pid)
                if name:
                    convs.append(chat_pb.Conversation(username=name,
                                                      display_name=self.users[name].get("display_name", name),
                                                      unread_count=unread.get(pid, 0), last_message=self._dm_pb(d)))
        return chat_pb.ConversationsResponse(success=True, conversations=convs)

    # ----------------------------------------------------------- users
    def GetOnlineUsers(self, request, context):
        if not self._verify(request.token):
            return chat_pb.UserListResponse(success=False, users=[])
        with self.lock:
            names = list(self.users)
            if request.channel_id and request.channel_id in self.channels:
                mem = self.channels[request.channel_id]["members"]
                names = [n for n in names if self.users[n]["id"] in mem]
            users = [self._user_info(n) for n in names]
        return chat_pb.UserListResponse(success=True, users=users)

    def UpdatePresence(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        status = request.status.strip().lower()
        if status not in ("online", "away", "busy", "offline"):
            return chat_pb.StatusResponse(success=False, message="Invalid status", code=400)
        with self.lock:
            u = self.users[p["username"]]
            u["status"], u["last_seen"] = status, _now()
            (self.online.add if status != "offline" else self.online.discard)(p["username"])
            self._save_users()
        return chat_pb.StatusResponse(success=True, message=f"Status set to {status}", code=200)

    def ManageUser(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.StatusResponse(success=False, message="Invalid token", code=401)
        with self.lock:
            if not self.users.get(p["username"], {}).get("is_admin"):
                return chat_pb.StatusResponse(success=False, message="Admin privileges required", code=403)
            name = self.users_by_id.get(request.target_user_id, request.target_user_id)
            u = self.users.get(name)
            if u is None:
                return chat_pb.StatusResponse(success=False, message="User not found", code=404)
            a = request.action
            if a == "promote":
                u["is_admin"] = True
            elif a == "demote":
                u["is_admin"] = False
            elif a == "disable":
                self.disabled.add(name)
                u["status"] = "offline"
            elif a == "enable":
                self.disabled.discard(name)
            else:
                return chat_pb.StatusResponse(success=False, message="Invalid action", code=400)
            self._save_users()
        return chat_pb.StatusResponse(success=True, message=f"{a} applied to {name}", code=200)

    def GetServerInfo(self, request, context):
        return chat_pb.ServerInfoResponse(is_leader=True, node_id=self.node_id, state="leader", current_term=0,
                                          leader_address=f"localhost:{self.port}", leader_id=self.node_id,
                                          log_size=0, commit_index=-1,
                                          cluster_nodes=[f"localhost:{self.port}"])

    # ----------------------------------------------------------- files
    def _store_file(self, p, name, data, mime, channel_id, recipient, desc):
        fid = str(uuid.uuid4())
        self.files[fid] = {"id": fid, "name": name, "data": bytes(data), "size": len(data),
                           "mime_type": mime or mimetypes.guess_type(name)[0] or "application/octet-stream",
                           "uploader_id": p["user_id"], "uploader_name": p["username"],
                           "channel_id": channel_id, "recipient": recipient, "description": desc,
                           "uploaded_at": _now()}
        return fid

    def _file_pb(self, fid, f):
        return chat_pb.FileMetadata(file_id=fid, file_name=f["name"], uploader_name=f["uploader_name"],
                                    file_size=f["size"], mime_type=f["mime_type"],
                                    uploaded_at=_ts(f["uploaded_at"]), channel_id=f.get("channel_id") or "")

    def UploadFile(self, request, context):
        p = self._verify(request.token)
        if not p:
            return chat_pb.FileUploadResponse(success=False, message="Invalid token")
        with self.lock:
            if request.channel_id and request.channel_id not in self.channels:
                return chat_pb.FileUploadResponse(success=False, message="Channel not found")
            fid = self._store_file(p, request.file_name, request.file_data, request.mime_type,
                                   request.channel_id or None, request.recipient_username or None,
                                   request.description)
            f = self.files[fid]
            members = set(self.channels[request.channel_id]["members"]) if request.channel_id else set()
        if request.channel_id:
            self.broker.broadcast(members, chat_pb.MessageEvent(event_type="file_uploaded",
                                                                file=self._file_pb(fid, f),
                                                                channel_id=request.channel_id),
                                  exclude=p["user_id"])
        return chat_pb.FileUploadResponse(success=True, message="File uploaded successfully", file_id=fid,
                                          file_url=f"file://{fid}")

    def DownloadFile(self, request, context):
        if not self._verify(request.token):
            return chat_pb.FileResponse(success=False)
        with self.lock:
            f = self.files.get(request.file_id)
        if f is None:
            return chat_pb.FileResponse(success=False)
        return chat_pb.FileResponse(success=True, file_name=f["name"], file_data=f["data"], mime_type=f["mime_type"])

    def ListFiles(self, request, context):
        if not self._verify(request.token):
            return chat_pb.FileListResponse(success=False, files=[])
        with self.lock:
            files = [self._file_pb(fid, f) for fid, f in self.files.items()
                     if f.get("channel_id") == request.channel_id]
        return chat_pb.FileListResponse(success=True, files=files)


def serve(port: int = 50050, data_dir: str = "server_data", block: bool = True, **kw):
    srv = LegacyChatServer(data_dir=data_dir, port=port, **kw)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=32), options=SERVER_QUEUE_OPTS)
    add_servicer(server, CHAT_SERVICE, srv)
    if server.add_insecure_port(f"[::]:{port}") == 0:
        raise RuntimeError(f"cannot bind {port}")
    server.start()
    if block:
        server.wait_for_termination()
    return srv, server


def main(argv=None):
    ap = argparse.ArgumentParser(description="legacy single-node chat.ChatService")
    # default differs from the reference's 50051, which collides with Raft node 1 (quirk Q26)
    ap.add_argument("--port", type=int, default=50050)
    ap.add_argument("--node_id", type=int, default=1)
    ap.add_argument("--data-dir", default="server_data")
    ap.add_argument("--log-level", default="INFO")
    a = parse_with_config(ap, argv)
    setup_logging(a.log_level)
    serve(a.port, a.data_dir, node_id=a.node_id)


if __name__ == "__main__":
    main()
