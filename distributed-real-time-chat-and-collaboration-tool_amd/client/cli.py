"""Interactive chat client: ``python -m drtc_amd.client.cli [--server host:port]``.

Same command set as the reference CLI (client/chat_client.py:466-1783, SURVEY
§2.9): signup, login, logout, channels, create_channel, switch, join, send,
dm, conversations, back, history, users, reconnect, status, clear, upload,
download, files, smart_reply, ask, suggest, summarize, add_user,
remove_user, members, help, help_all - plus ``exit``/``quit``/EOF, which the
reference's help text advertised but never implemented (quirk Q20).

Fixes: the login channel-restore path reads real fields (Q19), ``switch``
checks membership through GetChannelMembers (Q21), sends are synchronous
with leader-redirect that targets the new stub (Q18/Q25).
"""
from __future__ import annotations

import argparse
import cmd
import getpass
import mimetypes
import os
import shlex
import sys
import uuid
from datetime import datetime

import grpc

from ..protos import raft_pb
from ..utils.config import parse_with_config
from ..utils.logging_utils import setup_logging
from .connection import DEFAULT_CLUSTER, ClusterConnection, ClusterUnavailable

BANNER = """
    +----------------------------------------------+
    |     Distributed Chat & Collaboration Tool    |
    |  Raft Consensus + Real-time Chat + GPU AI    |
    +----------------------------------------------+

    Commands: 'signup' | 'login <username>' | 'help'
    Test users: alice/alice123, bob/bob123, charlie/charlie123
"""
MAX_UPLOAD = 10 * 1024 * 1024  # client/chat_client.py:1226


def _ts(ms: int) -> str:
    return datetime.fromtimestamp(ms / 1000).strftime("%H:%M")


class ChatShell(cmd.Cmd):
    intro = BANNER
    prompt = "(chat) > "

    def __init__(self, conn: ClusterConnection, stdout=None, password_fn=None, input_fn=None,
                 download_dir: str = "downloads"):
        super().__init__(stdout=stdout)
        self.conn = conn
        self.token: str | None = None
        self.username: str | None = None
        self.channel_id: str | None = None
        self.channel_name: str | None = None
        self.dm_partner: str | None = None
        self.last_smart: list[str] = []
        self.last_suggest: list[str] = []
        self.password_fn = password_fn or getpass.getpass
        self.input_fn = input_fn or input
        self.download_dir = download_dir
        conn.on_leader_change = self._after_failover

    # ----------------------------------------------------------- failover
    def _after_failover(self, addr: str) -> None:
        """Session recovery on a new leader (ref client/chat_client.py:147-228):
        probe the token with GetOnlineUsers; auto-logout if the new leader
        rejects it; otherwise restore the current channel by name."""
        self.say(f" Reconnected to new leader at {addr}")
        if not self.token:
            return
        stub = self.conn.stub
        try:
            valid = stub.GetOnlineUsers(raft_pb.GetOnlineUsersRequest(token=self.token),
                                        timeout=2.0).success
        except grpc.RpcError:
            return  # leave the session as is; the next call retries discovery
        if not valid:
            who = self.username
            self.say("   Session expired on new leader")
            self.say("    Auto-logging out...")
            self.token = self.username = self.channel_id = self.dm_partner = None
            self.say(f"\n Please re-login: login {who}")
            return
        if self.channel_name and not self.dm_partner:
            try:
                r = stub.GetChannels(raft_pb.GetChannelsRequest(token=self.token), timeout=3.0)
            except grpc.RpcError:
                return
            for c in r.channels if r.success else []:
                if c.name.lower() == self.channel_name.lower():
                    if c.channel_id != self.channel_id:
                        self.channel_id = c.channel_id
                    self.say(f" Restored channel #{self.channel_name}")
                    break

    def _auto_logout(self, why: str) -> None:
        who = self.username or "<username>"
        self.say(f" {why}")
        self.say(" Auto-logging out...")
        self.token = self.username = self.channel_id = self.channel_name = self.dm_partner = None
        self.say(f"\n Please login again: login {who}")

    @staticmethod
    def _rid() -> str:
        """Idempotency key of one logical write (survives client retries)."""
        return uuid.uuid4().hex

    # ----------------------------------------------------------- plumbing
    def say(self, *parts) -> None:
        print(*parts, file=self.stdout)

    def emptyline(self):
        return False

    def default(self, line):
        self.say(f"Unknown command: {line.split()[0] if line.split() else line}. Type 'help'.")

    def onecmd(self, line):
        try:
            return super().onecmd(line)
        except ClusterUnavailable as e:
            self.say(f" {e}. Type 'reconnect' to try again.")
        except grpc.RpcError as e:
            self.say(f"Error: {e.code().name}: {e.details()}")
            self.say("Tip: Try 'status' to check cluster health")
        return False

    def _need_login(self) -> bool:
        if not self.token:
            self.say("Please login first")
            return True
        return False

    def _channels(self) -> list:
        r = self.conn.call("GetChannels", raft_pb.GetChannelsRequest(token=self.token))
        return list(r.channels) if r.success else []

    def _find_channel(self, name: str):
        name = name.lstrip("#")
        for c in self._channels():
            if c.name == name or c.channel_id == name:
                return c
        return None

    def _enter_channel(self, cid: str, name: str, show: int = 10) -> None:
        self.channel_id, self.channel_name, self.dm_partner = cid, name, None
        self.say(f" Now in #{name}")
        if show:
            self._show_recent(show)

    def _show_recent(self, limit: int) -> None:
        r = self.conn.call("GetMessages", raft_pb.GetMessagesRequest(
            token=self.token, channel_id=self.channel_id, limit=limit))
        if r.success and r.messages:
            self.say("-" * 50)
            for m in r.messages:
                who = "You" if m.sender_name == self.username else m.sender_name
                self.say(f"[{_ts(m.timestamp)}] {who}: {m.content}")
            self.say("-" * 50)

    # ----------------------------------------------------------- account
    def do_signup(self, arg):
        """Create an account: signup"""
        username = self.input_fn("Username: ").strip()
        email = self.input_fn("Email: ").strip()
        display = self.input_fn("Display name (optional): ").strip()
        password = self.password_fn("Password: ")
        if not username or not password:
            self.say("Username and password are required")
            return
        r = self.conn.call("Signup", raft_pb.SignupRequest(username=username, password=password,
                                                             email=email, display_name=display),
                           timeout=15.0, retry_deadline=False)
        self.say(f" {r.message}" if r.success else f" Signup failed: {r.message}")
        if r.success:
            self.say(f"Now login with: login {username}")

    def do_login(self, arg):
        """Log in: login <username>"""
        username = arg.strip() or self.input_fn("Username: ").strip()
        if not username:
            self.say("Usage: login <username>")
            return
        password = self.password_fn("Password: ")
        self.conn.ensure()
        r = self.conn.call("Login", raft_pb.LoginRequest(username=username, password=password),
                           timeout=15.0)
        if not r.success:
            self.say(f" Login failed: {r.message}")
            return
        self.token, self.username = r.token, username
        self.say(f" Welcome, {r.user_info.display_name or username}!")
        g = self._find_channel("general")
        if g is not None:
            if g.member_count == 0 or not self._is_member(g.channel_id):
                self.conn.call("JoinChannel", raft_pb.JoinChannelRequest(token=self.token,
                                                                         channel_id=g.channel_id))
            self._enter_channel(g.channel_id, g.name)

    def do_logout(self, arg):
        """Log out"""
        if self._need_login():
            return
        try:
            self.conn.call("Logout", raft_pb.LogoutRequest(token=self.token))
        finally:
            self.token = self.username = self.channel_id = self.channel_name = self.dm_partner = None
        self.say(" Logged out")

    # ----------------------------------------------------------- channels
    def _is_member(self, cid: str) -> bool:
        r = self.conn.call("GetChannelMembers", raft_pb.GetChannelMembersRequest(token=self.token,
                                                                                 channel_id=cid))
        return r.success and any(m.username == self.username for m in r.members)

    def do_channels(self, arg):
        """List channels"""
        if self._need_login():
            return
        best = {}
        for c in self._channels():
            if c.name not in best or c.member_count > best[c.name].member_count:
                best[c.name] = c
        self.say("\n Channels:")
        for name in sorted(best):
            c = best[name]
            mark = "*" if c.channel_id == self.channel_id else " "
            lock = " (private)" if c.is_private else ""
            self.say(f" {mark} #{name}{lock} - {c.member_count} members - {c.description}")

    def do_create_channel(self, arg):
        """Create a channel: create_channel <name> [description]"""
        if self._need_login():
            return
        parts = arg.split(maxsplit=1)
        if not parts:
            self.say("Usage: create_channel <name> [description]")
            return
        name, desc = parts[0].lstrip("#"), parts[1] if len(parts) > 1 else ""
        r = self.conn.call("CreateChannel", raft_pb.CreateChannelRequest(
            token=self.token, channel_name=name, description=desc), retry_deadline=False)
        if not r.success:
            self.say(f" {r.message}")
            return
        self.say(f" {r.message}")
        self._enter_channel(r.channel_id, name, show=0)

    def do_switch(self, arg):
        """Switch to a channel you are a member of: switch <name>"""
        if self._need_login():
            return
        if not arg.strip():
            self.say("Usage: switch <channel>")
            return
        c = self._find_channel(arg.strip())
        if c is None:
            self.say(f" Channel #{arg.strip()} not found")
            return
        if not self._is_member(c.channel_id):
            self.say(f" You are not a member of #{c.name}. Try: join {c.name}")
            return
        self._enter_channel(c.channel_id, c.name)

    def do_join(self, arg):
        """Join a public default channel: join <name>"""
        if self._need_login():
            return
        if not arg.strip():
            self.say("Usage: join <channel>")
            return
        c = self._find_channel(arg.strip())
        if c is None:
            self.say(f" Channel #{arg.strip()} not found")
            return
        r = self.conn.call("JoinChannel", raft_pb.JoinChannelRequest(token=self.token,
                                                                     channel_id=c.channel_id),
                           timeout=10.0)
        self.say(f" {r.message}")
        if r.success:
            self._enter_channel(c.channel_id, c.name)

    def do_members(self, arg):
        """List members of the current channel: members"""
        if self._need_login():
            return
        if not self.channel_id:
            self.say(" Not in any channel")
            return
        r = self.conn.call("GetChannelMembers", raft_pb.GetChannelMembersRequest(
            token=self.token, channel_id=self.channel_id))
        if not r.success:
            self.say(" Could not load members")
            return
        self.say(f"\n Members of #{self.channel_name} ({r.total_count}):")
        for m in sorted(r.members, key=lambda m: m.username):
            badge = " [admin]" if m.is_admin else ""
            self.say(f"  {'+' if m.status == 'online' else '-'} {m.username}{badge} ({m.display_name})")

    def do_add_user(self, arg):
        """Add a user to the current channel (admins): add_user <username>"""
        self._admin("AddUserToChannel", arg)

    def do_remove_user(self, arg):
        """Remove a user from the current channel (admins): remove_user <username>"""
        self._admin("RemoveUserFromChannel", arg)

    def _admin(self, rpc: str, arg: str) -> None:
        if self._need_login():
            return
        if not arg.strip() or not self.channel_id:
            self.say(f"Usage: {'add_user' if rpc.startswith('Add') else 'remove_user'} <username> "
                     "(inside a channel)")
            return
        r = self.conn.call(rpc, raft_pb.ChannelAdminRequest(token=self.token, channel_id=self.channel_id,
                                                           target_username=arg.strip()), timeout=10.0)
        self.say(r.message)

    # ----------------------------------------------------------- messaging
    def do_send(self, arg):
        """Send a message to the current channel or DM: send <message>"""
        if self._need_login():
            return
        if not arg:
            self.say("Usage: send <message>")
            return
        if self.dm_partner:
            r = self.conn.call("SendDirectMessage", raft_pb.DirectMessageRequest(
                token=self.token, recipient_username=self.dm_partner, content=arg,
                request_id=self._rid()))
            self.say(f"[{datetime.now():%H:%M}] You: {arg}" if r.success else f" Failed: {r.message}")
            return
        if not self.channel_id:
            self.say(" No channel selected. Use 'join <channel>' first.")
            self.say("Available channels: general, random, tech")
            return
        # the channel may have been removed / access lost since it was entered
        # (ref client/chat_client.py:802-815)
        if not any(c.channel_id == self.channel_id for c in self._channels()):
            self.say(f" Channel #{self.channel_name} no longer exists or you lost access.")
            self.say("  Rejoining general channel...")
            g = self._find_channel("general")
            if g is not None:
                self.conn.call("JoinChannel", raft_pb.JoinChannelRequest(token=self.token,
                                                                         channel_id=g.channel_id))
                self._enter_channel(g.channel_id, g.name, show=0)
            else:
                self.channel_id = self.channel_name = None
            return
        r = self.conn.call("SendMessage", raft_pb.SendMessageRequest(
            token=self.token, channel_id=self.channel_id, content=arg, request_id=self._rid()))
        if r.success:
            self.say(f"[{datetime.now():%H:%M}] You -> #{self.channel_name}: {arg}")
        else:
            self.say(f" Failed: {r.message}")

    def do_dm(self, arg):
        """Open a direct-message conversation: dm <username>"""
        if self._need_login():
            return
        who = arg.strip()
        if not who:
            self.say("Usage: dm <username>")
            return
        if who == self.username:
            self.say("Cannot DM yourself")
            return
        r = self.conn.call("GetDirectMessages", raft_pb.GetDirectMessagesRequest(
            token=self.token, other_username=who, limit=20))
        if not r.success:
            self.say(f" User @{who} not found")
            return
        self.dm_partner, self.channel_id, self.channel_name = who, None, None
        self.say(f" Direct message with @{who}  ('send <message>' to chat, 'back' to leave)")
        if r.messages:
            self.say("-" * 50)
            for m in r.messages:
                who_s = "You" if m.sender_name == self.username else m.sender_name
                self.say(f"[{_ts(m.timestamp)}] {who_s}: {m.content}")
            self.say("-" * 50)
        else:
            self.say(" No previous messages with this user")

    def do_conversations(self, arg):
        """List your DM conversations"""
        if self._need_login():
            return
        r = self.conn.call("ListConversations", raft_pb.ListConversationsRequest(token=self.token))
        if not r.conversations:
            self.say("No conversations yet")
            return
        self.say("\n Your Conversations:")
        for c in r.conversations:
            unread = f" ({c.unread_count} unread)" if c.unread_count else ""
            self.say(f"  @{c.username}{unread} - {c.display_name}")

    def do_back(self, arg):
        """Leave DM mode"""
        if self.dm_partner:
            self.dm_partner = None
            self.say("Back to channel mode. Use 'switch <channel>' or 'join <channel>'")
        else:
            self.say("Already in channel mode")

    def do_history(self, arg):
        """Show channel history: history [n]"""
        if self._need_login():
            return
        if self.dm_partner:
            self.say("History only works in channels. Type 'back' to return to channel mode.")
            return
        if not self.channel_id:
            self.say(" Not in any channel. Try: switch general")
            return
        try:
            n = int(arg) if arg.strip() else 20
        except ValueError:
            self.say("Usage: history [n]")
            return
        r = self.conn.call("GetMessages", raft_pb.GetMessagesRequest(
            token=self.token, channel_id=self.channel_id, limit=n))
        if not r.success:  # the token is not valid on this node (ref :1011-1021)
            self._auto_logout("Your session is invalid on this server")
            return
        if not r.messages:
            self.say("No messages yet. Be the first to say something!")
            return
        self.say(f"\n History of #{self.channel_name} (last {n}):")
        self.say("-" * 50)
        for m in r.messages:
            who = "You" if m.sender_name == self.username else m.sender_name
            self.say(f"[{_ts(m.timestamp)}] {who}: {m.content}")
        self.say("-" * 50)

    def do_users(self, arg):
        """List users and presence"""
        if self._need_login():
            return
        r = self.conn.call("GetOnlineUsers", raft_pb.GetOnlineUsersRequest(token=self.token))
        on = [u for u in r.users if u.status == "online"]
        off = [u for u in r.users if u.status != "online"]
        self.say(f"\n Online ({len(on)}): " + ", ".join(u.username for u in on))
        self.say(f" Offline ({len(off)}): " + ", ".join(u.username for u in off))

    # ----------------------------------------------------------- cluster
    def do_reconnect(self, arg):
        """Re-discover the Raft leader"""
        addr = self.conn.discover()
        self.say(f" Connected to leader at {addr}")
        self.do_status("")

    def do_status(self, arg):
        """Show cluster and session status"""
        self.say(f"\n Connected to: {self.conn.address}")
        self.say(f" User: {self.username or '(not logged in)'}")
        where = f"@{self.dm_partner} (DM)" if self.dm_partner else (f"#{self.channel_name}" if self.channel_name else "-")
        self.say(f" Location: {where}")
        self.say(" Cluster:")
        for addr, state, term, is_leader, leader in self.conn.node_status():
            star = " <- leader" if is_leader else ""
            t = f"term {term}" if term is not None else ""
            self.say(f"   {addr}: {state} {t}{star}")

    def do_clear(self, arg):
        """Clear the screen"""
        self.say("\033[2J\033[H" + BANNER)

    # ----------------------------------------------------------- files
    def do_upload(self, arg):
        """Upload a file to the current channel/DM: upload <path> [description]"""
        if self._need_login():
            return
        parts = shlex.split(arg) if arg else []
        if not parts:
            self.say("Usage: upload <path> [description]")
            return
        path = parts[0]
        if not os.path.isfile(path):
            self.say(f" File not found: {path}")
            return
        size = os.path.getsize(path)
        if size > MAX_UPLOAD:
            self.say(f" File too large ({size} bytes, max {MAX_UPLOAD})")
            return
        with open(path, "rb") as f:
            data = f.read()
        r = self.conn.call("UploadFile", raft_pb.FileUploadRequest(
            token=self.token, file_name=os.path.basename(path), file_data=data,
            channel_id=self.channel_id or "", recipient_username=self.dm_partner or "",
            description=" ".join(parts[1:]), mime_type=mimetypes.guess_type(path)[0] or "",
            request_id=self._rid()),
            timeout=30.0)
        self.say(f" Uploaded {os.path.basename(path)} (id {r.file_id})" if r.success else f" {r.message}")

    def do_download(self, arg):
        """Download a file: download <file_id> [save_as]"""
        if self._need_login():
            return
        parts = arg.split()
        if not parts:
            self.say("Usage: download <file_id> [save_as]")
            return
        r = self.conn.call("DownloadFile", raft_pb.FileDownloadRequest(token=self.token, file_id=parts[0]),
                           timeout=30.0)
        if not r.success:
            self.say(" File not found")
            return
        d = os.path.join(self.download_dir, self.username)
        os.makedirs(d, exist_ok=True)
        dest = os.path.join(d, os.path.basename(parts[1] if len(parts) > 1 else r.file_name))
        with open(dest, "wb") as f:
            f.write(r.file_data)
        self.say(f" Saved {len(r.file_data)} bytes to {dest}")

    def do_files(self, arg):
        """List files shared in the current channel"""
        if self._need_login():
            return
        if not self.channel_id:
            self.say(" Not in any channel")
            return
        r = self.conn.call("ListFiles", raft_pb.ListFilesRequest(token=self.token, channel_id=self.channel_id))
        if not r.files:
            self.say(" No files in this channel")
            return
        for f in r.files:
            self.say(f"  {f.file_id}  {f.file_name}  {f.file_size} B  {f.mime_type}  by {f.uploader_name}")

    # ----------------------------------------------------------- AI
    def do_smart_reply(self, arg):
        """AI reply suggestions: smart_reply [k]  (k sends the k-th suggestion)"""
        if self._need_login():
            return
        if arg.strip().isdigit() and self.last_smart:
            k = int(arg) - 1
            if 0 <= k < len(self.last_smart):
                self.do_send(self.last_smart[k])
            else:
                self.say(f"Pick 1..{len(self.last_smart)}")
            return
        if not self.channel_id:
            self.say(" Not in any channel")
            return
        r = self.conn.call("GetSmartReply", raft_pb.SmartReplyRequest(
            token=self.token, channel_id=self.channel_id, recent_message_count=5), timeout=20.0)
        self.last_smart = list(r.suggestions)
        self.say("\n Smart replies:")
        for i, s in enumerate(self.last_smart, 1):
            self.say(f"  {i}. {s}")
        self.say(" Use 'smart_reply <n>' to send one")

    def do_ask(self, arg):
        """Ask the AI assistant: ask <question>"""
        if self._need_login():
            return
        if not arg.strip():
            self.say("Usage: ask <question>")
            return
        r = self.conn.call("GetLLMAnswer", raft_pb.LLMRequest(token=self.token, query=arg, context=[]),
                           timeout=60.0)
        self.say(f"\n AI: {r.answer}")

    def do_suggest(self, arg):
        """Context-aware suggestions: suggest [partial text | k]"""
        if self._need_login():
            return
        if arg.strip().isdigit() and self.last_suggest:
            k = int(arg) - 1
            if 0 <= k < len(self.last_suggest):
                self.do_send(self.last_suggest[k])
            return
        if not self.channel_id:
            self.say(" Not in any channel")
            return
        r = self.conn.call("GetContextSuggestions", raft_pb.ContextSuggestionsRequest(
            token=self.token, channel_id=self.channel_id, current_input=arg.strip(),
            context_message_count=5), timeout=20.0)
        self.last_suggest = list(r.suggestions)
        self.say("\n Suggestions:")
        for i, s in enumerate(self.last_suggest, 1):
            self.say(f"  {i}. {s}")
        if r.topics:
            self.say(" Topics: " + ", ".join(r.topics))

    def do_summarize(self, arg):
        """Summarize the channel: summarize [n]  (n clamped to 5..100, default 20)"""
        if self._need_login():
            return
        if not self.channel_id:
            self.say(" Not in any channel")
            return
        n = 20
        if arg.strip():
            try:
                n = int(arg)
            except ValueError:
                self.say("Usage: summarize [n]")
                return
        n = max(5, min(100, n))
        r = self.conn.call("SummarizeConversation", raft_pb.SummarizeRequest(
            token=self.token, channel_id=self.channel_id, message_count=n), timeout=30.0)
        self.say(f"\n Summary: {r.summary}")
        for p in r.key_points:
            self.say(f"  - {p}")

    # ----------------------------------------------------------- help/exit
    HELP_GROUPS = (
        ("Account", ("signup", "login <username>", "logout")),
        ("Channels", ("channels", "create_channel <name> [description]", "switch <channel>",
                      "join <channel>", "send <message>", "history [n]", "members",
                      "add_user <username>  (channel admins)",
                      "remove_user <username>  (channel admins)")),
        ("Direct messages", ("dm <username>", "conversations", "back")),
        ("Files", ("upload <path> [description]", "download <file_id> [name]", "files")),
        ("AI", ("smart_reply [k]", "summarize [n]", "ask <question>", "suggest [text|k]")),
        ("Cluster", ("users", "status", "reconnect")),
        ("Other", ("clear", "help", "help_all", "exit / quit / Ctrl-D")),
    )

    def do_help(self, arg):
        """Show the command overview (help <command> for one command)"""
        if arg:
            return super().do_help(arg)
        self.say("\n" + "=" * 60 + "\nCOMMANDS\n" + "=" * 60)
        for title, cmds in self.HELP_GROUPS:
            self.say(f" {title}:")
            for c in cmds:
                self.say(f"   {c}")
        self.say(" 'help_all' lists every command with a one-line description.")

    def do_help_all(self, arg):
        """Show every command with its usage"""
        for name in sorted(n[3:] for n in self.get_names() if n.startswith("do_")):
            if name == "EOF":
                continue
            doc = getattr(self, "do_" + name).__doc__ or ""
            self.say(f"  {name:<16} {doc.strip().splitlines()[0] if doc else ''}")

    def do_exit(self, arg):
        """Exit the client"""
        self.say("Goodbye!")
        return True

    do_quit = do_exit

    def do_EOF(self, arg):  # noqa: N802
        self.say("")
        return self.do_exit(arg)


def main(argv=None):
    ap = argparse.ArgumentParser(description="drtc_amd chat client")
    ap.add_argument("--server", default=None, help="any node address (default: 3-node localhost cluster)")
    ap.add_argument("--nodes", default=None, help="comma-separated cluster addresses")
    ap.add_argument("--log-level", default="WARNING")  # the reference client logs at WARNING
    a = parse_with_config(ap, argv)
    setup_logging(a.log_level)
    nodes = a.nodes.split(",") if a.nodes else list(DEFAULT_CLUSTER)
    if a.server and a.server not in nodes:
        nodes.insert(0, a.server)
    conn = ClusterConnection(nodes)
    try:
        addr = conn.discover()
        print(f"Connected to Raft leader at {addr}")
    except ClusterUnavailable:
        print("Could not find a Raft leader. Start the cluster: python -m drtc_amd.server.node ...")
        sys.exit(1)
    try:
        ChatShell(conn).cmdloop()
    except KeyboardInterrupt:
        print("\nGoodbye!")


if __name__ == "__main__":
    main()
