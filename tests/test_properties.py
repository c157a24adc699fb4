"""Property-based tests (hypothesis; SURVEY.md §4.2 unit-test plan): random
fault schedules against the Raft safety invariants, random command streams
against the replicated chat state machine, and the parsers / prompt fitting /
JWT / block allocator over arbitrary inputs.  CPU only."""
import string

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from drtc_amd.engine import ChatTokenizer
from drtc_amd.engine.block_allocator import BlockAllocator, PyBlockAllocator
from drtc_amd.llm import prompts as P
from drtc_amd.raft.core import NotLeaderError
from drtc_amd.raft.sim import SimCluster
from drtc_amd.raft.state_machine import ChatState
from drtc_amd.utils import auth

SLOW = settings(max_examples=20, deadline=None,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
FAST = settings(max_examples=150, deadline=None)


# ------------------------------------------------------------------ Raft
_raft_op = st.one_of(
    st.tuples(st.just("propose"), st.integers(1, 4)),
    st.tuples(st.just("partition"), st.integers(1, 4)),   # size of the first group
    st.tuples(st.just("heal"), st.just(0)),
    st.tuples(st.just("crash"), st.integers(1, 5)),
    st.tuples(st.just("restart"), st.integers(1, 5)),
    st.tuples(st.just("compact"), st.integers(1, 5)),
    st.tuples(st.just("run"), st.integers(1, 40)),          # x 10 ms
)


@SLOW
@given(seed=st.integers(0, 2**16), drop=st.sampled_from([0.0, 0.05, 0.2]),
       ops=st.lists(_raft_op, min_size=4, max_size=24))
def test_raft_safety_under_random_fault_schedules(seed, drop, ops):
    """Whatever the schedule of partitions, crashes, restarts, compactions and
    message loss/duplication: at most one leader per term, logs match, no two
    nodes apply different entries at one index, no entry any node applied is
    ever lost, and the healed cluster converges."""
    c = SimCluster(5, seed=seed, drop=drop, dup=0.05, delay=(0.001, 0.03))
    c.wait_leader(30)
    ever = {}  # log index -> entry applied there by some node at some point
    k = 0

    def record():
        for i in c.nodes:
            for idx, e in c.applied[i]:
                assert ever.setdefault(idx, e) == e, "two entries applied at one index"

    for op, arg in ops:
        ids = sorted(c.nodes)
        if op == "propose":
            for _ in range(arg):
                try:
                    c.propose("SEND_MESSAGE", str(k).encode())
                    k += 1
                except (RuntimeError, NotLeaderError):
                    pass
        elif op == "partition":
            c.partition = [set(ids[:arg]), set(ids[arg:])]
        elif op == "heal":
            c.partition = None
        elif op == "crash" and len(c.down) < 2:      # keep a majority able to exist
            c.crash(arg)
        elif op == "restart" and arg in c.down:
            c.restart(arg)
        elif op == "compact" and arg not in c.down:
            c.compact(arg)
        c.run(0.01 * (arg if op == "run" else 5))
        record()
    c.partition, c.drop = None, 0.0
    for i in list(c.down):
        c.restart(i)
    c.run(6.0)
    record()
    for t, ls in c.leaders_by_term.items():
        assert len(ls) == 1, f"two leaders in term {t}"
    applied = [c.applied[i] for i in sorted(c.nodes)]
    assert all(a == applied[0] for a in applied), "healed cluster did not converge"
    final = dict(applied[0])
    for idx, e in ever.items():
        assert final.get(idx) == e, f"applied entry {idx} lost"


# ------------------------------------------------------------ state machine
_name = st.text(string.ascii_lowercase, min_size=1, max_size=5)
_cmd = st.one_of(
    st.tuples(st.just("CREATE_USER"), _name),
    st.tuples(st.just("CREATE_CHANNEL"), _name),
    st.tuples(st.just("JOIN_CHANNEL"), st.tuples(_name, _name)),
    st.tuples(st.just("LEAVE_CHANNEL"), st.tuples(_name, _name)),
    st.tuples(st.just("SEND_MESSAGE"), st.tuples(_name, st.integers(0, 6), st.text(max_size=12))),
    st.tuples(st.just("SEND_DM"), st.tuples(_name, _name, st.integers(0, 6))),
    st.tuples(st.just("UPLOAD_FILE"), st.tuples(_name, st.binary(max_size=16))),
    st.tuples(st.just("REVOKE_TOKEN"), st.tuples(_name, st.integers(0, 100), st.integers(0, 100))),
)


def _entry(cmd, arg):
    if cmd == "CREATE_USER":
        return {"username": arg, "user_id": "u-" + arg, "password": "$2b$04$x", "email": "",
                "display_name": arg, "is_admin": False}
    if cmd == "CREATE_CHANNEL":
        return {"channel_id": "c-" + arg, "name": arg, "description": "", "is_private": False,
                "members": [], "admins": [], "created_at": "2025-01-01T00:00:00"}
    if cmd in ("JOIN_CHANNEL", "LEAVE_CHANNEL"):
        return {"channel_id": "c-" + arg[0], "user_id": "u-" + arg[1]}
    if cmd == "SEND_MESSAGE":
        return {"id": f"m{arg[1]}", "channel_id": "c-" + arg[0], "sender_id": "u", "content": arg[2]}
    if cmd == "SEND_DM":
        return {"id": f"d{arg[2]}", "sender_id": "u-" + arg[0], "sender_name": arg[0],
                "recipient_id": "u-" + arg[1], "recipient_name": arg[1], "content": "x"}
    if cmd == "UPLOAD_FILE":
        return {"file_id": "f-" + arg[0], "filename": arg[0], "data": arg[1].hex()}
    return {"token_hash": arg[0], "exp": arg[1], "ts": arg[2]}


def _view(s: ChatState):
    return (s.users, s.users_by_id, s.channels, s.channel_messages, s.direct_messages, s.files,
            s.revoked_tokens)


@FAST
@given(cmds=st.lists(_cmd, max_size=40))
def test_state_machine_replay_is_deterministic_idempotent_and_snapshots(cmds):
    """Replaying a committed stream gives the same state on every replica;
    re-applying an entry (retried RPC with the same request id) changes
    nothing; the Raft snapshot image restores an equal state with equal
    indexes (DM conversations)."""
    entries = [(c, _entry(c, a)) for c, a in cmds]
    a, b = ChatState(), ChatState()
    for c, d in entries:
        a.apply(c, dict(d))
    for c, d in entries:
        b.apply(c, dict(d))
        b.apply(c, dict(d))  # duplicate delivery of an idempotent write
    assert _view(a) == _view(b)
    msg_ids = [m["id"] for ms in a.channel_messages.values() for m in ms]
    assert len(msg_ids) == len(set(msg_ids))
    r = ChatState()
    r.restore_image(a.image())
    assert _view(r) == _view(a)
    names = sorted(a.users)
    for x in names[:3]:
        for y in names[:3]:
            assert r.conversation(x, y) == a.conversation(x, y)


# ---------------------------------------------------------------- parsers
@FAST
@given(text=st.text(max_size=300))
def test_smart_reply_parser_pads_to_the_reference_contract(text):
    """3 cleaned lines; fewer are padded from ["I agree", "Interesting point"],
    so a reply with no usable line yields those two (ref
    llm_server/llm_server.py:251-260, kept as is)."""
    out = P.parse_smart_replies(text)
    usable = [s.strip().lstrip("0123456789.-•*) ") for s in text.strip().split("\n")]
    n = sum(1 for s in usable if s)
    assert len(out) == (3 if n >= 1 else 2) and all(isinstance(s, str) and s for s in out)
    assert not any(s[0] in "0123456789.-•*) " for s in out[:min(n, 3)])


@FAST
@given(text=st.text(max_size=300), cur=st.text(max_size=10))
def test_suggestion_and_summary_parsers_bounds(text, cur):
    sug, top = P.parse_suggestions(text, cur)
    assert 1 <= len(sug) <= 5 and 1 <= len(top) <= 3
    msgs = [P.ChatLine("alice", "hi"), P.ChatLine("bob", "yo")]
    summary, points = P.parse_summary(text, msgs, 200)
    assert len(summary) <= 200 and 1 <= len(points) <= 3


_tok = ChatTokenizer(32000, 1, 2)


@FAST
@given(lines=st.lists(st.text(string.ascii_letters + " ,.?", min_size=1, max_size=40), min_size=1,
                      max_size=30), limit=st.integers(8, 200))
def test_fit_prompt_keeps_instruction_head_and_newest_tail(lines, limit):
    msgs = [P.ChatLine(f"u{i % 3}", s) for i, s in enumerate(lines)]
    text = P.summarize_prompt(msgs, 200)
    full = _tok.encode(text)
    ids = P.fit_prompt(_tok, text, limit)
    assert len(ids) <= max(limit, 1)
    if len(full) <= limit:
        assert ids == full
    else:
        head = _tok.encode(text.split("\n", 1)[0] + "\n")
        if len(head) <= limit // 2:
            assert ids[:len(head)] == head  # the "Summarize ..." instruction survives
        tail = len(ids) - len(head) if len(head) <= limit // 2 else len(ids) - max(1, limit // 4)
        assert ids[len(ids) - tail:] == full[len(full) - tail:]  # newest lines kept


# -------------------------------------------------------------------- JWT
_claims = st.dictionaries(st.text(string.ascii_letters, min_size=1, max_size=8),
                          st.one_of(st.text(max_size=20), st.integers(-10**6, 10**6)),
                          max_size=6)


@FAST
@given(claims=_claims, secret=st.text(min_size=1, max_size=32))
def test_jwt_roundtrip_and_tamper_detection(claims, secret):
    claims = {k: v for k, v in claims.items() if k not in ("exp", "nbf", "iat")}
    tok = auth.jwt_encode(claims, secret)
    assert auth.jwt_decode(tok, secret) == claims
    h, p, s = tok.split(".")
    bad = h + "." + p + "." + ("A" if s[0] != "A" else "B") + s[1:]
    with pytest.raises(auth.InvalidTokenError):
        auth.jwt_decode(bad, secret)
    with pytest.raises(auth.InvalidTokenError):
        auth.jwt_decode(tok, secret + "x")


# --------------------------------------------------------- block allocator
@FAST
@given(ops=st.lists(st.tuples(st.sampled_from(["alloc", "free", "incref"]), st.integers(0, 6)),
                    max_size=60))
def test_native_block_allocator_matches_python_twin(ops):
    nat, py = BlockAllocator(24, reserved=1), PyBlockAllocator(24, reserved=1)
    held: list[int] = []
    for op, n in ops:
        if op == "alloc":
            ok = py.can_allocate(n)
            assert nat.can_allocate(n) == ok
            if ok:
                a, b = nat.allocate(n), py.allocate(n)
                assert list(a) == b
                held += b
        elif op == "free" and held:
            blk = held.pop(n % len(held))
            nat.free([blk])
            py.free([blk])
        elif op == "incref" and held:
            blk = held[n % len(held)]
            nat.incref([blk])
            py.incref([blk])
            held.append(blk)
        assert (nat.num_free, nat.num_used) == (py.num_free, py.num_used)
    for blk in held:
        assert nat.refcount(blk) == py.refcount(blk) > 0


# ------------------------------------------------------------------ sampler
@FAST
@given(seed=st.integers(0, 2**20), V=st.integers(2, 300), k=st.integers(0, 40),
       p=st.floats(0.05, 1.0), t=st.floats(0.1, 2.0))
def test_sampler_reference_draws_inside_the_nucleus(seed, V, k, p, t):
    """ops.sampling.sample_ref (the HIP sampler's contract): a draw is inside
    the top-k set (ties kept) and inside the top-p nucleus of that set."""
    from drtc_amd.ops.sampling import sample_ref

    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(1, V, generator=g).round(decimals=1)  # rounding creates ties
    tok = int(sample_ref(logits, torch.tensor([t]), torch.tensor([k], dtype=torch.int32),
                         torch.tensor([p]), generator=g)[0])
    lf = logits[0]
    if 0 < k < V:
        assert lf[tok] >= torch.topk(lf, k).values[-1]
        cand = lf[lf >= torch.topk(lf, k).values[-1]]
    else:
        cand = lf
    probs = torch.softmax(cand / t, dim=-1)
    mass_above = probs[cand > lf[tok]].sum().item()
    assert mass_above < p + 1e-5
