"""Synthetic chat-log generator (no datasets in this environment).

Produces channel histories shaped like the reference's usage: short chat
lines from a handful of users (the seeded users alice/bob/charlie plus
others), 4-24 words each, drawn from a fixed chat vocabulary so they
tokenize at ~1 token per word.
"""
from __future__ import annotations

import random

from ..engine.tokenizer import COMMON_WORDS
from ..llm.prompts import ChatLine

USERS = ["alice", "bob", "charlie", "dana", "eve", "frank"]
_END = [".", "!", "?", "", "..."]


def chat_line(rng: random.Random) -> ChatLine:
    n = rng.randint(4, 24)
    words = [rng.choice(COMMON_WORDS) for _ in range(n)]
    words[0] = words[0].capitalize()
    if rng.random() < 0.3:
        words.insert(rng.randint(1, n - 1), ",")
    text = " ".join(words).replace(" ,", ",") + rng.choice(_END)
    return ChatLine(sender=rng.choice(USERS), content=text)


def channel_history(rng: random.Random, n: int) -> list[ChatLine]:
    return [chat_line(rng) for _ in range(n)]


def smart_reply_workload(num_requests: int, seed: int = 0, history: int = 5) -> list[list[ChatLine]]:
    """One 5-message context per smart-reply request (server/raft_node.py:1988)."""
    rng = random.Random(seed)
    return [channel_history(rng, history) for _ in range(num_requests)]
