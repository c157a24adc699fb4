"""Offline word-level tokenizer with a synthetic vocabulary of the model's size.

There are no vocab files or network in this environment, so the vocabulary
is generated deterministically: special tokens, the 256 byte tokens (lossless
fallback for any text), then English words (the reference's prompt templates,
a list of common chat words, and every word of the synthetic chat corpus)
with and without a leading space, then pseudo-words filling the remaining
ids up to ``vocab_size`` (128,256 for Llama-3, 32,000 for Mixtral, 256,000
for Gemma).  Text is pre-split GPT-style into `` ?word | ?punct | space``
pieces; each piece is one token when in the vocabulary, else its UTF-8 bytes.
Token counts of chat text therefore track a BPE tokenizer's (~1 token per
word), which is what matters for prefill/decode shapes.  (The reference
sends raw prompt text to a hosted API, llm_server/llm_server.py:167; the
prompt strings themselves are the reference's, see llm/prompts.py.)
"""
from __future__ import annotations

import importlib
import os
import random
import re

_PIECE = re.compile(r" ?[A-Za-z0-9_']+| ?[^\sA-Za-z0-9_']+|\s+")

COMMON_WORDS = """
the be to of and a in that have i it for not on with he as you do at this but his by from they we
say her she or an will my one all would there their what so up out if about who get which go me when
make can like time no just him know take people into year your good some could them see other than then
now look only come its over think also back after use two how our work first well way even new want
because any these give day most us is are was were been has had did does doing done said says going
yes yeah ok okay sure thanks thank please hello hi hey sounds great agree interesting point tell more
understand right maybe probably definitely really very much lot lets let's meeting tomorrow today tonight
project deadline review code bug fix deploy release build test tests plan design doc docs team channel
message messages reply replies question answer idea ideas discuss discussion topic topics summary key
points next step steps lunch coffee weekend friday monday call sync update status issue issues merge
branch server client cluster node leader raft vote term log commit gpu model latency throughput
performance benchmark chat file files upload download share join leave admin user users online offline
should would could might need needs help helps check checked looks good nice cool awesome perfect
""".split()

TEMPLATE_TEXT = """
Based on this conversation: Generate exactly 3 short, natural reply suggestions. Each suggestion should be:
- Under 10 words - Contextually relevant - Natural and conversational
Format: Just list the 3 suggestions, one per line, no numbering or bullets.
Summarize this conversation concisely in under characters: Then provide 3 key bullet points about the
discussion. Format: Summary: [your summary here] Key Points: - point 1 - point 2 - point 3
Based on this recent conversation context: User's question: Do not give more than 2 sentences in your
response. Provide a helpful, short, informative response that considers the conversation context:
Provide a short, helpful answer in 2 sentences or less. Based on this conversation context:
User started typing: Provide 3 natural completions for what they might want to say next, completing
their thought. Also suggest 2 related topics they could discuss. Format as simple lists: COMPLETIONS:
- completion 1 - completion 2 - completion 3 TOPICS: - topic 1 - topic 2 Suggest 3 natural things the
user might want to say next. - suggestion 1 - suggestion 2 - suggestion 3 No previous context
alice bob charlie Alice Bob Charlie
"""

SPECIALS = ["<pad>", "<bos>", "<eos>", "<unk>"]
_CONS = "bcdfghjklmnprstvwz"
_VOW = "aeiou"


def _pseudo_words(seed: int):
    rng = random.Random(seed)
    seen = set()
    while True:
        n = rng.randint(2, 4)
        w = "".join(rng.choice(_CONS) + rng.choice(_VOW) for _ in range(n))
        if w not in seen:
            seen.add(w)
            yield w


def _native_tokenizer(toks, byte_base, bos_id, skip_ids):
    """drtc_amd._native.WordTokenizer over ``toks``, or None without the native module
    (DRTC_NATIVE_TOKENIZER=0 forces the Python path)."""
    if os.environ.get("DRTC_NATIVE_TOKENIZER", "1") == "0":
        return None
    try:
        pkg = __name__.rsplit(".", 2)[0]
        mod = importlib.import_module(pkg + "._native")
        return mod.WordTokenizer(toks, byte_base, bos_id, skip_ids)
    except (ImportError, AttributeError):
        return None


class ChatTokenizer:
    def __init__(self, vocab_size: int, bos_id: int | None = None, eos_id: int | None = None,
                 seed: int = 1234):
        if vocab_size < len(SPECIALS) + 256 + 16:
            raise ValueError("vocab too small")
        self.vocab_size = vocab_size
        toks: list[str] = []
        seen: set[str] = set()

        def add(t: str):
            if t not in seen and len(toks) < vocab_size:
                seen.add(t)
                toks.append(t)

        for s in SPECIALS:
            add(s)
        self.byte_base = len(toks)
        for b in range(256):
            toks.append(f"<0x{b:02X}>")
        for p in ["\n", "\n\n", " ", "  ", ".", ",", ":", "-", "!", "?", "'", '"', "(", ")", "[", "]",
                  " -", " (", " [", " \"", "...", ")", "*", "•"]:
            add(p)
        words = list(dict.fromkeys(COMMON_WORDS + re.findall(r"[A-Za-z0-9_']+", TEMPLATE_TEXT)))
        for w in words:
            add(w)
            add(" " + w)
            add(w.capitalize())
            add(" " + w.capitalize())
        for d in range(10):
            add(str(d))
            add(" " + str(d))
        gen = _pseudo_words(seed)
        while len(toks) < vocab_size:
            w = next(gen)
            add(w)
            add(" " + w)
        self.id_to_tok = toks
        self.tok_to_id = {t: i for i, t in enumerate(toks)}
        self.pad_id, self.unk_id = 0, 3
        self.bos_id = 1 if bos_id is None else bos_id
        self.eos_id = 2 if eos_id is None else eos_id
        self._bytes = {i: bytes([i - self.byte_base]) for i in range(self.byte_base, self.byte_base + 256)}
        # native encode / decode (csrc/runtime/tokenizer.cpp, GIL released) for ASCII text;
        # this class stays the reference (non-ASCII input, no native build)
        self._nt = _native_tokenizer(toks, self.byte_base, self.bos_id,
                                     list(range(len(SPECIALS))) + [self.bos_id, self.eos_id])

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        if self._nt is not None and text.isascii():
            return self._nt.encode(text, add_bos)
        return self.encode_py(text, add_bos)

    def decode(self, ids, skip_special: bool = True) -> str:
        if self._nt is not None:
            try:
                return self._nt.decode(ids, skip_special).decode("utf-8", errors="replace")
            except TypeError:  # ids not convertible to int64 (e.g. a tensor): generic path
                pass
        return self.decode_py(ids, skip_special)

    def encode_py(self, text: str, add_bos: bool = True) -> list[int]:
        get = self.tok_to_id.get
        pieces = _PIECE.findall(text)
        ids = list(map(get, pieces))  # one C-level pass: the serving path's common case
        if None not in ids:
            return [self.bos_id, *ids] if add_bos else ids
        out = [self.bos_id] if add_bos else []
        for piece in pieces:
            t = get(piece)
            if t is not None:
                out.append(t)
                continue
            if piece.startswith(" ") and len(piece) > 1:
                sp = get(" ")
                t2 = get(piece[1:])
                if t2 is not None:
                    out.extend((sp, t2))
                    continue
            out.extend(self.byte_base + b for b in piece.encode("utf-8"))
        return out

    def decode_py(self, ids, skip_special: bool = True) -> str:
        buf = bytearray()
        for i in ids:
            i = int(i)
            if i in self._bytes:
                buf += self._bytes[i]
            elif 0 <= i < len(self.id_to_tok):
                if i < len(SPECIALS) or i in (self.bos_id, self.eos_id):
                    if not skip_special:
                        buf += self.id_to_tok[i].encode()
                    continue
                buf += self.id_to_tok[i].encode("utf-8")
        return buf.decode("utf-8", errors="replace")
