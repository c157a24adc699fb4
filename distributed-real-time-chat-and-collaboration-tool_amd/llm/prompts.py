"""Prompt templates and output parsers of the four LLM features.

These define the service contract the reference's LLM server exposes
(llm_server/llm_server.py): the prompt text sent to the model and the way
its text is turned into the RPC response (3 smart replies; "Summary:" +
"Key Points:" bullets; "COMPLETIONS:" / "TOPICS:" lists; a <=2-sentence
answer).  The parsers are pure functions over model text so the same
contract holds for any backend (on-GPU engine, stub, canned fallback).
"""
from __future__ import annotations

from dataclasses import dataclass

# ----------------------------------------------------------------- constants
SMART_REPLY_FALLBACK = ["I agree", "That's interesting", "Tell me more"]
SMART_REPLY_EMPTY = ["Hello!", "How can I help?", "What's on your mind?"]
SMART_REPLY_PAD = ["I agree", "Interesting point"]
ANSWER_ERROR = ("I apologize, but I'm having trouble processing your request. "
                "Please try again.")
# ref llm_server.py:180 (empty response after every retry)
ANSWER_EMPTY = ("I'm having trouble generating a response. "
                "Please try rephrasing your question.")
SUMMARY_ERROR = "Unable to generate summary at this time."
SUGGEST_ERROR = ["sounds interesting", "tell me more", "I see"]


@dataclass
class ChatLine:
    sender: str
    content: str


def _conversation(messages, last: int | None = None) -> str:
    msgs = list(messages)
    if last is not None:
        msgs = msgs[-last:]
    return "\n".join(f"{m.sender}: {m.content}" for m in msgs)


# ------------------------------------------------------------------ fitting
def fit_prompt(tokenizer, text: str, limit: int) -> list[int]:
    """Token ids of ``text`` within ``limit`` tokens.  Every prompt above is
    instruction head + conversation + instruction tail (the output format the
    parsers rely on), so an over-long prompt loses its OLDEST conversation
    lines: the first line (e.g. "Summarize this conversation concisely in
    under N characters:") and the newest tail are kept, the middle is cut."""
    ids = tokenizer.encode(text)
    if len(ids) <= limit:
        return ids
    head = tokenizer.encode(text.split("\n", 1)[0] + "\n")
    if len(head) > limit // 2:  # degenerate one-line prompt: keep its start and end
        head = ids[:max(1, limit // 4)]
    keep_tail = limit - len(head)
    return head + ids[len(ids) - keep_tail:]


# ------------------------------------------------------------------ prompts
def answer_prompt(query: str, context: list[str]) -> str:
    """Ask-AI (llm_server.py:150-161): last 5 context strings + the question."""
    if context:
        ctx = "\n".join(list(context)[-5:])
        return ("Based on this recent conversation context:\n\n"
                f"{ctx}\n\n"
                f"User's question: {query}\n"
                "Do not give more than 2 sentences in your response.\n"
                "Provide a helpful, short, informative response that considers the "
                "conversation context:")
    return f"{query}\n\nProvide a short, helpful answer in 2 sentences or less."


def smart_reply_prompt(messages) -> str:
    """Smart reply (llm_server.py:220-229): last 5 messages."""
    return ("Based on this conversation:\n"
            f"{_conversation(messages, 5)}\n\n"
            "Generate exactly 3 short, natural reply suggestions. Each suggestion should be:\n"
            "- Under 10 words\n"
            "- Contextually relevant\n"
            "- Natural and conversational\n\n"
            "Format: Just list the 3 suggestions, one per line, no numbering or bullets.")


def summarize_prompt(messages, max_length: int) -> str:
    """Summarize (llm_server.py:272-285): every message given."""
    return (f"Summarize this conversation concisely in under {max_length} characters:\n\n"
            f"{_conversation(messages)}\n\n"
            "Then provide 3 key bullet points about the discussion.\n\n"
            "Format:\n"
            "Summary: [your summary here]\n\n"
            "Key Points:\n"
            "- point 1\n"
            "- point 2\n"
            "- point 3")


def suggestions_prompt(messages, current_input: str) -> str:
    """Context suggestions (llm_server.py:362-401)."""
    ctx = _conversation(messages, 5) if list(messages) else "No previous context"
    if current_input:
        return ("Based on this conversation context:\n"
                f"{ctx}\n\n"
                f"User started typing: \"{current_input}\"\n\n"
                "Provide 3 natural completions for what they might want to say next, "
                "completing their thought.\n"
                "Also suggest 2 related topics they could discuss.\n\n"
                "Format as simple lists:\n"
                "COMPLETIONS:\n"
                "- completion 1\n"
                "- completion 2  \n"
                "- completion 3\n\n"
                "TOPICS:\n"
                "- topic 1\n"
                "- topic 2")
    return ("Based on this conversation context:\n"
            f"{ctx}\n\n"
            "Suggest 3 natural things the user might want to say next.\n"
            "Also suggest 2 related topics they could discuss.\n\n"
            "Format as simple lists:\n"
            "COMPLETIONS:\n"
            "- suggestion 1\n"
            "- suggestion 2\n"
            "- suggestion 3\n\n"
            "TOPICS:\n"
            "- topic 1\n"
            "- topic 2")


# ------------------------------------------------------------------ parsers
def parse_answer(text: str) -> str:
    return text.strip()


def parse_smart_replies(text: str) -> list[str]:
    """3 lines; bullets/numbering stripped; padded with canned replies."""
    lines = [s.strip() for s in text.strip().split("\n") if s.strip()]
    cleaned = []
    for s in lines:
        s = s.lstrip("0123456789.-•*) ")
        if s:
            cleaned.append(s)
    if len(cleaned) >= 3:
        return cleaned[:3]
    return cleaned + SMART_REPLY_PAD[: 3 - len(cleaned)]


def _participants(messages) -> list[str]:
    return list({m.sender for m in messages})


def parse_summary(text: str, messages, max_length: int) -> tuple[str, list[str]]:
    text = text.strip()
    summary, points, in_points = "", [], False
    for line in text.split("\n"):
        line = line.strip()
        if line.startswith("Summary:"):
            summary = line.replace("Summary:", "").strip()
        elif "Key Points:" in line or "Key points:" in line:
            in_points = True
        elif in_points and (line.startswith("-") or line.startswith("•")):
            p = line.lstrip("-•* ").strip()
            if p:
                points.append(p)
        elif not in_points and summary and line:
            summary += " " + line
    if len(summary) > max_length:
        summary = summary[: max_length - 3] + "..."
    if not summary:
        summary = text[: max_length - 3] + "..." if len(text) > max_length else text
    if not points:
        parts = _participants(messages)
        points = [f"{len(messages)} messages exchanged",
                  f"Participants: {', '.join(parts[:3])}",
                  "Active discussion"]
    return summary, points[:3]


def parse_suggestions(text: str, current_input: str) -> tuple[list[str], list[str]]:
    suggestions, topics, section = [], [], None
    for line in text.strip().split("\n"):
        line = line.strip()
        up = line.upper()
        if "COMPLETION" in up or "SUGGESTION" in up:
            section = "s"
        elif "TOPIC" in up:
            section = "t"
        elif line.startswith("-") or line.startswith("•"):
            item = line.lstrip("-•* ").strip()
            if item:
                if section == "s":
                    suggestions.append(item)
                elif section == "t":
                    topics.append(item)
    if not suggestions:
        if current_input:
            suggestions = [f"{current_input} be the best option", f"{current_input} work well",
                           f"{current_input} make sense"]
        else:
            suggestions = ["continue the thought", "ask a question", "share more details"]
    if not topics:
        topics = ["current discussion", "related ideas"]
    return suggestions[:5], topics[:3]
