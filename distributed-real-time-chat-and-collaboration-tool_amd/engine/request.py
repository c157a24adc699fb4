"""Request / sampling-parameter objects of the serving engine."""
from __future__ import annotations

import enum
import itertools
import threading
import time
from dataclasses import dataclass, field


@dataclass
class SamplingParams:
    """Per-request generation settings.

    Defaults mirror the hosted backend the reference called with SDK defaults
    (llm_server/llm_server.py:231,287,403); Ask-AI overrides temperature 0.7
    and 150 output tokens (llm_server/llm_server.py:168-172)."""
    max_new_tokens: int = 64
    temperature: float = 1.0
    top_k: int = 64
    top_p: float = 0.95
    ignore_eos: bool = False
    stop_token_ids: tuple = ()

    @staticmethod
    def greedy(max_new_tokens: int = 64, ignore_eos: bool = False) -> "SamplingParams":
        return SamplingParams(max_new_tokens=max_new_tokens, temperature=0.0, top_k=0,
                              top_p=1.0, ignore_eos=ignore_eos)


class RequestState(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    FINISHED = "finished"


_ids = itertools.count()
_ev_lock = threading.Lock()


@dataclass
class Request:
    prompt_ids: list
    params: SamplingParams = field(default_factory=SamplingParams)
    request_id: str = ""
    # engine-managed state
    output_ids: list = field(default_factory=list)
    blocks: list = field(default_factory=list)
    state: RequestState = RequestState.WAITING
    slot: int = -1
    finish_reason: str = ""
    arrival_time: float = field(default_factory=time.perf_counter)
    first_token_time: float = 0.0
    finish_time: float = 0.0
    num_preemptions: int = 0
    # completion Event, created by the first wait() only: a threading.Event costs ~4 us to
    # build, and a 1024-request wave creates its requests on the critical path between waves
    _done: threading.Event | None = field(default=None, repr=False)
    # called once with the request when it finishes (engine thread): lets a server
    # collect completions from a queue instead of polling every pending request
    on_done: object = field(default=None, repr=False, compare=False)

    def __post_init__(self):
        if not self.request_id:
            self.request_id = f"req-{next(_ids)}"

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def all_ids(self) -> list:
        return list(self.prompt_ids) + list(self.output_ids)

    @property
    def latency(self) -> float:
        return self.finish_time - self.arrival_time if self.finish_time else 0.0

    @property
    def ttft(self) -> float:
        return self.first_token_time - self.arrival_time if self.first_token_time else 0.0

    def wait(self, timeout: float | None = None) -> bool:
        # the Event exists before the state is read, and mark_finished sets the state before
        # it reads _done: a finish either sees this Event and sets it, or happened before
        # the state check below
        ev = self._done
        if ev is None:
            with _ev_lock:
                ev = self._done
                if ev is None:
                    ev = self._done = threading.Event()
        if self.state is RequestState.FINISHED:
            return True
        return ev.wait(timeout)

    def mark_finished(self, reason: str) -> None:
        self.finish_reason = reason
        self.finish_time = time.perf_counter()
        self.state = RequestState.FINISHED
        ev = self._done
        if ev is not None:
            ev.set()
        cb = self.on_done
        if cb is not None:
            self.on_done = None  # at most once (an abort may race a normal finish)
            cb(self)
