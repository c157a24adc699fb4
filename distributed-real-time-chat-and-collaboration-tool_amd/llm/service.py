"""``llm.LLMService``: all four RPCs (the reference registers only two:
survey quirk Q15) over a text backend (on-GPU engine, DP router, scripted).

Each handler: build the feature's prompt (llm/prompts.py), generate with the
feature's sampling settings, parse into the response contract; any backend
failure yields the same fallback responses as the reference service
(llm_server/llm_server.py:45-145).  Handlers run concurrently on the gRPC
thread pool and meet in the engine's continuous batch.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..engine.request import SamplingParams
from ..protos import llm_pb
from ..utils.metrics import METRICS
from . import prompts as P

log = logging.getLogger(__name__)


class FeatureParams:
    """Sampling per feature.  Ask-AI uses the reference's explicit settings
    (temperature 0.7, 150 tokens: llm_server.py:168-172); the other three
    used the hosted SDK defaults (temperature 1.0, top-k 64, top-p 0.95)
    with output budgets sized to their format contracts."""

    def __init__(self, ignore_eos: bool = False):
        sdk = dict(temperature=1.0, top_k=64, top_p=0.95, ignore_eos=ignore_eos)
        self.answer = SamplingParams(max_new_tokens=150, temperature=0.7, top_k=64, top_p=0.95,
                                     ignore_eos=ignore_eos)
        self.smart = SamplingParams(max_new_tokens=48, **sdk)
        self.summary = SamplingParams(max_new_tokens=128, **sdk)
        self.suggest = SamplingParams(max_new_tokens=96, **sdk)


def _backend_for(backend, feature: str):
    """The backend serving ``feature`` (a FeatureRouter hosts one per feature)."""
    route = getattr(backend, "route", None)
    return route(feature) if route is not None else backend


class FeatureRouter:
    """One LLM service hosting several models: each feature ("smart", "summary", "answer",
    "suggest") is served by its own backend (an engine replica pool or a TP group on its
    share of the node's GPUs), as BASELINE.json assigns a model per feature.  Backends
    shared by several features are listed once in ``backends``."""

    FEATURES = ("smart", "summary", "answer", "suggest")
    ALIAS = {"smart_reply": "smart", "summarize": "summary", "ask": "answer"}

    def __init__(self, by_feature: dict, default=None):
        self.by_feature = dict(by_feature)
        self.default = default
        missing = [f for f in self.FEATURES if f not in self.by_feature and default is None]
        if missing:
            raise ValueError(f"no backend for features {missing}")
        uniq = {id(b): b for b in list(self.by_feature.values()) + [default] if b is not None}
        self.backends = list(uniq.values())

    def route(self, feature: str):
        return self.by_feature.get(self.ALIAS.get(feature, feature), self.default)

    def generate(self, prompts, params, timeout=None):  # feature-less callers: the default
        return (self.default or self.by_feature["smart"]).generate(prompts, params, timeout=timeout)

    def close(self) -> None:
        for b in self.backends:
            c = getattr(b, "close", None)
            if c is not None:
                c()


class LLMServicer:
    def __init__(self, backend, params: FeatureParams | None = None, timeout: float = 60.0,
                 answer_retries: int = 3, answer_backoff: float = 1.0):
        self.backend = backend
        self.p = params or FeatureParams()
        self.timeout = timeout
        # Ask-AI retries a failed or empty generation with exponential backoff
        # (answer_backoff * 2**attempt: 1 s, 2 s), as ref llm_server.py:164-208
        self.answer_retries = max(1, answer_retries)
        self.answer_backoff = answer_backoff

    def _gen(self, feature: str, prompt: str, params: SamplingParams, context=None) -> str:
        """Generate under the service timeout, shortened to the caller's RPC
        deadline: when the caller gives up, the backend aborts the request
        (its batch slot and KV blocks are freed) instead of finishing it."""
        t0 = time.perf_counter()
        timeout = self.timeout
        left = context.time_remaining() if context is not None else None
        if left is not None:
            timeout = min(timeout, max(0.05, left))
        text = _backend_for(self.backend, feature).generate([prompt], [params],
                                                            timeout=timeout)[0]
        METRICS.observe(f"llm.{feature}.latency_s", time.perf_counter() - t0)
        METRICS.inc(f"llm.{feature}.requests")
        return text

    def GetLLMAnswer(self, request, context):
        """Ask-AI with retry + exponential backoff (ref llm_server.py:164-208):
        an exception or an empty answer is retried up to ``answer_retries``
        attempts, never sleeping past the RPC deadline; the final failure maps
        to the reference's fallback strings (confidence 0)."""
        prompt = P.answer_prompt(request.query, list(request.context))
        empty = False
        for attempt in range(self.answer_retries):
            try:
                answer = P.parse_answer(self._gen("answer", prompt, self.p.answer, context))
                if answer:
                    return llm_pb.LLMResponse(request_id=request.request_id, answer=answer,
                                              confidence=0.95)
                empty = True
                log.warning("empty LLM answer (attempt %d)", attempt + 1)
            except Exception as e:
                empty = False
                log.warning("LLM answer attempt %d/%d failed: %s", attempt + 1,
                            self.answer_retries, str(e)[:120])
            if attempt + 1 < self.answer_retries:
                wait = self.answer_backoff * (2 ** attempt)
                left = context.time_remaining() if context is not None else None
                if left is not None and left < wait + 1.0:
                    break  # no time for another attempt before the caller's deadline
                METRICS.inc("llm.answer.retries")
                time.sleep(wait)
        log.error("LLM answer failed after retries")
        return llm_pb.LLMResponse(request_id=request.request_id,
                                  answer=P.ANSWER_EMPTY if empty else P.ANSWER_ERROR,
                                  confidence=0.0)

    # Each RPC other than ask-AI is (early answer | prompt, params, parse, fallback); the
    # thread-pool handlers below and the asyncio ones (AsyncLLMServicer) share these parts.
    def _smart_parts(self, request):
        msgs = list(request.recent_messages)
        rid = request.request_id
        if not msgs:
            return llm_pb.SmartReplyResponse(request_id=rid, suggestions=P.SMART_REPLY_EMPTY), None
        return None, ("smart_reply", P.smart_reply_prompt(msgs), self.p.smart,
                      lambda text: llm_pb.SmartReplyResponse(
                          request_id=rid, suggestions=P.parse_smart_replies(text)),
                      lambda: llm_pb.SmartReplyResponse(request_id=rid,
                                                        suggestions=P.SMART_REPLY_FALLBACK))

    def _summary_parts(self, request):
        msgs = list(request.messages)
        max_len = request.max_length if request.max_length > 0 else 200
        rid = request.request_id
        if not msgs:
            return llm_pb.SummarizeResponse(request_id=rid, summary="No messages to summarize",
                                            key_points=[]), None

        def ok(text):
            summary, points = P.parse_summary(text, msgs, max_len)
            return llm_pb.SummarizeResponse(request_id=rid, summary=summary, key_points=points)
        return None, ("summarize", P.summarize_prompt(msgs, max_len), self.p.summary, ok,
                      lambda: llm_pb.SummarizeResponse(request_id=rid, summary=P.SUMMARY_ERROR,
                                                       key_points=[]))

    def _suggest_parts(self, request):
        msgs = list(request.context)
        rid = request.request_id

        def ok(text):
            s, t = P.parse_suggestions(text, request.current_input)
            return llm_pb.SuggestionsResponse(request_id=rid, suggestions=s, topics=t)
        return None, ("suggest", P.suggestions_prompt(msgs, request.current_input),
                      self.p.suggest, ok,
                      lambda: llm_pb.SuggestionsResponse(request_id=rid,
                                                         suggestions=P.SUGGEST_ERROR, topics=[]))

    def _run(self, parts, context):
        early, job = parts
        if early is not None:
            return early
        feature, prompt, params, ok, fail = job
        try:
            return ok(self._gen(feature, prompt, params, context))
        except Exception as e:
            log.error("%s failed: %s", feature, e)
            return fail()

    def GetSmartReply(self, request, context):
        return self._run(self._smart_parts(request), context)

    def SummarizeConversation(self, request, context):
        return self._run(self._summary_parts(request), context)

    def GetContextSuggestions(self, request, context):
        return self._run(self._suggest_parts(request), context)


class AsyncLLMServicer(LLMServicer):
    """The same four RPCs as coroutines for a ``grpc.aio`` server: one event-loop thread
    serves every in-flight request (no handler thread per generation), and a replica's
    completions resolve their futures from the pool's collector thread.  Backends without
    an ``agenerate`` coroutine run ``generate`` on the loop's default executor."""

    async def _agen(self, feature: str, prompt: str, params: SamplingParams, context=None) -> str:
        t0 = time.perf_counter()
        timeout = self.timeout
        left = context.time_remaining() if context is not None else None
        if left is not None:
            timeout = min(timeout, max(0.05, left))
        backend = _backend_for(self.backend, feature)
        agen = getattr(backend, "agenerate", None)
        if agen is not None:
            text = await agen(prompt, params, timeout=timeout)
        else:
            loop = asyncio.get_running_loop()
            text = (await loop.run_in_executor(
                None, lambda: backend.generate([prompt], [params], timeout=timeout)))[0]
        METRICS.observe(f"llm.{feature}.latency_s", time.perf_counter() - t0)
        METRICS.inc(f"llm.{feature}.requests")
        return text

    async def _arun(self, parts, context):
        early, job = parts
        if early is not None:
            return early
        feature, prompt, params, ok, fail = job
        try:
            return ok(await self._agen(feature, prompt, params, context))
        except Exception as e:
            log.error("%s failed: %s", feature, e)
            return fail()

    async def GetLLMAnswer(self, request, context):
        """Ask-AI with the retry + backoff of LLMServicer.GetLLMAnswer (asyncio sleeps)."""
        prompt = P.answer_prompt(request.query, list(request.context))
        empty = False
        for attempt in range(self.answer_retries):
            try:
                answer = P.parse_answer(await self._agen("answer", prompt, self.p.answer, context))
                if answer:
                    return llm_pb.LLMResponse(request_id=request.request_id, answer=answer,
                                              confidence=0.95)
                empty = True
                log.warning("empty LLM answer (attempt %d)", attempt + 1)
            except Exception as e:
                empty = False
                log.warning("LLM answer attempt %d/%d failed: %s", attempt + 1,
                            self.answer_retries, str(e)[:120])
            if attempt + 1 < self.answer_retries:
                wait = self.answer_backoff * (2 ** attempt)
                left = context.time_remaining() if context is not None else None
                if left is not None and left < wait + 1.0:
                    break
                METRICS.inc("llm.answer.retries")
                await asyncio.sleep(wait)
        log.error("LLM answer failed after retries")
        return llm_pb.LLMResponse(request_id=request.request_id,
                                  answer=P.ANSWER_EMPTY if empty else P.ANSWER_ERROR,
                                  confidence=0.0)

    async def GetSmartReply(self, request, context):
        return await self._arun(self._smart_parts(request), context)

    async def SummarizeConversation(self, request, context):
        return await self._arun(self._summary_parts(request), context)

    async def GetContextSuggestions(self, request, context):
        return await self._arun(self._suggest_parts(request), context)
