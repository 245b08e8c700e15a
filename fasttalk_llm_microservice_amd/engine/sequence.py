"""Request / sequence state tracked by the scheduler."""
from __future__ import annotations

import dataclasses
import enum
import time
from typing import Any, Callable, List, Optional

import numpy as np

from .sampling_params import SamplingParams


class SeqStatus(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    SWAPPED = "swapped"     # preempted with its KV blocks parked in host memory
    FINISHED = "finished"


@dataclasses.dataclass
class RequestOutput:
    """One streamed event for a request (what the engine hands the API layer)."""
    request_id: str
    text: str                       # text delta (complete UTF-8 characters)
    token_ids: List[int]            # new token ids in this delta
    finished: bool = False
    finish_reason: Optional[str] = None   # "stop" | "length" | "abort" | "error"
    num_prompt_tokens: int = 0
    num_cached_tokens: int = 0
    num_output_tokens: int = 0
    ttft_s: Optional[float] = None
    error: Optional[str] = None


class Sequence:
    __slots__ = ("request_id", "params", "prompt_len", "_tok", "n_tokens", "status", "block_ids",
                 "num_computed", "num_committed_blocks", "num_cached_tokens", "arrival",
                 "first_token_time", "finish_reason", "detok_stream", "on_output", "grammar",
                 "grammar_state", "stop_buf", "text_len", "aborted", "preemptions", "admit_order",
                 "meta", "host_slots", "background", "jf_text", "jf_ids", "lazy", "inflight",
                 "drop_next", "pf_sched", "epoch")

    def __init__(self, request_id: str, prompt_ids: List[int], params: SamplingParams,
                 on_output: Optional[Callable[[RequestOutput], None]] = None, meta: Any = None):
        self.request_id = request_id
        self.params = params
        self.prompt_len = len(prompt_ids)
        cap = max(64, len(prompt_ids) + min(params.max_tokens, 4096) + 1)
        self._tok = np.zeros(cap, dtype=np.int32)
        self._tok[: len(prompt_ids)] = prompt_ids
        self.n_tokens = len(prompt_ids)
        self.status = SeqStatus.WAITING
        self.block_ids: List[int] = []
        self.num_computed = 0
        self.num_committed_blocks = 0
        self.num_cached_tokens = 0
        self.arrival = time.perf_counter()
        self.first_token_time: Optional[float] = None
        self.finish_reason: Optional[str] = None
        self.detok_stream = -1
        self.on_output = on_output
        self.grammar = None
        self.grammar_state = -1
        self.stop_buf = ""
        self.text_len = 0
        self.aborted = False
        self.background = False   # prefix-cache warm-up: prefilled only into spare step room
        self.preemptions = 0
        self.admit_order = 0
        self.meta = meta
        self.host_slots: List[int] = []
        # jump-forward tokens appended at admission (guided decoding), reported with
        # the first sampled token's output
        self.jf_text = ""
        self.jf_ids: List[int] = []
        self.lazy = False   # grammar not bound yet (SamplingParams.guided_lazy)
        # queued (launched, not yet collected) steps that sample this sequence: its
        # next step's position / sampling step run this many tokens ahead of n_tokens
        self.inflight = 0
        # samples of queued steps to discard: a jump-forward (pipelined guided decoding)
        # appended forced tokens after the step behind it was already queued
        self.drop_next = 0
        # prompt tokens of prefill chunks in queued (launched, not yet post-stepped)
        # steps: the next chunk starts at num_computed + pf_sched
        self.pf_sched = 0
        # bumped when the sequence's KV is dropped (_reset_to_waiting): a queued
        # chunk scheduled before that is not counted when its step completes
        self.epoch = 0

    # ---------------------------------------------------------------- tokens
    @property
    def tokens(self) -> np.ndarray:
        return self._tok[: self.n_tokens]

    def append(self, tok: int):
        if self.n_tokens >= self._tok.shape[0]:
            self._tok = np.concatenate([self._tok, np.zeros(self._tok.shape[0], dtype=np.int32)])
        self._tok[self.n_tokens] = tok
        self.n_tokens += 1

    @property
    def num_output(self) -> int:
        return self.n_tokens - self.prompt_len

    @property
    def output_ids(self) -> List[int]:
        return self._tok[self.prompt_len: self.n_tokens].tolist()

    @property
    def last_token(self) -> int:
        return int(self._tok[self.n_tokens - 1])

    @property
    def is_finished(self) -> bool:
        return self.status == SeqStatus.FINISHED


def coalesce(first: RequestOutput, q) -> RequestOutput:
    """``first`` merged with the outputs already waiting in asyncio queue ``q``
    (text deltas concatenated, token ids appended, the last one's finish state).
    A consumer that fell behind the engine (e.g. one service process streaming
    many replicas' tokens) then sends one WS frame per wake-up instead of one per
    token, so it catches up instead of queueing without bound."""
    if q.empty() or first.finished:
        return first
    text = [first.text]
    ids = list(first.token_ids)
    o = first
    while not q.empty() and not o.finished:
        o = q.get_nowait()
        text.append(o.text)
        ids.extend(o.token_ids)
    return RequestOutput(first.request_id, "".join(text), ids, finished=o.finished,
                         finish_reason=o.finish_reason,
                         num_prompt_tokens=first.num_prompt_tokens or o.num_prompt_tokens,
                         num_cached_tokens=first.num_cached_tokens or o.num_cached_tokens,
                         num_output_tokens=o.num_output_tokens,
                         ttft_s=first.ttft_s if first.ttft_s is not None else o.ttft_s, error=o.error)
