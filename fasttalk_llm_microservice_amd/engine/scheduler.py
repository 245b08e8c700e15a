"""Iteration-level (continuous batching) scheduler -- E4/E5/E6/E12 in SURVEY.md §2.3.

Replaces vLLM's scheduler behind ``--max-num-seqs`` / ``--max-num-batched-tokens``
(``docker-compose.vllm.yml:47-48``).  Policy:

* Every step carries one decode token for every running sequence AND, in the
  same forward pass, prefill chunks of waiting requests up to the step's token
  budget (mixed continuous batching with chunked prefill): a new conversation
  turn is prefilled in the very next step without stalling the sessions that
  are streaming, which is what keeps p50 TTFT low at 50+ concurrent sessions.
  A prompt longer than the remaining budget is chunked and resumes next step.
* On admission the longest cached prefix (full KV blocks of an earlier turn of
  the same conversation, or a shared system prompt) is attached from the C++
  block manager, so only new tokens are computed.
* A sequence that needs a new KV block when the pool is empty preempts the
  most recently admitted sequence (its blocks are released and it is
  recomputed later -- "recompute" preemption; cached prefix blocks usually make
  the recompute cheap).
"""
from __future__ import annotations

import collections
import dataclasses
from typing import Deque, Dict, List, Optional

from .sequence import SeqStatus, Sequence


@dataclasses.dataclass
class ScheduledBatch:
    decode_seqs: List[Sequence]
    prefill_seqs: List[Sequence]
    prefill_tokens: List[int]
    prefill_sample: List[bool]
    rejected: List[Sequence] = dataclasses.field(default_factory=list)

    @property
    def is_prefill(self) -> bool:
        return not self.decode_seqs

    @property
    def has_prefill(self) -> bool:
        return bool(self.prefill_seqs)

    @property
    def seqs(self) -> List[Sequence]:
        return self.decode_seqs + self.prefill_seqs

    @property
    def total_tokens(self) -> int:
        return len(self.decode_seqs) + sum(self.prefill_tokens)

    def sampled_seqs(self) -> List[Sequence]:
        return self.decode_seqs + [s for s, sm in zip(self.prefill_seqs, self.prefill_sample) if sm]


class Scheduler:
    def __init__(self, block_manager, block_size: int, max_num_seqs: int,
                 max_num_batched_tokens: int, max_model_len: int):
        self.bm = block_manager
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[Sequence] = []
        self.by_id: Dict[str, Sequence] = {}
        self._admit_counter = 0
        self.num_preemptions = 0

    # ------------------------------------------------------------------ queue ops
    def add(self, seq: Sequence):
        self.by_id[seq.request_id] = seq
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting) or bool(self.running)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running)

    def release(self, seq: Sequence):
        """Free a sequence's KV blocks (full blocks stay cached for reuse)."""
        if seq.block_ids:
            self.bm.free(seq.block_ids)
            seq.block_ids = []

    def finish(self, seq: Sequence, reason: str):
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        self.release(seq)
        if seq in self.running:
            self.running.remove(seq)
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass
        self.by_id.pop(seq.request_id, None)

    def abort(self, request_id: str) -> Optional[Sequence]:
        seq = self.by_id.get(request_id)
        if seq is None:
            return None
        seq.aborted = True
        self.finish(seq, "abort")
        return seq

    # ------------------------------------------------------------------ scheduling
    def _blocks_needed(self, seq: Sequence, upto_tokens: int) -> int:
        return max(0, (upto_tokens + self.bs - 1) // self.bs - len(seq.block_ids))

    def schedule(self) -> Optional[ScheduledBatch]:
        decode = self._schedule_decode()
        budget = self.max_tokens - len(decode)
        pseqs, ptok, psamp, rejected = self._schedule_prefill(budget, len(decode))
        if not decode and not pseqs and not rejected:
            return None
        return ScheduledBatch(decode, pseqs, ptok, psamp, rejected)

    def _reset_to_waiting(self, seq: Sequence):
        """Drop a sequence's KV blocks (full blocks stay in the prefix cache, so a
        later admission re-attaches them) and restart its prefill from scratch."""
        self.release(seq)
        seq.num_computed = 0
        seq.num_committed_blocks = 0
        seq.num_cached_tokens = 0

    def _schedule_prefill(self, budget: int, n_decode: int):
        seqs, ntok, samp, rejected = [], [], [], []
        retried = None
        while self.waiting and budget > 0 and n_decode + len(seqs) < self.max_num_seqs:
            seq = self.waiting[0]
            if seq.num_computed == 0 and not seq.block_ids:
                max_blocks = (seq.n_tokens - 1) // self.bs
                if max_blocks > 0:
                    hit = self.bm.match_prefix(seq.tokens, max_blocks)
                    if hit:
                        seq.block_ids = list(hit)
                        seq.num_computed = len(hit) * self.bs
                        seq.num_committed_blocks = len(hit)
                        seq.num_cached_tokens = seq.num_computed
            remaining = seq.n_tokens - seq.num_computed
            chunk = min(remaining, budget)
            need = self._blocks_needed(seq, seq.num_computed + chunk)
            if need and not self.bm.can_allocate(need):
                # A waiting sequence must not sit on blocks (matched prefix or an
                # unfinished chunked prefill): they would starve the running
                # sequences, which then preempt themselves into a deadlock.
                self._reset_to_waiting(seq)
                if seqs or self.running:
                    break
                if retried is not seq:
                    # nothing is running: drop whatever other waiting sequences hold
                    # (an unfinished chunked prefill) and try once from scratch
                    retried = seq
                    for w in self.waiting:
                        if w.block_ids:
                            self._reset_to_waiting(w)
                    continue
                # nothing else holds memory and it still does not fit
                self.waiting.popleft()
                seq.status = SeqStatus.FINISHED
                seq.finish_reason = "error"
                rejected.append(seq)
                continue
            if need:
                seq.block_ids.extend(self.bm.allocate(need))
            seqs.append(seq)
            ntok.append(chunk)
            full = chunk == remaining
            samp.append(full)
            budget -= chunk
            if full:
                self.waiting.popleft()
            else:
                break  # the partially prefilled prompt continues next step
        return seqs, ntok, samp, rejected

    def _preempt_one(self, keep: Sequence) -> bool:
        # a waiting sequence in the middle of a chunked prefill gives its blocks up first
        for w in self.waiting:
            if w.block_ids:
                self._reset_to_waiting(w)
                self.num_preemptions += 1
                return True
        for victim in reversed(self.running):
            if victim is keep:
                continue
            self.running.remove(victim)
            self._reset_to_waiting(victim)
            victim.status = SeqStatus.WAITING
            victim.preemptions += 1
            self.waiting.appendleft(victim)
            self.num_preemptions += 1
            return True
        return False

    def _schedule_decode(self) -> List[Sequence]:
        if not self.running:
            return []
        for seq in list(self.running):
            if seq not in self.running:  # preempted while making room
                continue
            need = self._blocks_needed(seq, seq.n_tokens)
            while need and not self.bm.can_allocate(need):
                if not self._preempt_one(seq):
                    break
            if need:
                if not self.bm.can_allocate(need):
                    # cannot grow even alone: recompute later
                    self.running.remove(seq)
                    self._reset_to_waiting(seq)
                    seq.status = SeqStatus.WAITING
                    self.waiting.appendleft(seq)
                    continue
                seq.block_ids.extend(self.bm.allocate(need))
        return list(self.running)

    def post_step(self, batch: ScheduledBatch):
        items = [(s, 1, False) for s in batch.decode_seqs] + \
            list(zip(batch.prefill_seqs, batch.prefill_tokens, batch.prefill_sample))
        for seq, n, smp in items:
            if seq.status == SeqStatus.FINISHED:
                continue
            seq.num_computed += n
            if smp:
                seq.status = SeqStatus.RUNNING
                self._admit_counter += 1
                seq.admit_order = self._admit_counter
                self.running.append(seq)
            nfull = seq.num_computed // self.bs
            if nfull > seq.num_committed_blocks:
                self.bm.commit(seq.block_ids, seq.tokens, seq.num_computed, seq.num_committed_blocks)
                seq.num_committed_blocks = nfull
