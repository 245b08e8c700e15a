"""Iteration-level (continuous batching) scheduler -- E4/E5/E6/E12 in SURVEY.md §2.3.

Replaces vLLM's scheduler behind ``--max-num-seqs`` / ``--max-num-batched-tokens``
(``docker-compose.vllm.yml:47-48``).  Policy:

* Prefill first: waiting requests are admitted FIFO while the step's token
  budget lasts; a prompt longer than the remaining budget is chunked (chunked
  prefill) and resumes on the next step.  On admission the longest cached
  prefix (full KV blocks of an earlier turn of the same conversation, or a shared
  system prompt) is attached from the C++ block manager, so only new tokens are
  computed.
* Otherwise one decode step for every running sequence.  A sequence that needs
  a new KV block when the pool is empty preempts the most recently admitted
  sequence (its blocks are released and it is recomputed later -- "recompute"
  preemption; cached prefix blocks usually make the recompute cheap).
"""
from __future__ import annotations

import collections
import dataclasses
from typing import Deque, Dict, List, Optional

from .sequence import SeqStatus, Sequence


@dataclasses.dataclass
class ScheduledBatch:
    is_prefill: bool
    seqs: List[Sequence]
    num_tokens: List[int]
    sample: List[bool]

    @property
    def total_tokens(self) -> int:
        return sum(self.num_tokens)


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
        b = self._schedule_prefill()
        if b is not None:
            return b
        return self._schedule_decode()

    def _schedule_prefill(self) -> Optional[ScheduledBatch]:
        if not self.waiting:
            return None
        budget = self.max_tokens
        seqs, ntok, samp = [], [], []
        while self.waiting and budget > 0 and len(self.running) + len(seqs) < self.max_num_seqs:
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
                if not seqs and not self.running:
                    # nothing can free memory: the prompt cannot fit at all
                    self.waiting.popleft()
                    self.release(seq)
                    seq.status = SeqStatus.FINISHED
                    seq.finish_reason = "error"
                    seqs.append(seq)
                    ntok.append(0)
                    samp.append(False)
                break
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
        if not seqs:
            return None
        return ScheduledBatch(True, seqs, ntok, samp)

    def _preempt_one(self, keep: Sequence) -> bool:
        for victim in reversed(self.running):
            if victim is keep:
                continue
            self.running.remove(victim)
            self.release(victim)
            victim.num_computed = 0
            victim.num_committed_blocks = 0
            victim.status = SeqStatus.WAITING
            victim.preemptions += 1
            self.waiting.appendleft(victim)
            self.num_preemptions += 1
            return True
        return False

    def _schedule_decode(self) -> Optional[ScheduledBatch]:
        if not self.running:
            return None
        seqs = []
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
                    self.release(seq)
                    seq.num_computed = 0
                    seq.num_committed_blocks = 0
                    seq.status = SeqStatus.WAITING
                    self.waiting.appendleft(seq)
                    continue
                seq.block_ids.extend(self.bm.allocate(need))
            seqs.append(seq)
        seqs = [s for s in seqs if s in self.running]
        if not seqs:
            return None
        return ScheduledBatch(False, seqs, [1] * len(seqs), [True] * len(seqs))

    def post_step(self, batch: ScheduledBatch):
        for seq, n, smp in zip(batch.seqs, batch.num_tokens, batch.sample):
            if seq.status == SeqStatus.FINISHED:
                continue
            seq.num_computed += n
            if batch.is_prefill and smp:
                seq.status = SeqStatus.RUNNING
                self._admit_counter += 1
                seq.admit_order = self._admit_counter
                self.running.append(seq)
            nfull = seq.num_computed // self.bs
            if nfull > seq.num_committed_blocks:
                self.bm.commit(seq.block_ids, seq.tokens, seq.num_computed, seq.num_committed_blocks)
                seq.num_committed_blocks = nfull
