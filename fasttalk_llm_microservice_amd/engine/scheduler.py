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
  most recently admitted sequence.  With host swap space (``--swap-space``,
  ``docker-compose.vllm.yml:49``) the victim's blocks are copied to pinned host
  memory and copied back when blocks free up (its generation continues exactly
  where it stopped, sampling stream included); without it, or when the host
  pool is full, its blocks are released and it is recomputed later
  ("recompute" preemption; cached prefix blocks usually make that cheap).
  Swapped sequences resume before new prompts are admitted.
"""
from __future__ import annotations

import collections
import dataclasses
import time
from typing import Deque, Dict, List, Optional, Tuple

from .sequence import SeqStatus, Sequence


@dataclasses.dataclass
class ScheduledBatch:
    decode_seqs: List[Sequence]
    prefill_seqs: List[Sequence]
    prefill_tokens: List[int]
    prefill_sample: List[bool]
    rejected: List[Sequence] = dataclasses.field(default_factory=list)
    # (device block, host slot) copies to run BEFORE this step's forward pass,
    # swap-outs first: a block freed by a swap-out may be reused by this step
    swap_out: List[Tuple[int, int]] = dataclasses.field(default_factory=list)
    swap_in: List[Tuple[int, int]] = dataclasses.field(default_factory=list)
    # per prefill chunk: first prompt position and the sequence's epoch when it was
    # scheduled (Scheduler.stamp); empty for batches built outside the scheduler
    prefill_start: List[int] = dataclasses.field(default_factory=list)
    prefill_epoch: List[int] = dataclasses.field(default_factory=list)

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


class HostSwapPool:
    """Slots of the pinned host KV pool (one slot = one KV block of every layer)."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))

    def num_free(self) -> int:
        return len(self._free)

    def can_allocate(self, n: int) -> bool:
        return len(self._free) >= n

    def allocate(self, n: int) -> List[int]:
        return [self._free.pop() for _ in range(n)]

    def release(self, slots: List[int]):
        self._free.extend(reversed(slots))


class Scheduler:
    def __init__(self, block_manager, block_size: int, max_num_seqs: int,
                 max_num_batched_tokens: int, max_model_len: int, host_blocks: int = 0,
                 prefill_chunk: int = 0, chunk_counts_decode: bool = False,
                 guided_prefill_cap: int = 0):
        self.bm = block_manager
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.admit_trace: Optional[list] = None   # the engine's step trace list, when on
        # Soft prefill budget (0 = off): the first waiting prompt may fill the whole
        # step budget (a lone long prompt prefills in one step), further prompts join
        # only up to this many prefill tokens per step.  A burst of many short turns
        # (every session of a voice chat answering at once) is then served in several
        # short steps instead of one long one, so most of them see their first token
        # after a fraction of the burst: p50 TTFT 127 -> 62 ms at 50 sessions for
        # -1% throughput (profiles/ab_prefill_chunk_r02.log).  chunk_counts_decode:
        # the budget bounds decode rows + prefill tokens, so burst steps stay inside
        # four 256-row prefill GEMM tiles (mixed steps at 953-1050 rows 32.4/31.5 ms
        # -> 28.6 ms at <= 1024 rows, profiles/ab_prefill_chunk_rows_r02.log).  The
        # default budget is 512 rows: p50 TTFT 63 -> 39-42 ms at unchanged tok/s vs
        # 1024; 384 / 256 cost 2.5-3.5% tok/s (profiles/ab_prefill_chunk_512_r02.log).
        self.prefill_chunk = int(prefill_chunk)
        self.chunk_counts_decode = bool(chunk_counts_decode)
        # Prefill tokens a step may carry while it decodes a guided (tool-call) row
        # (0 = no cap): the free argument string of a call (~14 tokens) is decoded one
        # token per step, and a step carrying a full prefill chunk takes ~2x a decode
        # step, so a tool turn's time to its re-prompt grows with every chunk it rides
        # along (tool-turn p99 406 ms).
        self.guided_prefill_cap = int(guided_prefill_cap)
        self.guided_capped = 0
        self.max_model_len = max_model_len
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[Sequence] = []
        self.by_id: Dict[str, Sequence] = {}
        self._admit_counter = 0
        self.num_preemptions = 0
        self.stale_chunks = 0   # chained prefill chunks whose sequence was reset in flight
        self.swapped: Deque[Sequence] = collections.deque()
        # background (prefix-cache warm-up) prompts: prefilled only into the room a
        # step has left after every waiting prompt, within the soft budget
        self.background: Deque[Sequence] = collections.deque()
        self.host = HostSwapPool(host_blocks) if host_blocks > 0 else None
        self._swap_out: List[Tuple[int, int]] = []
        self.num_swap_out = 0
        self.num_swap_in = 0

    # ------------------------------------------------------------------ queue ops
    def add(self, seq: Sequence):
        self.by_id[seq.request_id] = seq
        if seq.background:
            self.background.append(seq)
            return
        # SamplingParams.priority (opt-in, default 0; NativeHandler.stream_events(priority=)):
        # a prompt of priority p > 0 is prefilled ahead of every waiting prompt of lower
        # priority that has not started yet.  A chunked prefill in progress keeps its place,
        # and so does a sequence re-queued by preemption (it was admitted before the new
        # prompt arrived; jumping it again would starve it under memory pressure).
        pr = getattr(seq.params, "priority", 0)
        if pr > 0 and self.waiting:
            i = 0
            for i, q in enumerate(self.waiting):
                if q.num_computed == 0 and q.preemptions == 0 and \
                        getattr(q.params, "priority", 0) < pr:
                    break
            else:
                i = len(self.waiting)
            self.waiting.insert(i, seq)
            return
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting) or bool(self.running) or bool(self.swapped) or bool(self.background)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running) + len(self.swapped) + len(self.background)

    def release(self, seq: Sequence):
        """Free a sequence's KV blocks (full blocks stay cached for reuse) and its
        host swap slots."""
        if seq.block_ids:
            self.bm.free(seq.block_ids)
            seq.block_ids = []
        if seq.host_slots:
            self.host.release(seq.host_slots)
            seq.host_slots = []

    def finish(self, seq: Sequence, reason: str):
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        self.release(seq)
        if seq in self.running:
            self.running.remove(seq)
        else:
            for q in (self.waiting, self.swapped, self.background):
                try:
                    q.remove(seq)
                    break
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
        self._swap_out = []
        decode = self._schedule_decode()
        swap_in: List[Tuple[int, int]] = []
        if self.swapped and not self._swap_out:
            resumed, swap_in = self._schedule_swap_in(len(decode))
            decode += resumed
        # jump-forward (guided decoding): a running sequence whose grammar forced a run
        # of tokens has them pending past the sampled one; they are prefilled as one
        # chunk (sampled at its last row) instead of one decode step each
        jumps = [s for s in decode if s.n_tokens - s.num_computed > 1]
        if jumps:
            decode = [s for s in decode if s.n_tokens - s.num_computed <= 1]
        jtok = [s.n_tokens - s.num_computed for s in jumps]
        budget = self.max_tokens - len(decode) - sum(jtok)
        if self.guided_prefill_cap > 0 and any(
                s.grammar is not None and not s.lazy for s in decode):
            budget = min(budget, self.guided_prefill_cap)
            self.guided_capped += 1
        n_rows = len(decode) + len(jumps)
        if self.swapped:  # swapped sequences go first; only unfinished chunks continue
            pseqs, ptok, psamp, rejected = [], [], [], []
        else:
            pseqs, ptok, psamp, rejected = self._schedule_prefill(budget, n_rows)
        if jumps:
            pseqs, ptok, psamp = jumps + pseqs, jtok + ptok, [True] * len(jumps) + psamp
        swap_out, self._swap_out = self._swap_out, []
        if not decode and not pseqs and not rejected and not swap_out and not swap_in:
            return None
        return self.stamp(ScheduledBatch(decode, pseqs, ptok, psamp, rejected, swap_out, swap_in))

    @staticmethod
    def stamp(batch: ScheduledBatch) -> ScheduledBatch:
        """Records where each prefill chunk starts and counts it as scheduled
        (``pf_sched``) until its step's post_step, so a step queued behind this one
        before it completes (engine mixed chain) continues a chunked prompt after it
        instead of repeating it."""
        batch.prefill_start = [s.num_computed + s.pf_sched for s in batch.prefill_seqs]
        batch.prefill_epoch = [s.epoch for s in batch.prefill_seqs]
        for s, n in zip(batch.prefill_seqs, batch.prefill_tokens):
            s.pf_sched += n
        return batch

    def _swap_out_seq(self, seq: Sequence) -> bool:
        """Parks a running sequence's KV blocks in host memory (False if there is no
        host pool or it is full: the caller falls back to recompute)."""
        n = len(seq.block_ids)
        if self.host is None or n == 0 or not self.host.can_allocate(n):
            return False
        slots = self.host.allocate(n)
        self._swap_out.extend(zip(seq.block_ids, slots))
        self.bm.free(seq.block_ids)  # reusable in this step: the copies run first
        seq.block_ids = []
        seq.host_slots = slots
        seq.status = SeqStatus.SWAPPED
        self.swapped.append(seq)
        self.num_swap_out += 1
        return True

    def _schedule_swap_in(self, n_running: int):
        """Brings swapped sequences back (FIFO) while their blocks, plus the one
        this step's decode token needs, fit.  Full blocks still in the device
        prefix cache are re-attached instead of copied."""
        resumed, pairs = [], []
        while self.swapped and n_running + len(resumed) < self.max_num_seqs:
            seq = self.swapped[0]
            hit = self.bm.match_prefix(seq.tokens, seq.num_committed_blocks) \
                if seq.num_committed_blocks else []
            nslots = len(seq.host_slots)
            total = max((seq.n_tokens + self.bs - 1) // self.bs, nslots)
            need = total - len(hit)
            if not self.bm.can_allocate(need):
                if hit:
                    self.bm.free(hit)
                break
            new = self.bm.allocate(need)
            # blocks [len(hit), nslots) come back from host; the tail (if any) is new
            pairs.extend(zip(seq.host_slots[len(hit):], new[:nslots - len(hit)]))
            self.host.release(seq.host_slots)
            seq.host_slots = []
            seq.block_ids = list(hit) + new
            # the restored blocks are fresh (unhashed) device blocks: let the next
            # post_step commit them to the prefix cache again
            seq.num_committed_blocks = len(hit)
            seq.status = SeqStatus.RUNNING
            self.swapped.popleft()
            self.running.append(seq)
            resumed.append(seq)
            self.num_swap_in += 1
        return resumed, pairs

    def _reset_to_waiting(self, seq: Sequence):
        """Drop a sequence's KV blocks (full blocks stay in the prefix cache, so a
        later admission re-attaches them) and restart its prefill from scratch."""
        self.release(seq)
        seq.num_computed = 0
        seq.num_committed_blocks = 0
        seq.num_cached_tokens = 0
        seq.pf_sched = 0
        seq.epoch += 1

    def _schedule_prefill(self, budget: int, n_decode: int):
        seqs, ntok, samp, rejected = [], [], [], []
        retried = None
        used = 0
        # the soft budget is for latency when the queue head is short (one turn of
        # every session: short new messages on a cached history); when the head
        # itself needs more than the soft budget (a long first prompt, or every
        # session re-rendering its history window at once) the step is filled to the
        # hard budget instead, for throughput.  (Prefilling such a head alone was
        # measured neutral in round 5 -- config 5 4,811 / 4,679 vs 4,793 / 4,799 tok/s,
        # tool-turn p99 396 / 364 vs 363 / 382 ms, profiles/ab_prefill_flood_r05.log.)
        soft = self.prefill_chunk
        if soft and self.chunk_counts_decode:
            # the soft budget bounds the step's GEMM rows (decode rows + prefill
            # tokens), so a burst step stays inside the prefill GEMMs' 256-row tiles
            soft = max(self.bs, soft - n_decode)
        while self.waiting and budget > 0 and n_decode + len(seqs) < self.max_num_seqs:
            if seqs and soft and used >= soft:
                break
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
                if self.admit_trace is not None:   # FT_STEP_TRACE: what each admission costs
                    self.admit_trace.append(("admit", time.perf_counter(), seq.request_id, seq.n_tokens,
                                             seq.num_computed, seq.grammar is not None, seq.background))
            start = seq.num_computed + seq.pf_sched   # chunks already queued come first
            remaining = seq.n_tokens - start
            if not seqs and remaining >= soft:
                soft = 0
            limit = budget if not seqs or not soft else min(budget, soft - used)
            chunk = min(remaining, limit)
            need = self._blocks_needed(seq, start + chunk)
            if need and not self.bm.can_allocate(need) and self._release_background():
                pass  # a warm-up's blocks went back to the pool first (optional work)
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
            used += chunk
            if full:
                self.waiting.popleft()
            else:
                break  # the partially prefilled prompt continues next step
        if self.background and not self.waiting and budget > 0 \
                and n_decode + len(seqs) < self.max_num_seqs:
            room = min(budget, soft - used) if soft else budget
            if room > 0:
                self._schedule_background(room, seqs, ntok, samp, rejected)
        return seqs, ntok, samp, rejected

    def _release_background(self) -> bool:
        """Background warm-ups give up the blocks of their unfinished prefill (full
        blocks stay in the prefix cache) so a real prompt can be admitted; they
        only run when nothing is waiting, so otherwise they would hold the blocks
        without progressing.  True if anything was released."""
        freed = False
        for w in self.background:
            if w.block_ids:
                self._reset_to_waiting(w)
                freed = True
        return freed

    def _schedule_background(self, room: int, seqs, ntok, samp, rejected):
        """One chunk of the oldest background prompt into ``room`` spare tokens.
        Warm-up is optional work: under KV pressure it is dropped, not waited for."""
        seq = self.background[0]
        if seq.num_computed == 0 and not seq.block_ids:
            max_blocks = (seq.n_tokens - 1) // self.bs
            hit = self.bm.match_prefix(seq.tokens, max_blocks) if max_blocks > 0 else []
            if hit:
                seq.block_ids = list(hit)
                seq.num_computed = len(hit) * self.bs
                seq.num_committed_blocks = len(hit)
                seq.num_cached_tokens = seq.num_computed
        start = seq.num_computed + seq.pf_sched
        remaining = seq.n_tokens - start
        chunk = min(remaining, room)
        need = self._blocks_needed(seq, start + chunk)
        if need and not self.bm.can_allocate(need):
            self.background.popleft()
            self.release(seq)
            seq.status = SeqStatus.FINISHED
            seq.finish_reason = "abort"
            rejected.append(seq)
            return
        if need:
            seq.block_ids.extend(self.bm.allocate(need))
        seqs.append(seq)
        ntok.append(chunk)
        samp.append(chunk == remaining)
        if chunk == remaining:
            self.background.popleft()

    def _preempt_one(self, keep: Sequence) -> bool:
        # a background warm-up gives its blocks up first (it is optional work)
        for w in self.background:
            if w.block_ids:
                self._reset_to_waiting(w)
                self.num_preemptions += 1
                return True
        # a waiting sequence in the middle of a chunked prefill gives its blocks up next
        for w in self.waiting:
            if w.block_ids:
                self._reset_to_waiting(w)
                self.num_preemptions += 1
                return True
        for victim in reversed(self.running):
            if victim is keep:
                continue
            self.running.remove(victim)
            self.num_preemptions += 1
            if self._swap_out_seq(victim):
                return True
            self._reset_to_waiting(victim)
            victim.status = SeqStatus.WAITING
            victim.preemptions += 1
            self.waiting.appendleft(victim)
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
        items = [(s, 1, False, None) for s in batch.decode_seqs] + \
            list(zip(batch.prefill_seqs, batch.prefill_tokens, batch.prefill_sample,
                     batch.prefill_epoch or [None] * len(batch.prefill_seqs)))
        for seq, n, smp, ep in items:
            if ep is not None:
                if ep != seq.epoch:   # its KV was dropped after this chunk was queued
                    self.stale_chunks += 1
                    continue
                seq.pf_sched = max(0, seq.pf_sched - n)
            if seq.status == SeqStatus.FINISHED:
                continue
            seq.num_computed += n
            if smp and seq.status != SeqStatus.RUNNING:   # (a jump-forward chunk already runs)
                seq.status = SeqStatus.RUNNING
                self._admit_counter += 1
                seq.admit_order = self._admit_counter
                self.running.append(seq)
            nfull = seq.num_computed // self.bs
            if nfull > seq.num_committed_blocks:
                self.bm.commit(seq.block_ids, seq.tokens, seq.num_computed, seq.num_committed_blocks)
                seq.num_committed_blocks = nfull
