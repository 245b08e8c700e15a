"""LLMEngine (synchronous step loop) and AsyncEngine (engine thread + asyncio
streams).  Together they replace the vLLM server the reference reaches over
HTTP/SSE (``app/core/vllm_handler.py:216-308``): ``AsyncEngine.generate`` is an
async iterator of text deltas, ``abort`` is E12 (frees KV blocks mid-stream),
``is_healthy`` / ``model_info`` are E13.
"""
from __future__ import annotations

import asyncio
import collections
import itertools
import os
import logging
import queue
import threading
import time
import uuid
from typing import Any, AsyncIterator, Callable, Dict, List, Optional, Sequence as Seq

import numpy as np

from ..models.config import resolve_model
from ..parallel.comm import SINGLE, TPComm
from ..runtime import rt
from .chat_template import ChatTemplate
from .config import EngineConfig
from .sampling_params import SamplingParams
from .scheduler import ScheduledBatch, Scheduler
from .sequence import coalesce, RequestOutput, SeqStatus, Sequence
from .tokenizer import get_tokenizer

log = logging.getLogger("fasttalk.engine")


class EngineError(RuntimeError):
    pass


class _Inflight:
    """A queued (launched, not yet collected) step: its batch, the runner's handle,
    whether it is a mixed (prefill) step, and when the host launched it."""
    __slots__ = ("batch", "handle", "mixed", "t_launch")

    def __init__(self, batch: ScheduledBatch, handle, mixed: bool):
        self.batch = batch
        self.handle = handle
        self.mixed = mixed
        self.t_launch = 0.0


class LLMEngine:
    def __init__(self, cfg: EngineConfig, comm: TPComm = SINGLE, runner=None):
        self.cfg = cfg
        self.model_cfg = resolve_model(cfg.weights if cfg.weights not in ("random", None, "")
                                       else cfg.model)
        tok_path = cfg.tokenizer
        if tok_path is None and cfg.weights not in ("random", None, ""):
            tok_path = cfg.weights
        self.tokenizer = get_tokenizer(tok_path)
        self.template = ChatTemplate(self.tokenizer)
        if runner is None:
            from .synthetic import make_synthetic_runner, synthetic_step_ms

            if synthetic_step_ms() > 0:   # service load tests (ENGINE_SYNTHETIC_STEP_MS)
                runner = make_synthetic_runner(cfg, self.model_cfg)
            else:
                from .runner import ModelRunner

                runner = ModelRunner(cfg, self.model_cfg, comm)
        self.runner = runner
        self.max_model_len = runner.max_model_len
        R = rt()
        self.bm = R.BlockManager(runner.num_blocks, cfg.block_size, cfg.enable_prefix_caching)
        self.detok = R.Detokenizer(self.tokenizer.id_to_bytes)
        self.scheduler = Scheduler(self.bm, cfg.block_size, cfg.max_num_seqs,
                                   cfg.max_num_batched_tokens, self.max_model_len,
                                   host_blocks=getattr(runner, "num_host_blocks", 0),
                                   prefill_chunk=cfg.prefill_chunk,
                                   chunk_counts_decode=cfg.prefill_chunk_rows,
                                   guided_prefill_cap=cfg.guided_prefill_cap)
        self.stop_ids = set(self.tokenizer.stop_ids) | set(self.model_cfg.eos_token_ids)
        self._trie = None
        # jump-forward over grammar-forced runs (ENGINE_JUMP_FORWARD=0 disables)
        self.jump_forward = os.environ.get("ENGINE_JUMP_FORWARD", "1") != "0"
        # a grammar that is complete ends the sequence without decoding its EOS
        self.grammar_eos_shortcut = self.jump_forward
        # token-exact assistant history (ChatTemplate.remember_assistant;
        # ENGINE_TOKEN_HISTORY=0 re-encodes every reply from its text)
        self.token_history = os.environ.get("ENGINE_TOKEN_HISTORY", "1") != "0"
        self._jf_cache: Dict[bytes, List[int]] = {}
        self._guided_lens = collections.deque(maxlen=4096)
        self.stats = collections.Counter()
        self.step_times = collections.deque(maxlen=512)
        # FT_STEP_TRACE=<path>: per-step timeline (kind, rows, tokens, start/end) and
        # request arrivals, written at shutdown -- what the GPU waits on between turns
        self._trace_path = os.environ.get("FT_STEP_TRACE") or None
        self._trace: List[tuple] = []
        if self._trace_path:
            self.scheduler.admit_trace = self._trace
        self.host_prof = collections.Counter()
        # queued decode steps, oldest first: [(batch, DecodeHandle)], at most
        # cfg.pipeline_depth + 1 of them (ENGINE_PIPELINE_DEPTH)
        self._inflight: List[_Inflight] = []
        self._executing: Optional[ScheduledBatch] = None   # drained step being executed
        self.pipeline_depth = max(1, int(getattr(cfg, "pipeline_depth", 1)))
        # ENGINE_MIXED_AHEAD (default on): waiting prompts are scheduled into a mixed
        # step queued behind the running decode step instead of draining the queue.
        # (A just-in-time queue top-up was built and measured in round 3: the host's view
        # of step ends jitters with the GIL, late top-ups cost the decode step 7.6 ->
        # 8.0 ms, p50 TTFT did not improve -- profiles/ab_mixed_ahead_r03.log; removed.)
        self.mixed_ahead = os.environ.get("ENGINE_MIXED_AHEAD", "1") != "0"
        self.poll_hook = None
        # ENGINE_PIPELINE_SHRINK=1: a stop shrinks the queued steps instead of draining
        # them.  Off by default: in the voice-agent loop the session's next prompt
        # follows its stop within a step, and a drained queue lets it start one step
        # sooner (driver config, same box: p50 TTFT 36-41 ms drained vs 50-51 ms shrunk
        # at equal tok/s, profiles/ab_pipeline_shrink_r03.log).  Workloads with think
        # time between turns keep the GPU busy with it on.
        self.pipeline_shrink = os.environ.get("ENGINE_PIPELINE_SHRINK", "0") == "1"
        # ENGINE_MIXED_CHAIN: mixed steps are queued like decode steps -- a drained
        # queue launches its mixed step without waiting for it, and the next mixed
        # step (more prompts, the next chunk of a long or background prompt) is
        # queued behind a running one -- instead of running each synchronously with
        # the GPU idle while the host collects it and builds the next
        self.mixed_chain = self.mixed_ahead and os.environ.get("ENGINE_MIXED_CHAIN", "1") != "0"
        # ENGINE_MIXED_CHAIN_GUIDED: the chain also covers guided (grammar-masked) rows
        # and prompts -- a mixed step queued behind guided decode rows defers its
        # sampler until their masks are known (runner.sample_launch), like the split
        # decode graphs do
        self.mixed_chain_guided = self.mixed_chain and \
            os.environ.get("ENGINE_MIXED_CHAIN_GUIDED", "1") != "0"
        self._last_complete = 0.0
        from .debug import FaultInjector, StepProfiler

        self._faults = FaultInjector()
        self._profiler = StepProfiler()
        self.last_step_end = time.time()

    # ------------------------------------------------------------------ requests
    def add_request(self, request_id: str, prompt_ids: Seq[int], params: SamplingParams,
                    on_output: Optional[Callable[[RequestOutput], None]] = None,
                    meta: Any = None, background: bool = False) -> Sequence:
        prompt_ids = list(prompt_ids)
        if not prompt_ids:
            prompt_ids = [self.tokenizer.bos_id]
        if len(prompt_ids) >= self.max_model_len:
            raise EngineError(f"prompt of {len(prompt_ids)} tokens exceeds max_model_len "
                              f"{self.max_model_len}")
        seq = Sequence(request_id, prompt_ids, params, on_output, meta)
        seq.background = bool(background)
        if self._trace_path:
            self._trace.append(("arrive", time.perf_counter(), len(prompt_ids)))
        seq.detok_stream = self.detok.new_stream()
        if params.guided is not None:
            seq.grammar = params.guided.grammar(self)
            seq.grammar_state = seq.grammar.initial()
            if params.guided_lazy:   # the model decides with its first token (_process_token)
                seq.lazy = True
            else:
                # the grammar's fixed head (e.g. '{"name": "' of a tool call) is output the
                # model cannot choose: appended now, prefilled with the prompt
                # bounded by max_model_len too: the head is prefilled with the prompt, and
                # positions past max_model_len have no RoPE row / KV room
                room = min(params.max_tokens - 1, self.max_model_len - 1 - len(prompt_ids))
                seq.jf_text, seq.jf_ids = self._jump_forward(seq, room=max(0, room))
        self.scheduler.add(seq)
        self.stats["requests"] += 1
        return seq

    def abort(self, request_id: str) -> bool:
        seq = self.scheduler.abort(request_id)
        if seq is None:
            return False
        self._finalize(seq, "abort", emit=True)
        return True

    def has_work(self) -> bool:
        return bool(self._inflight) or self.scheduler.has_work()

    # ------------------------------------------------------------------ helpers
    def token_trie(self):
        if self._trie is None:
            self._trie = rt().TokenTrie(self.tokenizer.id_to_bytes)
        return self._trie

    def _masks_for(self, seqs: List[Sequence]) -> Optional[np.ndarray]:
        if not any(s.grammar is not None for s in seqs):
            return None
        words = (self.runner.mcfg.vocab_size + 31) // 32
        m = np.full((len(seqs), words), -1, dtype=np.int32)
        for i, s in enumerate(seqs):
            if s.grammar is not None and s.grammar_state >= 0 and not s.lazy:
                raw = np.frombuffer(s.grammar.mask(s.grammar_state), dtype=np.int32)
                m[i, : raw.shape[0]] = raw
                m[i, raw.shape[0]:] = 0
        return m

    # ------------------------------------------------------------------ stepping
    # ------------------------------------------------------------------ pipelined decode
    def _pipeline_ok(self, batch: ScheduledBatch) -> bool:
        """Decode-only steps of graph-replayable batches run pipelined: step n+1 is
        queued on the GPU (inputs = step n's sampled ids, on the device) before the
        host processes step n, so detokenizing / streaming / scheduling overlap the
        GPU instead of idling it between graph replays."""
        return (self.cfg.async_output and not batch.has_prefill and bool(batch.decode_seqs)
                and self.runner.__class__.__name__ == "ModelRunner"
                and self.runner.can_pipeline(len(batch.decode_seqs))
                and (all(s.grammar is None for s in batch.decode_seqs) or self._guided_pipeline()))

    def _guided_pipeline(self) -> bool:
        """Guided (grammar-masked) batches pipeline too: the next step's forward pass
        is queued before this step's tokens are known, and only its sampler waits
        for the masks the tokens decide (runner.sample_launch)."""
        return getattr(self.runner, "can_defer_sample", lambda: False)()

    def _launch_decode(self, seqs, from_device: bool, rowmap=None, masks=None):
        """Queues a graph-replayed decode step.  Positions come from each sequence's
        ``inflight`` count (steps queued ahead of it); with ``from_device`` the
        input ids are the previous queued step's sampled rows (``rowmap``: the row
        of that step each sequence sat in; None = the same rows).  A guided batch
        queued ahead (``from_device``) defers its sampler until its masks are known."""
        defer = from_device and any(q.grammar is not None for q in seqs)
        h = self.runner.decode_launch(seqs, ahead=int(from_device), masks=masks,
                                      rowmap=rowmap if from_device else None,
                                      **({"defer_sample": True} if defer else {}))
        for q in seqs:
            q.inflight += 1
        return _Inflight(ScheduledBatch(list(seqs), [], [], []), h, False)

    def _speculate(self):
        """Queue the step after the queued ones, assuming none of their sequences
        stops.  Rows of sequences that do stop are discarded; their extra KV writes
        land in blocks beyond the sequence's end, which are not in the prefix cache
        (a freed block that is re-allocated meanwhile is written by its new owner
        later in stream order).

        * New prompts waiting: a MIXED step (ahead-of-time prefill injection,
          :meth:`_speculate_mixed`) is queued behind the running decode step, its
          decode rows' ids gathered on the device, instead of draining the queue
          and leaving the GPU idle while the host schedules and builds the step.
        * A sequence known to have finished: with ``pipeline_shrink`` the queued
          step drops its row and gathers the survivors' ids by row map; otherwise
          the queue drains (the session's next prompt usually follows within a
          step and then starts sooner)."""
        sched = self.scheduler
        if getattr(self._inflight[-1].handle, "pending", False):
            return None   # its sampled ids (the next step's inputs) are not queued yet
        last = self._inflight[-1].batch.sampled_seqs()
        # a background warm-up ends the pipeline unless the batch is full (it could
        # not join a step anyway)
        warm = bool(sched.background) and len(sched.running) < sched.max_num_seqs
        if sched.waiting or warm:
            return self._speculate_mixed(last) if self.mixed_ahead else None
        seqs = [q for q in last if q.status != SeqStatus.FINISHED]
        # every row ends with the queued steps' tokens (length limits): nothing to
        # speculate -- a lone request would otherwise queue a decode step whose only
        # row is discarded, and the next prompt would wait behind it
        if all(self._at_length(q) for q in seqs):
            return None
        rowmap = None
        if len(seqs) != len(last):
            if not self.pipeline_shrink or not seqs or not self.runner.can_pipeline(len(seqs)):
                return None
            rowmap = [i for i, q in enumerate(last) if q.status != SeqStatus.FINISHED]
        if self.mixed_chain:
            # running sequences that are not rows of the last queued step joined after
            # it was built (a prompt completed by an earlier, collected mixed step):
            # with nothing queued for them their ids come from the host (rowmap -1)
            rows = {id(q) for q in last}
            extra = [q for q in sched.running if id(q) not in rows]
            if extra:
                if any(q.inflight or q.grammar is not None or q.drop_next for q in extra):
                    return None
                rowmap = (rowmap if rowmap is not None else list(range(len(seqs)))) + [-1] * len(extra)
                seqs = seqs + extra
        if not self.runner.can_pipeline(len(seqs)):
            return None
        if any(q.grammar is not None for q in seqs) and not self._guided_pipeline():
            return None
        # a jump-forward appended forced tokens behind a queued step: they are
        # prefilled by the drained path (their sequence's queued sample is dropped)
        if any(q.drop_next for q in seqs):
            return None
        if not self._grow_for_next(seqs):
            return None
        if rowmap is not None and len(seqs) < len(last):
            self.stats["pipeline_shrinks"] += 1
        return self._launch_decode(seqs, True, rowmap)

    def _at_length(self, q: Sequence) -> bool:
        """The tokens of the steps queued for ``q`` reach its max_tokens / the model
        length, so it finishes when they are processed."""
        return q.num_output + q.inflight >= q.params.max_tokens or \
            q.n_tokens + q.inflight >= self.max_model_len

    def _grow_for_next(self, seqs) -> bool:
        """KV blocks for one more token past everything queued (no preemption: a
        sequence that cannot grow ends the pipeline and the scheduler decides)."""
        sched = self.scheduler
        need = 0
        for q in seqs:
            if q.n_tokens + q.inflight >= self.max_model_len:
                return False
            need += sched._blocks_needed(q, q.n_tokens + q.inflight)
        if need and not self.bm.can_allocate(need):
            return False
        for q in seqs:
            k = sched._blocks_needed(q, q.n_tokens + q.inflight)
            if k:
                q.block_ids.extend(self.bm.allocate(k))
        return True

    def _speculate_mixed(self, last):
        """Schedules the waiting prompts into a mixed step queued behind the running
        decode step: decode rows = the running sequences (each a row of the last
        queued step, ids gathered from its sampled rows on the device), prefill
        rows as the scheduler picks them.  At most one mixed step is in flight
        (a prompt's next chunk needs the previous chunk's post-step state), and
        only for grammar-free, single-process (no TP broadcast) engines."""
        sched = self.scheduler

        def skip(why: str):
            self.stats["mixed_ahead_skip_" + why] += 1
            return None

        if sched.swapped:
            return skip("swapped")
        if not self.mixed_chain and any(e.mixed for e in self._inflight):
            return skip("queued_mixed")
        if not hasattr(self.runner, "mixed_launch") or getattr(self.runner, "bcast", None) is not None:
            return None
        guided = self.mixed_chain_guided and self.pipeline_depth == 1 and self._guided_pipeline()
        # (a guided prompt's jump-forward head, jf_ids, is part of its prompt: prefilled
        # like the rest, reported with its first sampled token)
        if any(not guided and (q.grammar is not None or q.lazy or q.jf_ids) for q in sched.waiting) \
                or any(q.grammar is not None for q in sched.background):
            return skip("grammar")
        running = list(sched.running)
        if not running:   # nothing to overlap: the drained path schedules it
            return skip("no_running")
        pos = {id(q): i for i, q in enumerate(last)}
        # (guided decode rows: round 4 queued a mixed step behind them, sampler deferred
        # until their masks were known, without the chain -- more, smaller mixed steps
        # and a worse tool-turn tail, profiles/ab_guided_mixed_ahead_r04.log.  With the
        # round-5 chain the same deferral measured +5.2% tok/s at config 5 and a lower
        # p99 TTFT, profiles/ab_mixed_chain_guided_r05.log: ENGINE_MIXED_CHAIN_GUIDED)
        # a running sequence that is not a row of the last queued step joined after it
        # was built (its prompt completed in an earlier, collected step): with nothing
        # queued for it, its id is its last token (rowmap -1)
        if any((id(q) not in pos and q.inflight) or (q.grammar is not None and not guided)
               or q.drop_next for q in running):
            return skip("rows")
        if not self._grow_for_next(running):
            return skip("blocks")
        pseqs, ptok, psamp, rejected = sched._schedule_prefill(sched.max_tokens - len(running),
                                                               len(running))
        for q in rejected:   # only background warm-ups are dropped while sequences run
            sched.by_id.pop(q.request_id, None)
            self._finalize(q, "abort", emit=False)
        if not pseqs:
            return skip("no_prefill")
        mb = sched.stamp(ScheduledBatch(running, pseqs, ptok, psamp))
        rowmap = [pos.get(id(q), -1) for q in running]
        # guided decode rows: their masks wait for the tokens of the step queued ahead,
        # so the sampler is queued once those are processed (_step_pipelined); guided
        # prompts alone (initial grammar states) have their masks now
        defer = any(q.grammar is not None for q in running)
        masks = None if defer else self._masks_for(mb.sampled_seqs())
        h = self.runner.mixed_launch(mb, rowmap, masks=masks, defer_sample=defer) \
            if (defer or masks is not None) else self.runner.mixed_launch(mb, rowmap)
        for q in mb.sampled_seqs():
            q.inflight += 1
        self.stats["mixed_ahead"] += 1
        if defer:
            self.stats["mixed_deferred_sample"] += 1
        if self._inflight[-1].mixed:
            self.stats["mixed_chain"] += 1
        return _Inflight(mb, h, True)

    def _launch_mixed_drained(self, batch: ScheduledBatch, masks) -> bool:
        """Mixed chain: the drained path's mixed step is launched and queued (ids
        from the host) instead of run synchronously, so the steps behind it can be
        queued while it runs.  False where only the synchronous path applies: TP
        broadcast, allow-masks, jump-forward chunks, swaps."""
        if not self.mixed_chain or (masks is not None and not self.mixed_chain_guided) \
                or batch.swap_out or batch.swap_in \
                or not hasattr(self.runner, "mixed_launch") \
                or getattr(self.runner, "bcast", None) is not None \
                or self.runner.__class__.__name__ != "ModelRunner" or not self.cfg.async_output:
            return False
        guided = self.mixed_chain_guided
        if any(q.status == SeqStatus.RUNNING or (not guided and (q.grammar is not None or q.lazy or q.jf_ids))
               for q in batch.prefill_seqs) or \
                (not guided and any(q.grammar is not None for q in batch.decode_seqs)):
            return False
        h = self.runner.mixed_launch(batch, None, masks=masks) if masks is not None \
            else self.runner.mixed_launch(batch, None)
        for q in batch.sampled_seqs():
            q.inflight += 1
        e = _Inflight(batch, h, True)
        e.t_launch = time.perf_counter()
        self._inflight = [e]
        self.stats["mixed_drained_launch"] += 1
        return True

    def _wait_mark(self, e: "_Inflight"):
        """A step is about to be queued behind the mixed step ``e``: wait (admitting
        new requests) until the GPU has passed ``e``'s mark, 60% into its layers by
        default (runner ENGINE_MIXED_CHAIN_AT), so prompts that arrive
        meanwhile still make the next step -- built at once, the next step would
        leave them a step behind (+9 ms p50 engine TTFT at the driver config) --
        while the host has the rest of ``e`` to build and queue it."""
        mark = getattr(e.handle, "mark", None)
        poll = self.poll_hook
        if mark is None or poll is None or not self.mixed_chain:
            return
        while not mark.query() and not self.runner.step_done(e.handle):
            poll()
            time.sleep(0.0002)

    def _drain_wait(self, e: "_Inflight"):
        """The queue is draining (nothing could be queued behind ``e``: a stop, or no
        room).  While ``e`` runs, new requests are admitted (``poll_hook``), and the
        first prompt that arrives is scheduled into a mixed step queued behind ``e``
        (:meth:`_speculate_mixed`), so the prefill starts the moment ``e`` ends
        instead of after the host has collected it and built the step."""
        poll = self.poll_hook
        while not self.runner.step_done(e.handle):
            poll()
            if self.scheduler.waiting:
                nxt = self._speculate_mixed(e.batch.sampled_seqs())
                if nxt is not None:
                    nxt.t_launch = time.perf_counter()
                    self._inflight.append(nxt)
                    self.stats["mixed_ahead_drain"] += 1
                return
            time.sleep(0.0002)

    def _step_pipelined(self) -> List[RequestOutput]:
        e = self._inflight[0]
        batch, handle = e.batch, e.handle
        t0 = time.perf_counter()
        # top the queue up to depth + 1 steps before waiting on the oldest
        while len(self._inflight) <= self.pipeline_depth:
            if self._inflight[-1].mixed:
                self._wait_mark(self._inflight[-1])
            nxt = self._speculate()
            if nxt is None:
                break
            nxt.t_launch = time.perf_counter()
            self._inflight.append(nxt)
        if len(self._inflight) == 1 and not e.mixed and self.mixed_ahead and self.poll_hook is not None:
            self._drain_wait(e)
        tl = time.perf_counter()
        toks = self.runner.mixed_collect(handle) if e.mixed else self.runner.decode_collect(handle)
        t1 = time.perf_counter()
        self._inflight.pop(0)
        sampled = batch.sampled_seqs()
        for q in sampled:
            q.inflight -= 1
        outs = self._complete(batch, sampled, toks)
        # the guided step queued behind this one: its forward pass is running; its
        # sampler goes in now that this step's tokens have moved the grammars
        if self._inflight and getattr(self._inflight[0].handle, "pending", False):
            nxt = self._inflight[0]
            self.runner.sample_launch(nxt.handle, self._masks_for(nxt.batch.sampled_seqs()))
            self.stats["guided_pipelined_mixed" if nxt.mixed else "guided_pipelined_steps"] += 1
        t2 = time.perf_counter()
        dt = t2 - self._last_complete if self._last_complete else t2 - t0
        self._last_complete = t2
        self.step_times.append((batch.has_prefill, len(batch.decode_seqs), batch.total_tokens, dt))
        if self._trace_path:
            self._trace.append(("mixed_p" if e.mixed else "decode_p", t0, t2, len(batch.decode_seqs),
                                sum(batch.prefill_tokens), len(batch.prefill_seqs)))
        if e.mixed:
            self.stats["mixed_steps"] += 1
            self.stats["prefill_tokens"] += sum(batch.prefill_tokens)
            return outs
        self.stats["decode_ms_sum"] += 1e3 * dt
        self.stats["decode_steps"] += 1
        self.stats["pipelined_steps"] += 1
        self._count_ctx(batch.decode_seqs)
        hp = self.host_prof
        hp["launch_next"] += tl - t0
        hp["collect"] += t1 - tl
        hp["process"] += t2 - t1
        hp["steps"] += 1
        return outs

    def _complete(self, batch: ScheduledBatch, sampled_seqs, toks) -> List[RequestOutput]:
        outs: List[RequestOutput] = []
        self.scheduler.post_step(batch)
        for seq, tok in zip(sampled_seqs, toks):
            if seq.drop_next:   # its forced tokens replaced this sample (jump-forward)
                seq.drop_next -= 1
                self.stats["pipelined_jump_drops"] += 1
                continue
            o = self._process_token(seq, int(tok))
            if o is not None:
                outs.append(o)
        self.stats["generated_tokens"] += len(sampled_seqs)
        self.last_step_end = time.time()
        return outs

    def step(self) -> List[RequestOutput]:
        self._faults.check()
        self._profiler.before_step()
        try:
            return self._step()
        finally:
            self._profiler.after_step()

    def _count_ctx(self, seqs):
        """Decode-step context counters: rows, tokens attended over, longest context
        (bench.py reports the measured mean / max context of the timed turns)."""
        st = self.stats
        m = 0
        tot = 0
        for q in seqs:
            c = q.n_tokens
            tot += c
            if c > m:
                m = c
        st["ctx_rows"] += len(seqs)
        st["ctx_tokens"] += tot
        if m > st["ctx_max"]:
            st["ctx_max"] = m

    def reset_inflight(self):
        """Forget the queued steps (after a failed step)."""
        for e in self._inflight:
            for q in e.batch.sampled_seqs():
                q.inflight = 0
                q.drop_next = 0
            for q in e.batch.prefill_seqs:
                q.pf_sched = 0
        self._inflight = []
        discard = getattr(self.runner, "discard_pending", None)
        if discard is not None:
            discard()

    def fail_unfinished(self, error: str, reset_cache: bool = False):
        """After a failed step: every unfinished sequence ends with an error and
        gives back its KV blocks and host swap slots -- swapped-out ones too (if
        the failing step was the swap itself their host copies may be garbage).
        ``reset_cache`` (a collective fault: KV written from un-reduced partial sums
        may sit in committed blocks) also empties the prefix cache."""
        # sequences of queued / executing steps first: a mixed-ahead step's prompts left
        # `waiting` when it was scheduled and join `running` only in post_step, so
        # without this they would never finish and their KV blocks would leak
        limbo = []
        for e in self._inflight:
            limbo += list(e.batch.prefill_seqs) + list(e.batch.sampled_seqs())
        if self._executing is not None:
            limbo += list(self._executing.prefill_seqs) + list(self._executing.decode_seqs)
            self._executing = None
        self.reset_inflight()
        sched = self.scheduler
        seen = set()
        for seq in limbo + list(sched.running) + list(sched.waiting) + list(sched.swapped) + \
                list(sched.background):
            if id(seq) in seen or seq.status == SeqStatus.FINISHED:
                continue
            seen.add(id(seq))
            self._finalize(seq, "error", emit=True, error=error)
        if reset_cache and hasattr(self.bm, "reset_prefix_cache"):
            self.bm.reset_prefix_cache()

    def _step(self) -> List[RequestOutput]:
        if self._inflight:
            return self._step_pipelined()
        self._last_complete = 0.0
        ts = time.perf_counter()
        batch = self.scheduler.schedule()
        if batch is None:
            return []
        t0 = time.perf_counter()
        outs: List[RequestOutput] = []
        if batch.swap_out or batch.swap_in:  # E6: host swap copies precede the forward
            self.runner.swap(batch.swap_out, batch.swap_in)
            self.stats["swapped_out_blocks"] += len(batch.swap_out)
            self.stats["swapped_in_blocks"] += len(batch.swap_in)
        # sequences the scheduler had to reject (cannot fit in the KV pool)
        for s in batch.rejected:
            self.scheduler.by_id.pop(s.request_id, None)
            if s.background:  # a dropped warm-up is not a failed request
                self._finalize(s, "abort", emit=False)
                continue
            outs.append(self._finalize(s, "error", emit=True,
                                       error="prompt does not fit in the KV cache"))
        if not batch.decode_seqs and not batch.prefill_seqs:
            return outs
        if not outs and self._pipeline_ok(batch):
            e = self._launch_decode(batch.decode_seqs, False,
                                    masks=self._masks_for(batch.decode_seqs))
            e.t_launch = time.perf_counter()
            self._inflight = [e]
            return self._step_pipelined()
        sampled_seqs = batch.sampled_seqs()
        masks = self._masks_for(sampled_seqs)
        if not outs and batch.has_prefill and self._launch_mixed_drained(batch, masks):
            return self._step_pipelined()
        self._executing = batch
        toks = self.runner.execute(batch, masks)
        self._executing = None
        t1 = time.perf_counter()
        self.scheduler.post_step(batch)
        for seq, tok in zip(sampled_seqs, toks):
            o = self._process_token(seq, int(tok))
            if o is not None:
                outs.append(o)
        t2 = time.perf_counter()
        dt = t2 - t0
        if not batch.has_prefill:  # host-side anatomy of decode steps (ms sums)
            hp = self.host_prof
            hp["schedule"] += t0 - ts
            hp["execute"] += t1 - t0
            hp["process"] += t2 - t1
            hp["steps"] += 1
        self.step_times.append((batch.has_prefill, len(batch.decode_seqs), batch.total_tokens, dt))
        if not batch.has_prefill:
            self.stats["decode_ms_sum"] += 1e3 * dt
            self._count_ctx(batch.decode_seqs)
        if self._trace_path:
            self._trace.append(("mixed" if batch.has_prefill else "decode", ts, t2,
                                len(batch.decode_seqs), sum(batch.prefill_tokens),
                                len(batch.prefill_seqs)))
        self.stats["mixed_steps" if batch.has_prefill else "decode_steps"] += 1
        self.stats["generated_tokens"] += len(sampled_seqs)
        self.stats["prefill_tokens"] += sum(batch.prefill_tokens)
        self.last_step_end = time.time()
        return outs

    def _forced_ids(self, fb: bytes) -> List[int]:
        """Token ids whose bytes are exactly ``fb`` (cut at the last complete UTF-8
        character), or [] when the tokenizer does not round-trip them."""
        cache = self._jf_cache
        ids = cache.get(fb)
        if ids is None:
            text = fb.decode("utf-8", errors="ignore")
            while text and text.encode("utf-8") != fb[:len(text.encode("utf-8"))]:
                text = text[:-1]
            ids = self.tokenizer.encode(text) if text else []
            tb = self.tokenizer.id_to_bytes
            if b"".join(tb[i] for i in ids) != text.encode("utf-8"):
                ids = []
            if len(cache) < 4096:
                cache[fb] = ids
        return ids

    def _jump_forward(self, seq: Sequence, room: int):
        """Appends the bytes the grammar forces from the sequence's current state (the
        rest of a key, '": "', closing braces, a tool name once its prefix is unique)
        as tokens, advancing the grammar and the detokenizer; returns (text, ids).
        They are prefilled in the next step instead of decoded one step each."""
        if not self.jump_forward or room <= 0 or seq.grammar_state < 0:
            return "", []
        fb = seq.grammar.forced(seq.grammar_state)
        if not fb:
            return "", []
        text, used = "", []
        for t in self._forced_ids(fb)[:room]:
            st = seq.grammar.advance_token(seq.grammar_state, t)
            if st < 0:
                break
            seq.grammar_state = st
            seq.append(t)
            text += self.detok.push(seq.detok_stream, t)
            used.append(t)
        if used:
            self.stats["jump_forward_tokens"] += len(used)
        return text, used

    def _process_token(self, seq: Sequence, tok: int) -> Optional[RequestOutput]:
        if seq.status == SeqStatus.FINISHED:
            return None
        p = seq.params
        now = time.perf_counter()
        first = seq.first_token_time is None
        if first:
            seq.first_token_time = now
        seq.append(tok)
        n_out = seq.num_output
        reason = None
        is_stop_tok = (tok in self.stop_ids and not p.ignore_eos) or \
            (p.stop_token_ids is not None and tok in p.stop_token_ids)
        if seq.grammar is not None and seq.lazy:
            # lazy grammar: bound iff the model's first token starts a valid string of it
            seq.lazy = False
            st = seq.grammar.advance_token(seq.grammar_state, tok)
            if st >= 0:
                seq.grammar_state = st
                self.stats["lazy_grammar_bound"] += 1
            else:
                seq.grammar = None
        elif seq.grammar is not None:
            if seq.grammar.is_eos(tok) and seq.grammar.accepting(seq.grammar_state):
                is_stop_tok = True
            else:
                seq.grammar_state = seq.grammar.advance_token(seq.grammar_state, tok)
                if seq.grammar_state < 0:
                    reason = "stop"
        pre_text, pre_ids, post_ids = "", [], []
        if first and seq.jf_ids:   # the head forced at admission goes out with the first token
            pre_text, pre_ids = seq.jf_text, seq.jf_ids
            seq.jf_text, seq.jf_ids = "", []
        if is_stop_tok and n_out > p.min_tokens:
            reason = "stop"
            delta = pre_text
        else:
            delta = pre_text + self.detok.push(seq.detok_stream, tok)
            if seq.grammar is not None and reason is None:
                room = min(p.max_tokens - n_out, self.max_model_len - 1 - seq.n_tokens)
                jtext, post_ids = self._jump_forward(seq, room)
                delta += jtext
                n_out = seq.num_output
                if post_ids and seq.inflight:
                    # steps already queued behind this one sampled past a position the
                    # grammar has now filled with forced tokens: drop their samples
                    seq.drop_next = seq.inflight
                # the grammar is complete (accepting, no byte can follow: the mask would
                # allow EOS alone): end here instead of decoding that EOS -- for a tool
                # call the step that prefills its forced closing and samples the EOS is
                # skipped (the uncomputed tail is never committed to the prefix cache)
                if self.grammar_eos_shortcut and n_out >= p.min_tokens and \
                        seq.grammar.complete(seq.grammar_state):
                    reason = "stop"
                    self.stats["grammar_complete_stops"] += 1
        if reason is None:
            if n_out >= p.max_tokens or seq.n_tokens >= self.max_model_len:
                reason = "length"
        if p.stop and delta:
            delta, hit = self._apply_stop(seq, delta)
            if hit:
                reason = "stop"
        elif p.stop and reason is not None:
            pass
        ids = pre_ids + ([] if (is_stop_tok and reason == "stop") else [tok]) + post_ids
        if reason is not None:
            return self._finalize(seq, reason, emit=True, delta=delta, ids=ids)
        if not delta and not first:
            # nothing printable yet (partial UTF-8): still report progress
            out = RequestOutput(seq.request_id, "", ids, num_output_tokens=n_out)
        else:
            out = RequestOutput(seq.request_id, delta, ids, num_output_tokens=n_out,
                                num_prompt_tokens=seq.prompt_len,
                                num_cached_tokens=seq.num_cached_tokens,
                                ttft_s=(seq.first_token_time - seq.arrival) if first else None)
        if seq.on_output is not None:
            seq.on_output(out)
        return out

    def _apply_stop(self, seq: Sequence, delta: str):
        """Hold back text that could be the start of a stop string."""
        stops = seq.params.stop
        buf = seq.stop_buf + delta
        for s in stops:
            i = buf.find(s)
            if i >= 0:
                seq.stop_buf = ""
                return buf[:i], True
        keep = max(len(s) for s in stops) - 1
        if keep <= 0:
            seq.stop_buf = ""
            return buf, False
        # emit all but the longest suffix that is a prefix of some stop string
        hold = 0
        for k in range(min(keep, len(buf)), 0, -1):
            tail = buf[-k:]
            if any(s.startswith(tail) for s in stops):
                hold = k
                break
        seq.stop_buf = buf[len(buf) - hold:] if hold else ""
        return buf[: len(buf) - hold], False

    def _finalize(self, seq: Sequence, reason: str, emit: bool, delta: str = "",
                  ids: Optional[List[int]] = None, error: Optional[str] = None) -> RequestOutput:
        if seq.status != SeqStatus.FINISHED or seq.block_ids:
            self.scheduler.finish(seq, reason)
        seq.finish_reason = reason
        if seq.grammar is not None:   # output lengths of guided sequences (tool calls, JSON)
            self._guided_lens.append(seq.num_output)
        tail = ""
        if seq.detok_stream >= 0:
            if reason != "abort":
                tail = self.detok.flush(seq.detok_stream)
            self.detok.release(seq.detok_stream)
            seq.detok_stream = -1
        text = delta + (seq.stop_buf if reason != "stop" else "") + tail
        seq.stop_buf = ""
        if self.token_history and reason in ("length", "stop") and seq.grammar is None \
                and not seq.params.stop:
            out_ids = seq.output_ids
            while out_ids and self.tokenizer.is_special(out_ids[-1]):   # the EOS that ended it
                out_ids.pop()
            self.template.remember_assistant(out_ids)
        out = RequestOutput(seq.request_id, text, ids or [], finished=True, finish_reason=reason,
                            num_prompt_tokens=seq.prompt_len,
                            num_cached_tokens=seq.num_cached_tokens,
                            num_output_tokens=seq.num_output, error=error)
        self.stats["finished_" + reason] += 1
        if emit and seq.on_output is not None:
            seq.on_output(out)
        return out

    # ------------------------------------------------------------------ convenience
    def generate(self, prompts: List[List[int]], params: SamplingParams) -> List[List[int]]:
        """Blocking batch generation (tests / offline use)."""
        ids = []
        for i, p in enumerate(prompts):
            rid = f"gen-{uuid.uuid4().hex[:8]}-{i}"
            self.add_request(rid, p, SamplingParams(**{**params.__dict__}))
            ids.append(rid)
        results: Dict[str, List[int]] = {r: [] for r in ids}
        done = set()
        while len(done) < len(ids):
            if not self.has_work():
                break
            for o in self.step():
                if o.request_id in results:
                    results[o.request_id].extend(o.token_ids)
                    if o.finished:
                        done.add(o.request_id)
        return [results[r] for r in ids]

    def write_trace(self):
        if self._trace_path and self._trace:
            import json

            with open(self._trace_path, "w") as f:
                json.dump(self._trace, f)

    def shutdown(self):
        """Stops tensor-parallel workers (if any)."""
        self.write_trace()
        g = getattr(self, "tp_group", None)
        if g is not None:
            g.shutdown()
            self.tp_group = None

    def kv_usage(self) -> float:
        n = self.bm.num_blocks
        return 1.0 - self.bm.num_free() / n if n else 0.0

    def metrics(self) -> Dict[str, Any]:
        st = list(self.step_times)
        dec = [x for x in st if not x[0]]
        pre = [x for x in st if x[0]]
        return {
            "running": len(self.scheduler.running),
            "waiting": len(self.scheduler.waiting),
            "kv_blocks_total": self.bm.num_blocks,
            "kv_blocks_free": self.bm.num_free(),
            "kv_blocks_cached": self.bm.num_cached(),
            "kv_usage": self.kv_usage(),
            "prefix_cache_hit_rate": (self.bm.hits / self.bm.queries) if self.bm.queries else 0.0,
            "preemptions": self.scheduler.num_preemptions,
            "guided_capped_steps": self.scheduler.guided_capped,
            "swapped": len(self.scheduler.swapped),
            "swap_outs": self.scheduler.num_swap_out,
            "swap_ins": self.scheduler.num_swap_in,
            "decode_step_ms_avg": 1e3 * sum(x[3] for x in dec) / len(dec) if dec else 0.0,
            "decode_batch_avg": sum(x[1] for x in dec) / len(dec) if dec else 0.0,
            "prefill_step_ms_avg": 1e3 * sum(x[3] for x in pre) / len(pre) if pre else 0.0,
            **{k: v for k, v in self.stats.items()},
            "runner": {**getattr(self.runner, "stats", {}),
                       **({"gpu_gaps": self.runner.gap_summary()}
                          if getattr(self.runner, "_gaps", None) else {})},
            "decode_host_ms": {k: round(1e3 * v / max(1, self.host_prof["steps"]), 3)
                               for k, v in self.host_prof.items() if k != "steps"},
            "guided_output_tokens": self._len_summary(self._guided_lens),
        }

    @staticmethod
    def _len_summary(lens) -> Dict[str, Any]:
        if not lens:
            return {}
        v = sorted(lens)
        q = lambda f: v[min(len(v) - 1, int(round(f * (len(v) - 1))))]  # noqa: E731
        hist = collections.Counter(min(64, (x + 7) // 8 * 8) for x in v)
        return {"n": len(v), "p50": q(0.5), "p90": q(0.9), "max": v[-1],
                "hist_le": {str(k): hist[k] for k in sorted(hist)}}


class AsyncEngine:
    """Runs an :class:`LLMEngine` on a dedicated thread and multiplexes every
    WebSocket session into its batched step loop (E16).  Outputs are handed to
    the asyncio loop once per engine step (one ``call_soon_threadsafe`` per step,
    not per token)."""

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._cmds: "queue.SimpleQueue" = queue.SimpleQueue()
        self._wake = threading.Event()
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self._streams: Dict[str, "asyncio.Queue"] = {}
        self._loops: Dict[str, asyncio.AbstractEventLoop] = {}
        self._pending: Dict[asyncio.AbstractEventLoop, list] = {}
        self._ids = itertools.count()
        self.error: Optional[BaseException] = None
        self.heartbeat = time.time()
        self._fail_streak = 0
        # consecutive failed steps after which the engine is declared broken even
        # when each failure looked recoverable (ENGINE_MAX_FAIL_STREAK)
        import os as _os

        self.max_fail_streak = int(_os.environ.get("ENGINE_MAX_FAIL_STREAK", "3"))

    @classmethod
    def from_config(cls, cfg: EngineConfig) -> "AsyncEngine":
        if cfg.tp_size > 1:
            import os as _os

            from ..parallel.tp import spawn_tp_engine

            # a DP service worker owns GPUs [ENGINE_DEVICE_BASE, +tp) (app/server/workers.py)
            base = int(_os.environ.get("ENGINE_DEVICE_BASE", "0") or 0)
            return cls(spawn_tp_engine(cfg, device_base=base))
        return cls(LLMEngine(cfg))

    # ------------------------------------------------------------------ lifecycle
    def start(self):
        # the engine thread and the asyncio (WebSocket) thread share the GIL: a short
        # switch interval keeps token frames flowing while the engine runs Python
        import sys

        if sys.getswitchinterval() > 0.001:
            sys.setswitchinterval(0.001)
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="fasttalk-engine", daemon=True)
            self._thread.start()
        return self

    def shutdown(self):
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None
        self.engine.shutdown()

    def is_healthy(self, stall_s: float = 120.0) -> bool:
        """Watchdog: the step loop must be alive and, when busy, making progress;
        every tensor-parallel worker process must be running (a dead worker leaves
        rank 0 blocked in a collective: /health turns 503 at once, not after the
        stall timeout)."""
        if self.error is not None or self._thread is None or not self._thread.is_alive():
            return False
        group = getattr(self.engine, "tp_group", None)
        if group is not None and hasattr(group, "alive") and not group.alive():
            return False
        if self.engine.has_work() and time.time() - self.heartbeat > stall_s:
            return False
        return True

    # ------------------------------------------------------------------ engine thread
    def _deliver(self, out: RequestOutput):
        loop = self._loops.get(out.request_id)
        if loop is None:
            return
        self._pending.setdefault(loop, []).append(out)

    def _flush(self):
        for loop, items in self._pending.items():
            if items:
                try:
                    loop.call_soon_threadsafe(self._dispatch, items)
                except RuntimeError:
                    pass
        self._pending = {}

    def _dispatch(self, items: List[RequestOutput]):
        # a request's first output (a new turn's first token) wakes its consumer
        # ahead of the step's streaming deltas: the loop runs woken consumers in
        # put order, and ~50 deltas of the other sessions share each step
        for first in (True, False):
            for o in items:
                if (o.ttft_s is not None) == first:
                    q = self._streams.get(o.request_id)
                    if q is not None:
                        q.put_nowait(o)

    def _poll_cmds(self):
        while True:
            try:
                cmd = self._cmds.get_nowait()
            except queue.Empty:
                return
            self._handle(cmd)

    def _run(self):
        eng = self.engine
        if hasattr(eng, "poll_hook"):
            # requests that arrive while the last queued step runs are admitted and
            # scheduled into a mixed step behind it (LLMEngine._drain_wait)
            eng.poll_hook = self._poll_cmds
        while not self._stop:
            self.heartbeat = time.time()
            self._poll_cmds()
            if not eng.has_work():
                self._flush()
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                eng.step()
            except Exception as e:  # surfaced through health / streams (FT_FAULT_* tests)
                log.exception("engine step failed")
                self._fail_streak += 1
                fatal = not self._recoverable(e) or self._fail_streak >= self.max_fail_streak
                if fatal:  # set before the error outputs go out: no new request slips in
                    self.error = e
                from .runner import CommFault, DecodeBlockFault, KernelCheckError

                # KV written from un-reduced partials, clamped indices or a timed-out
                # decode block must not be re-attached from the prefix cache
                eng.fail_unfinished(str(e), reset_cache=isinstance(
                    e, (CommFault, DecodeBlockFault, KernelCheckError)))
                self._flush()
                continue
            self._fail_streak = 0
            self._flush()

    # RuntimeError texts of device faults that leave the HIP context unusable
    _FATAL_DEVICE_ERRORS = ("illegal memory access", "illegal instruction", "hipErrorLaunchFailure",
                            "unspecified launch failure", "device-side assert", "HIP error: an illegal",
                            "hipErrorIllegalAddress", "memory access fault", "out of memory",
                            "hipErrorOutOfMemory", "GPU hang", "hipErrorECCNotCorrectable")

    @classmethod
    def _recoverable(cls, e: BaseException) -> bool:
        """A step failure that only failed its own requests (bad input, a transient
        host error) vs one after which the device cannot be trusted: host OOM,
        device OOM (torch.cuda.OutOfMemoryError) and sticky HIP faults are fatal,
        so /health turns unhealthy instead of every later step failing silently."""
        if isinstance(e, MemoryError):
            return False
        from ..parallel.shm_broadcast import PeerDied

        if isinstance(e, PeerDied):  # a TP worker is gone: the group cannot step again
            return False
        try:
            import torch

            if isinstance(e, torch.cuda.OutOfMemoryError):
                return False
        except Exception:  # pragma: no cover
            pass
        msg = str(e)
        return not any(pat in msg for pat in cls._FATAL_DEVICE_ERRORS)

    def _handle(self, cmd):
        kind = cmd[0]
        if kind == "add":
            _, rid, prompt, params = cmd
            try:
                self.engine.add_request(rid, prompt, params, on_output=self._deliver)
            except Exception as e:
                self._deliver(RequestOutput(rid, "", [], finished=True, finish_reason="error",
                                            error=str(e)))
        elif kind == "warm":
            _, rid, prompt = cmd
            try:
                self.engine.add_request(rid, prompt, SamplingParams(temperature=0.0, max_tokens=1),
                                        background=True)
            except Exception as e:  # optional work: never fails a session
                log.warning("prefix warm-up %s not queued: %s", rid, e)
        elif kind == "abort":
            self.engine.abort(cmd[1])

    # ------------------------------------------------------------------ public API
    def new_request_id(self) -> str:
        return f"req-{next(self._ids)}-{uuid.uuid4().hex[:6]}"

    async def generate(self, prompt_ids: Seq[int], params: SamplingParams,
                       request_id: Optional[str] = None) -> AsyncIterator[RequestOutput]:
        if self.error is not None:
            raise EngineError(f"engine failed: {self.error}")
        rid = request_id or self.new_request_id()
        if rid in self._streams:
            raise EngineError(f"duplicate request id {rid}")
        q: asyncio.Queue = asyncio.Queue()
        self._streams[rid] = q
        self._loops[rid] = asyncio.get_running_loop()
        self._cmds.put(("add", rid, list(prompt_ids), params))
        self._wake.set()
        finished = False
        try:
            while True:
                o = coalesce(await q.get(), q)
                if o.finished:
                    finished = True
                yield o
                if finished:
                    break
        finally:
            self._streams.pop(rid, None)
            if not finished:
                # consumer went away before the end: free the KV blocks
                self._cmds.put(("abort", rid))
                self._wake.set()
            self._loops.pop(rid, None)

    def prefill_background(self, prompt_ids: Seq[int], session_id: Optional[str] = None) -> str:
        """Queue a prompt whose only purpose is to leave its KV blocks in the
        prefix cache (e.g. the window a conversation will be cut back to on its
        next turn).  It is prefilled in the room steps leave after every waiting
        prompt and produces no output.  ``session_id`` keys the request id like the
        session's turns (``<session>#...``), which is what DP routing is affine to."""
        rid = f"{session_id}#warm-{next(self._ids)}" if session_id else f"warm-{next(self._ids)}"
        self._cmds.put(("warm", rid, list(prompt_ids)))
        self._wake.set()
        return rid

    def abort(self, request_id: str) -> bool:
        if request_id not in self._loops:
            return False
        self._cmds.put(("abort", request_id))
        self._wake.set()
        return True

    def active_requests(self) -> List[str]:
        return list(self._loops.keys())

    def model_info(self) -> Dict[str, Any]:
        e = self.engine
        m = e.model_cfg
        return {
            "model": m.name, "num_layers": m.num_layers, "hidden_size": m.hidden_size,
            "num_heads": m.num_heads, "num_kv_heads": m.num_kv_heads, "vocab_size": m.vocab_size,
            "max_model_len": e.max_model_len, "dtype": str(e.runner.dtype).replace("torch.", ""),
            "device": str(e.runner.device), "weights": e.cfg.weights,
            "tensor_parallel_size": e.cfg.tp_size, "kv_cache_tokens": e.bm.num_blocks * e.cfg.block_size,
        }
