"""Model runner: turns a :class:`ScheduledBatch` into device metadata, runs the
forward pass + sampler, returns sampled token ids.

Decode steps replay hipGraphs (``torch.cuda.CUDAGraph`` is hipGraph on ROCm),
one per (batch bucket, split bucket): the graph covers embedding -> 32 layers ->
final norm -> LM head -> sampler, with every input in static device buffers
that are refreshed by one pinned-host -> device copy per step.  Prefill steps
run eagerly (variable token counts) through the same HIP kernels.
"""
from __future__ import annotations

import logging
import math
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..models.config import ModelConfig
from ..models.llama import AttnMeta, LlamaModel
from ..parallel.comm import SINGLE, TPComm
from .config import EngineConfig
from .scheduler import ScheduledBatch

log = logging.getLogger("fasttalk.engine.runner")


def _pow2_ceil(x: int) -> int:
    return 1 << max(0, (x - 1).bit_length())


class ModelRunner:
    def __init__(self, cfg: EngineConfig, model_cfg: ModelConfig, comm: TPComm = SINGLE,
                 device: Optional[str] = None):
        self.cfg = cfg
        self.mcfg = model_cfg
        self.comm = comm
        dev = device or cfg.resolved_device()
        if dev == "cuda":
            dev = f"cuda:{torch.cuda.current_device()}"
        self.device = torch.device(dev)
        self.is_gpu = self.device.type == "cuda"
        self.dtype = cfg.torch_dtype()
        self.bs = cfg.block_size
        self.max_model_len = min(cfg.max_model_len, model_cfg.max_position_embeddings)
        self.max_blocks_per_seq = (self.max_model_len + self.bs - 1) // self.bs

        t0 = time.time()
        self.model = LlamaModel(model_cfg, self.device, self.dtype, comm, self.max_model_len)
        if cfg.weights and cfg.weights != "random":
            self.model.load_checkpoint(cfg.weights)
        else:
            self.model.init_random(seed=cfg.seed)
        if self.is_gpu:
            torch.cuda.synchronize(self.device)
        log.info("weights ready in %.1fs", time.time() - t0)

        self.num_blocks = self._decide_num_blocks()
        self.kv = self.model.allocate_kv_cache(self.num_blocks, self.bs)
        self.part = ops.decode_partition_size()
        self.max_splits_cap = _pow2_ceil(math.ceil(self.max_model_len / self.part))
        nq, d = self.model.nq, self.model.d

        # -------- static decode buffers (graph inputs) --------
        self.graph_sizes = sorted(b for b in cfg.graph_batch_sizes if b <= cfg.max_num_seqs) or [1]
        if self.graph_sizes[-1] < cfg.max_num_seqs:
            self.graph_sizes.append(cfg.max_num_seqs)
        mb = self.graph_sizes[-1]
        self.max_decode_batch = mb
        dv = self.device
        i32 = torch.int32
        pin = self.is_gpu
        # Static graph inputs live in a few device buffers whose layout mirrors a
        # pinned host staging copy, so a decode step refreshes all inputs with 4
        # async H2D copies.  int32 fields: ids | pos | slots | seq_lens | top_k | steps
        self.h_small = torch.zeros(6 * mb, dtype=i32, pin_memory=pin)
        self.d_small = torch.zeros(6 * mb, dtype=i32, device=dv)
        self.d_input_ids = self.d_small[0:mb]
        self.d_positions = self.d_small[mb:2 * mb]
        self.d_slots = self.d_small[2 * mb:3 * mb]
        self.d_seq_lens = self.d_small[3 * mb:4 * mb]
        self.d_top_k = self.d_small[4 * mb:5 * mb]
        self.d_steps = self.d_small[5 * mb:6 * mb]
        self.h_bt = torch.zeros(mb, self.max_blocks_per_seq, dtype=i32, pin_memory=pin)
        self.d_bt = torch.zeros(mb, self.max_blocks_per_seq, dtype=i32, device=dv)
        self.h_f32 = torch.zeros(2 * mb, dtype=torch.float32, pin_memory=pin)
        self.d_f32 = torch.zeros(2 * mb, dtype=torch.float32, device=dv)
        self.d_temp = self.d_f32[0:mb]
        self.d_top_p = self.d_f32[mb:2 * mb]
        self.h_seeds = torch.zeros(mb, dtype=torch.int64, pin_memory=pin)
        self.d_seeds = torch.zeros(mb, dtype=torch.int64, device=dv)
        self.d_out = torch.zeros(mb, dtype=i32, device=dv)
        self.h_out = torch.zeros(mb, dtype=i32, pin_memory=pin)
        self.d_logits_idx = torch.arange(mb, dtype=torch.int64, device=dv)
        self.tmp_out = torch.empty(mb * nq * self.max_splits_cap * d, dtype=torch.float32, device=dv)
        self.tmp_ml = torch.empty(mb * nq * self.max_splits_cap * 2, dtype=torch.float32, device=dv)
        self._hs = self.h_small.numpy()
        self._hbt = self.h_bt.numpy()
        self._hf = self.h_f32.numpy()
        self._hseed = self.h_seeds.numpy()
        self._done_event = torch.cuda.Event() if self.is_gpu else None
        self.graphs: Dict[Tuple[int, int], torch.cuda.CUDAGraph] = {}
        self.graph_pool = None
        self.use_graphs = self.is_gpu and not cfg.enforce_eager
        self.stats = {"graph_replays": 0, "eager_decode": 0, "prefill_steps": 0, "captures": 0}

    # ------------------------------------------------------------------ memory
    def _decide_num_blocks(self) -> int:
        cfg = self.cfg
        per_block = self.mcfg.num_layers * 2 * self.model.nkv * self.model.d * self.bs * \
            torch.tensor([], dtype=self.dtype).element_size()
        if cfg.num_kv_blocks:
            n = cfg.num_kv_blocks
        elif self.is_gpu:
            free, total = torch.cuda.mem_get_info(self.device)
            reserve = 6 << 30  # activations (8k-token prefill), graphs, sampler workspace
            budget = int(total * cfg.gpu_memory_utilization) - (total - free) - reserve
            n = max(budget // per_block, 64)
        else:
            n = max(1024, (self.max_model_len // self.bs) * 4)
        n = int(min(n, 4_000_000))
        log.info("KV cache: %d blocks x %d tokens = %d tokens (%.1f GiB)", n, self.bs, n * self.bs,
                 n * per_block / 2**30)
        return n

    # ------------------------------------------------------------------ helpers
    def _splits_for(self, max_len: int) -> int:
        return min(self.max_splits_cap, _pow2_ceil(math.ceil(max_len / self.part)))

    def _bucket(self, b: int) -> Optional[int]:
        for s in self.graph_sizes:
            if s >= b:
                return s
        return None

    # ------------------------------------------------------------------ execution
    @torch.inference_mode()
    def execute(self, batch: ScheduledBatch, masks: Optional[np.ndarray] = None) -> List[int]:
        """Runs one step; returns sampled ids for sequences with ``sample=True``
        (in batch order)."""
        if batch.is_prefill:
            return self._prefill(batch, masks)
        return self._decode(batch, masks)

    def _sampling_arrays(self, seqs):
        n = len(seqs)
        temp = np.empty(n, np.float32)
        topp = np.empty(n, np.float32)
        topk = np.empty(n, np.int32)
        seeds = np.empty(n, np.int64)
        steps = np.empty(n, np.int32)
        for i, s in enumerate(seqs):
            p = s.params
            temp[i] = p.temperature
            topp[i] = p.top_p
            topk[i] = p.top_k
            seeds[i] = p.seed
            steps[i] = s.num_output + 131 * s.preemptions
        return temp, topp, topk, seeds, steps

    def _prefill(self, batch: ScheduledBatch, masks) -> List[int]:
        self.stats["prefill_steps"] += 1
        seqs = [s for s, n in zip(batch.seqs, batch.num_tokens) if n > 0]
        ntoks = [n for n in batch.num_tokens if n > 0]
        samp = [sm for sm, n in zip(batch.sample, batch.num_tokens) if n > 0]
        if not seqs:
            return []
        bs = self.bs
        ids, pos, slots = [], [], []
        seq_lens = np.empty(len(seqs), np.int32)
        qsl = np.zeros(len(seqs) + 1, np.int32)
        maxb = max(len(s.block_ids) for s in seqs)
        bt = np.zeros((len(seqs), maxb), np.int32)
        for i, (s, n) in enumerate(zip(seqs, ntoks)):
            a = s.num_computed
            ids.append(s.tokens[a:a + n])
            p = np.arange(a, a + n, dtype=np.int32)
            pos.append(p)
            blk = np.asarray(s.block_ids, dtype=np.int32)
            bt[i, : len(blk)] = blk
            slots.append(blk[p // bs] * bs + p % bs)
            seq_lens[i] = a + n
            qsl[i + 1] = qsl[i] + n
        tiles = ops.build_prefill_tiles(ntoks, ops.prefill_tile_tokens(self.model.nq, self.model.nkv))
        dv = self.device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dv, non_blocking=True)  # noqa: E731
        meta = AttnMeta(
            is_prefill=True,
            positions=t(np.concatenate(pos)),
            slot_mapping=t(np.concatenate(slots).astype(np.int32)),
            block_tables=t(bt),
            seq_lens=t(seq_lens),
            logits_indices=t((qsl[1:] - 1).astype(np.int64)),
            q_start_loc=t(qsl) if self.is_gpu else torch.from_numpy(qsl),
            tile_info=t(np.asarray(tiles, np.int32).reshape(-1)),
            num_tiles=len(tiles),
        )
        if not self.is_gpu:
            meta.q_start_loc = torch.from_numpy(qsl)
        input_ids = t(np.concatenate(ids).astype(np.int32))
        h = self.model.forward(input_ids, meta, self.kv)
        idx = [i for i, sm in enumerate(samp) if sm]
        if not idx:
            return []
        if len(idx) != len(seqs):
            h = h[torch.tensor(idx, device=dv)]
        sseqs = [seqs[i] for i in idx]
        return self._sample(h, sseqs, masks)

    def _sample(self, h, seqs, masks) -> List[int]:
        logits = self.model.compute_logits(h)
        temp, topp, topk, seeds, steps = self._sampling_arrays(seqs)
        dv = self.device
        m = None
        if masks is not None:
            m = torch.from_numpy(masks).to(dv)
        out = ops.sample(logits, torch.from_numpy(temp).to(dv), torch.from_numpy(topp).to(dv),
                         torch.from_numpy(topk).to(dv), torch.from_numpy(seeds).to(dv),
                         torch.from_numpy(steps).to(dv), mask=m)
        return out.cpu().tolist()

    def _decode(self, batch: ScheduledBatch, masks) -> List[int]:
        seqs = batch.seqs
        n = len(seqs)
        bucket = self._bucket(n) if (self.use_graphs and masks is None) else None
        maxlen = max(s.n_tokens for s in seqs)
        splits = self._splits_for(maxlen)
        if bucket is None:
            return self._decode_eager(seqs, splits, masks)
        nb = bucket
        mb = self.max_decode_batch
        hs = self._hs
        ids = hs[0:mb]
        pos = hs[mb:2 * mb]
        slots = hs[2 * mb:3 * mb]
        sl = hs[3 * mb:4 * mb]
        bt = self._hbt
        bs = self.bs
        for i, s in enumerate(seqs):
            p = s.n_tokens - 1
            ids[i] = s.last_token
            pos[i] = p
            slots[i] = s.block_ids[p // bs] * bs + p % bs
            sl[i] = p + 1
            bt[i, :len(s.block_ids)] = s.block_ids
        temp, topp, topk, seeds, steps = self._sampling_arrays(seqs)
        hs[4 * mb:4 * mb + n] = topk
        hs[5 * mb:5 * mb + n] = steps
        self._hf[:n] = temp
        self._hf[mb:mb + n] = topp
        self._hseed[:n] = seeds
        if nb > n:  # padding rows: no KV write, 1-token context, greedy
            ids[n:nb] = 0
            pos[n:nb] = 0
            slots[n:nb] = -1
            sl[n:nb] = 1
            bt[n:nb, 0] = 0
            hs[4 * mb + n:4 * mb + nb] = 0
            hs[5 * mb + n:5 * mb + nb] = 0
            self._hf[n:nb] = 0.0
            self._hf[mb + n:mb + nb] = 1.0
        self.d_small.copy_(self.h_small, non_blocking=True)
        self.d_bt[:nb].copy_(self.h_bt[:nb], non_blocking=True)
        self.d_f32.copy_(self.h_f32, non_blocking=True)
        self.d_seeds.copy_(self.h_seeds, non_blocking=True)
        g = self.graphs.get((nb, splits))
        if g is None:
            g = self._capture(nb, splits)
        g.replay()
        self.stats["graph_replays"] += 1
        self.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
        self._done_event.record()
        self._done_event.synchronize()
        return self.h_out[:n].tolist()

    def _decode_meta(self, nb: int, splits: int) -> AttnMeta:
        return AttnMeta(is_prefill=False, positions=self.d_positions[:nb],
                        slot_mapping=self.d_slots[:nb], block_tables=self.d_bt[:nb],
                        seq_lens=self.d_seq_lens[:nb], logits_indices=self.d_logits_idx[:nb],
                        max_splits=splits, tmp_out=self.tmp_out, tmp_ml=self.tmp_ml)

    def _graph_body(self, nb: int, splits: int):
        meta = self._decode_meta(nb, splits)
        h = self.model.forward(self.d_input_ids[:nb], meta, self.kv)
        logits = self.model.compute_logits(h)
        ops.sample(logits, self.d_temp[:nb], self.d_top_p[:nb], self.d_top_k[:nb],
                   self.d_seeds[:nb], self.d_steps[:nb], out=self.d_out[:nb])

    def _capture(self, nb: int, splits: int):
        t0 = time.time()
        # inputs must be valid for the warm-up/capture run: no KV writes, 1-token contexts
        saved = (self.d_slots[:nb].clone(), self.d_seq_lens[:nb].clone())
        self.d_slots[:nb].fill_(-1)
        self.d_seq_lens[:nb].fill_(1)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._graph_body(nb, splits)  # warm-up (allocator, lazy init)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.graph_pool is None:
            self.graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.graph_pool):
            self._graph_body(nb, splits)
        self.d_slots[:nb].copy_(saved[0])
        self.d_seq_lens[:nb].copy_(saved[1])
        self.graphs[(nb, splits)] = g
        self.stats["captures"] += 1
        log.info("captured decode graph batch=%d splits=%d in %.2fs", nb, splits, time.time() - t0)
        return g

    def _decode_eager(self, seqs, splits, masks) -> List[int]:
        self.stats["eager_decode"] += 1
        n = len(seqs)
        bs = self.bs
        maxb = max(len(s.block_ids) for s in seqs)
        ids = np.empty(n, np.int32)
        pos = np.empty(n, np.int32)
        slots = np.empty(n, np.int32)
        sl = np.empty(n, np.int32)
        bt = np.zeros((n, maxb), np.int32)
        for i, s in enumerate(seqs):
            p = s.n_tokens - 1
            ids[i] = s.last_token
            pos[i] = p
            slots[i] = s.block_ids[p // bs] * bs + p % bs
            sl[i] = p + 1
            bt[i, : len(s.block_ids)] = s.block_ids
        dv = self.device
        t = lambda a: torch.from_numpy(a).to(dv)  # noqa: E731
        nq, d = self.model.nq, self.model.d
        if n > self.max_decode_batch:
            tmp_out = torch.empty(n * nq * splits * d, dtype=torch.float32, device=dv)
            tmp_ml = torch.empty(n * nq * splits * 2, dtype=torch.float32, device=dv)
        else:
            tmp_out, tmp_ml = self.tmp_out, self.tmp_ml
        meta = AttnMeta(is_prefill=False, positions=t(pos), slot_mapping=t(slots),
                        block_tables=t(bt), seq_lens=t(sl),
                        logits_indices=torch.arange(n, device=dv), max_splits=splits,
                        tmp_out=tmp_out, tmp_ml=tmp_ml)
        h = self.model.forward(t(ids), meta, self.kv)
        return self._sample(h, seqs, masks)

    def warmup(self, batch_sizes=None, max_len: int = 256):
        """Pre-capture decode graphs so the first requests do not pay for capture."""
        if not self.use_graphs:
            return
        for b in batch_sizes or self.graph_sizes:
            b = self._bucket(b)
            if b is None:
                continue
            sp = self._splits_for(max_len)
            if (b, sp) not in self.graphs:
                self._capture(b, sp)
