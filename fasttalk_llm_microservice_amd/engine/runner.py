"""Model runner: turns a :class:`ScheduledBatch` into device metadata, runs the
forward pass + sampler, returns sampled token ids.

Decode steps replay hipGraphs (``torch.cuda.CUDAGraph`` is hipGraph on ROCm),
one per (batch bucket, split bucket): the graph covers embedding -> 32 layers ->
final norm -> LM head -> sampler, with every input in static device buffers
that are refreshed by one pinned-host -> device copy per step.  Prefill steps
run eagerly (variable token counts) through the same HIP kernels.
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
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


class DecodeBlockFault(RuntimeError):
    """A persistent decode-block launch gave up at a grid barrier: the step's rows
    (and the K/V they wrote) are garbage."""


class KernelCheckError(RuntimeError):
    """The bounds-checked kernel build (FT_KERNEL_CHECKS=1) caught an out-of-range
    index (block-table entry, KV slot, rotary position, token id) in a step."""

    CODES = {1: "block-table entry >= num_blocks", 2: "KV slot >= pool capacity",
             3: "position >= rotary table rows", 4: "input token id >= vocab",
             5: "sampled token id >= vocab", 6: "KV copy/swap block id >= num_blocks"}

    def __init__(self, word):
        count, code, ctx, value = (int(x) for x in word[:4])
        self.count, self.code, self.ctx, self.value = count, code, ctx, value
        super().__init__(f"kernel bounds check: {self.CODES.get(code, f'code {code}')} "
                         f"(row/token {ctx}, value {value}; {count} violation(s))")


class CommFault(RuntimeError):
    """A tensor-parallel collective of this step timed out (custom all-reduce spin
    budget): the step's tokens are discarded and the group now runs on RCCL."""


def _pow2_ceil(x: int) -> int:
    return 1 << max(0, (x - 1).bit_length())


def input_words(mb: int, max_blocks: int) -> int:
    return 10 * mb + mb * max_blocks


def _input_views(buf: torch.Tensor, mb: int, max_blocks: int):
    """(small int32 [6mb], f32 [2mb], seeds int64 [mb], block tables int32 [mb, max_blocks])
    views of one int32 buffer of input_words() elements."""
    return (buf[0:6 * mb], buf[6 * mb:8 * mb].view(torch.float32), buf[8 * mb:10 * mb].view(torch.int64),
            buf[10 * mb:].view(mb, max_blocks))


class _Uploader:
    """Eager (mixed decode + prefill) step inputs in ONE host -> device copy: the
    numpy arrays are packed into a pinned int32 image (64-B aligned fields, int64
    and float32 bit-cast) and come back as typed device views.  Two images
    alternate; an image is refilled only after its previous copy retired (event).
    Replaces ~15 pageable ``torch.from_numpy(a).to(dev)`` copies per step, each a
    blit launch with the GPU idle in front of it."""

    ALIGN = 16  # int32 words

    def __init__(self, device, pin: bool):
        self.device = device
        self.pin = pin
        self.host = [torch.zeros(0, dtype=torch.int32) for _ in range(2)]
        self.events = [None, None]
        self.dev = torch.zeros(0, dtype=torch.int32, device=device)
        self.k = 0

    def __call__(self, arrays):
        arrs = [np.ascontiguousarray(a) for a in arrays]
        offs, n = [], 0
        for a in arrs:
            offs.append(n)
            w = (a.nbytes + 3) // 4
            n += (w + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        n = max(n, self.ALIGN)
        k = self.k
        self.k ^= 1
        if self.events[k] is not None:
            self.events[k].synchronize()
        if self.host[k].numel() < n:
            self.host[k] = torch.zeros(2 * n, dtype=torch.int32, pin_memory=self.pin)
        if self.dev.numel() < n:
            # the old buffer may still feed queued kernels: the caching allocator only
            # reuses its memory after the stream has passed this point
            self.dev = torch.zeros(2 * n, dtype=torch.int32, device=self.device)
        hb = self.host[k].numpy().view(np.uint8)
        for a, o in zip(arrs, offs):
            hb[4 * o:4 * o + a.nbytes] = a.reshape(-1).view(np.uint8)
        self.dev[:n].copy_(self.host[k][:n], non_blocking=True)
        if self.pin:
            ev = self.events[k] or torch.cuda.Event()
            ev.record()
            self.events[k] = ev
        outs = []
        for a, o in zip(arrs, offs):
            w = (a.nbytes + 3) // 4
            v = self.dev[o:o + w]
            if a.dtype.itemsize == 8:
                v = v.view(torch.int64 if a.dtype.kind in "iu" else torch.float64)
            elif a.dtype == np.float32:
                v = v.view(torch.float32)
            elif a.dtype.itemsize != 4:
                raise TypeError(f"upload: unsupported dtype {a.dtype}")
            outs.append(v.view(a.shape) if a.ndim != 1 else v)
        return outs


class _Staging:
    """Pinned host mirror of the decode graph's device inputs + its output copy.
    int32 ``small`` fields: ids | pos | slots | seq_lens | top_k | steps."""

    def __init__(self, mb: int, max_blocks: int, pin: bool, gpu: bool):
        i32 = torch.int32
        # one pinned int32 image, laid out like the device inputs (_input_views), so a
        # step's inputs go up in ONE copy: small | f32 | seeds (int64) | block tables
        self.h_in = torch.zeros(input_words(mb, max_blocks), dtype=i32, pin_memory=pin)
        self.h_small, self.h_f32, self.h_seeds, self.h_bt = _input_views(self.h_in, mb, max_blocks)
        self.h_out = torch.zeros(mb, dtype=i32, pin_memory=pin)
        self.h_err = torch.zeros(1, dtype=i32, pin_memory=pin)  # TP collective error flag
        # pipelined row gather: [source rows | destination rows] (partial gathers)
        self.h_map = torch.zeros(2 * mb, dtype=torch.int64, pin_memory=pin)
        self.err_armed = False
        self.hs = self.h_small.numpy()
        self.hbt = self.h_bt.numpy()
        self.hf = self.h_f32.numpy()
        self.hseed = self.h_seeds.numpy()
        self.event = torch.cuda.Event() if gpu else None


class MixedHandle:
    """A queued mixed step's sampled ids (pinned host copy), completion event and
    ``mark``: an event recorded after MIXED_MARK_FRAC of its layers (the engine
    builds the step queued behind it once the GPU passes it).  They rotate; a
    handle is reused only after MIXED_HANDLES - 1 later mixed launches, more than
    the steps the engine keeps queued (ENGINE_PIPELINE_DEPTH + 1)."""
    __slots__ = ("host", "event", "mark", "n", "pending", "logits", "samp")

    def __init__(self, rows: int, pin: bool, gpu: bool):
        self.host = torch.zeros(rows, dtype=torch.int32, pin_memory=pin)
        self.event = torch.cuda.Event() if gpu else None
        self.mark = torch.cuda.Event() if gpu else None
        self.n = 0
        # deferred sampler (guided rows behind a queued step): the logits and the
        # device sampling arrays wait here for sample_launch
        self.pending = False
        self.logits = None
        self.samp = None


MIXED_HANDLES = 4


class DecodeHandle:
    """A queued graph-replayed decode step.  ``pending``: only its forward pass is
    queued; its sampler waits for the allow-masks (``ModelRunner.sample_launch``)."""
    __slots__ = ("stage", "n", "nb", "pending")

    def __init__(self, stage: "_Staging", n: int, nb: int, pending: bool = False):
        self.stage = stage
        self.n = n
        self.nb = nb
        self.pending = pending


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
        self.model = LlamaModel(model_cfg, self.device, self.dtype, comm, self.max_model_len,
                                quantization=cfg.quantization)
        if cfg.weights and cfg.weights != "random":
            self.model.load_checkpoint(cfg.weights)
        else:
            self.model.init_random(seed=cfg.seed)
        if self.is_gpu:
            torch.cuda.synchronize(self.device)
        log.info("weights ready in %.1fs", time.time() - t0)

        # batch-invariant numerics (cfg.batch_invariant): rows of a step up to the token
        # budget plus a decode row per sequence
        self.invariant = bool(getattr(cfg, "batch_invariant", False))
        if self.invariant:
            self.model.set_batch_invariant(max(cfg.max_num_batched_tokens, cfg.max_num_seqs)
                                           + cfg.max_num_seqs)
        self.kv_dtype = cfg.kv_torch_dtype(self.dtype)
        self.num_blocks = self._decide_num_blocks()
        self.kv = self.model.allocate_kv_cache(self.num_blocks, self.bs, self.kv_dtype)
        # FT_KERNEL_CHECKS=1: the bounds-checked kernel build validates every index it
        # is handed against the tensors of the launch (this pool's blocks, the rotary
        # table's rows, the vocab) and reports into this word, read after each step
        self.d_check: Optional[torch.Tensor] = None
        if self.is_gpu and getattr(ops.native(), "kernel_checks", False):
            self.d_check = torch.zeros(4, dtype=torch.int32, device=self.device)
            ops.native().set_kernel_checks(self.d_check)
            log.warning("FT_KERNEL_CHECKS: bounds-checked kernels (KV pool %d blocks x %d, "
                        "rotary rows %d, vocab %d)", self.num_blocks, self.bs,
                        self.model.cos_sin.shape[0], self.mcfg.vocab_size)
        # E6 host swap pool (--swap-space): capped at 2x the device pool, allocated
        # (pinned) on the first swap-out so an idle server does not pin host memory
        k0 = self.kv[0][0]
        self.kv_block_elems = k0.numel() // k0.shape[0]
        host_block_bytes = 2 * len(self.kv) * self.kv_block_elems * k0.element_size()
        self.num_host_blocks = min(int(cfg.swap_space_gb * (1 << 30)) // host_block_bytes,
                                   2 * self.num_blocks)
        self.host_kv = None
        self.swap_staging = None
        self.kv_ptrs = None
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
        # Static graph inputs live in ONE device buffer whose layout mirrors a pinned
        # host staging image, so a decode step refreshes all its inputs with one async
        # H2D copy (each copy is a blit launch, and the GPU idled ~20 us in front of
        # each of the four it used to take: profiles/prof_driver_config_r02b.txt).
        # int32 fields: ids | pos | slots | seq_lens | top_k | steps, then temperature |
        # top_p (f32), seeds (int64), block tables
        self.d_in = torch.zeros(input_words(mb, self.max_blocks_per_seq), dtype=i32, device=dv)
        self.d_small, self.d_f32, self.d_seeds, self.d_bt = _input_views(self.d_in, mb, self.max_blocks_per_seq)
        self.d_input_ids = self.d_small[0:mb]
        self.d_positions = self.d_small[mb:2 * mb]
        self.d_slots = self.d_small[2 * mb:3 * mb]
        self.d_seq_lens = self.d_small[3 * mb:4 * mb]
        self.d_top_k = self.d_small[4 * mb:5 * mb]
        self.d_steps = self.d_small[5 * mb:6 * mb]
        self.d_temp = self.d_f32[0:mb]
        self.d_top_p = self.d_f32[mb:2 * mb]
        self.d_out = torch.zeros(mb, dtype=i32, device=dv)
        self.d_map = torch.zeros(2 * mb, dtype=torch.int64, device=dv)
        # pinned staging sets: while decode step n runs, steps n+1 .. n+depth are
        # filled and queued behind it from the other sets (pipelined decode)
        nstg = max(2, int(getattr(cfg, "pipeline_depth", 1)) + 1)
        self.stg = [_Staging(mb, self.max_blocks_per_seq, pin, self.is_gpu) for _ in range(nstg)]
        self._mx_handles = [MixedHandle(mb, pin, self.is_gpu) for _ in range(MIXED_HANDLES)]
        # ENGINE_MIXED_CHAIN_AT: fraction of a queued mixed step's layers after which
        # its mark event is recorded (0: no mark, the next step is built at once).
        # 0.6: 5,751 / 5,782 / 5,694 vs 5,701-5,711 tok/s at 0.75, same p50 TTFT
        # (profiles/ab_sched_screen_r05.log)
        self.mixed_mark_frac = float(os.environ.get("ENGINE_MIXED_CHAIN_AT", "0.6"))
        self._mx_next = 0
        self._stg_next = 0
        self._upload = _Uploader(dv, pin) if self.is_gpu else None
        self.h_out = torch.zeros(mb, dtype=i32, pin_memory=pin)  # eager-step sampler output
        self.h_err = torch.zeros(1, dtype=i32, pin_memory=pin)
        # TP rank 0 decides about collective faults; workers only follow its messages
        self.checks_comm = comm.world_size > 1 and comm.rank == 0
        # guided decoding (E19): the token allow-mask is a STATIC input of every
        # decode graph -- all-ones rows for unguided sequences -- so a batch with
        # one tool-calling session stays on the graph path (it only loses the
        # one-step-ahead pipelining: the next mask depends on this step's token)
        self.mask_words = (model_cfg.vocab_size + 31) // 32
        self.d_mask = torch.full((mb, self.mask_words), -1, dtype=i32, device=dv) if self.is_gpu else None
        self.h_mask = torch.full((mb, self.mask_words), -1, dtype=i32, pin_memory=pin) if self.is_gpu else None
        self._mask_rows = 0   # leading rows of d_mask that may hold a non-trivial mask
        self.d_logits_idx = torch.arange(mb, dtype=torch.int64, device=dv)
        # decode-attention partials: one slot per (sequence, kv head) + one per wave
        # of the kernel's grid (any step has at most max_num_seqs decode rows)
        self.max_decode_rows = max(mb, cfg.max_num_seqs)
        n_out, n_ml = ops.decode_workspace(self.max_decode_rows, nq, self.model.nkv, d,
                                           waves=None if self.is_gpu else 0,
                                           piece=ops.DECODE_INV_PIECE if self.invariant else 0,
                                           max_len=self.max_blocks_per_seq * self.bs)
        self.tmp_out = torch.empty(max(1, n_out), dtype=torch.float32, device=dv)
        self.tmp_ml = torch.empty(max(1, n_ml), dtype=torch.float32, device=dv)
        # split-KV prefill partials (ops.build_prefill_tiles): 128 slots = 128 MiB fp32
        # for Llama-3-8B; FT_PREFILL_SPLIT=0 keeps one workgroup per query block
        self.num_cus = torch.cuda.get_device_properties(dv).multi_processor_count if self.is_gpu else 256
        self.pf_part_o = self.pf_part_ml = None
        # batch-invariant plans cut every KV range at fixed pieces and never fall back
        # to an unsplit item: room for every query block of a full step (the budget's
        # 64-token blocks + a partial one per prompt) times the pieces of max_model_len
        self.pf_max_partials = ops.PREFILL_MAX_PARTIALS
        if self.invariant:
            pieces = -(-self.max_model_len // (ops.PREFILL_BK * ops.PREFILL_INV_CHUNK))
            qblocks = -(-cfg.max_num_batched_tokens // ops.prefill_tile_tokens(nq, self.model.nkv))
            self.pf_max_partials = max(ops.PREFILL_MAX_PARTIALS,
                                       (qblocks + cfg.max_num_seqs) * pieces)
        if self.is_gpu and (self.invariant or os.environ.get("FT_PREFILL_SPLIT", "1") == "1"):
            n_po, n_pml = ops.prefill_partials(self.model.nkv, d, self.pf_max_partials)
            self.pf_part_o = torch.empty(n_po, dtype=torch.float32, device=dv)
            self.pf_part_ml = torch.empty(n_pml, dtype=torch.float32, device=dv)
        # in-launch combine tickets (FT_DECODE_FUSED_COMBINE=0: separate combine kernel):
        # with the kernel at one workgroup per CU the last-arriver merge matches or beats
        # the combine kernel and saves a launch per layer (csrc/kernels/attn_decode.hip)
        self.dec_counters = ops.decode_counters(self.max_decode_rows, self.model.nkv, dv) \
            if self.is_gpu and (self.invariant or os.environ.get("FT_DECODE_FUSED_COMBINE", "1") == "1") \
            else None
        self._done_event = torch.cuda.Event() if self.is_gpu else None
        # persistent decode block: its sticky give-up word (ctl[2]) is copied to pinned
        # memory every BLOCK_CHECK_EVERY waits and read at the next check (never a sync)
        self._blk_host = torch.zeros(1, dtype=torch.int32, pin_memory=True) \
            if self.is_gpu and self.model.block else None
        self._blk_event = torch.cuda.Event() if self._blk_host is not None else None
        self._blk_armed = False
        self._blk_waits = 0
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        # guided decoding, pipelined: per bucket a forward graph (-> logits) and a
        # sampler graph, so the next step's forward is queued before this step's
        # tokens are known and only its sampler waits for the grammar masks
        self.graphs_split: Dict[int, tuple] = {}
        self._fwd_logits: Dict[int, torch.Tensor] = {}
        self._pending_split: Optional["DecodeHandle"] = None   # forward queued, sampler not yet
        # ENGINE_GUIDED_PIPELINE=0: guided batches run one synchronous step at a time
        self.guided_pipeline = os.environ.get("ENGINE_GUIDED_PIPELINE", "1") != "0"
        self.graph_pool = None
        self.use_graphs = self.is_gpu and not cfg.enforce_eager and comm.graph_safe()
        # FT_FAULT_TP_STALL="<n>:<seconds>" (TP workers): before executing the n-th
        # decode graph message, stall until rank 0's custom all-reduce has run out of
        # spin budget (its error word is set; at most <seconds>) -- the fault test
        # of the collective timeout contract
        # "m<n>:<seconds>" stalls before the n-th eager (mixed / prefill) message instead
        stall = os.environ.get("FT_FAULT_TP_STALL", "") if comm.rank > 0 else ""
        self._stall_mixed = stall.startswith("m")
        stall = stall.lstrip("m")
        self._stall_at, self._stall_s = (int(stall.split(":")[0]), float(stall.split(":")[1])) \
            if stall else (None, 0.0)
        self._graph_msgs = 0
        self._mixed_msgs = 0
        # the first eager steps and graph warm-ups of a TP group wait for peers with a
        # long spin budget (every rank counts the same steps: same message order)
        self._warm_left = int(os.environ.get("ENGINE_TP_WARM_STEPS", "4")) \
            if comm.world_size > 1 else 0
        self._trace_tp = os.environ.get("FT_TP_TRACE", "0") == "1" and comm.world_size > 1
        self.stats = {"graph_replays": 0, "eager_decode": 0, "prefill_steps": 0, "captures": 0}
        # tests: a list here collects every step's logits (fp32; eager steps on the host,
        # graph-replayed and mixed-ahead steps as stream-ordered device copies) -- TP-vs-TP=1
        # numerics are compared on logits, not on greedy tokens of random weights.  With
        # logits_tap_ids a list too, each entry gets the request ids of its rows.
        self.logits_tap: Optional[list] = None
        self.logits_tap_ids: Optional[list] = None
        self._tap_rows: Optional[list] = None
        self._graph_logits: Dict[int, torch.Tensor] = {}   # logits tensor of each graph
        # FT_GPU_GAPS=1: timing events around every graph-replayed decode step, so
        # gap_summary() can report how long the GPU sat idle BETWEEN consecutive
        # decode steps (the host enqueued the next one late), without a profiler
        self._gaps = [] if self.is_gpu and os.environ.get("FT_GPU_GAPS", "0") == "1" else None
        self.bcast = None  # TP rank 0: parallel.shm_broadcast.ShmBroadcast writer

    # ------------------------------------------------------------------ memory
    # ------------------------------------------------------------------ host swap (E6)
    SWAP_CHUNK = 32  # blocks per gather/scatter launch (64 MiB of staging for 8B)

    def swap(self, swap_out, swap_in):
        """Copies preempted sequences' KV blocks device -> host (``swap_out``:
        (block, slot) pairs) and resumed ones host -> device (``swap_in``: (slot,
        block) pairs), in stream order before the step that follows."""
        if self.bcast is not None:
            self.bcast.send(("swap", (list(swap_out), list(swap_in)), None))
        self._swap(swap_out, swap_in)

    def _swap(self, swap_out, swap_in):
        nl = 2 * len(self.kv)
        be = self.kv_block_elems
        if self.host_kv is None:
            t0 = time.time()
            self.host_kv = torch.empty(self.num_host_blocks, nl * be, dtype=self.kv_dtype,
                                       pin_memory=self.is_gpu)
            self.swap_staging = torch.empty(self.SWAP_CHUNK, nl * be, dtype=self.kv_dtype,
                                            device=self.device)
            if self.is_gpu:
                self.kv_ptrs = torch.tensor([c.data_ptr() for kv in self.kv for c in kv],
                                            dtype=torch.int64, device=self.device)
            log.info("host KV swap pool: %d blocks (%.2f GiB) in %.2fs", self.num_host_blocks,
                     self.host_kv.numel() * self.host_kv.element_size() / (1 << 30),
                     time.time() - t0)
        for pairs, out in ((swap_out, True), (swap_in, False)):
            for c0 in range(0, len(pairs), self.SWAP_CHUNK):
                chunk = pairs[c0:c0 + self.SWAP_CHUNK]
                dev_blocks = [p[0] if out else p[1] for p in chunk]
                slots = [p[1] if out else p[0] for p in chunk]
                if min(dev_blocks) < 0 or max(dev_blocks) >= self.num_blocks or \
                        min(slots) < 0 or max(slots) >= self.num_host_blocks:
                    raise ValueError("swap block id out of range")
                ids = torch.tensor(dev_blocks, dtype=torch.int32, device=self.device)
                st = self.swap_staging[:len(chunk)]
                if not out:
                    for i, h in enumerate(slots):
                        st[i].copy_(self.host_kv[h], non_blocking=True)
                ops.kv_swap(self.kv, self.kv_ptrs, ids, st, to_staging=out)
                if out:
                    for i, h in enumerate(slots):
                        self.host_kv[h].copy_(st[i], non_blocking=True)
        self.stats["swap_blocks"] = self.stats.get("swap_blocks", 0) + len(swap_out) + len(swap_in)

    def _decide_num_blocks(self) -> int:
        cfg = self.cfg
        per_block = self.mcfg.num_layers * 2 * self.model.nkv * self.model.d * self.bs * \
            torch.tensor([], dtype=self.kv_dtype).element_size()
        if cfg.num_kv_blocks:
            n = cfg.num_kv_blocks
        elif self.is_gpu:
            free, total = torch.cuda.mem_get_info(self.device)
            reserve = 6 << 30  # activations (8k-token prefill), graphs, sampler workspace
            used = total - free
            if os.environ.get("ENGINE_KV_SIZING", "device") == "own":
                # several engines time-share this device (FT_BENCH_SHARED_GPU rehearsals):
                # count only this process's allocations, so the pool does not depend on
                # whether the other engines have sized theirs yet
                used = torch.cuda.memory_reserved(self.device)
            budget = int(total * cfg.gpu_memory_utilization) - used - reserve
            n = max(budget // per_block, 64)
        else:
            n = max(1024, (self.max_model_len // self.bs) * 4)
        n = self.comm.min_int(int(min(n, 4_000_000)))  # every TP rank holds the same pool
        log.info("KV cache: %d blocks x %d tokens = %d tokens (%.1f GiB, %s)", n, self.bs, n * self.bs,
                 n * per_block / 2**30, str(self.kv_dtype).replace("torch.", ""))
        return n

    # ------------------------------------------------------------------ helpers
    def _bucket(self, b: int) -> Optional[int]:
        for s in self.graph_sizes:
            if s >= b:
                return s
        return None

    # ------------------------------------------------------------------ execution
    @torch.inference_mode()
    def execute(self, batch: ScheduledBatch, masks: Optional[np.ndarray] = None) -> List[int]:
        """Runs one step; returns sampled ids for ``batch.sampled_seqs()`` in order.

        Decode-only steps replay a hipGraph; steps that carry prefill chunks run
        eagerly as one mixed forward pass (decode rows first)."""
        self._assert_no_pending_split("execute")
        if batch.has_prefill:
            if self._gaps is not None:
                self._gap_mark(True, "m")   # closed by _wait, right after the last launch
            return self._mixed(batch, masks)
        if not batch.decode_seqs:
            return []
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
            steps[i] = s.num_output + s.inflight + 131 * s.preemptions
        return temp, topp, topk, seeds, steps

    def _mixed(self, batch: ScheduledBatch, masks) -> List[int]:
        host = self._mixed_host(batch)
        if self.bcast is not None:
            self.bcast.send(("mixed", host, masks))
        return self._mixed_run(host, masks)

    def _mixed_host(self, batch: ScheduledBatch) -> Dict[str, object]:
        """Host-side (numpy) inputs of an eager mixed decode+prefill step; this is
        also the message tensor-parallel workers receive."""
        dseqs = batch.decode_seqs
        pseqs = [s for s, n in zip(batch.prefill_seqs, batch.prefill_tokens) if n > 0]
        ntoks = [n for n in batch.prefill_tokens if n > 0]
        # chunk starts as scheduled (a chunk queued behind an in-flight chunk of the
        # same prompt starts after it; num_computed only moves in post_step)
        starts = [a for a, n in zip(batch.prefill_start or [None] * len(batch.prefill_seqs),
                                    batch.prefill_tokens) if n > 0]
        psamp = [sm for sm, n in zip(batch.prefill_sample, batch.prefill_tokens) if n > 0]
        bs = self.bs
        nd = len(dseqs)
        ids, pos, slots = [], [], []
        host: Dict[str, object] = {"nd": nd}
        # decode rows
        if nd:
            d_ids = np.empty(nd, np.int32)
            d_pos = np.empty(nd, np.int32)
            d_slot = np.empty(nd, np.int32)
            d_bt = np.zeros((nd, max(len(s.block_ids) for s in dseqs)), np.int32)
            for i, s in enumerate(dseqs):
                p = s.n_tokens - 1 + s.inflight   # queued ahead: ids come from the device
                d_ids[i] = s.last_token
                d_pos[i] = p
                d_slot[i] = s.block_ids[p // bs] * bs + p % bs
                d_bt[i, : len(s.block_ids)] = s.block_ids
            ids.append(d_ids)
            pos.append(d_pos)
            slots.append(d_slot)
            host["d_bt"] = d_bt
            host["d_sl"] = d_pos + 1
        # prefill rows
        seq_lens = np.empty(len(pseqs), np.int32)
        qsl = np.zeros(len(pseqs) + 1, np.int32)
        maxb = max([len(s.block_ids) for s in pseqs] or [1])
        bt = np.zeros((max(1, len(pseqs)), maxb), np.int32)
        for i, (s, n, a) in enumerate(zip(pseqs, ntoks, starts)):
            if a is None:
                a = s.num_computed
            ids.append(s.tokens[a:a + n])
            p = np.arange(a, a + n, dtype=np.int32)
            pos.append(p)
            blk = np.asarray(s.block_ids, dtype=np.int32)
            bt[i, : len(blk)] = blk
            slots.append(blk[p // bs] * bs + p % bs)
            seq_lens[i] = a + n
            qsl[i + 1] = qsl[i] + n
        tiles, combine = ops.build_prefill_tiles(
            ntoks, ops.prefill_tile_tokens(self.model.nq, self.model.nkv),
            seq_lens=seq_lens if self.pf_part_o is not None else None, nkv=self.model.nkv,
            num_cus=self.num_cus, max_partials=self.pf_max_partials,
            fixed_chunk=ops.PREFILL_INV_CHUNK if self.invariant else 0)
        # logits rows: every decode row + the last row of each prompt that completes
        lrows = list(range(nd)) + [nd + int(qsl[i + 1]) - 1 for i, sm in enumerate(psamp) if sm]
        host.update(ids=np.concatenate(ids).astype(np.int32), pos=np.concatenate(pos).astype(np.int32),
                    slots=np.concatenate(slots).astype(np.int32), lrows=np.asarray(lrows, np.int64),
                    bt=bt, seq_lens=seq_lens, qsl=qsl, tiles=np.asarray(tiles, np.int32).reshape(-1),
                    num_tiles=len(tiles), combine=np.asarray(combine, np.int32).reshape(-1),
                    num_combine=len(combine),
                    num_partials=sum(c[3] for c in combine))
        sseqs = dseqs + [s for s, sm in zip(pseqs, psamp) if sm]
        host["sampling"] = self._sampling_arrays(sseqs)
        if self.logits_tap_ids is not None:
            self._tap_rows = [s.request_id for s in sseqs]
        return host

    def _long_waits(self):
        """Context: the custom collectives' first-steps spin budget while warm steps last."""
        if self._warm_left <= 0 or self.comm.custom is None:
            return contextlib.nullcontext()
        self._warm_left -= 1
        return self.comm.custom.long_waits()

    def _mixed_run(self, host: Dict[str, object], masks) -> List[int]:
        t0 = time.perf_counter() if self._trace_tp else 0.0
        with self._long_waits():
            out = self._mixed_run_inner(host, masks)
        if self._trace_tp:
            log.warning("TP trace rank %d: mixed step %d rows in %.1f ms", self.comm.rank,
                        len(host["ids"]), 1e3 * (time.perf_counter() - t0))
        return out

    def _mixed_run_inner(self, host: Dict[str, object], masks) -> List[int]:
        self.stats["prefill_steps"] += 1
        nd = host["nd"]
        qsl = host["qsl"]
        names = ["pos", "slots", "lrows", "bt", "seq_lens", "qsl", "tiles", "ids", "combine"]
        if nd:
            if nd > self.max_decode_rows:
                raise ValueError(f"{nd} decode rows exceed max_num_seqs {self.max_decode_rows}")
            names += ["d_bt", "d_sl"]
        arrays = [host[k] for k in names]
        has_logits = len(host["lrows"]) > 0
        if has_logits:
            arrays += list(host["sampling"])
            if masks is not None:
                arrays.append(masks)
        if self.is_gpu:
            dev = self._upload(arrays)
        else:
            dev = [torch.from_numpy(np.ascontiguousarray(a)) for a in arrays]
        d = dict(zip(names, dev))
        meta = AttnMeta(
            positions=d["pos"], slot_mapping=d["slots"], logits_indices=d["lrows"], num_decode=nd,
            block_tables=d["bt"], seq_lens=d["seq_lens"],
            q_start_loc=d["qsl"] if self.is_gpu else torch.from_numpy(qsl),
            tile_info=d["tiles"], num_tiles=host["num_tiles"])
        if host.get("num_combine", 0):
            meta.pf_part_o, meta.pf_part_ml = self.pf_part_o, self.pf_part_ml
            meta.pf_combine, meta.pf_num_combine = d["combine"], host["num_combine"]
            meta.pf_num_partials = host["num_partials"]
        if nd:
            meta.dec_block_tables = d["d_bt"]
            meta.dec_seq_lens = d["d_sl"]
            meta.tmp_out, meta.tmp_ml = self.tmp_out, self.tmp_ml
            meta.dec_counters = self.dec_counters
        h = self.model.forward(d["ids"], meta, self.kv)
        if not has_logits:
            # a middle chunk of a chunked prefill samples nothing, but its all-reduces
            # wrote KV blocks that post_step commits to the prefix cache: check the
            # custom collectives' error word before anything is committed
            flag = self._arm_comm_check() if self.is_gpu else None
            if flag is not None:
                self.h_err.copy_(flag, non_blocking=True)
                self._wait()
                if int(self.h_err[0]):
                    self._comm_fault()
            return []
        k = len(names)
        samp = dev[k:k + 5]
        dmask = dev[k + 5] if masks is not None else None
        return self._sample(h, host["sampling"], masks, dev_sampling=samp, dev_mask=dmask)

    def _wait(self, ev=None):
        """Block until the GPU work queued so far (or up to ``ev``) is done WITHOUT
        holding the GIL: a plain ``.cpu()`` / ``synchronize`` keeps the GIL for the
        whole step and starves the asyncio thread that streams to the WebSockets."""
        if ev is None:
            if self._gaps and self._gaps[-1][1] is None:
                self._gap_mark(False)
            ev = self._done_event
            ev.record()
        t0 = time.perf_counter()
        while not ev.query():
            time.sleep(0.0001)
        self.stats["wait_ms"] = self.stats.get("wait_ms", 0.0) + 1e3 * (time.perf_counter() - t0)
        if self.d_check is not None:
            self.kernel_check()
        if self._blk_host is not None:
            self._block_check()

    BLOCK_CHECK_EVERY = 64

    def _block_check(self):
        """Decode block give-up word: a grid barrier that timed out (a grid that was
        not fully resident) leaves garbage rows; the step fails loudly and the model
        falls back to the unfused layer (graphs recaptured on demand)."""
        self._blk_waits += 1
        if self._blk_armed and self._blk_event.query():
            self._blk_armed = False
            if int(self._blk_host[0]) and self.model.block_fault():
                self._blk_host = None
                self.graphs.clear()
                self._graph_logits.clear()
                self.graphs_split.clear()
                self._fwd_logits.clear()
                self._pending_split = None
                raise DecodeBlockFault("decode block grid barrier timed out; step discarded, "
                                       "unfused decode layer from now on")
        if not self._blk_armed and self._blk_waits % self.BLOCK_CHECK_EVERY == 0:
            self._blk_host.copy_(self.model.db_ctl[2:3], non_blocking=True)
            self._blk_event.record()
            self._blk_armed = True

    def kernel_check(self):
        """Checked build: raise KernelCheckError if a kernel has reported an out-of-range
        index since the last reset (the word is sticky until kernel_check_reset)."""
        if self.d_check is None:
            return
        w = self.d_check.cpu()
        if int(w[0]):
            # clear the sticky word as the error is raised: the serving loop fails the
            # affected requests and carries on, and later steps must not re-raise it
            self.d_check.zero_()
            raise KernelCheckError(w.tolist())

    def kernel_check_reset(self):
        if self.d_check is not None:
            self.d_check.zero_()

    def _sample(self, h, sampling, masks, dev_sampling=None, dev_mask=None) -> List[int]:
        logits = self.model.compute_logits(h)
        if self.logits_tap is not None:
            self._tap(logits.float().cpu())
        if dev_sampling is None:
            arrays = list(sampling) + ([masks] if masks is not None else [])
            if self.is_gpu:
                dev = self._upload(arrays)
            else:
                dev = [torch.from_numpy(np.ascontiguousarray(a)) for a in arrays]
            dev_sampling = dev[:5]
            dev_mask = dev[5] if masks is not None else None
        temp, topp, topk, seeds, steps = dev_sampling
        out = ops.sample(logits, temp, topp, topk, seeds, steps, mask=dev_mask)
        if not self.is_gpu:
            return out.tolist()
        n = out.shape[0]
        flag = self._arm_comm_check()
        if flag is not None:
            self.h_err.copy_(flag, non_blocking=True)
        if n <= self.h_out.shape[0]:
            self.h_out[:n].copy_(out, non_blocking=True)
            self._wait()
            host = self.h_out[:n]
        else:
            host = torch.empty(n, dtype=out.dtype, pin_memory=True)
            host.copy_(out, non_blocking=True)
            self._wait()
        if flag is not None and int(self.h_err[0]):
            self._comm_fault()
        return host.tolist()

    def _tap(self, logits: torch.Tensor):
        self.logits_tap.append(logits)
        if self.logits_tap_ids is not None:
            self.logits_tap_ids.append(self._tap_rows)
            self._tap_rows = None

    # ------------------------------------------------------------------ TP fault contract
    def _arm_comm_check(self) -> Optional[torch.Tensor]:
        """Queues the fold of every rank's collective error word into the device
        flag (eager steps; decode graphs carry it) and returns the flag, or None
        when this rank does not check (single GPU, workers, RCCL only)."""
        flag = self.comm.error_flag
        if flag is None or not self.checks_comm:
            return None
        self.comm.export_error()
        return flag

    def _comm_fault(self):
        """Rank 0 saw a timed-out custom collective: every rank drops to RCCL (in
        message order, so the collectives stay matched) and the step fails."""
        if self.bcast is not None:
            self.bcast.send(("comm_fault", None, None))
        self._drop_custom_collectives()
        raise CommFault("tensor-parallel all-reduce timed out waiting for a peer; "
                        "step discarded, group switched to RCCL")

    def _drop_custom_collectives(self):
        if self.is_gpu:
            torch.cuda.synchronize(self.device)  # no graph of the old kind still running
        self.comm.disable_custom("custom collective timed out")
        self.graphs.clear()  # they captured the custom kernels; recaptured on demand
        self._graph_logits.clear()
        self.graphs_split.clear()
        self._fwd_logits.clear()
        self._pending_split = None   # the in-flight step is discarded with its graphs
        if not self.comm.graph_safe():
            self.use_graphs = False
        for st in self.stg:
            st.err_armed = False
            st.h_err.zero_()

    def _decode(self, batch: ScheduledBatch, masks) -> List[int]:
        seqs = batch.decode_seqs
        n = len(seqs)
        bucket = self._bucket(n) if self.use_graphs else None
        if bucket is None:
            return self._decode_eager(seqs, masks)
        return self.decode_collect(self.decode_launch(seqs, masks=masks))

    def can_pipeline(self, n: int) -> bool:
        return self.use_graphs and self._bucket(n) is not None

    def can_defer_sample(self) -> bool:
        """Can a decode step be queued with its sampler deferred until its allow-masks
        are known (pipelined guided decoding)?  Single process only (TP workers replay
        whole steps from the broadcast)."""
        return self.use_graphs and self.guided_pipeline and self.bcast is None \
            and not self.checks_comm and self.d_mask is not None

    def decode_launch(self, seqs, ahead: int = 0, masks: Optional[np.ndarray] = None,
                      rowmap: Optional[List[int]] = None, defer_sample: bool = False
                      ) -> DecodeHandle:
        """Fills a staging set and queues a graph-replayed decode step (returns at
        once).  Positions are ``inflight`` tokens past each sequence's collected
        state (steps queued ahead of it); with ``ahead`` the input ids are the last
        queued step's sampled ids, copied device-to-device, so the host never waits
        between steps.  ``rowmap[i]`` (with ``ahead``): the row of that step that
        sequence i sat in (None: the same row).  ``defer_sample``: queue the forward
        pass only; ``sample_launch`` queues its sampler once the masks are known."""
        n = len(seqs)
        nb = self._bucket(n)
        st = self.stg[self._stg_next]
        self._stg_next = (self._stg_next + 1) % len(self.stg)
        maxblk = self._decode_fill(seqs, nb, st)
        gather = None
        if ahead and rowmap is not None:
            gather = np.zeros(nb, dtype=np.int64)   # padding rows read row 0 (ignored)
            gather[:n] = rowmap   # -1: no queued step has the row, its id comes from the host
        self._assert_no_pending_split("decode_launch")
        if defer_sample:
            assert self.can_defer_sample()
            self._decode_enqueue(st, nb, n, from_device=bool(ahead), gather=gather, fwd_only=True)
            h = DecodeHandle(st, n, nb, pending=True)
            self._pending_split = h
            return h
        if self.bcast is not None:
            self.bcast.send(("graph", {"nb": nb, "n": n, "small": st.hs.copy(),
                                       "bt": st.hbt[:nb, :maxblk].copy(), "f32": st.hf.copy(),
                                       "seeds": st.hseed.copy(), "from_device": bool(ahead),
                                       "rowmap": gather}, masks))
        self._set_masks(masks, n)
        self._decode_enqueue(st, nb, n, from_device=bool(ahead), gather=gather)
        if self.logits_tap is not None and nb in self._graph_logits:
            # copied in stream order: the next queued replay overwrites the graph's logits
            if self.logits_tap_ids is not None:
                self._tap_rows = [s.request_id for s in seqs]
            self._tap(self._graph_logits[nb][:n].float().clone())
        return DecodeHandle(st, n, nb)

    @torch.inference_mode()
    def sample_launch(self, h, masks: Optional[np.ndarray]):
        """Queues the sampler of a step whose forward pass ``decode_launch(...,
        defer_sample=True)`` queued: its allow-masks go up, the sampler graph reads
        the forward graph's logits, the ids land in ``d_out`` (the next step's
        inputs) and in the staging set's pinned copy.  A mixed step's
        (``mixed_launch(..., defer_sample=True)``) eager sampler reads its held logits."""
        if isinstance(h, MixedHandle):
            assert h.pending
            dmask = None
            if masks is not None:
                dmask = self._upload([masks])[0] if self.is_gpu else torch.from_numpy(masks)
            self._mixed_sample(h, h.logits, h.samp, dmask)
            return
        assert h.pending and self._pending_split is h
        self._set_masks(masks, h.n)
        self.graphs_split[h.nb][1].replay()
        self._pending_split = None
        st = h.stage
        st.h_out[:h.n].copy_(self.d_out[:h.n], non_blocking=True)
        st.err_armed = False
        st.event.record()
        h.pending = False
        if self._gaps is not None:
            self._gap_mark(False)

    def discard_pending(self):
        """Forget a deferred-sample step whose sampler will never be queued (the
        engine dropped its in-flight steps after a failure)."""
        self._pending_split = None

    def _assert_no_pending_split(self, where: str):
        """A split step's logits (``_fwd_logits``) live in the graph pool every graph
        shares: nothing may be replayed or run between its forward and its sampler, or
        that work can overwrite them before they are sampled."""
        if self._pending_split is not None:
            raise RuntimeError(f"{where}: a deferred-sample decode step is pending; "
                               "sample_launch() must be queued first")

    def _set_masks(self, masks: Optional[np.ndarray], n: int):
        """Uploads the step's allow-masks into the graph's static mask rows (stream
        ordered before the replay); resets rows a previous guided step dirtied."""
        if self.d_mask is None:
            return
        if masks is None:
            if self._mask_rows:
                self.d_mask[:self._mask_rows].fill_(-1)
                self._mask_rows = 0
            return
        rows = max(n, self._mask_rows)
        hm = self.h_mask.numpy()
        hm[:n, : masks.shape[1]] = masks[:n]
        hm[n:rows] = -1
        self.d_mask[:rows].copy_(self.h_mask[:rows], non_blocking=True)
        self._mask_rows = n

    def decode_collect(self, h: DecodeHandle) -> List[int]:
        st = h.stage
        self._wait(st.event)
        if st.err_armed and int(st.h_err[0]):
            self._comm_fault()
        return st.h_out[:h.n].tolist()

    def step_done(self, h) -> bool:
        """Non-blocking: has the queued step behind handle ``h`` finished on the GPU?"""
        ev = h.stage.event if isinstance(h, DecodeHandle) else h.event
        return ev is None or ev.query()

    @torch.inference_mode()
    def mixed_launch(self, batch: ScheduledBatch, rowmap: Optional[List[int]],
                     masks: Optional[np.ndarray] = None, defer_sample: bool = False) -> "MixedHandle":
        """Queues a mixed (decode + prefill) step behind the queued step(s) without
        waiting (engine ``_speculate_mixed``): decode row i's input id is row
        ``rowmap[i]`` of the last queued step's sampled ids (``d_out``), gathered on
        the device; its position is ``inflight`` tokens ahead.  ``rowmap`` None:
        nothing is queued, the ids are the sequences' last tokens (host).  The
        sampled ids land in ``d_out`` (rows = ``batch.sampled_seqs()``) for the
        decode step queued next, and in a pinned host buffer for the collect.
        ``masks``: the sampled rows' allow-masks when they are known at launch;
        ``defer_sample``: they are not (guided rows whose grammar waits for the step
        queued ahead) -- the forward pass is queued now, the sampler by
        :meth:`sample_launch` once the engine has the masks.  Single process only
        (no TP broadcast)."""
        self._assert_no_pending_split("mixed_launch")
        if self._gaps is not None:
            self._gap_mark(True, "a")
        tp0 = time.perf_counter()
        host = self._mixed_host(batch)
        tp1 = time.perf_counter()
        nd = host["nd"]
        self.stats["prefill_steps"] += 1
        self.stats["mixed_ahead"] = self.stats.get("mixed_ahead", 0) + 1
        names = ["pos", "slots", "lrows", "bt", "seq_lens", "qsl", "tiles", "ids", "combine"]
        if nd:
            names += ["d_bt", "d_sl"]
        arrays = [host[k] for k in names] + list(host["sampling"])
        # rowmap[i] < 0: row i's sequence has no queued step (it joined after the last
        # queued step was built); its id is its last token, already in host["ids"]
        rm = np.asarray(rowmap if rowmap is not None else [], dtype=np.int64)
        dst = np.nonzero(rm >= 0)[0].astype(np.int64)
        partial = nd and rowmap is not None and len(dst) < nd
        arrays.append(rm[dst] if nd and len(dst) else np.zeros(1, np.int64))
        arrays.append(dst if partial and len(dst) else np.zeros(1, np.int64))
        if masks is not None and not defer_sample:
            arrays.append(masks)
        if self.is_gpu:
            dev = self._upload(arrays)
        else:
            dev = [torch.from_numpy(np.ascontiguousarray(a)) for a in arrays]
        d = dict(zip(names, dev))
        tp2 = time.perf_counter()
        if nd and len(dst):
            src_t, dst_t = dev[len(names) + 5], dev[len(names) + 6]
            if partial:
                d["ids"].index_copy_(0, dst_t, self.d_out.index_select(0, src_t))
            else:
                torch.index_select(self.d_out, 0, src_t, out=d["ids"][:nd])
        tp3 = time.perf_counter()
        meta = AttnMeta(
            positions=d["pos"], slot_mapping=d["slots"], logits_indices=d["lrows"], num_decode=nd,
            block_tables=d["bt"], seq_lens=d["seq_lens"],
            q_start_loc=d["qsl"] if self.is_gpu else torch.from_numpy(host["qsl"]),
            tile_info=d["tiles"], num_tiles=host["num_tiles"])
        if host.get("num_combine", 0):
            meta.pf_part_o, meta.pf_part_ml = self.pf_part_o, self.pf_part_ml
            meta.pf_combine, meta.pf_num_combine = d["combine"], host["num_combine"]
            meta.pf_num_partials = host["num_partials"]
        if nd:
            meta.dec_block_tables = d["d_bt"]
            meta.dec_seq_lens = d["d_sl"]
            meta.tmp_out, meta.tmp_ml = self.tmp_out, self.tmp_ml
            meta.dec_counters = self.dec_counters
        mh = self._mx_handles[self._mx_next]
        self._mx_next = (self._mx_next + 1) % len(self._mx_handles)
        nl = len(getattr(self.model, "layers", ()))
        if mh.mark is not None and nl and self.mixed_mark_frac > 0:
            self.model.mark_at = (min(nl - 1, int(self.mixed_mark_frac * nl)), mh.mark)
        try:
            h = self.model.forward(d["ids"], meta, self.kv)
        finally:
            self.model.mark_at = None
        logits = self.model.compute_logits(h)
        if self.logits_tap is not None:
            self._tap(logits.float().cpu())   # taps are host tensors (tests)
        n = logits.shape[0]
        samp = dev[len(names):len(names) + 5]
        if mh.host.shape[0] < n:
            mh.host = torch.zeros(2 * n, dtype=torch.int32, pin_memory=self.is_gpu)
        mh.n = n
        if defer_sample:
            # the sampling arrays are views into the shared upload buffer, which the
            # masks' upload (sample_launch) overwrites first: keep copies
            mh.pending, mh.logits, mh.samp = True, logits, [t.clone() for t in samp]
            self.stats["deferred_mixed"] = self.stats.get("deferred_mixed", 0) + 1
        else:
            dmask = dev[len(names) + 7] if masks is not None else None
            self._mixed_sample(mh, logits, samp, dmask)
        if self._gaps is not None:
            self._gap_mark(False)
        tp4 = time.perf_counter()
        ml = self.stats.setdefault("mixed_launch_ms", {"host": 0.0, "upload": 0.0, "gather": 0.0,
                                                        "forward": 0.0, "n": 0})
        ml["host"] += 1e3 * (tp1 - tp0)
        ml["upload"] += 1e3 * (tp2 - tp1)
        ml["gather"] += 1e3 * (tp3 - tp2)
        ml["forward"] += 1e3 * (tp4 - tp3)
        ml["n"] += 1
        return mh

    def _mixed_sample(self, mh: "MixedHandle", logits, samp, dmask):
        temp, topp, topk, seeds, steps = samp
        ops.sample(logits, temp, topp, topk, seeds, steps, out=self.d_out[:mh.n], mask=dmask)
        mh.host[:mh.n].copy_(self.d_out[:mh.n], non_blocking=self.is_gpu)
        if mh.event is not None:
            mh.event.record()
        mh.pending, mh.logits, mh.samp = False, None, None

    def mixed_collect(self, h: "MixedHandle") -> List[int]:
        if h.event is not None:
            self._wait(h.event)
        return h.host[:h.n].tolist()

    def _decode_fill(self, seqs, nb: int, st: "_Staging") -> int:
        """Writes a decode step's inputs into a pinned staging set."""
        n = len(seqs)
        mb = self.max_decode_batch
        hs = st.hs
        ids = hs[0:mb]
        pos = hs[mb:2 * mb]
        slots = hs[2 * mb:3 * mb]
        sl = hs[3 * mb:4 * mb]
        bt = st.hbt
        bs = self.bs
        maxblk = 1
        for i, s in enumerate(seqs):
            p = s.n_tokens - 1 + s.inflight   # steps queued ahead of this one
            ids[i] = s.last_token  # replaced on the device when queued ahead
            pos[i] = p
            slots[i] = s.block_ids[p // bs] * bs + p % bs
            sl[i] = p + 1
            nbk = len(s.block_ids)
            bt[i, :nbk] = s.block_ids
            maxblk = max(maxblk, nbk)
        temp, topp, topk, seeds, steps = self._sampling_arrays(seqs)
        hs[4 * mb:4 * mb + n] = topk
        hs[5 * mb:5 * mb + n] = steps
        st.hf[:n] = temp
        st.hf[mb:mb + n] = topp
        st.hseed[:n] = seeds
        if nb > n:  # padding rows: no KV write, empty context (no attention work), greedy
            ids[n:nb] = 0
            pos[n:nb] = 0
            slots[n:nb] = -1
            sl[n:nb] = 0
            bt[n:nb, 0] = 0
            hs[4 * mb + n:4 * mb + nb] = 0
            hs[5 * mb + n:5 * mb + nb] = 0
            st.hf[n:nb] = 0.0
            st.hf[mb + n:mb + nb] = 1.0
        return maxblk

    def _gap_mark(self, start: bool, kind: str = "d"):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if start:
            if self._gaps and self._gaps[-1][1] is None:   # an unclosed step: drop it
                self._gaps.pop()
            self._gaps.append([ev, None, kind])
        elif self._gaps and self._gaps[-1][1] is None:
            self._gaps[-1][1] = ev

    def gap_summary(self) -> Dict[str, float]:
        """FT_GPU_GAPS: idle GPU time between consecutive steps, by transition
        (d = graph-replayed decode, m = synchronous mixed step, a = mixed step
        queued ahead), and each kind's mean span from its first to its last
        launch (a mixed step's span includes any wait for the host's launches)."""
        if not self._gaps:
            return {}
        torch.cuda.synchronize(self.device)
        out: Dict[str, float] = {}
        busy: Dict[str, List[float]] = {}
        trans: Dict[str, List[float]] = {}
        prev = None
        for e0, e1, kind in self._gaps:
            if e1 is None:
                prev = None
                continue
            busy.setdefault(kind, []).append(e0.elapsed_time(e1))
            if prev is not None:
                trans.setdefault(prev[1] + kind, []).append(max(0.0, prev[0].elapsed_time(e0)))
            prev = (e1, kind)
        if not trans:
            return {}
        gaps = [g for v in trans.values() for g in v]
        out.update(idle_ms_total=round(sum(gaps), 1), idle_ms_per_step=round(sum(gaps) / len(gaps), 3),
                   idle_ms_max=round(max(gaps), 2), steps=sum(len(v) for v in busy.values()))
        for k, v in sorted(busy.items()):
            out[f"span_ms_{k}"] = round(sum(v) / len(v), 3)
            out[f"n_{k}"] = len(v)
        if "d" in busy:
            out["gpu_ms_per_step"] = out["span_ms_d"]
        for k, v in sorted(trans.items()):
            out[f"idle_ms_{k}"] = round(sum(v), 1)
            out[f"n_{k}"] = len(v)
        return out

    def _decode_enqueue(self, st: "_Staging", nb: int, n: int, from_device: bool = False,
                        gather: Optional[np.ndarray] = None, fwd_only: bool = False):
        nw = 10 * self.max_decode_batch + nb * self.max_blocks_per_seq
        if self._gaps is not None:   # g: a split step, closed by its sampler (sample_launch)
            self._gap_mark(True, "g" if fwd_only else "d")
        self.d_in[:nw].copy_(st.h_in[:nw], non_blocking=True)
        if from_device:  # the previous step's sampled ids feed this step
            if gather is None:
                self.d_input_ids[:nb].copy_(self.d_out[:nb])
            elif (gather >= 0).all():   # rows of the previous step, survivors only
                st.h_map[:nb].numpy()[:] = gather
                self.d_map[:nb].copy_(st.h_map[:nb], non_blocking=True)
                torch.index_select(self.d_out, 0, self.d_map[:nb], out=self.d_input_ids[:nb])
            else:   # gather < 0: a sequence with no queued step keeps its host id
                dst = np.nonzero(gather >= 0)[0]
                k = len(dst)
                if k:
                    hm = st.h_map.numpy()
                    hm[:k] = gather[dst]
                    hm[k:2 * k] = dst
                    self.d_map[:2 * k].copy_(st.h_map[:2 * k], non_blocking=True)
                    self.d_input_ids.index_copy_(0, self.d_map[k:2 * k],
                                                 self.d_out.index_select(0, self.d_map[:k]))
        if fwd_only:
            pair = self.graphs_split.get(nb)
            if pair is None:
                pair = self._capture_split(nb)
            pair[0].replay()
            self.stats["graph_replays"] += 1
            self.stats["deferred_samples"] = self.stats.get("deferred_samples", 0) + 1
            return
        g = self.graphs.get(nb)
        if g is None:
            g = self._capture(nb)
        g.replay()
        self.stats["graph_replays"] += 1
        st.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
        flag = self.comm.error_flag if self.checks_comm else None
        st.err_armed = flag is not None
        if flag is not None:  # the graph folded the ranks' error words into it
            st.h_err.copy_(flag, non_blocking=True)
        st.event.record()
        if self._gaps is not None:
            self._gap_mark(False)

    # ------------------------------------------------------------------ TP workers
    @torch.inference_mode()
    def run_remote(self, msg) -> bool:
        """Executes one message broadcast by TP rank 0 (same kernels, same
        collectives, same order).  Returns False on ``stop``."""
        kind, host, masks = msg
        if kind == "stop":
            return False
        if kind == "mixed":
            self._mixed_msgs += 1
            if self._stall_mixed and self._mixed_msgs == self._stall_at:
                self._fault_stall()
            self._mixed_run(host, masks)
        elif kind == "graph":
            self._graph_msgs += 1
            if not self._stall_mixed and self._graph_msgs == self._stall_at:
                self._fault_stall()
            nb, n = host["nb"], host["n"]
            self._set_masks(masks, n)
            st = self.stg[0]
            st.hs[:] = host["small"]
            bt = host["bt"]
            st.hbt[:nb, :bt.shape[1]] = bt
            st.hf[:] = host["f32"]
            st.hseed[:] = host["seeds"]
            self._decode_enqueue(st, nb, n, from_device=host.get("from_device", False),
                                 gather=host.get("rowmap"))
            self._wait(st.event)
        elif kind == "warmup":
            self.warmup(host)
        elif kind == "swap":
            self._swap(*host)
        elif kind == "comm_fault":
            self._drop_custom_collectives()
        else:
            raise ValueError(f"unknown TP message {kind!r}")
        return True

    def _fault_stall(self):
        log.warning("FT_FAULT_TP_STALL: rank %d stalls", self.comm.rank)
        t_end = time.time() + self._stall_s
        while time.time() < t_end and not (self.comm.custom is not None
                                           and self.comm.custom.peer_error(0)):
            time.sleep(0.01)

    def _decode_meta(self, nb: int) -> AttnMeta:
        assert nb <= self.max_decode_rows
        return AttnMeta(positions=self.d_positions[:nb], slot_mapping=self.d_slots[:nb],
                        logits_indices=self.d_logits_idx[:nb], num_decode=nb,
                        dec_block_tables=self.d_bt[:nb], dec_seq_lens=self.d_seq_lens[:nb],
                        tmp_out=self.tmp_out, tmp_ml=self.tmp_ml, dec_counters=self.dec_counters)

    def _graph_body(self, nb: int, keep: bool = False):
        meta = self._decode_meta(nb)
        h = self.model.forward(self.d_input_ids[:nb], meta, self.kv)
        logits = self.model.compute_logits(h)
        if keep:   # graph-pool memory: holds each replay's logits until the next one
            self._graph_logits[nb] = logits
        ops.sample(logits, self.d_temp[:nb], self.d_top_p[:nb], self.d_top_k[:nb],
                   self.d_seeds[:nb], self.d_steps[:nb], out=self.d_out[:nb],
                   mask=self.d_mask[:nb] if self.d_mask is not None else None)
        if self.checks_comm:
            self.comm.export_error()

    @torch.inference_mode()
    def _capture_split(self, nb: int):
        """The forward graph (-> logits, held in ``_fwd_logits``) and the sampler graph
        of bucket ``nb`` for pipelined guided decoding, captured like ``_capture``.
        Nothing replays between a step's two halves (its sampler is queued before
        the next forward), so the pool may share their temporaries with every other
        graph; the logits stay allocated."""
        self._assert_no_pending_split("split-graph capture")
        t0 = time.time()
        saved = (self.d_slots[:nb].clone(), self.d_seq_lens[:nb].clone())
        self.d_slots[:nb].fill_(-1)
        self.d_seq_lens[:nb].fill_(0)

        def fwd():
            h = self.model.forward(self.d_input_ids[:nb], self._decode_meta(nb), self.kv)
            return self.model.compute_logits(h)

        def samp(lg):
            ops.sample(lg, self.d_temp[:nb], self.d_top_p[:nb], self.d_top_k[:nb],
                       self.d_seeds[:nb], self.d_steps[:nb], out=self.d_out[:nb],
                       mask=self.d_mask[:nb])

        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            samp(fwd())  # warm-up (allocator, lazy init)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.graph_pool is None:
            self.graph_pool = torch.cuda.graph_pool_handle()
        gf = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gf, pool=self.graph_pool):
            lg = fwd()
        self._fwd_logits[nb] = lg
        gs = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gs, pool=self.graph_pool):
            samp(lg)
        self.d_slots[:nb].copy_(saved[0])
        self.d_seq_lens[:nb].copy_(saved[1])
        self.graphs_split[nb] = (gf, gs)
        self.stats["captures"] += 1
        log.info("captured split decode graphs batch=%d in %.2fs", nb, time.time() - t0)
        return gf, gs

    @torch.inference_mode()
    def _capture(self, nb: int):
        """Captures the decode graph of batch bucket ``nb``.  Always under
        inference mode, whichever path triggers it (pipelined launches run outside
        ``execute``): the CUDA generator's graph-safe RNG state is created by the
        first capture and must be of the same kind for every later one."""
        self._assert_no_pending_split("graph capture")
        t0 = time.time()
        # inputs must be valid for the warm-up/capture run: no KV writes, empty contexts
        saved = (self.d_slots[:nb].clone(), self.d_seq_lens[:nb].clone())
        self.d_slots[:nb].fill_(-1)
        self.d_seq_lens[:nb].fill_(0)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s), self._long_waits():
            self._graph_body(nb)  # warm-up (allocator, lazy init)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.graph_pool is None:
            self.graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.graph_pool):
            self._graph_body(nb, keep=True)
        self.d_slots[:nb].copy_(saved[0])
        self.d_seq_lens[:nb].copy_(saved[1])
        self.graphs[nb] = g
        self.stats["captures"] += 1
        log.info("captured decode graph batch=%d in %.2fs", nb, time.time() - t0)
        return g

    def _decode_eager(self, seqs, masks) -> List[int]:
        self.stats["eager_decode"] += 1
        from .scheduler import ScheduledBatch as _SB

        return self._mixed(_SB(list(seqs), [], [], []), masks)

    @staticmethod
    def _warm_split_graphs() -> bool:
        """Pre-capture the split (forward | sampler) graphs of pipelined guided decoding?
        Guided rows come from grammar-constrained tool calls or JSON-schema requests.
        ``ENGINE_WARM_SPLIT_GRAPHS`` decides when set; otherwise only a service with
        guided tool calls on (``AGENT_GUIDED_TOOL_CALLS``) pays for them at start-up, and
        any other deployment captures a bucket's pair on its first guided step."""
        env = os.environ.get("ENGINE_WARM_SPLIT_GRAPHS")
        if env is not None:
            return env.strip().lower() not in ("0", "false", "no", "off", "")
        return os.environ.get("AGENT_GUIDED_TOOL_CALLS", "false").strip().lower() == "true"

    def warmup(self, batch_sizes=None):
        """Pre-capture decode graphs (one per batch bucket, any context length) so
        serving never pays for a capture."""
        if not self.use_graphs:
            return
        if self.bcast is not None:
            self.bcast.send(("warmup", list(batch_sizes or self.graph_sizes), None))
        t0 = time.time()
        split = self.can_defer_sample() and self._warm_split_graphs()
        for b in batch_sizes or self.graph_sizes:
            b = self._bucket(b)
            if b is not None and b not in self.graphs:
                self._capture(b)
            if b is not None and split and b not in self.graphs_split:
                self._capture_split(b)
        log.info("decode graphs ready (%d + %d split) in %.1fs", len(self.graphs),
                 len(self.graphs_split), time.time() - t0)
