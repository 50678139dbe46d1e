"""In-process LLM serving engine (one per GPU, or per TP group on its leader).

Replaces the reference's out-of-tree inference hop (core -> Ollama /api/chat,
worker -> /api/generate).  Pieces:

* native continuous-batching scheduler + paged-KV block manager
  (csrc/runtime/scheduler.cpp) decides every step;
* the step's metadata is packed into ONE pinned buffer and moved with ONE
  host->device copy;
* pure-decode steps replay a captured hipGraph per batch bucket (the whole
  forward + sampling), mixed/prefill steps run eagerly;
* results leave the engine thread as one batched event list per step
  (``event_sink``), so the asyncio side wakes once per step, not per token.

Thread model: a single engine thread owns the GPU stream, the scheduler and
all device buffers.  ``submit`` / ``abort`` are thread-safe and only enqueue.
"""
from __future__ import annotations

import itertools
import logging
import math
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch

from .. import ops
from ..models.config import LlamaConfig
from ..models.llama import LlamaModel, StepInputs, TPContext
from ..utils.faults import faults

log = logging.getLogger("lmx.engine")

BLOCK_SIZE = 32
FINISH_REASONS = {1: "stop", 2: "length", 3: "abort"}


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    max_tokens: int = 256
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    logprobs: bool = False
    # repetition (HF / Ollama repeat_penalty) over the last penalty_last_n
    # context tokens; presence / frequency (OpenAI) over the generated tokens
    # inside that window (window <= 64 tokens, the penalty kernel's wave)
    repetition_penalty: float = 1.0
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    penalty_last_n: int = 64

    def penalized(self) -> bool:
        return self.penalty_last_n > 0 and (self.repetition_penalty != 1.0 or
                                            self.presence_penalty != 0.0 or
                                            self.frequency_penalty != 0.0)


@dataclass
class GenRequest:
    prompt_ids: list[int]
    params: SamplingParams
    id: int = 0
    priority: int = 0
    user: object = None             # opaque handle for the event sink
    arrival: float = 0.0
    first_token_at: float = 0.0
    num_generated: int = 0
    finished: bool = False


@dataclass
class TokenEvent:
    req: GenRequest
    token: int
    logprob: float
    finish: str | None  # None while running


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name, "")
    return int(v) if v.strip() else default


@dataclass
class EngineConfig:
    """One set of serving defaults for ``serve`` / ``worker`` and bench.py
    (environment-overridable, settings.py): a step takes up to
    max_batched_tokens tokens -- an idle engine takes a whole burst of
    prompts in few steps -- but a step that also carries at least
    mixed_min_decodes decode rows of streams that were running before the
    newest request with prompt tokens left arrived (>= mixed_later_steps
    scheduler steps earlier) takes at most mixed_prefill_tokens prompt
    tokens.  One burst's rows never cap each other, so a wave of requests is
    prefilled at the full budget, while in steady serving a new request's
    prefill is chunked so it cannot stall the running streams for a
    full-budget step (closed loop at 256 streams: per-token gap p99 251 -> 35
    ms, TTFT p50 756 -> 454 ms; profiles/r6_serving.md).  36864-token steps
    take a 256 x 512-token wave in 4 steps instead of 6: equal throughput and
    TTFT to 24576, fewer stalled decode gaps (token-gap p99 168 -> 13 ms;
    profiles/r6_serving.md "Prefill budget")."""
    model: str = "llama-3-8b"
    max_num_seqs: int = 256
    max_batched_tokens: int = field(
        default_factory=lambda: _env_int("LMX_MAX_BATCHED_TOKENS", 36864))
    mixed_prefill_tokens: int = field(
        default_factory=lambda: _env_int("LMX_MIXED_PREFILL_TOKENS", 2048))
    mixed_min_decodes: int = field(
        default_factory=lambda: _env_int("LMX_MIXED_MIN_DECODES", 32))
    # the cap counts only decode rows whose request came >= this many
    # scheduler steps before the newest request with prompt tokens left
    # (0: every decode row): one burst's rows never cap each other
    mixed_later_steps: int = field(
        default_factory=lambda: _env_int("LMX_MIXED_LATER_STEPS", 8))
    max_model_len: int = 8192
    kv_fraction: float = 0.6        # of free HBM after weights
    kv_cache_gb: float | None = None
    prefix_cache: bool = field(
        default_factory=lambda: _env_int("LMX_PREFIX_CACHE", 1) != 0)
    use_graphs: bool = True
    part_tokens: int = 512
    seed: int = 0


class _Packer:
    """Packs numpy arrays into one pinned host buffer and one device buffer
    (16-byte aligned regions) so a step's metadata moves in one copy."""

    def __init__(self, nbytes: int, device):
        self.nbytes = nbytes
        self.device = device
        pin = device.type == "cuda"
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=pin)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.hnp = self.host.numpy()

    def pack(self, items: list[tuple[str, np.ndarray]]) -> dict[str, torch.Tensor]:
        off, spans = 0, []
        for name, a in items:
            a = np.ascontiguousarray(a)
            n = a.nbytes
            if off + n > self.nbytes:
                raise RuntimeError("step metadata exceeds packer capacity")
            self.hnp[off:off + n] = a.view(np.uint8).reshape(-1)
            spans.append((name, off, a.dtype, a.shape))
            off += (n + 15) & ~15
        if off:
            self.dev[:off].copy_(self.host[:off], non_blocking=True)
        out = {}
        for name, o, dt, shape in spans:
            n = int(np.prod(shape)) * np.dtype(dt).itemsize
            out[name] = self.dev[o:o + n].view(_TORCH_DT[np.dtype(dt)]).view(shape)
        return out


PEN_WINDOW = 64   # kPenWindow of csrc/runtime/scheduler.h (one wave per row in the kernel)

_PLAN_KEY = {"ids": "input_ids", "pos": "positions", "ctx": "context_lens"}

_TORCH_DT = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
             np.dtype(np.float32): torch.float32}


class _FixedMeta:
    """Fixed-layout metadata block (pinned host mirrors + device buffer): the
    static inputs of the captured decode graphs are device views into it, so
    a replay needs exactly one host->device copy.

    Two host mirrors, alternated per step (``next()``): under lookahead
    stepping step n's non-blocking upload is queued behind step n-1's
    kernels, and the host writes step n+1's metadata after waiting only for
    step n-1's tokens, i.e. possibly before step n's copy has read the
    mirror.  Step n+1 writes the other mirror; ``next()`` also waits for the
    event recorded after that mirror's last copy (already complete in the
    steady state: it precedes the output event the host waited for)."""

    def __init__(self, fields: list[tuple[str, type, tuple]], device):
        off, spans = 0, []
        for name, dt, shape in fields:
            n = int(np.prod(shape)) * np.dtype(dt).itemsize
            spans.append((name, off, dt, shape, n))
            off += (n + 15) & ~15
        self.nbytes = off
        self._cuda = device.type == "cuda"
        self.host_ts = [torch.empty(off, dtype=torch.uint8, pin_memory=self._cuda)
                        for _ in range(2)]
        self.dev_t = torch.empty(off, dtype=torch.uint8, device=device)
        self._hs = []
        for host_t in self.host_ts:
            hnp = host_t.numpy()
            self._hs.append({name: hnp[o:o + n].view(dt).reshape(shape)
                             for name, o, dt, shape, n in spans})
        self.d = {name: self.dev_t[o:o + n].view(_TORCH_DT[np.dtype(dt)]).view(shape)
                  for name, o, dt, shape, n in spans}
        self._evs = [None, None]
        self._k = 0
        self.h = self._hs[0]

    def mirror_all(self):
        """Copy the current host mirror into the other one (initial fill)."""
        self.host_ts[self._k ^ 1].numpy()[:] = self.host_ts[self._k].numpy()

    def next(self):
        """Switch to the other host mirror before writing a step's fields."""
        self._k ^= 1
        ev = self._evs[self._k]
        if ev is not None:
            ev.synchronize()
        self.h = self._hs[self._k]

    def upload(self):
        self.dev_t.copy_(self.host_ts[self._k], non_blocking=True)
        if self._cuda:
            if self._evs[self._k] is None:
                self._evs[self._k] = torch.cuda.Event()
            self._evs[self._k].record()


_TUNING_LOADED = False


def _load_gemm_tuning() -> None:
    """Load the cold-cache hipBLASLt solution table for the served shapes
    (bench/tune_gemms.py) into PyTorch TunableOp, tuning disabled at serve
    time.  LMX_TUNABLEOP=0 turns it off; shapes absent from the table keep
    the library heuristic; a table from another ROCm / hipBLASLt build is
    rejected by TunableOp's validators."""
    global _TUNING_LOADED
    if _TUNING_LOADED or os.environ.get("LMX_TUNABLEOP", "1") != "1":
        return
    _TUNING_LOADED = True
    path = os.environ.get("LMX_TUNABLEOP_FILE") or os.path.join(
        os.path.dirname(os.path.dirname(__file__)), "config", "tunableop_gfx950.csv")
    if not os.path.exists(path):
        return
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    ok = tun.read_file(path)
    log.info("GEMM tuning table %s: %s", path, "loaded" if ok else "rejected")
    if not ok:
        tun.enable(False)


class LLMEngine:
    def __init__(self, ecfg: EngineConfig, device: str | torch.device = "cuda",
                 model_cfg: LlamaConfig | None = None, tp: TPContext | None = None,
                 event_sink: Callable[[list[TokenEvent]], None] | None = None,
                 weights: dict | None = None, plan_channel=None):
        """``tp`` + ``plan_channel``: member of a tensor-parallel group.  The
        leader (rank 0) schedules, publishes every step's plan and samples;
        followers run ``run_follower()`` and execute the same forward on
        their shard (parallel/tp_worker.py)."""
        from ..models import config as mc
        from ..native import runtime
        _runtime = runtime()
        self.ecfg = ecfg
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.cfg = model_cfg or mc.resolve(ecfg.model)
        self.max_model_len = min(ecfg.max_model_len, self.cfg.max_position)
        if self.device.type == "cuda":
            _load_gemm_tuning()
        self.model = LlamaModel(self.cfg, self.device, tp=tp, seed=ecfg.seed, weights=weights)
        self.tp = self.model.tp
        self.is_leader = self.tp.rank == 0
        self.chan = plan_channel
        # live TP all-reduce samples every LMX_TP_PROBE_STEPS engine steps (0 = off)
        self._comm_every = int(os.environ.get("LMX_TP_PROBE_STEPS", "2000"))
        self.tp_comm_live: dict = {}
        self._upload_ev = None
        self.Hq, self.Hkv, self.D = self.model.Hq, self.model.Hkv, self.model.D
        self.q_per_tile = ops.prefill_q_per_tile(self.Hq, self.Hkv, self.D)
        self._alloc_kv()
        self.sched = _runtime.Scheduler(self.num_blocks, BLOCK_SIZE, ecfg.max_num_seqs,
                                        ecfg.max_batched_tokens, self.max_model_len,
                                        ecfg.prefix_cache)
        if ecfg.mixed_prefill_tokens and ecfg.mixed_prefill_tokens < ecfg.max_batched_tokens:
            self.sched.set_mixed_prefill_cap(ecfg.mixed_prefill_tokens, ecfg.mixed_min_decodes,
                                             ecfg.mixed_later_steps)
        self.max_blocks = math.ceil(self.max_model_len / BLOCK_SIZE)
        self.max_parts = max(1, min(16, math.ceil(self.max_model_len / ecfg.part_tokens)))
        self.decode_ws = ops.DecodeWorkspace(ecfg.max_num_seqs, self.Hq, self.D, self.max_parts,
                                             self.device)
        T = ecfg.max_batched_tokens + ecfg.max_num_seqs
        cap = 4 * (4 * T + ecfg.max_num_seqs * (self.max_blocks + 8) + 2 * T) + 16 * 64 + \
            8 * ecfg.max_num_seqs * 4 + 4 * ecfg.max_num_seqs * (PEN_WINDOW + 4) + \
            4 * ecfg.max_num_seqs + 16          # decode dispatch order
        self.packer = _Packer(cap, self.device)
        self.event_sink = event_sink
        self._intake: queue.SimpleQueue = queue.SimpleQueue()
        self._aborts: queue.SimpleQueue = queue.SimpleQueue()
        self._reqs: dict[int, GenRequest] = {}
        self._ids = itertools.count(1)
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.graphs: dict[int, dict] = {}
        self.stats = {"steps": 0, "decode_steps": 0, "graph_steps": 0, "prefill_tokens": 0,
                      "generated_tokens": 0, "step_time_s": 0.0, "finished": 0,
                      "t_schedule": 0.0, "t_launch": 0.0, "t_events": 0.0, "t_wait": 0.0,
                      "t_update": 0.0, "t_gpu": 0.0, "decode_step_s": 0.0,
                      "g_schedule": 0.0, "g_launch": 0.0, "g_update": 0.0, "g_upload": 0.0,
                      "g_replay": 0.0}
        self._pending = None
        self._fetch_cpu = [None, None]
        # (arrival, first token) wall times of recent requests: engine-side TTFT
        import collections
        self.ttft_samples: collections.deque = collections.deque(maxlen=65536)
        self._step_started = 0.0
        self._last_error = None
        # LMX_TORCH_PROFILE=/dir[:steps]: torch.profiler timeline of N steps
        self._prof = None
        self._prof_spec = os.environ.get("LMX_TORCH_PROFILE", "")
        if self.device.type == "cuda":
            # two slots: under lookahead stepping step n+1's copy is queued
            # while step n's is still being read
            self._hout = torch.zeros((2, 2, ecfg.max_num_seqs), dtype=torch.int32,
                                     pin_memory=True)
            self._hout_np = self._hout.numpy()
            self._out_evs = [torch.cuda.Event(), torch.cuda.Event()]
        self._slot = 0
        # lookahead stepping (step n+1 scheduled and launched before step n's
        # tokens are read back): on by default for GPU engines, TP groups
        # included (every rank then samples the all-gathered logits itself:
        # sample_all below).  The TP form runs in captured decode graphs with
        # the peer-memory collectives inside and gives the eager path's greedy
        # tokens (tests/test_00_tp_gpu.py::test_tp_group_captured_decode_graphs);
        # one-GPU TP8 rehearsal: decode step 6.44 -> 6.16 ms
        # (profiles/r5_tp_rehearsal.md).  LMX_LOOKAHEAD=0 turns it off.
        if os.environ.get("LMX_STEP_TRACE", "0") == "1":
            import collections
            self.step_trace = collections.deque(maxlen=4096)   # bounded in long runs
        self._idle = True
        self._admit_quiet_s = float(os.environ.get("LMX_ADMIT_QUIET_MS", "2")) / 1e3
        self._admit_max_s = float(os.environ.get("LMX_ADMIT_MAX_MS", "25")) / 1e3
        la_env = os.environ.get("LMX_LOOKAHEAD", "")
        # TP groups: vocab-sharded sampling (ops.sample_race) by default --
        # every rank samples its own logits shard and a B x 32-B record
        # exchange per phase picks the same token everywhere, so no rank
        # gathers logits and every rank holds each step's tokens on its device
        # (LMX_TP_SAMPLER=gather: the logits gathered to the sampling ranks)
        self.race_tp = self.tp.size > 1 and os.environ.get("LMX_TP_SAMPLER", "race") != "gather"
        self.tp.shard_logits = self.race_tp
        # LMX_SAMPLER=race: the race form at TP = 1 too (one shard: the same
        # tokens a TP group draws for the same seeds; the default K6 kernel is
        # 2.7x faster over full rows, profiles/r6_sampling.md)
        self.race = self.race_tp or os.environ.get("LMX_SAMPLER", "") == "race"
        rccl_tp = (self.tp.size > 1 and self.tp.group is not None
                   and torch.distributed.get_backend(self.tp.group) == "nccl")
        # lookahead: on by default for GPU engines and one-GPU (gloo) TP
        # rehearsals; an RCCL TP group opts in with LMX_LOOKAHEAD=1 until a
        # multi-GPU run has covered it
        self.lookahead = la_env == "1" or (la_env != "0" and self.device.type == "cuda"
                                           and not rccl_tp)
        # every rank samples: the race sampler is a collective; the gather
        # form all-gathers the logits under lookahead (each rank then holds
        # step n's tokens for step n+1's ids_from_prev gather)
        self.sample_all = self.tp.size > 1 and (self.race_tp or self.lookahead)
        self.tp.logits_to_all = self.sample_all and not self.race_tp
        self._la = None                    # the launched step not yet read back
        self._la_end = 0.0                 # when the last launched step was read back
        self._penalized: set[int] = set()  # active requests with penalty windows
        # a gloo TP group (one-GPU rehearsals) captures its decode graphs when
        # every decode collective runs on the peer-memory kernels (all-reduces
        # and the logits gather within a slot); host-staged gloo collectives
        # synchronise inside the step and cannot be captured
        host_tp = self.tp.size > 1 and self.tp.group is not None and \
            torch.distributed.get_backend(self.tp.group) == "gloo" and \
            not self.tp.device_collectives_cover(max(self._graph_buckets(), default=1),
                                                 self.cfg.hidden_size,
                                                 16 if self.race_tp else self.model.vocab_shard)
        if ecfg.use_graphs and self.device.type == "cuda" and not ops.debug_sync() and not host_tp:
            self._capture_graphs()
        self._bucket_list = sorted(self.graphs)

    # ------------------------------------------------------------ memory ----
    def _alloc_kv(self):
        cfg = self.cfg
        per_block = cfg.num_layers * 2 * self.Hkv * BLOCK_SIZE * self.D * 2
        if self.ecfg.kv_cache_gb is not None:
            kv_bytes = int(self.ecfg.kv_cache_gb * (1 << 30))
        elif self.device.type == "cuda":
            free, _ = torch.cuda.mem_get_info(self.device)
            kv_bytes = int(free * self.ecfg.kv_fraction)
        else:
            kv_bytes = 64 * per_block
        self.num_blocks = max(16, kv_bytes // per_block)
        if self.tp.size > 1:
            # the leader's scheduler hands out page ids for every rank
            gloo = torch.distributed.get_backend(self.tp.group) == "gloo"
            t = torch.tensor([self.num_blocks], dtype=torch.int64,
                             device="cpu" if gloo else self.device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN,
                                         group=self.tp.group)
            self.num_blocks = int(t.item())
        # zero-filled: masked keys multiply P = 0 with V, which must be finite
        self.kv = torch.zeros((cfg.num_layers, 2, self.num_blocks, self.Hkv, BLOCK_SIZE * self.D),
                              dtype=torch.bfloat16, device=self.device)
        self.k_caches = [self.kv[l, 0].view(self.num_blocks, self.Hkv, BLOCK_SIZE, self.D)
                         for l in range(cfg.num_layers)]
        self.v_caches = [self.kv[l, 1].view(self.num_blocks, self.Hkv, BLOCK_SIZE // 4, self.D, 4)
                         for l in range(cfg.num_layers)]
        log.info("KV cache: %d blocks x %d tokens (%.1f GB)", self.num_blocks, BLOCK_SIZE,
                 self.kv.numel() * 2 / 1e9)

    # ----------------------------------------------------------- sampling ---
    def _sample(self, logits, temp, topk, topp, seeds, offs, out_tok=None, out_lp=None):
        """Sample the step's rows: the K6 kernel over full rows, or under TP
        the vocab-sharded race sampler over this rank's shard (collective:
        every rank of the group calls it with the same rows)."""
        if not self.race:
            return ops.sample(logits, temp, topk, topp, seeds, offs, out_tok, out_lp)
        tp = self.tp
        if tp.size == 1:
            return ops.sample_race(logits, temp, topk, topp, seeds, offs, out_tok=out_tok,
                                   out_lp=out_lp)
        return ops.sample_race(logits, temp, topk, topp, seeds, offs,
                               exchange=tp.all_gather_records,
                               v0=tp.rank * self.model.vocab_shard, vocab=self.cfg.vocab_size,
                               world=tp.size, out_tok=out_tok, out_lp=out_lp)

    def _penalize(self, logits, win, ngen, pen):
        v0 = self.tp.rank * self.model.vocab_shard if self.race_tp else 0
        return ops.apply_penalties(logits, win, ngen, pen, v0=v0)

    # ------------------------------------------------------------- graphs ---
    def _graph_buckets(self) -> list[int]:
        base = [1, 2, 4, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256,
                320, 384, 448, 512]
        return [b for b in base if b <= self.ecfg.max_num_seqs]

    def _graph_parts(self, B: int) -> int:
        """Split-K partitions of the decode attention for B rows: one as soon
        as the batch has a workgroup per CU (B x Hkv >= 256); a split adds
        the partial write, the reduce launch and per-workgroup start-up and
        measured 20-27 % slower at 32-128 rows, context ~660
        (profiles/r2_decode_attention.md).  Smaller batches split to fill the
        chip; the kernel grows the partition length when a context needs
        more."""
        return max(1, min(self.max_parts, -(-256 // max(1, B * self.Hkv))))

    def _decode_ws(self, B: int):
        """The decode workspace seen by a B-row step (max_parts = policy)."""
        ws = ops.DecodeWorkspace.__new__(ops.DecodeWorkspace)
        ws.max_parts, ws.part_o, ws.part_ml = (self._graph_parts(B), self.decode_ws.part_o,
                                               self.decode_ws.part_ml)
        return ws

    def _capture_graphs(self):
        t0 = time.time()
        Bmax = max(self._graph_buckets())
        dev = self.device
        meta = _FixedMeta([
            ("ids", np.int32, (Bmax,)), ("pos", np.int32, (Bmax,)), ("slots", np.int32, (Bmax,)),
            ("ctx", np.int32, (Bmax,)), ("bt", np.int32, (Bmax, self.max_blocks)),
            ("temp", np.float32, (Bmax,)), ("topk", np.int32, (Bmax,)),
            ("topp", np.float32, (Bmax,)), ("seeds", np.int64, (Bmax,)),
            ("offs", np.int32, (Bmax,)), ("order", np.int32, (Bmax,)),
            ("src", np.int32, (Bmax,))], dev)
        # penalty inputs: uploaded only on steps with penalised rows, read by
        # the lazily captured penalty variants of the decode graphs
        pmeta = _FixedMeta([("win", np.int32, (Bmax, PEN_WINDOW)), ("ngen", np.int32, (Bmax,)),
                            ("pen", np.float32, (Bmax, 3))], dev)
        pmeta.h["win"][:] = -1; pmeta.h["ngen"][:] = 0; pmeta.h["pen"][:] = 0
        pmeta.mirror_all()
        pmeta.upload()
        self._pmeta = pmeta
        h = meta.h
        h["ids"][:] = 0; h["pos"][:] = 0; h["slots"][:] = -1; h["ctx"][:] = 1; h["bt"][:] = 0
        h["temp"][:] = 0; h["topk"][:] = 0; h["topp"][:] = 1; h["seeds"][:] = 0; h["offs"][:] = 0
        h["order"][:] = np.arange(Bmax, dtype=np.int32)
        h["src"][:] = -1
        meta.mirror_all()
        meta.upload()
        self._gmeta = meta
        g = dict(meta.d)
        g.update({
            "cu": torch.arange(Bmax + 1, dtype=torch.int32, device=dev),
            "tiles": torch.zeros(2, dtype=torch.int32, device=dev),
            "rows": torch.arange(Bmax, dtype=torch.int64, device=dev),
            # every sample of a step (an eager step may sample more rows than
            # the largest bucket): the next graph step's ids_from_prev source
            "tok": torch.zeros(max(Bmax, self.ecfg.max_num_seqs), dtype=torch.int32,
                               device=dev),
            "lp": torch.zeros(Bmax, dtype=torch.float32, device=dev),
        })
        self._gbuf = g
        self._gpool = None
        self._gstream = torch.cuda.Stream(device=dev)
        self.pen_graphs: dict[int, dict] = {}
        for B in sorted(self._graph_buckets(), reverse=True):
            self.graphs[B] = self._capture_bucket(B)
        torch.cuda.synchronize(dev)
        log.info("captured %d decode graphs in %.1fs", len(self.graphs), time.time() - t0)

    def _capture_bucket(self, B: int) -> dict:
        """Capture the decode step of bucket B (forward + sampling)."""
        g, dev, stream = self._gbuf, self.device, self._gstream
        inp = StepInputs(g["ids"][:B], g["pos"][:B], g["slots"][:B], B, g["bt"][:B],
                         g["ctx"][:B], g["cu"][:B + 1], g["tiles"], g["rows"][:B], B, B,
                         decode_order=g["order"][:B])
        ws = self._decode_ws(B)
        out = {}

        def run():
            # lookahead rows: input tokens still on the device (previous step's samples)
            ops.ids_from_prev(g["ids"][:B], g["src"][:B], g["tok"])
            logits = self.model.forward(inp, self.k_caches, self.v_caches, ws,
                                        self.ecfg.part_tokens)
            if self.is_leader or self.sample_all:
                self._sample(logits, g["temp"][:B], g["topk"][:B], g["topp"][:B],
                             g["seeds"][:B], g["offs"][:B], g["tok"][:B], g["lp"][:B])
            out["logits"] = logits

        if self.tp.size > 1:
            # every rank enters a bucket's warm-up together: its collectives
            # (peer kernels with bounded waits, or RCCL) pair up across ranks
            from ..parallel.peer_allreduce import _cpu_group
            torch.distributed.barrier(group=self.tp.cpu_group or _cpu_group(self.tp.group))
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            run()  # warm-up (allocator, kernels, library heuristics)
            run()
        torch.cuda.current_stream(dev).wait_stream(stream)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._gpool, stream=stream):
            run()
        self._gpool = graph.pool()
        return {"graph": graph, "parts": ws.max_parts, "logits": out["logits"]}

    def _capture_penalty(self, B: int) -> dict:
        """Penalty variant of bucket B, captured lazily the first time a step
        of that bucket carries a penalised row: the penalty kernel and a
        second sampling pass over the logits the bucket's decode graph left in
        its pool (replayed right after it).  No forward pass runs in this
        capture; under vocab-sharded TP sampling its sampler exchanges records
        with the other ranks, which capture it at the same step (every rank
        replays the same plans) -- nothing runs during a capture, so the
        ranks need not meet there."""
        g, dev, stream = self._gbuf, self.device, self._gstream
        pd = self._pmeta.d
        logits = self.graphs[B]["logits"]

        def run():
            self._penalize(logits, pd["win"][:B], pd["ngen"][:B], pd["pen"][:B])
            self._sample(logits, g["temp"][:B], g["topk"][:B], g["topp"][:B],
                         g["seeds"][:B], g["offs"][:B], g["tok"][:B], g["lp"][:B])

        stream.wait_stream(torch.cuda.current_stream(dev))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._gpool, stream=stream):
            run()
        self._gpool = graph.pool()
        torch.cuda.current_stream(dev).wait_stream(stream)
        return {"graph": graph}

    # --------------------------------------------------------- public API ---
    step_trace = None   # a bounded deque of eager steps with LMX_STEP_TRACE=1 (see _step_la)

    def submit(self, req: GenRequest) -> GenRequest:
        if not req.id:
            req.id = next(self._ids)
        req.arrival = req.arrival or time.time()
        self._intake.put(req)
        self._wake.set()
        return req

    def abort(self, req_id: int) -> None:
        self._aborts.put(req_id)
        self._wake.set()

    def start(self):
        if self._thread is None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._loop, name="lmx-engine", daemon=True)
            self._thread.start()

    def stop(self):
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None

    def release_followers(self):
        """Leader: tell the TP followers to leave ``run_follower``."""
        if self.chan is not None and self.is_leader:
            self.chan.publish({"cmd": "stop"})

    def run_follower(self) -> int:
        """TP follower loop: execute the leader's plans until told to stop.
        Returns the number of steps executed."""
        from ..parallel.plan_channel import decode_plan
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        n = 0
        while True:
            msg = self.chan.receive()
            if msg.get("cmd") != "step":
                return n
            plan, bucket = decode_plan(msg)
            if self._upload_ev is not None:
                # the pinned staging buffers are reused: wait for the previous
                # step's H2D copies only (not for its kernels)
                self._upload_ev.synchronize()
            if bucket is not None:
                self._run_graph(plan, bucket)
            else:
                tok, _ = self._run_eager(plan)
                N = len(plan["sample_rows"])
                if self.sample_all and self.graphs and N:
                    # the next (graph) step gathers its inputs from here
                    self._gbuf["tok"][:N].copy_(tok[:N], non_blocking=True)
            if msg.get("probe"):
                self._comm_probe()
            n += 1

    def _mark_upload(self):
        """Event after this step's metadata H2D copies (TP followers reuse the
        pinned staging buffers as soon as it has completed)."""
        if self.device.type == "cuda" and self.chan is not None and not self.is_leader:
            if self._upload_ev is None:
                self._upload_ev = torch.cuda.Event()
            self._upload_ev.record()

    def _comm_probe(self):
        """Live all-reduce sample of the TP group (collective: the leader
        flags it in the step's plan, every rank runs it after the step): one
        decode-sized message (batch x hidden bf16) per path, exported as
        rccl_allreduce_seconds{group=path} next to the start-up probe."""
        from ..parallel.tp_worker import probe_allreduce
        n = max(1, self.ecfg.max_num_seqs) * self.cfg.hidden_size * 2
        res = probe_allreduce(self.tp, self.device, sizes=(n,), iters=3)
        seq = int(self.tp_comm_live.get("seq", 0)) + 1
        self.tp_comm_live = {"seq": seq, "bytes": n,
                             "us": {p: next(iter(v.values())) for p, v in res.items() if v}}

    @property
    def num_active(self) -> int:
        return len(self._reqs)

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        if self._prof_spec:
            d, _, n = self._prof_spec.partition(":")
            self.start_profile(d, int(n or 20))
        while not self._stop.is_set():
            try:
                did = self.step()
            except Exception as e:  # keep serving: fail the in-flight requests
                log.exception("engine step failed")
                if "hip" in str(e).lower():
                    self._last_error = str(e)[:200]
                self._fail_all("engine_error")
                did = False
            if not did:
                self._wake.wait(timeout=0.05)
                self._wake.clear()

    def _fail_all(self, why: str):
        self._pending = None
        if self.lookahead:       # whatever step was in flight or half read back
            self._la = None
            self.sched.discard_lookahead()
        self._penalized.clear()
        evs = []
        for rid, req in list(self._reqs.items()):
            self.sched.abort(rid)
            req.finished = True
            evs.append(TokenEvent(req, -1, 0.0, "error"))
        self._reqs.clear()
        if evs and self.event_sink:
            self.event_sink(evs)

    def _drain(self):
        evs = []
        while True:
            try:
                rid = self._aborts.get_nowait()
            except queue.Empty:
                break
            req = self._reqs.pop(rid, None)
            if req is not None:
                self._penalized.discard(rid)
                self.sched.abort(rid)
                req.finished = True
                evs.append(TokenEvent(req, -1, 0.0, "abort"))
        while True:
            try:
                req = self._intake.get_nowait()
            except queue.Empty:
                break
            p = req.params
            stop_ids = list(p.stop_token_ids) + list(getattr(self.cfg, "eos_token_ids", ()))
            seed = p.seed if p.seed is not None else (req.id * 2654435761) & 0x7FFFFFFF
            try:
                self.sched.add(req.id, list(req.prompt_ids), int(p.max_tokens), stop_ids,
                               bool(p.ignore_eos), int(req.priority), float(p.temperature),
                               int(p.top_k), float(p.top_p), int(seed))
                if p.penalized():
                    self.sched.set_penalties(req.id, float(p.repetition_penalty),
                                             float(p.presence_penalty),
                                             float(p.frequency_penalty), int(p.penalty_last_n))
                    self._penalized.add(req.id)
                self._reqs[req.id] = req
            except Exception as e:
                req.finished = True
                evs.append(TokenEvent(req, -1, 0.0, f"error:{e}"))
        if evs and self.event_sink:
            self.event_sink(evs)

    # -------------------------------------------------------------- step ----
    def healthy(self, timeout_s: float | None = None) -> tuple[bool, str]:
        """Watchdog view for the worker agent: a step in flight for longer
        than LMX_STEP_TIMEOUT (default 120 s) or an engine error means the
        GPU is hung or broken."""
        limit = timeout_s if timeout_s is not None else float(
            os.environ.get("LMX_STEP_TIMEOUT", "120"))
        if self._last_error is not None:
            return False, f"engine error: {self._last_error}"
        t = self._step_started
        if t and time.monotonic() - t > limit:
            return False, f"engine step running for {time.monotonic() - t:.0f}s"
        return True, ""

    def step(self) -> bool:
        """One engine step, software-pipelined against the GPU:

            schedule(n) -> upload + launch(n) -> emit events of step n-1
            -> wait for step n's tokens -> scheduler.update(n)

        Building and delivering step n-1's events (TokenEvents, IPC msgpack,
        SSE wake-ups) overlaps step n's kernels, so the host critical path is
        only schedule + upload + launch + update (all native / array code;
        sampling parameters come out of the native plan as flat arrays)."""
        self._drain()
        if not self.sched.has_work and self._la is None:
            self._flush_pending()
            self._idle = True
            return False
        if self._idle:
            self._idle = False
            self._admission_window()
        self._step_started = time.monotonic()
        try:
            return self._step_la() if self.lookahead else self._step()
        finally:
            self._step_started = 0.0

    def _admission_window(self) -> None:
        """Idle -> busy: a burst of requests (a client wave, a batch job)
        reaches the engine over tens of ms through the front door; the first
        step would otherwise prefill whichever request came first alone and
        the rest one step later.  Wait while requests keep arriving -- until
        LMX_ADMIT_QUIET_MS (2) pass without one, LMX_ADMIT_MAX_MS (25) pass in
        all, or a step's token budget is queued -- then schedule.  A lone
        request pays the quiet interval once; a busy engine never waits."""
        quiet = self._admit_quiet_s
        if quiet <= 0 or self.sched.num_running:
            return
        t0 = time.monotonic()
        n = len(self._reqs)                # all waiting: nothing was running

        def queued_tokens():
            return sum(len(r.prompt_ids) for r in self._reqs.values())
        self._wake.clear()
        last = t0                          # the latest arrival seen
        while (n < self.ecfg.max_num_seqs and queued_tokens() < self.ecfg.max_batched_tokens):
            now = time.monotonic()
            if now - last >= quiet or now - t0 >= self._admit_max_s:
                break
            self._wake.wait(timeout=min(quiet - (now - last), self._admit_max_s - (now - t0)))
            self._wake.clear()
            self._drain()
            m = len(self._reqs)
            if m != n:
                n, last = m, time.monotonic()

    def _step(self) -> bool:
        fl = faults()
        if fl:
            if fl.hit("step_hang"):
                time.sleep(float(os.environ.get("LMX_FAULT_HANG_S", "5")))
            fl.maybe_raise("gpu_error", "HIP error: injected device fault")
        if self._prof is not None:
            self._prof_tick()
        t0 = time.perf_counter()
        plan = self.sched.schedule(self.q_per_tile)
        T = plan["num_tokens"]
        if T == 0:
            self._flush_pending()
            return False
        S = len(plan["seq_ids"])
        nd = plan["num_decode"]
        N = len(plan["sample_seq"])
        bucket = None
        if nd == S == T and self.graphs:
            bucket = next((b for b in self._bucket_list if b >= nd), None)
        probe = (self.tp.size > 1 and self._comm_every > 0
                 and self.stats["steps"] % self._comm_every == self._comm_every - 1)
        self._publish(plan, bucket, probe)
        t1 = time.perf_counter()
        if bucket is not None:
            tok, lp = self._run_graph(plan, bucket)
        else:
            tok, lp = self._run_eager(plan)
        self._start_fetch(tok, lp, N)
        t2 = time.perf_counter()
        self._flush_pending()
        t3 = time.perf_counter()
        toks, lps = self._finish_fetch(N)
        t4 = time.perf_counter()
        finished = self.sched.update(toks)
        if probe:
            self._comm_probe()
        t5 = time.perf_counter()
        self._pending = (plan["seq_ids"], plan["sample_seq"], toks, lps, finished)
        if not self.sched.has_work:
            self._flush_pending()
        st = self.stats
        st["t_schedule"] += t1 - t0
        st["t_launch"] += t2 - t1
        st["t_events"] += t3 - t2
        st["t_wait"] += t4 - t3
        st["t_update"] += t5 - t4
        st["t_gpu"] += t4 - t1
        st["steps"] += 1
        st["step_time_s"] += t5 - t0
        st["decode_steps"] += int(nd == S)
        st["graph_steps"] += int(bucket is not None)
        if bucket is not None:
            st["decode_step_s"] += t5 - t0
            # host phases of graph (pure decode) steps alone: schedule,
            # launch (metadata + upload + replay), update
            st["g_schedule"] += t1 - t0
            st["g_launch"] += t2 - t1
            st["g_update"] += t5 - t4
        st["prefill_tokens"] += plan["num_prefill_tokens"]
        if self.step_trace is not None and bucket is None:
            self.step_trace.append((time.time(), T, nd, int(plan["num_prefill_tokens"]),
                                    int(self.sched.num_waiting)))
        return True

    def _publish(self, plan, bucket, probe: bool) -> None:
        """TP leader: hand the step's plan to the followers (no-op alone)."""
        if self.chan is None:
            return
        from ..parallel.plan_channel import encode_plan
        msg = encode_plan(plan, bucket, full=self.sample_all)
        msg["probe"] = int(probe)
        self.chan.publish(msg)

    def _step_la(self) -> bool:
        """Lookahead step (one-step asynchronous scheduling):

            consume step n (tokens unknown) -> schedule(n+1) -> launch(n+1)
            -> wait for step n's tokens (n+1 queued behind it) -> patch(n)
            -> emit step n's events

        so the GPU always has the next step queued and the host's schedule /
        metadata / launch work runs under the previous step's kernels.  Rows
        whose input is step n's sample carry its index (plan input_src); the
        decode graphs gather those tokens on the device (ops.ids_from_prev),
        an eager (prefill / mixed) step waits for them first.  Sequences that
        stop on a sampled stop token one step late cost one dropped row
        (native Scheduler::patch)."""
        fl = faults()
        if fl:
            if fl.hit("step_hang"):
                time.sleep(float(os.environ.get("LMX_FAULT_HANG_S", "5")))
            fl.maybe_raise("gpu_error", "HIP error: injected device fault")
        if self._prof is not None:
            self._prof_tick()
        t0 = time.perf_counter()
        la = self._la
        if la is not None:
            self.sched.update_lookahead()
            if self._penalized:     # penalty windows are built from the real tokens
                self._la_resolve()
                la = None
        plan = self.sched.schedule(self.q_per_tile)
        T = plan["num_tokens"]
        if T == 0:
            if la is not None:
                self._la_resolve()
            self._flush_pending()
            return la is not None
        S = len(plan["seq_ids"])
        nd = plan["num_decode"]
        N = len(plan["sample_seq"])
        bucket = None
        if nd == S == T and self.graphs:
            bucket = next((b for b in self._bucket_list if b >= nd), None)
        probe = (self.tp.size > 1 and self._comm_every > 0
                 and self.stats["steps"] % self._comm_every == self._comm_every - 1)
        t1 = time.perf_counter()
        tw = 0.0
        if bucket is not None:
            self._publish(plan, bucket, probe)
            tok, lp = self._run_graph(plan, bucket)
        else:
            if la is not None:      # this step's inputs need step n's tokens on the host
                tw = time.perf_counter()
                prev = self._la_resolve()
                tw = time.perf_counter() - tw
                la = None
                if plan["num_pending_inputs"]:
                    src = plan["input_src"]
                    m = src >= 0
                    plan["input_ids"][m] = prev[src[m]]
            elif plan["num_pending_inputs"]:
                raise RuntimeError("lookahead plan references an unread step")
            self._publish(plan, None, probe)
            tok, lp = self._run_eager(plan)
            if self.graphs and N:
                # the next (graph) step gathers its input tokens from here
                self._gbuf["tok"][:N].copy_(tok[:N], non_blocking=True)
        k = self._start_fetch(tok, lp, N)
        t2 = time.perf_counter()
        if la is not None:
            self._la_resolve()
        t3 = time.perf_counter()
        self._la = {"seq_ids": plan["seq_ids"], "sample_seq": plan["sample_seq"], "N": N,
                    "slot": k, "graph": bucket is not None, "t_launch": t1}
        if probe:
            self._comm_probe()
        st = self.stats
        st["t_schedule"] += t1 - t0
        st["t_launch"] += t2 - t1 - tw
        st["t_wait"] += t3 - t2 + tw
        st["t_gpu"] += t3 - t1
        st["steps"] += 1
        st["step_time_s"] += t3 - t0
        st["decode_steps"] += int(nd == S)
        st["graph_steps"] += int(bucket is not None)
        if bucket is not None:      # (decode_step_s: timed when the step resolves)
            st["g_schedule"] += t1 - t0
            st["g_launch"] += t2 - t1
        st["prefill_tokens"] += plan["num_prefill_tokens"]
        if self.step_trace is not None and bucket is None:
            # eager (prefill / mixed) steps: launch time, rows, decode rows,
            # prefill tokens, sequences still waiting (LMX_STEP_TRACE=1)
            self.step_trace.append((time.time(), T, nd, int(plan["num_prefill_tokens"]),
                                    int(self.sched.num_waiting)))
        return True

    def _la_resolve(self) -> np.ndarray:
        """Read back the launched step's tokens, fill the scheduler's
        placeholders and emit that step's events; returns its tokens."""
        la, self._la = self._la, None
        t = time.perf_counter()
        toks, lps = self._finish_fetch(la["N"], la["slot"])
        t2 = time.perf_counter()
        if la["graph"]:
            # a queued step runs from the previous step's end (or from its own
            # launch if the GPU was idle), so a decode step queued behind a
            # prefill step is not charged that prefill's time
            self.stats["decode_step_s"] += t2 - max(la["t_launch"], self._la_end)
        self._la_end = t2
        fin = self.sched.patch(toks)
        self.stats["t_update"] += time.perf_counter() - t2
        self.stats["t_events"] += t2 - t
        self._pending = (la["seq_ids"], la["sample_seq"], toks, lps, fin)
        self._flush_pending()
        return toks

    def start_profile(self, out_dir: str, steps: int = 20):
        """Record a torch.profiler (ROCm/roctracer) timeline of the next
        ``steps`` engine steps into ``out_dir`` (chrome trace)."""
        from torch.profiler import ProfilerActivity, profile
        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA]
                                         if self.device.type == "cuda" else [])
        self._prof = profile(activities=acts, record_shapes=False)
        self._prof.__enter__()
        self._prof_left = steps
        self._prof_dir = out_dir

    def _prof_tick(self):
        self._prof_left -= 1
        if self._prof_left < 0:
            self._prof.__exit__(None, None, None)
            os.makedirs(self._prof_dir, exist_ok=True)
            path = os.path.join(self._prof_dir, f"engine_steps_{os.getpid()}.json")
            self._prof.export_chrome_trace(path)
            log.info("engine profile written to %s", path)
            self._prof = None

    def _flush_pending(self):
        """Turn the previous step's sampled tokens into TokenEvents."""
        pend, self._pending = self._pending, None
        if pend is None:
            return
        seq_ids, sample_seq, toks, lps, finished = pend
        fin = {rid: FINISH_REASONS.get(r, "stop") for rid, r in finished}
        evs = []
        now = time.time()
        reqs = self._reqs
        rids = seq_ids[sample_seq].tolist()
        tl, ll = toks.tolist(), lps.tolist()
        for i, rid in enumerate(rids):
            req = reqs.get(rid)
            if req is None:
                continue
            if req.num_generated == 0:
                req.first_token_at = now
                self.ttft_samples.append((req.arrival, now))
            req.num_generated += 1
            reason = fin.get(rid)
            if reason is not None:
                req.finished = True
                del reqs[rid]
                self._penalized.discard(rid)
                self.stats["finished"] += 1
            evs.append(TokenEvent(req, tl[i], ll[i], reason))
        # counted where the tokens are delivered: lookahead's dropped rows
        # (a stopped or aborted sequence's extra sample) never reach here
        self.stats["generated_tokens"] += len(evs)
        if evs and self.event_sink:
            self.event_sink(evs)

    def _run_eager(self, plan):
        T = plan["num_tokens"]
        S = len(plan["seq_ids"])
        mb = plan["max_blocks"]
        rows = plan["sample_rows"].astype(np.int64)
        items = [
            ("ids", plan["input_ids"]), ("pos", plan["positions"]), ("slots", plan["slots"]),
            ("ctx", plan["context_lens"]), ("cu", plan["cu_q"]),
            ("bt", plan["block_tables"].reshape(S, mb)),
            ("tiles", plan["prefill_tiles"] if len(plan["prefill_tiles"]) else
             np.zeros(2, np.int32)),
            ("rows", rows), ("temp", plan["temp"]), ("topk", plan["topk"]),
            ("topp", plan["topp"]), ("seeds", plan["seeds"]), ("offs", plan["offs"])]
        nd = plan["num_decode"]
        if nd > 1:
            items.append(("order", ops.decode_order(plan["context_lens"][:nd])))
        samples = self.is_leader or self.sample_all
        pen = bool(plan.get("any_penalty")) and samples
        if pen:   # one pack, one upload: the pinned staging buffer is reused per call
            N = len(plan["sample_rows"])
            items += [("win", plan["pen_window"].reshape(N, PEN_WINDOW)),
                      ("ngen", plan["pen_ngen"]), ("pen", plan["pen_params"].reshape(N, 3))]
        d = self.packer.pack(items)
        self._mark_upload()
        inp = StepInputs(d["ids"], d["pos"], d["slots"], plan["num_decode"], d["bt"], d["ctx"],
                         d["cu"], d["tiles"], d["rows"], T, S, decode_order=d.get("order"),
                         host={"cu_q": plan["cu_q"], "tiles": plan["prefill_tiles"], "rows": rows})
        ws = self._decode_ws(plan["num_decode"]) if plan["num_decode"] else self.decode_ws
        logits = self.model.forward(inp, self.k_caches, self.v_caches, ws, self.ecfg.part_tokens)
        self._peer_check()
        if not samples:
            return None, None
        if pen:
            self._penalize(logits, d["win"], d["ngen"], d["pen"])
        return self._sample(logits, d["temp"], d["topk"], d["topp"], d["seeds"], d["offs"])

    def _run_graph(self, plan, B):
        self._gmeta.next()
        g, h = self._gbuf, self._gmeta.h
        n = len(plan["seq_ids"])
        mb = plan["max_blocks"]
        pen = bool(plan.get("any_penalty")) and (self.is_leader or self.sample_all)
        if pen and B not in self.pen_graphs:
            t0 = time.time()
            self.pen_graphs[B] = self._capture_penalty(B)
            log.info("captured the penalty sampling graph of bucket %d in %.2fs", B,
                     time.time() - t0)
        # rows n..B-1 are padding: no cache write (slot -1), a 1-token context
        for k, fill in (("ids", 0), ("pos", 0), ("slots", -1), ("ctx", 1), ("temp", 0),
                        ("topk", 0), ("topp", 1), ("seeds", 0), ("offs", 0)):
            a = h[k]
            a[:n] = plan[_PLAN_KEY.get(k, k)]
            a[n:B] = fill
        src = plan.get("input_src")
        if src is not None and plan.get("num_pending_inputs"):
            h["src"][:n] = src
        else:
            h["src"][:n] = -1
        h["src"][n:B] = -1
        # only the live columns: stale entries beyond a row's context are
        # never read (and always hold valid page ids)
        h["bt"][:n, :mb] = plan["block_tables"].reshape(n, mb)
        h["bt"][n:B, 0] = 0
        h["order"][:B] = ops.decode_order(h["ctx"][:B])
        if pen:
            self._pmeta.next()
            ph = self._pmeta.h
            ph["win"][:n] = plan["pen_window"].reshape(n, -1)
            ph["win"][n:B] = -1
            ph["ngen"][:n] = plan["pen_ngen"]
            ph["pen"][:n] = plan["pen_params"].reshape(n, 3)
            self._pmeta.upload()
        ta = time.perf_counter()
        self._gmeta.upload()
        self._mark_upload()
        tb = time.perf_counter()
        self.graphs[B]["graph"].replay()
        if pen:
            self.pen_graphs[B]["graph"].replay()
        self._peer_check()
        st = self.stats
        st["g_upload"] += tb - ta
        st["g_replay"] += time.perf_counter() - tb
        return g["tok"][:B], g["lp"][:B]

    def _peer_check(self) -> None:
        """TP: a peer-memory collective of this rank that gave up waiting for a
        peer (bounded spin) produced a wrong sum.  Behind every step its error
        word is copied to pinned memory, ahead of the step's token D2H copy on
        the same stream, so it has landed once the tokens have: the ranks that
        emit tokens check it where the tokens are read back (``_peer_raise``
        in ``_finish_fetch``), before any of that step's tokens reach the
        scheduler or a client.  Followers emit nothing and raise as soon as
        they see it.  Raised as a HIP error: the engine turns unhealthy and
        the worker is restarted instead of serving corrupted tokens."""
        peer = self.tp.peer
        if peer is None:
            return
        if not (self.is_leader or self.sample_all):
            self._peer_raise()
        if self.device.type == "cuda":
            peer.check_async(torch.cuda.current_stream(self.device))
        else:
            peer.check_async(None)

    def _peer_raise(self) -> None:
        peer = self.tp.peer
        if peer is not None and peer.failed():
            raise RuntimeError("HIP error: peer all-reduce timed out waiting for a TP peer")

    def _start_fetch(self, tok: torch.Tensor, lp: torch.Tensor, n: int) -> int:
        """Queue the D2H copy of the sampled tokens/logprobs into pinned
        memory behind the step's kernels (no sync here); returns the slot."""
        k = self._slot = self._slot ^ 1
        if not tok.is_cuda:
            self._fetch_cpu[k] = (tok[:n].numpy().copy(), lp[:n].numpy().copy())
            return k
        self._hout[k, 0, :n].copy_(tok[:n], non_blocking=True)
        self._hout[k, 1, :n].copy_(lp[:n].view(torch.int32), non_blocking=True)
        self._out_evs[k].record()
        return k

    def _finish_fetch(self, n: int, k: int | None = None):
        k = self._slot if k is None else k
        if self.device.type != "cuda":
            self._peer_raise()
            return self._fetch_cpu[k]
        self._out_evs[k].synchronize()
        self._peer_raise()      # this step's collectives were sound (see _peer_check)
        h = self._hout_np[k]
        return h[0, :n].copy(), h[1, :n].view(np.float32).copy()

    # ----------------------------------------------------- offline helper ---
    def generate(self, prompts: list[list[int]], params: SamplingParams,
                 timeout: float = 600.0) -> list[list[int]]:
        """Blocking batch generation (smoke tests, offline use); must not be
        mixed with a running engine thread."""
        outs: dict[int, list[int]] = {}
        done: set[int] = set()
        prev_sink = self.event_sink

        def sink(evs):
            for e in evs:
                if e.token >= 0:
                    outs.setdefault(e.req.id, []).append(e.token)
                if e.finish is not None:
                    done.add(e.req.id)

        self.event_sink = sink
        try:
            reqs = [self.submit(GenRequest(list(p), params)) for p in prompts]
            t_end = time.time() + timeout
            while len(done) < len(reqs):
                if not self.step() and time.time() > t_end:
                    raise TimeoutError("generate timed out")
                if time.time() > t_end:
                    raise TimeoutError("generate timed out")
        finally:
            self.event_sink = prev_sink
        return [outs.get(r.id, []) for r in reqs]
