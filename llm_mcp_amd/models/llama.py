"""Llama-3 family decoder (8B / 70B / 3.x) for the in-process serving engine.

What the reference delegates to Ollama's /api/generate and /api/chat
(worker/llm_worker/main.py:222-243, core/internal/api/handlers.go:2308-2587)
runs here, on the GPU the worker owns:

  embed_gather (K10) -> per layer:
      rms_norm(+residual, K1) -> QKV GEMM (hipBLASLt) -> rope_and_cache (K2+K5)
      -> paged attention: decode rows (K4) / prefill rows (K3)
      -> O GEMM [+ RCCL all-reduce under TP] -> rms_norm(+residual)
      -> gate|up GEMM -> silu_mul (K8) -> down GEMM [+ all-reduce]
  -> final rms_norm on the sampled rows only -> LM head -> sampling (K6).

Weights are fused per layer (QKV, gate|up) so each step issues 4 GEMMs per
layer.  Tensor parallelism (Megatron column/row split) is built in: QKV and
gate|up are split by heads / intermediate columns, O and down by rows, with
one all-reduce after each (X1, X2); the LM head is vocab-split and gathered
(X3).  Embeddings are replicated -- on a 288 GB part their memory is cheaper
than an extra collective per step.  Long steps (>= LMX_SP_MIN_TOKENS tokens)
switch to sequence parallelism: each all-reduce becomes a reduce-scatter over
token rows, RMSNorm + residual run on the rank's row block, and an all-gather
feeds the next column-parallel GEMM (TPContext.reduce_scatter_rows /
all_gather_rows).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import ref
from .config import LlamaConfig
from .weights import vocab_shard


@dataclass
class StepInputs:
    """Device tensors of one engine step (built from the scheduler's plan)."""
    input_ids: torch.Tensor       # int32 [T]
    positions: torch.Tensor       # int32 [T]
    slots: torch.Tensor           # int32 [T]
    num_decode: int               # first num_decode rows are decode rows (1 per seq)
    block_tables: torch.Tensor    # int32 [S, max_blocks]
    context_lens: torch.Tensor    # int32 [S]
    cu_q: torch.Tensor            # int32 [S+1] (absolute token rows)
    prefill_tiles: torch.Tensor   # int32 [2 * n_tiles] (prefill-seq index, q_start)
    sample_rows: torch.Tensor     # int64 [N] token rows whose logits are needed
    num_tokens: int
    num_seqs: int
    decode_order: torch.Tensor | None = None   # int32 [num_decode] (ops.decode_order)
    # host copies of the plan's cu_q / prefill_tiles / sample_rows (numpy), when
    # the caller has them: lets the model split a step without a device sync
    host: dict | None = None


class TPContext:
    """Tensor-parallel placement of this rank (size 1 = no TP)."""

    def __init__(self, rank: int = 0, size: int = 1, group=None,
                 sp_min_tokens: int | None = None, cpu_group=None):
        """``group``: the TP process group (RCCL on GPUs); ``cpu_group``: a
        gloo group over the same ranks for host-side control values (built
        by the caller when several TP groups share one world, where a
        subgroup cannot be created lazily by one group alone)."""
        self.rank, self.size, self.group = rank, size, group
        self.cpu_group = cpu_group
        # lookahead TP (engine.sample_all): every rank keeps the full logits
        # and samples them itself, so each rank holds the step's tokens on
        # its device for the next step's ids_from_prev gather
        self.logits_to_all = False
        # vocab-sharded sampling (engine race_tp): forward returns this rank's
        # logits shard; nothing is gathered
        self.shard_logits = False
        self.peer = None      # parallel.peer_allreduce.PeerAllReduce when enabled
        # Sequence parallelism (SURVEY.md §2.4 "SP" row): steps with at least
        # this many tokens keep the residual stream row-sharded across the TP
        # group -- reduce-scatter after the row-parallel O / down GEMMs,
        # RMSNorm + residual add on T/size rows, all-gather before the
        # column-parallel QKV / gate-up GEMMs.  Same bytes on the wire as the
        # all-reduce, 1/size of the norm work and residual memory.
        if sp_min_tokens is None:
            sp_min_tokens = int(os.environ.get("LMX_SP_MIN_TOKENS", "0"))
        self.sp_min_tokens = sp_min_tokens if sp_min_tokens > 0 else 1 << 62

    def use_sp(self, num_tokens: int) -> bool:
        return self.size > 1 and num_tokens >= self.sp_min_tokens

    def reduce_scatter_rows(self, t: torch.Tensor, padded_rows: int) -> torch.Tensor:
        """Sum ``t`` [T, d] over the group and return this rank's block of
        ``padded_rows // size`` rows (rows past T count as zero)."""
        rows, d = t.shape
        if rows < padded_rows:
            p = torch.zeros((padded_rows, d), dtype=t.dtype, device=t.device)
            p[:rows] = t
            t = p
        s = padded_rows // self.size
        if not t.is_cuda or self._host_staged(t):
            # gloo: no reduce-scatter of device tensors -> all-reduce + slice
            self.all_reduce(t)
            return t[self.rank * s:(self.rank + 1) * s].clone()
        out = torch.empty((s, d), dtype=t.dtype, device=t.device)
        torch.distributed.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate every rank's [s, d] block into [size * s, d]."""
        src = t.contiguous()
        if not src.is_cuda or self._host_staged(src):
            src = src.cpu()
            parts = [torch.empty_like(src) for _ in range(self.size)]
            torch.distributed.all_gather(parts, src, group=self.group)
            return torch.cat(parts, dim=0).to(t.device, non_blocking=True)
        out = torch.empty((self.size * src.shape[0], src.shape[1]), dtype=src.dtype,
                          device=src.device)
        torch.distributed.all_gather_into_tensor(out, src, group=self.group)
        return out

    def device_collectives_cover(self, rows: int, hidden: int, logit_cols: int) -> bool:
        """Every collective of a pure-decode step of ``rows`` rows runs as one
        peer-memory kernel (no RCCL / gloo call): the O / down all-reduces of
        [rows, hidden] bf16 and the vocab-split logits gather of
        [rows, logit_cols] bf16 fit a slot, and no decode step is
        sequence-parallel.  Such a step captures into a hipGraph whatever the
        group's backend -- a gloo group (one-GPU rehearsals) included."""
        if self.size == 1:
            return True
        if self.peer is None or self.use_sp(rows):
            return False
        slot = self.peer.slot
        return rows * hidden * 2 <= slot and rows * logit_cols * 2 <= slot

    def global_rank(self, group_rank: int) -> int:
        """World rank of a rank of this TP group (collectives that name a
        root take world ranks)."""
        if self.group is None or self.group == torch.distributed.group.WORLD:
            return group_rank
        return torch.distributed.get_global_rank(self.group, group_rank)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.peer is not None and self.peer.supports(t):
                self.peer(t)     # one kernel over peer memory (decode sizes)
            elif self._host_staged(t):
                h = t.cpu()
                torch.distributed.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                torch.distributed.all_reduce(t, group=self.group)
        return t

    def all_reduce_async(self, t: torch.Tensor):
        """Start the sum of ``t`` over the group in place; returns a handle
        whose ``wait()`` orders the caller's stream after it (RCCL: the
        collective runs on its own stream, overlapping the compute issued
        meanwhile).  Host-staged (gloo) and peer-slot messages complete here;
        a message the peer slot does not hold (prefill sizes) goes to RCCL
        asynchronously even when the group has the peer kernel."""
        if self.size > 1 and self._async_rccl(t):
            return torch.distributed.all_reduce(t, group=self.group, async_op=True)
        self.all_reduce(t)
        return _Done()

    def _async_rccl(self, t: torch.Tensor) -> bool:
        """``all_reduce_async`` hands ``t`` to RCCL with async_op=True."""
        if self.peer is not None and self.peer.supports(t):
            return False
        return not self._host_staged(t)

    def all_reduce_norm(self, t: torch.Tensor, w: torch.Tensor, eps: float,
                        residual: torch.Tensor) -> torch.Tensor:
        """residual += all_reduce(t); returns rms_norm(residual) * w.  One
        peer-memory kernel when it covers the message (decode sizes), else the
        group's all-reduce followed by the residual-add RMSNorm."""
        if self.peer is not None and self.peer.norm_supports(t, residual):
            return self.peer.all_reduce_norm(t, w, eps, residual)
        return ops.rms_norm(self.all_reduce(t), w, eps, residual=residual)

    def all_gather_records(self, rec: torch.Tensor) -> torch.Tensor:
        """Every rank's fp32 [B, 8] sampler records in rank order, [size, B, 8]
        (ops.sample_race's exchange: B x 32 B per rank).  Peer slots when the
        group has them (graph-capturable, no RCCL call), else the group's
        all-gather."""
        shape = (self.size,) + tuple(rec.shape)
        if self.size == 1:
            return rec.view(shape)
        src = rec.contiguous()
        raw = src.view(torch.bfloat16).reshape(-1)
        if self.peer is not None and self.peer.gather_supports(raw):
            return self.peer.all_gather(raw, None, to_all=True).view(torch.float32).view(shape)
        if not src.is_cuda or self._host_staged(src):
            h = src.cpu()
            parts = [torch.empty_like(h) for _ in range(self.size)]
            torch.distributed.all_gather(parts, h, group=self.group)
            return torch.stack(parts).to(rec.device, non_blocking=True)
        out = torch.empty(shape, dtype=rec.dtype, device=rec.device)
        torch.distributed.all_gather_into_tensor(out, src, group=self.group)
        return out

    def _host_staged(self, t: torch.Tensor) -> bool:
        # gloo only reduces device tensors; it gathers host tensors
        return t.is_cuda and torch.distributed.get_backend(self.group) == "gloo"

    def gather_last_to_leader(self, t: torch.Tensor) -> torch.Tensor | None:
        """Vocab-parallel logits [B, V/size] -> [B, V] on rank 0 (the only rank
        that samples); followers get None and assemble nothing.  RCCL: one
        all_gather_into_tensor (graph-capturable, one collective per step) and
        the column interleave on the leader only; gloo: a gather to rank 0."""
        if self.size == 1:
            return t
        src = t.contiguous()
        B, Vs = src.shape
        peer = self.peer is not None and self.peer.gather_supports(src)
        if not peer and (not src.is_cuda or self._host_staged(src)):
            h = src.cpu()
            if self.logits_to_all:
                parts = [torch.empty_like(h) for _ in range(self.size)]
                torch.distributed.all_gather(parts, h, group=self.group)
                return torch.cat(parts, dim=-1).to(t.device, non_blocking=True)
            parts = [torch.empty_like(h) for _ in range(self.size)] if self.rank == 0 else None
            torch.distributed.gather(h, parts, dst=self.global_rank(0), group=self.group)
            if self.rank:
                return None
            return torch.cat(parts, dim=-1).to(t.device, non_blocking=True)
        if peer:
            # one kernel over the peer-memory slots: no RCCL collective in the
            # captured decode graph (followers only publish unless every rank
            # samples)
            out = self.peer.all_gather(src, None, to_all=self.logits_to_all)
            if out is None:
                return None
        else:
            out = torch.empty((self.size * B, Vs), dtype=src.dtype, device=src.device)
            torch.distributed.all_gather_into_tensor(out, src, group=self.group)
            if self.rank and not self.logits_to_all:
                return None
        return out.view(self.size, B, Vs).permute(1, 0, 2).reshape(B, self.size * Vs)


class _Done:
    def wait(self):
        return True


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, device: torch.device | str = "cuda",
                 dtype=torch.bfloat16, tp: TPContext | None = None, seed: int = 0,
                 weights: dict | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPContext()
        T = self.tp.size
        if cfg.num_heads % T or cfg.intermediate_size % T:
            raise ValueError("TP size must divide heads and intermediate size")
        self.Hq = cfg.num_heads // T
        self.Hkv = max(1, cfg.num_kv_heads // T)
        if cfg.num_kv_heads % T and T % cfg.num_kv_heads:
            raise ValueError("TP size incompatible with kv heads")
        self.kv_replicas = max(1, T // cfg.num_kv_heads)
        self.D = cfg.head_dim
        self.I = cfg.intermediate_size // T
        self.vocab_shard = vocab_shard(cfg.vocab_size, T)
        self.scale = 1.0 / math.sqrt(self.D)
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, self.D, cfg.rope_theta, self.device,
                                        cfg.rope_scaling)
        # K2 + K5 inside K4 for decode rows (LMX_FUSED_DECODE_ROPE=0: separate kernels)
        self.fuse_decode_rope = os.environ.get("LMX_FUSED_DECODE_ROPE", "1") == "1"
        self.fuse_prefill_rope = os.environ.get("LMX_FUSED_PREFILL_ROPE", "1") == "1"
        if weights is None:
            weights = self._random_weights(seed)
        else:
            # the folds / interleaves / packing below replace entries of the
            # layer dicts: work on copies so the caller's dict keeps the
            # checkpoint's tensors (export_weights gives the served form back)
            weights = {**weights, "layers": [dict(L) for L in weights["layers"]]}
        self.w = weights
        # fused-SwiGLU decode GEMM (K11 epi=1): gate|up rows interleaved per
        # BN/2 channels when the measured dispatch table uses it for this shape
        self.gu_block = 0
        # the RMSNorm gains folded into the projections they feed (QKV <- ln1,
        # gate/up <- ln2; W' = W diag(g) at load, the norms then run with unit
        # gains): prefill steps may then skip the per-layer norm pass entirely
        # (_norm_fold_step) -- TP = 1 only
        self.norm_folded = False
        if (self.device.type == "cuda" and self.tp.size == 1 and not cfg.proxy_tp
                and os.environ.get("LMX_NORM_FOLD", "1") != "0"):
            for L in self.w["layers"]:
                for g, wk in (("ln1", "wqkv"), ("ln2", "w_gate_up")):
                    L[wk] = (L[wk].float() * L[g].float()[None, :]).to(L[wk].dtype)
                    L[g] = torch.ones_like(L[g])
            self.norm_folded = True
        if self.device.type == "cuda":
            blk = ops.swiglu_block(2 * self.I, cfg.hidden_size)
            if blk:
                for L in self.w["layers"]:
                    L["w_gate_up"] = ops.interleave_gate_up(L["w_gate_up"], blk)
                self.gu_block = blk
            # one copy of the MLP weights: gate/up (SwiGLU16 interleave) and
            # down stored only in K14's packed layout when every consumer
            # reads it (K14 decode, K13 prefill with packed W; TP = 1 path)
            if (self.tp.size == 1 and not cfg.proxy_tp
                    and ops.rs_single_wanted(self.weight_bytes(), self.device)):
                for L in self.w["layers"]:
                    if self.gu_block == ops.SWIGLU16 and ops.rs_single_ok(L["w_gate_up"], True):
                        L["w_gate_up"] = ops.rs_pack_only(L["w_gate_up"])
                    if ops.rs_single_ok(L["w_down"]):
                        L["w_down"] = ops.rs_pack_only(L["w_down"])
            # K14 decode shapes the table runs on packed weights get their
            # packed copies now, all or nothing per shape (row-major entries
            # need nothing)
            ops.rs_prepare_all([L[k] for L in self.w["layers"]
                                for k in ("wqkv", "wo", "w_gate_up", "w_down") if k in L]
                               + [self.w["lm_head"]])

    # ----------------------------------------------------------- weights ----
    def _random_weights(self, seed: int) -> dict:
        """Deterministic random init of this rank's shard (synthetic benchmark
        weights; std 0.02 keeps activations finite through 80 layers)."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed * 1000 + self.tp.rank)
        d = cfg.hidden_size

        def rnd(*shape, std=0.02):
            t = torch.empty(shape, dtype=dt, device=dev)
            t.normal_(0.0, std, generator=g)
            return t

        layers = []
        qkv_rows = (self.Hq + 2 * self.Hkv) * self.D
        for _ in range(cfg.num_layers):
            layers.append({})
            if cfg.qkv_bias:
                layers[-1]["bqkv"] = rnd(qkv_rows, std=0.02)
            if cfg.qk_norm:          # around 1, like trained q/k norm gains
                layers[-1]["q_norm"] = (1.0 + rnd(self.D, std=0.1)).to(dt)
                layers[-1]["k_norm"] = (1.0 + rnd(self.D, std=0.1)).to(dt)
            layers[-1].update({
                "ln1": torch.ones(d, dtype=dt, device=dev),
                "ln2": torch.ones(d, dtype=dt, device=dev),
                "wqkv": rnd(qkv_rows, d),
                "wo": rnd(d, self.Hq * self.D, std=0.02 / math.sqrt(2 * cfg.num_layers)),
                "w_gate_up": rnd(2 * self.I, d),
                "w_down": rnd(d, self.I, std=0.02 / math.sqrt(2 * cfg.num_layers)),
            })
        embed = rnd(cfg.vocab_size, d, std=1.0)
        vs = self.vocab_shard
        if cfg.tie_embeddings:
            lm_head = embed[self.tp.rank * vs:(self.tp.rank + 1) * vs]
            if lm_head.shape[0] < vs:        # the last shard: zero rows past the vocabulary
                lm_head = torch.cat([lm_head, lm_head.new_zeros(vs - lm_head.shape[0], d)])
        else:
            lm_head = rnd(vs, d)
        return {"embed": embed, "norm": torch.ones(d, dtype=dt, device=dev), "lm_head": lm_head,
                "layers": layers}

    def export_weights(self) -> dict:
        """The served weights as a plain fused dict (``weights.save_hf_llama``,
        ``shard_llama``): row-major (K14-packed copies unpacked), gate/up back
        in [gate; up] row order.  With the norm gains folded at load the
        projections carry them and ln1 / ln2 are ones: the exact model that is
        served, and loading it folds nothing further."""
        layers = []
        for L in self.w["layers"]:
            d = {k: ops.dense_weight(v) for k, v in L.items()}
            if self.gu_block:
                d["w_gate_up"] = ops.deinterleave_gate_up_rows(d["w_gate_up"], self.gu_block)
            layers.append(d)
        return {"embed": self.w["embed"], "norm": self.w["norm"],
                "lm_head": ops.dense_weight(self.w["lm_head"]), "layers": layers}

    def weight_bytes(self, copies: bool = False) -> int:
        """Bytes of the model's weights; ``copies``: plus the K14 packed
        copies kept beside row-major weights (HBM the weights hold)."""
        n = 0
        ts = [t for k, v in self.w.items() if k != "layers" for t in [v]]
        ts += [t for l in self.w["layers"] for t in l.values()]
        for t in ts:
            n += t.numel() * t.element_size()
            p = getattr(t, "_lmx_rs_packed", None) if copies else None
            if p is not None:
                n += p.numel() * p.element_size()
        return n

    # ----------------------------------------------------------- forward ----
    # ------------------------------------------- TP prefill micro-batches ----
    def _microbatch_split(self, inp: StepInputs) -> int:
        """Pure-prefill TP step split point (prefill-sequence index) for two
        micro-batches whose row-parallel all-reduces overlap the other
        micro-batch's compute, or 0 for one batch.  LMX_TP_MICROBATCH: auto
        (RCCL groups, steps of >= LMX_TP_MICROBATCH_MIN tokens, default 2048),
        1 (any group, any size: tests), 0 (off)."""
        tp = self.tp
        mode = os.environ.get("LMX_TP_MICROBATCH", "auto")
        if (tp.size < 2 or mode == "0" or inp.num_decode or inp.host is None
                or tp.use_sp(inp.num_tokens) or tp.group is None):
            return 0
        if mode != "1":
            if torch.distributed.get_backend(tp.group) != "nccl":
                return 0
            if inp.num_tokens < int(os.environ.get("LMX_TP_MICROBATCH_MIN", "2048")):
                return 0
        cu = inp.host["cu_q"]
        S = len(cu) - 1
        if S < 2:
            return 0
        half = cu[-1] / 2.0
        j = int(min(range(1, S), key=lambda k: abs(cu[k] - half)))
        return j

    def _microbatch(self, inp: StepInputs, s0: int, s1: int) -> StepInputs:
        """Rows of prefill sequences [s0, s1) of a pure-prefill step as a step
        of their own (device slices and rebased index tensors; no sync)."""
        import numpy as np
        h = inp.host
        cu, tiles, rows = h["cu_q"], h["tiles"].reshape(-1, 2), h["rows"]
        r0, r1 = int(cu[s0]), int(cu[s1])
        t0 = int(np.searchsorted(tiles[:, 0], s0, "left"))
        t1 = int(np.searchsorted(tiles[:, 0], s1, "left"))
        k0 = int(np.searchsorted(rows, r0, "left"))
        k1 = int(np.searchsorted(rows, r1, "left"))
        dev_tiles = inp.prefill_tiles.view(-1, 2)[t0:t1]
        shift = torch.tensor([s0, 0], dtype=dev_tiles.dtype, device=dev_tiles.device)
        return StepInputs(
            inp.input_ids[r0:r1], inp.positions[r0:r1], inp.slots[r0:r1], 0,
            inp.block_tables[s0:s1], inp.context_lens[s0:s1], inp.cu_q[s0:s1 + 1] - r0,
            (dev_tiles - shift).reshape(-1).contiguous(), inp.sample_rows[k0:k1] - r0,
            r1 - r0, s1 - s0,
            host={"cu_q": cu[s0:s1 + 1] - r0, "tiles": tiles[t0:t1] - [s0, 0],
                  "rows": rows[k0:k1] - r0})

    def _mb_pipeline(self, inp: StepInputs, k_caches: list, v_caches: list):
        """One micro-batch's layer loop as a generator: it yields the handle of
        each row-parallel all-reduce it starts and resumes (after the caller
        waited on it) with the next stage; returns the final normed rows."""
        cfg, w, tp = self.cfg, self.w, self.tp
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        x = ops.embed_gather(w["embed"], inp.input_ids)
        residual = x
        layers = w["layers"]
        h = ops.rms_norm(x, layers[0]["ln1"], cfg.rms_eps)
        for li, L in enumerate(layers):
            qkv = ops.linear(h, L["wqkv"], bias=L.get("bqkv"))
            kc, vc = k_caches[li], v_caches[li]
            fuse_pf = self.fuse_prefill_rope and "q_norm" not in L and qkv.is_cuda
            ops.rope_and_cache(qkv, inp.positions, self.cos_sin, Hq, Hkv, D, inp.slots, kc, vc,
                               tile_from=0, q_norm=L.get("q_norm"), k_norm=L.get("k_norm"),
                               eps=cfg.rms_eps, skip_q=fuse_pf)
            attn = torch.empty((inp.num_tokens, Hq * D), dtype=self.dtype, device=self.device)
            ops.paged_prefill_attention(qkv, kc, vc, inp.block_tables, inp.cu_q,
                                        inp.context_lens, inp.prefill_tiles, self.scale, attn,
                                        Hq=Hq, rope=(inp.positions, self.cos_sin) if fuse_pf
                                        else None)
            o = ops.linear(attn, L["wo"])
            yield tp.all_reduce_async(o)
            h = ops.rms_norm(o, L["ln2"], cfg.rms_eps, residual=residual)
            if self.gu_block:
                a = ops.linear_swiglu(h, L["w_gate_up"], self.gu_block)
            else:
                a = ops.silu_mul(ops.linear(h, L["w_gate_up"]))
            x = ops.linear(a, L["w_down"])
            yield tp.all_reduce_async(x)
            nxt = layers[li + 1]["ln1"] if li + 1 < len(layers) else None
            if nxt is not None:
                h = ops.rms_norm(x, nxt, cfg.rms_eps, residual=residual)
        rows = inp.sample_rows
        return ops.rms_norm(x.index_select(0, rows), w["norm"], cfg.rms_eps,
                            residual=residual.index_select(0, rows))

    def _forward_tp_mb(self, inp: StepInputs, j: int, k_caches: list,
                       v_caches: list) -> torch.Tensor | None:
        """Pure-prefill TP step as two micro-batches (prefill sequences [0, j)
        and [j, S)) stepped alternately: micro-batch A's all-reduce after its
        O (or down) GEMM runs on the collective stream while B's attention /
        GEMMs run, and the other way round; every rank issues the collectives
        in the same order (A, B, A, B, ...)."""
        S = inp.num_seqs
        gens = [self._mb_pipeline(self._microbatch(inp, 0, j), k_caches, v_caches),
                self._mb_pipeline(self._microbatch(inp, j, S), k_caches, v_caches)]
        handles = [next(g) for g in gens]
        outs: list = [None, None]
        live = [True, True]
        while any(live):
            for i in (0, 1):
                if not live[i]:
                    continue
                handles[i].wait()
                try:
                    handles[i] = gens[i].send(None)
                except StopIteration as stop:
                    outs[i] = stop.value
                    live[i] = False
        hs = torch.cat(outs, dim=0)
        return self._tp_logits(ops.linear(hs, self.w["lm_head"]))

    def _tp_logits(self, logits: torch.Tensor) -> torch.Tensor | None:
        """The vocab-parallel LM head's output under TP: this rank's valid
        shard columns (vocab-sharded sampling) or the rows gathered to the
        sampling ranks (None on the others)."""
        tp, V = self.tp, self.cfg.vocab_size
        if tp.shard_logits:
            return logits[:, :max(1, min(self.vocab_shard, V - tp.rank * self.vocab_shard))]
        logits = tp.gather_last_to_leader(logits)
        return None if logits is None else logits[:, :V]

    def _norm_fold_step(self, T: int, fold: bool) -> bool:
        """This step runs the folded norm: gains folded at load, TP = 1, and
        every projection of the layer on K13 (prefill-sized T, no QKV bias,
        the 16-row gate/up interleave, residual epilogues on)."""
        if not (self.norm_folded and fold and ops.RESIDUAL_EPILOGUE and T > 256
                and self.gu_block == ops.SWIGLU16):
            return False
        L = self.w["layers"][0]
        if "bqkv" in L:
            return False
        d = self.cfg.hidden_size
        shapes = ((L["wqkv"], ops.ACT_NONE), (L["wo"], ops.ACT_NONE),
                  (L["w_gate_up"], ops.ACT_SWIGLU), (L["w_down"], ops.ACT_NONE))
        if torch.device(self.device).type == "cuda" and any(
                ops.rows_split(T, w.shape[0], w.shape[1], 3 if act else 0, w) for w, act in shapes):
            return False      # a decode-sized step split into <= 256-row pieces
        return d % 64 == 0 and all(
            ops.large_gemm_backend(T, w.shape[0], w.shape[1], act) == "k13"
            and ops.pgemm_supported(w.shape[0], w.shape[1], act) for w, act in shapes)

    def forward(self, inp: StepInputs, k_caches: list, v_caches: list,
                decode_ws: ops.DecodeWorkspace | None, part_tokens: int = 512) -> torch.Tensor:
        """Returns logits [len(sample_rows), vocab] (bf16)."""
        j = self._microbatch_split(inp)
        if j:
            return self._forward_tp_mb(inp, j, k_caches, v_caches)
        cfg, w = self.cfg, self.w
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        T, nd = inp.num_tokens, inp.num_decode
        tp = self.tp
        sp = tp.use_sp(T)
        if sp:
            # residual stream row-sharded: this rank owns rows [rank*s, (rank+1)*s)
            Tp = -(-T // tp.size) * tp.size
            s = Tp // tp.size
            ids = inp.input_ids
            if Tp > T:
                ids = torch.cat([ids, ids.new_zeros(Tp - T)])
            x = ops.embed_gather(w["embed"], ids[tp.rank * s:(tp.rank + 1) * s].contiguous())
        else:
            x = ops.embed_gather(w["embed"], inp.input_ids)
        residual = None
        attn = torch.empty((T, Hq * D), dtype=self.dtype, device=self.device)
        all_rows = inp.sample_rows.numel() == T     # decode: rows 0..T-1, each sampled
        # TP = 1 prefill: O / down on K13 add into the residual stream in their
        # epilogue (ops.residual_gemm_ok); x is then None and the next norm
        # reads the residual alone (two passes over the hidden rows fewer)
        # (a TP-rank proxy preset keeps the rank's bf16 O / down outputs)
        solo = tp.size == 1 and not cfg.proxy_tp
        fold = solo and not sp
        pending = None            # h of this layer from the previous layer's fused AR + norm
        layers = w["layers"]
        # the folded norm (prefill-sized TP = 1 steps): no norm pass at all --
        # O / down's residual epilogue leaves per-64-column sums of squares,
        # ops.row_scale turns them into rsqrt(mean + eps), and QKV / gate-up
        # (gains folded into their weights) scale their output rows by it
        nf = self._norm_fold_step(T, fold)
        part = (torch.empty((T, cfg.hidden_size // 64), dtype=torch.float32, device=self.device)
                if nf else None)
        s_row = None
        for li, L in enumerate(layers):
            h = None
            if pending is not None:
                h, pending = pending, None
            elif residual is None:
                residual = x
                if nf:
                    s_row = ops.row_scale(cfg.rms_eps, x=x)
                else:
                    h = ops.rms_norm(x, L["ln1"], cfg.rms_eps)
            elif x is None:
                if nf:
                    s_row = ops.row_scale(cfg.rms_eps, part=part, cols=cfg.hidden_size)
                else:
                    h = ops.rms_norm(residual, L["ln1"], cfg.rms_eps)
            else:
                h = ops.rms_norm(x, L["ln1"], cfg.rms_eps, residual=residual)
            if sp:
                h = tp.all_gather_rows(h)[:T]
            if nf:
                qkv = ops.pgemm(residual, L["wqkv"], row_scale=s_row)
            else:
                qkv = ops.linear(h, L["wqkv"], bias=L.get("bqkv"))   # Qwen2: biased q/k/v
            kc, vc = k_caches[li], v_caches[li]
            # decode rows: rotary + cache write fused into the decode attention
            # kernel (one launch and one boundary fewer per layer); prefill rows
            # (and q/k-norm models) keep the rope/cache kernels
            fuse = nd > 0 and self.fuse_decode_rope and "q_norm" not in L
            # prefill rows: q rotated inside the prefill attention kernel (the
            # rope/cache kernel then only rotates k and writes the cache)
            fuse_pf = T > nd and self.fuse_prefill_rope and "q_norm" not in L and qkv.is_cuda
            if fuse_pf:
                if nd > 0 and not fuse:
                    ops.rope_and_cache(qkv[:nd], inp.positions[:nd], self.cos_sin, Hq, Hkv, D,
                                       inp.slots[:nd], kc, vc, tile_from=nd, eps=cfg.rms_eps)
                ops.rope_and_cache(qkv[nd:], inp.positions[nd:], self.cos_sin, Hq, Hkv, D,
                                   inp.slots[nd:], kc, vc, tile_from=0, eps=cfg.rms_eps,
                                   skip_q=True)
            elif not fuse:
                ops.rope_and_cache(qkv, inp.positions, self.cos_sin, Hq, Hkv, D, inp.slots, kc,
                                   vc, tile_from=nd, q_norm=L.get("q_norm"),
                                   k_norm=L.get("k_norm"), eps=cfg.rms_eps)
            elif T > nd:
                ops.rope_and_cache(qkv[nd:], inp.positions[nd:], self.cos_sin, Hq, Hkv, D,
                                   inp.slots[nd:], kc, vc, tile_from=0, eps=cfg.rms_eps)
            if nd > 0:
                ops.paged_decode_attention(qkv[:nd], kc, vc, inp.block_tables,
                                           inp.context_lens, self.scale, attn[:nd], decode_ws,
                                           part_tokens, Hq=Hq, order=inp.decode_order,
                                           rope=(inp.positions, self.cos_sin, inp.slots)
                                           if fuse else None)
            if T > nd:
                ops.paged_prefill_attention(qkv, kc, vc, inp.block_tables[nd:],
                                            inp.cu_q[nd:], inp.context_lens[nd:],
                                            inp.prefill_tiles, self.scale, attn, Hq=Hq,
                                            rope=(inp.positions, self.cos_sin) if fuse_pf
                                            else None)
            # TP = 1: the O projection may hand its split-K partials straight
            # to the residual-add RMSNorm (ops.Partials; K11 epi 2)
            if nf:
                ops.pgemm(attn, L["wo"], residual=residual, ssq=part)
                s_row = ops.row_scale(cfg.rms_eps, part=part, cols=cfg.hidden_size)
            elif fold and ops.residual_gemm_ok(attn, L["wo"], residual):
                ops.pgemm(attn, L["wo"], residual=residual)
                h = ops.rms_norm(residual, L["ln2"], cfg.rms_eps)
            else:
                o = ops.linear(attn, L["wo"], defer=solo)
                if tp.size > 1 and not sp:
                    # one kernel: all-reduce + residual add + RMSNorm (peer memory)
                    h = tp.all_reduce_norm(o, L["ln2"], cfg.rms_eps, residual)
                else:
                    if sp:
                        o = tp.reduce_scatter_rows(o, Tp)
                    h = ops.rms_norm(o, L["ln2"], cfg.rms_eps, residual=residual)
            if sp:
                h = tp.all_gather_rows(h)[:T]
            if nf:
                a = ops.pgemm(residual, L["w_gate_up"], act=ops.ACT_SWIGLU, row_scale=s_row)
            elif self.gu_block:
                a = ops.linear_swiglu(h, L["w_gate_up"], self.gu_block)
            else:
                a = ops.silu_mul(ops.linear(h, L["w_gate_up"]))
            # down's partials go to the next layer's input norm (not after the
            # last layer: the final norm runs on the sampled rows only)
            # the last layer's partials go to the final norm when every row is
            # sampled (pure decode): no gather of the sampled rows is needed
            if nf:
                ops.pgemm(a, L["w_down"], residual=residual, ssq=part)
                x = None
                continue
            if fold and ops.residual_gemm_ok(a, L["w_down"], residual):
                ops.pgemm(a, L["w_down"], residual=residual)
                x = None
                continue
            x = ops.linear(a, L["w_down"], defer=solo and
                           (li + 1 < len(layers) or all_rows))
            if tp.size > 1:
                if sp:
                    x = tp.reduce_scatter_rows(x, Tp)
                elif li + 1 < len(layers):
                    # the next layer's input norm fused into this all-reduce
                    pending = tp.all_reduce_norm(x, layers[li + 1]["ln1"], cfg.rms_eps,
                                                 residual)
                    x = None
                elif all_rows:
                    pending = tp.all_reduce_norm(x, w["norm"], cfg.rms_eps, residual)
                    x = None
                else:
                    x = tp.all_reduce(x)
        # final norm only on the rows we sample from
        rows = inp.sample_rows
        if pending is not None:
            hs = pending          # decode under TP: the final norm fused into the last all-reduce
        elif x is None:
            hs = ops.rms_norm(residual if all_rows else residual.index_select(0, rows),
                              w["norm"], cfg.rms_eps)
        elif sp:
            hs = tp.all_gather_rows(ops.rms_norm(x, w["norm"], cfg.rms_eps,
                                                 residual=residual))[:T].index_select(0, rows)
        elif all_rows:
            hs = ops.rms_norm(x, w["norm"], cfg.rms_eps, residual=residual)
        else:
            xs = x.index_select(0, rows)
            rs = residual.index_select(0, rows)
            hs = ops.rms_norm(xs, w["norm"], cfg.rms_eps, residual=rs)
        logits = ops.linear(hs, w["lm_head"])
        if self.tp.size > 1:
            logits = self._tp_logits(logits)
        return logits
