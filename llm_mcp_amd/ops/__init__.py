"""Device ops of llm_mcp_amd.

Every op dispatches on the tensor's device:
  * GPU (ROCm/HIP) tensors -> the hand-written gfx950 kernels in
    ``_lmx_kernels`` (csrc/kernels/*.hip).  If that extension is missing on a
    GPU host the op raises -- there is no silent eager fallback.
  * CPU tensors -> the PyTorch reference in ``ops.ref`` (tests and the CPU
    plumbing configuration).

Shapes, dtypes, contiguity and strides are validated here, on the host,
before any launch, so a kernel never runs on operands that disagree with its
grid assumptions.
"""
from __future__ import annotations

import importlib
import os

import torch

from . import ref

_K = None
_K_ERR: Exception | None = None


class _SyncedKernels:
    """LMX_DEBUG_SYNC=1: every kernel launch is followed by a device
    synchronize, so an asynchronous fault (bad address, NaN trap, a hung
    wave) is reported by the launch that caused it, named, instead of by a
    later unrelated call -- the HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL
    style debug mode of SURVEY §5.2 for this package's own kernels.  The
    engine disables hipGraph capture in this mode."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn

        def call(*a, **kw):
            r = fn(*a, **kw)
            if not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    raise RuntimeError(f"lmx kernel {name} faulted: {e}") from e
            return r
        return call


def debug_sync() -> bool:
    import os
    return os.environ.get("LMX_DEBUG_SYNC", "0") == "1"


def native():
    """The loaded kernel extension (raises with the build hint if absent)."""
    global _K, _K_ERR
    if _K is None and _K_ERR is None:
        try:
            _K = importlib.import_module("llm_mcp_amd._lmx_kernels")
            if debug_sync():
                _K = _SyncedKernels(_K)
        except Exception as e:  # pragma: no cover - depends on the build
            _K_ERR = e
    if _K is None:
        raise RuntimeError(
            "llm_mcp_amd HIP kernels are not built (python -m llm_mcp_amd.build): "
            f"{_K_ERR}")
    return _K


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _chk(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _bf16(t: torch.Tensor, name: str) -> None:
    _chk(t.dtype == torch.bfloat16, f"{name} must be bfloat16, got {t.dtype}")


# ------------------------------------------------------------------ norms ---
class Partials:
    """Split-K fp32 partial slabs [S, M, N] of a projection whose K reduction
    is deferred to the consuming kernel (dgemm epi 2 -> rms_norm)."""
    __slots__ = ("slabs", "S", "M", "N")

    def __init__(self, slabs: torch.Tensor, S: int, M: int, N: int):
        self.slabs, self.S, self.M, self.N = slabs, S, M, N

    @property
    def shape(self):
        return (self.M, self.N)

    def sum(self) -> torch.Tensor:
        return self.slabs.sum(0)


def rms_norm(x, w: torch.Tensor, eps: float,
             residual: torch.Tensor | None = None,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """y = rmsnorm(x [+ residual]) * w.  With ``residual`` the sum is written
    back into ``residual`` (fused residual add).  ``x`` may be row-strided, or
    ``Partials`` (deferred split-K slabs, summed here; needs ``residual``)."""
    if isinstance(x, Partials):
        _chk(residual is not None and residual.is_contiguous()
             and residual.shape == (x.M, x.N), "rms_norm over partials needs the residual")
        if out is None:
            out = torch.empty((x.M, x.N), dtype=residual.dtype, device=residual.device)
        native().rmsnorm_slabs(_ptr(out), _ptr(residual), _ptr(x.slabs), x.S, x.M * x.N,
                               _ptr(w), x.M, x.N, out.stride(0), float(eps), _stream())
        return out
    if not x.is_cuda:
        y = ref.rms_norm(x, w, eps, residual)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(x, "x"); _bf16(w, "w")
    rows, cols = x.shape
    _chk(x.stride(1) == 1 and w.numel() == cols and cols % 8 == 0, "rms_norm shape/stride")
    if residual is not None:
        _chk(residual.is_contiguous() and residual.shape == (rows, cols), "residual shape")
    if out is None:
        out = torch.empty((rows, cols), dtype=x.dtype, device=x.device)
    native().rmsnorm(_ptr(out), _ptr(residual), _ptr(x), _ptr(w), rows, cols, x.stride(0),
                     out.stride(0), float(eps), _stream())
    return out


def layer_norm(x, w, b, eps, residual=None):
    if not x.is_cuda:
        return ref.layer_norm(x, w, b, eps, residual)
    _bf16(x, "x")
    rows, cols = x.shape
    _chk(x.is_contiguous() and cols % 8 == 0, "layer_norm shape")
    out = torch.empty_like(x)
    native().layernorm(_ptr(out), _ptr(x), _ptr(residual), _ptr(w), _ptr(b), rows, cols,
                       float(eps), _stream())
    return out


# ------------------------------------------------------- rope / kv cache ----
def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                   Hq: int, Hkv: int, D: int, slots: torch.Tensor | None,
                   k_cache: torch.Tensor | None, v_cache: torch.Tensor | None,
                   rotate_k_inplace: bool = False, tile_from: int | None = None,
                   q_norm: torch.Tensor | None = None, k_norm: torch.Tensor | None = None,
                   eps: float = 1e-6, skip_q: bool = False) -> None:
    """In-place rotary on q (and k) heads of the fused QKV rows; k and v are
    scattered into the paged cache at ``slots`` (-1 = skip).  Rows from
    ``tile_from`` on (prefill chunks: consecutive slots) use the 32-token
    tiled kernel with coalesced transposed-V page writes; rows before it
    (decode: one token per page) the per-token kernel.  Default: all tiled.
    ``q_norm`` / ``k_norm`` ([D] weights, D = 128): per-head RMSNorm of q and
    k before the rotation (Qwen3), fused into the same pass.  ``skip_q``
    (tiled rows only, no norms): leave the q heads unrotated -- the prefill
    attention rotates q itself (``paged_prefill_attention(rope=...)``)."""
    if not qkv.is_cuda:
        q_keep = qkv[:, :Hq * D].clone() if skip_q else None
        ref.rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache,
                       rotate_k_inplace, q_norm, k_norm, eps)
        if skip_q:
            qkv[:, :Hq * D] = q_keep
        return
    _chk(not skip_q or (q_norm is None and not tile_from), "skip_q: tiled rows without q/k norms")
    if q_norm is not None:
        _chk(k_norm is not None and D == 128 and q_norm.numel() == D and k_norm.numel() == D
             and q_norm.dtype == torch.bfloat16 and k_norm.dtype == torch.bfloat16,
             "q_norm / k_norm: bf16 [128] both")
    _bf16(qkv, "qkv")
    T = qkv.shape[0]
    _chk(qkv.stride(1) == 1 and qkv.shape[1] >= (Hq + 2 * Hkv) * D, "qkv shape")
    _chk(positions.dtype == torch.int32 and positions.numel() >= T, "positions int32[T]")
    _chk(cos_sin.dtype == torch.float32 and cos_sin.shape[1] == D, "cos_sin [P, D] fp32")
    BS = 0
    if k_cache is not None:
        _chk(slots is not None and slots.dtype == torch.int32, "slots int32")
        _chk(k_cache.shape[1] == Hkv and k_cache.shape[3] == D and v_cache.dim() == 5
             and v_cache.shape[3] == D and v_cache.shape[4] == 4,
             "cache layout [NB,Hkv,BS,D] / [NB,Hkv,BS/4,D,4]")
        BS = k_cache.shape[2]
    native().rope_cache(_ptr(qkv), qkv.stride(0), _ptr(positions), _ptr(cos_sin), T, Hq, Hkv, D,
                        _ptr(slots), _ptr(k_cache), _ptr(v_cache), BS,
                        int(rotate_k_inplace), 0 if tile_from is None else int(tile_from),
                        _ptr(q_norm), _ptr(k_norm), float(eps), int(skip_q), _stream())


def kv_write(k, v, slots, k_cache, v_cache):
    if not k.is_cuda:
        ref.write_cache(k, v, slots, k_cache, v_cache)
        return
    T, Hkv, D = k.shape
    _chk(k.stride(2) == 1 and k.stride(1) == D and v.stride(0) == k.stride(0), "k/v layout")
    native().kv_write(_ptr(k), _ptr(v), k.stride(0), _ptr(slots), T, Hkv, D, _ptr(k_cache),
                      _ptr(v_cache), k_cache.shape[2], _stream())


# --------------------------------------------------------------- attention ---
class DecodeWorkspace:
    """Split-K scratch of the paged decode kernel, sized once (graph-safe)."""

    def __init__(self, max_batch: int, Hq: int, D: int, max_parts: int, device):
        self.max_parts = max_parts
        self.part_o = torch.empty((max_batch, Hq, max_parts, D), dtype=torch.float32,
                                  device=device)
        self.part_ml = torch.empty((max_batch, Hq, max_parts, 2), dtype=torch.float32,
                                   device=device)


def paged_decode_attention(q: torch.Tensor, k_cache, v_cache, block_tables, context_lens,
                           scale: float, out: torch.Tensor, ws: DecodeWorkspace | None = None,
                           part_tokens: int = 512, Hq: int | None = None,
                           order: torch.Tensor | None = None, rope: tuple | None = None
                           ) -> torch.Tensor:
    """q: [B, Hq*D] rows (row stride = q.stride(0)); out: [B, Hq*D].
    ``order`` (int32 [B], optional): a permutation of the rows, longest
    context first -- the workgroup dispatch order (``decode_order``).
    ``rope`` = (positions int32[B], cos_sin fp32[P, D], slots int32[B]): q is
    the UNROTATED fused QKV row ([q | k | v] heads); the kernel rotates q in
    registers and writes the step's rotated k and v into the cache at
    ``slots`` itself (K2 + K5 fused into K4: ``rope_and_cache`` is skipped for
    these rows; no q/k-norm models)."""
    B = q.shape[0]
    NB, Hkv, BS, D = k_cache.shape
    Hq = Hq or (q.shape[1] // D)
    if rope is not None and not q.is_cuda:
        positions, cos_sin, slots = rope
        ref.rope_cache(q, positions[:B], cos_sin, Hq, Hkv, D, slots[:B], k_cache, v_cache, False)
        rope = None
    if not q.is_cuda:
        o = ref.paged_decode(q[:, : Hq * D].reshape(B, Hq, D), k_cache, v_cache, block_tables,
                             context_lens, scale)
        out.copy_(o.reshape(B, Hq * D))
        return out
    _bf16(q, "q")
    _chk(D in (64, 128) and BS == 32, "paged decode kernel needs D in (64,128), BS=32")
    _chk(Hq % Hkv == 0 and Hq // Hkv <= 16, "GQA group must be <= 16")
    _chk(block_tables.dtype == torch.int32 and context_lens.dtype == torch.int32, "int32 meta")
    _chk(block_tables.shape[0] >= B and context_lens.numel() >= B, "meta rows")
    _chk(part_tokens % 128 == 0, "part_tokens % 128")
    if order is not None:
        _chk(order.dtype == torch.int32 and order.numel() >= B and order.is_cuda, "order int32[B]")
    max_parts = ws.max_parts if ws is not None else 1
    pos = cs = slots = None
    if rope is not None:
        pos, cs, slots = rope
        _chk(q.shape[1] >= (Hq + 2 * Hkv) * D, "fused rope: q rows must be whole QKV rows")
        _chk(pos.dtype == torch.int32 and pos.numel() >= B and slots.dtype == torch.int32
             and slots.numel() >= B, "fused rope: positions / slots int32[B]")
        _chk(cs.dtype == torch.float32 and cs.shape[1] == D and cs.is_contiguous(),
             "fused rope: cos_sin [P, D] fp32")
    native().paged_decode(_ptr(q), q.stride(0), _ptr(k_cache), _ptr(v_cache), _ptr(block_tables),
                          block_tables.stride(0), _ptr(context_lens), _ptr(order), _ptr(out),
                          out.stride(0),
                          _ptr(ws.part_o) if ws else 0, _ptr(ws.part_ml) if ws else 0, B, Hq, Hkv,
                          D, BS, float(scale), part_tokens, max_parts, _ptr(pos), _ptr(cs),
                          _ptr(slots), _stream())
    return out


def decode_order(context_lens) -> "np.ndarray":
    """Dispatch order of the decode attention workgroups: rows by context
    length, longest first (stable).  Measured at 256 rows with contexts
    535-791: 5.2-5.4 TB/s in row order, 5.5-5.7 sorted
    (tools/decode_attn_probe.py)."""
    import numpy as np
    return np.argsort(-np.asarray(context_lens, dtype=np.int64), kind="stable").astype(np.int32)


def paged_prefill_attention(q: torch.Tensor, k_cache, v_cache, block_tables, cu_q,
                            context_lens, tiles, scale: float, out: torch.Tensor,
                            causal: bool = True, Hq: int | None = None,
                            q_per_tile: int | None = None, rope=None) -> torch.Tensor:
    """Varlen prefill. q/out: [T, Hq*D] rows; tiles: int32 [(seq, q_start)]
    built with ``q_per_tile`` queries per tile (default
    ``prefill_q_per_tile(Hq, Hkv, D)``; the kernel's workgroup width follows
    from it).  ``rope`` = (positions int32 [rows], cos_sin fp32 [P, D]): q is
    unrotated and the kernel applies the rotary embedding (the rope/cache
    kernel ran with ``skip_q``)."""
    NB, Hkv, BS, D = k_cache.shape
    T = q.shape[0]
    Hq = Hq or (q.shape[1] // D)
    if rope is not None and not q.is_cuda:
        qr = q[:, :Hq * D].clone()
        ref.rope_cache(qr, rope[0], rope[1], Hq, 0, D, None, None, None, False, None, None, 1e-6)
        q = qr
    if not q.is_cuda:
        o = ref.paged_prefill(q[:, : Hq * D].reshape(T, Hq, D), k_cache, v_cache, block_tables,
                              cu_q, context_lens, scale, causal)
        a, b = int(cu_q[0]), int(cu_q[len(context_lens)])
        out[a:b].copy_(o.reshape(T, Hq * D)[a:b])
        return out
    _bf16(q, "q")
    _chk(D in (64, 128) and BS == 32, "paged prefill kernel needs D in (64,128), BS=32")
    _chk(Hq % Hkv == 0 and Hq // Hkv <= 16, "GQA group must be <= 16")
    _chk(tiles.dtype == torch.int32 and cu_q.dtype == torch.int32, "int32 meta")
    num_tiles = tiles.numel() // 2
    native().paged_prefill(_ptr(q), q.stride(0), _ptr(k_cache), _ptr(v_cache),
                           _ptr(block_tables), block_tables.stride(0), _ptr(cu_q),
                           _ptr(context_lens), _ptr(tiles), num_tiles, _ptr(out), out.stride(0),
                           Hq, Hkv, D, BS, float(scale), int(causal),
                           q_per_tile or prefill_q_per_tile(Hq, Hkv, D),
                           _ptr(rope[0]) if rope is not None else 0,
                           _ptr(rope[1]) if rope is not None else 0, _stream())
    return out


PREFILL_GROUPS_PER_WAVE = 2   # PF_NG in csrc/kernels/attention.hip
# waves per prefill workgroup at head dim 128 (4 or 8; head dim 64: 4).
# LMX_PREFILL_WAVES overrides (A/B).
PREFILL_WAVES_D128 = 4


def prefill_waves(D: int) -> int:
    import os
    if D != 128:
        return 4
    return int(os.environ.get("LMX_PREFILL_WAVES", PREFILL_WAVES_D128))


def prefill_q_per_tile(Hq: int, Hkv: int, D: int = 128) -> int:
    """Queries per prefill workgroup: waves (prefill_waves) x column groups
    x 16/G (column groups per wave: 4 at head dim 64, 2 at 128 --
    attention.hip pf_groups)."""
    return prefill_waves(D) * (4 if D == 64 else PREFILL_GROUPS_PER_WAVE) * (16 // (Hq // Hkv))


# ---------------------------------------------------------------- sampling ---
# race rounds of sample_race: a row still rejected after them (top-p 0.95:
# ~0.05^4) takes the argmax
RACE_ROUNDS = int(os.environ.get("LMX_RACE_ROUNDS", "4"))     # max_rounds + 1 exchanges


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           top_p: torch.Tensor, seeds: torch.Tensor, offsets: torch.Tensor,
           out_tok: torch.Tensor | None = None, out_lp: torch.Tensor | None = None,
           max_rounds: int = 32):
    B, V = logits.shape
    if not logits.is_cuda:
        return ref.sample(logits, temperature, top_k, top_p, seeds, offsets)
    _chk(logits.dtype in (torch.bfloat16, torch.float32) and logits.stride(1) == 1, "logits")
    _chk(temperature.dtype == torch.float32 and top_p.dtype == torch.float32, "fp32 params")
    _chk(top_k.dtype == torch.int32 and offsets.dtype == torch.int32, "int32 params")
    _chk(seeds.dtype == torch.int64, "int64 seeds")
    for t in (temperature, top_k, top_p, seeds, offsets):
        _chk(t.numel() >= B and t.is_cuda, "sampling param rows")
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=logits.device)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=logits.device)
    native().sample(_ptr(logits), int(logits.dtype == torch.bfloat16), logits.stride(0), B, V,
                    _ptr(temperature), _ptr(top_k), _ptr(top_p), _ptr(seeds), _ptr(offsets),
                    _ptr(out_tok), _ptr(out_lp), max_rounds, _stream())
    return out_tok, out_lp


def sample_race(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
                top_p: torch.Tensor, seeds: torch.Tensor, offsets: torch.Tensor,
                exchange=None, v0: int = 0, vocab: int | None = None, world: int = 1,
                out_tok: torch.Tensor | None = None, out_lp: torch.Tensor | None = None,
                max_rounds: int = RACE_ROUNDS):
    """K6-R: the truncated sampler in exponential-race form over a vocabulary
    shard (sampling.hip ``race_kernel``).  ``logits`` [B, Vs]: columns
    [v0, v0 + Vs) of the vocabulary (``vocab`` columns in all);
    ``exchange(rec)`` all-gathers the fp32 [B, 8] records of the ``world``
    shards in rank order ([world, B, 8]; None: one shard).  Every rank
    returns the same (tokens int32 [B], logprobs fp32 [B]); at ``world`` 1
    over the whole row it is the single-GPU form of the same sampler."""
    B, Vs = logits.shape
    V = Vs if vocab is None else vocab
    if exchange is None:
        exchange = lambda r: r.view(1, B, 8)   # noqa: E731 (slots keep an alias safe)
    if not logits.is_cuda:
        return ref.sample_race(logits, temperature, top_k, top_p, seeds, offsets, exchange,
                               v0, V, max_rounds)
    _chk(logits.dtype in (torch.bfloat16, torch.float32) and logits.stride(1) == 1, "logits")
    _chk(temperature.dtype == torch.float32 and top_p.dtype == torch.float32, "fp32 params")
    _chk(top_k.dtype == torch.int32 and offsets.dtype == torch.int32, "int32 params")
    _chk(seeds.dtype == torch.int64, "int64 seeds")
    for t in (temperature, top_k, top_p, seeds, offsets):
        _chk(t.numel() >= B and t.is_cuda, "sampling param rows")
    dev = logits.device
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=dev)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=dev)
    rec = torch.empty((B, 8), dtype=torch.float32, device=dev)
    st = torch.empty((B, 12), dtype=torch.float32, device=dev)
    k, bf, stream = native(), int(logits.dtype == torch.bfloat16), _stream()
    common = (_ptr(logits), bf, logits.stride(0), B, Vs, v0, V, _ptr(temperature), _ptr(top_k),
              _ptr(top_p), _ptr(seeds), _ptr(offsets))

    def phase(ph, rnd, g):
        _chk(g.shape == (world, B, 8) and g.is_contiguous() and g.dtype == torch.float32,
             "race records exchange")
        k.race_sample_phase(ph, rnd, max_rounds, *common, _ptr(g), world, _ptr(rec), _ptr(st),
                            _ptr(out_tok), _ptr(out_lp), stream)

    k.race_sample_phase(0, 0, max_rounds, *common, _ptr(rec), world, _ptr(rec), _ptr(st),
                        _ptr(out_tok), _ptr(out_lp), stream)    # phase 0 reads no records
    for rnd in range(max_rounds):       # one exchange per round (race_kernel phase 1)
        phase(1, rnd, exchange(rec))
    phase(2, max_rounds, exchange(rec))
    return out_tok, out_lp


def apply_penalties(logits: torch.Tensor, window: torch.Tensor, ngen: torch.Tensor,
                    pen: torch.Tensor, on: torch.Tensor | None = None,
                    v0: int = 0) -> torch.Tensor:
    """Repetition / presence / frequency penalties on logits [B, V] in place
    (K6 prologue).  window int32 [B, W<=64] right-aligned context tokens (-1
    padded), ngen int32 [B] generated tokens at its tail, pen fp32 [B, 3] =
    (repetition, presence, frequency); ``on`` int32 [1] device flag.  ``v0``:
    the logits are vocabulary columns [v0, v0 + V) (a TP rank's shard)."""
    B, V = logits.shape
    if not logits.is_cuda:
        if on is not None and int(on[0]) == 0:
            return logits
        return ref.apply_penalties(logits, window, ngen, pen, v0)
    _chk(logits.dtype == torch.bfloat16 and logits.stride(1) == 1, "bf16 logits rows")
    _chk(window.dtype == torch.int32 and window.is_contiguous() and window.shape[0] >= B
         and window.shape[1] <= 64, "penalty window")
    _chk(ngen.dtype == torch.int32 and pen.dtype == torch.float32 and pen.is_contiguous(),
         "penalty params")
    native().apply_penalties(_ptr(logits), logits.stride(0), B, V, _ptr(window), _ptr(ngen),
                             _ptr(pen), _ptr(on), window.shape[1], v0, _stream())
    return logits


# ------------------------------------------------------------ elementwise ---
def deinterleave_gate_up(x: torch.Tensor, block: int) -> torch.Tensor:
    """Inverse column permutation of ``interleave_gate_up(w, block)``'s output."""
    I = x.shape[-1] // 2
    return x.view(*x.shape[:-1], I // block, 2, block).transpose(-3, -2).reshape(x.shape)


def silu_mul(x: torch.Tensor, out: torch.Tensor | None = None, block: int = 0) -> torch.Tensor:
    """silu(gate) * up of a fused gate|up projection output; ``block`` > 0:
    the columns are interleaved per block (``interleave_gate_up(w, block)``)."""
    if not x.is_cuda:
        y = ref.silu_mul(deinterleave_gate_up(x, block) if block else x)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(x, "x")
    _chk(x.is_contiguous() and x.shape[-1] % 16 == 0, "silu_mul shape")
    I = x.shape[-1] // 2
    _chk(block % 8 == 0 and (block == 0 or I % block == 0), "silu_mul interleave block")
    rows = x.numel() // x.shape[-1]
    if out is None:
        out = torch.empty(x.shape[:-1] + (I,), dtype=x.dtype, device=x.device)
    native().glu(_ptr(out), _ptr(x), rows, I, 0, block, _stream())
    return out


def gelu_mul(x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        return ref.gelu_mul(x)
    _chk(x.is_contiguous() and x.shape[-1] % 16 == 0, "gelu_mul shape")
    I = x.shape[-1] // 2
    rows = x.numel() // x.shape[-1]
    out = torch.empty(x.shape[:-1] + (I,), dtype=x.dtype, device=x.device)
    native().glu(_ptr(out), _ptr(x), rows, I, 1, 0, _stream())
    return out


def embed_gather(table: torch.Tensor, ids: torch.Tensor, vocab_start: int = 0,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Rows of ``table`` (a vocab shard starting at vocab_start); ids outside
    the shard give zero rows."""
    rows, d = table.shape
    if not table.is_cuda:
        local = ids.long() - vocab_start
        own = (local >= 0) & (local < rows)
        y = table[local.clamp(0, rows - 1)] * own[:, None].to(table.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _chk(ids.dtype == torch.int32 and table.is_contiguous() and d % 8 == 0, "embed_gather")
    T = ids.numel()
    if out is None:
        out = torch.empty((T, d), dtype=table.dtype, device=table.device)
    native().embed_gather(_ptr(out), _ptr(table), _ptr(ids), T, d, vocab_start, rows, _stream())
    return out


def ids_from_prev(ids: torch.Tensor, src: torch.Tensor, prev: torch.Tensor) -> torch.Tensor:
    """In place: ids[i] = prev[src[i]] where src[i] >= 0 (lookahead decode: the
    input token of a row is the previous step's sample src[i], still on the
    device when the step is launched)."""
    if not ids.is_cuda:
        m = src >= 0
        ids[m] = prev[src[m].long()]
        return ids
    _chk(ids.dtype == src.dtype == prev.dtype == torch.int32 and ids.numel() == src.numel()
         and ids.is_contiguous() and src.is_contiguous(), "ids_from_prev")
    native().ids_from_prev(_ptr(ids), _ptr(src), _ptr(prev), ids.numel(), _stream())
    return ids


def mean_pool_l2(h: torch.Tensor, cu: torch.Tensor, dims: int | None = None,
                 normalize: bool = True) -> torch.Tensor:
    T, d = h.shape
    dims = dims or d
    if not h.is_cuda:
        return ref.mean_pool_l2(h, cu, dims, normalize)
    _chk(h.is_contiguous() and d % 8 == 0 and 0 < dims <= d and cu.dtype == torch.int32,
         "mean_pool_l2")
    nseq = cu.numel() - 1
    out = torch.empty((nseq, dims), dtype=torch.float32, device=h.device)
    # one block per sequence when that already gives >= half the row-tiled
    # grid (many short sequences); row-tiled two-stage pooling otherwise
    acc = None if 2 * nseq >= (T + POOL_ROWS - 1) // POOL_ROWS else \
        torch.empty((nseq, d), dtype=torch.float32, device=h.device)
    native().mean_pool_l2(_ptr(out), 0 if acc is None else _ptr(acc), _ptr(h), _ptr(cu), nseq, T,
                          d, dims, int(normalize), _stream())
    return out


POOL_ROWS = 32  # rows per block of the two-stage pooling kernel (elementwise.hip)


ACT_NONE, ACT_GELU, ACT_SILU = 0, 1, 2


ACT_SWIGLU = 3
ACT_GELU_ERF = 4   # exact (erf) GELU, BERT FFNs


def interleave_gate_up(w: torch.Tensor, block: int = 64) -> torch.Tensor:
    """[gate(I); up(I)] rows -> per ``block`` channels [gate block | up block],
    the layout of the fused SwiGLU epilogues (gemm_nt act=3: block 64;
    dgemm epi=1: block BN/2)."""
    I2, d = w.shape
    I = I2 // 2
    _chk(I % block == 0, f"intermediate size must be a multiple of {block}")
    return w.view(2, I // block, block, d).transpose(0, 1).reshape(I2, d).contiguous()


def deinterleave_gate_up_rows(w: torch.Tensor, block: int) -> torch.Tensor:
    """Inverse of ``interleave_gate_up`` (weight rows): back to [gate(I); up(I)]."""
    I2, d = w.shape
    I = I2 // 2
    return w.view(I // block, 2, block, d).transpose(0, 1).reshape(I2, d).contiguous()


def gemm_nt(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: int = 0,
            residual: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """act(a @ w^T + bias) (+ residual) on the hand-written MFMA GEMM.
    act=3 (ACT_SWIGLU): ``w`` from ``interleave_gate_up``; returns
    silu(gate) * up with N/2 columns.
    (A 256-row ring variant was measured and dropped: profiles/r1_gemm256_study.md.)"""
    M, K = a.shape
    N = w.shape[0]
    if act == ACT_SWIGLU:
        _chk(bias is None and residual is None, "SwiGLU epilogue takes no bias/residual")
        if not a.is_cuda:
            I = N // 2
            y = (a.float() @ w.float().t()).view(M, I // 64, 2, 64)
            y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, I).to(a.dtype)
            if out is not None:
                out.copy_(y)
                return out
            return y
    if not a.is_cuda:
        y = ref.gemm_nt(a, w, bias, act, residual)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(a, "a"); _bf16(w, "w")
    _chk(w.shape[1] == K and a.stride(1) == 1 and w.stride(1) == 1, "gemm_nt shapes")
    _chk(N % 128 == 0 and K % 64 == 0, "gemm_nt needs N % 128 == 0 and K % 64 == 0")
    if out is None:
        out = torch.empty((M, N // 2 if act == ACT_SWIGLU else N), dtype=a.dtype,
                          device=a.device)
    # the epilogue stores / loads 4 bf16 (8 B) per lane
    _chk(out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0,
         "gemm_nt output rows must be 8-B aligned")
    _chk(bias is None or bias.data_ptr() % 8 == 0, "gemm_nt bias must be 8-B aligned")
    if residual is not None:
        _chk(residual.shape == (M, N) and residual.stride(0) == out.stride(0)
             and residual.data_ptr() % 8 == 0, "residual")
    native().gemm_nt(_ptr(out), _ptr(a), _ptr(w), _ptr(bias), _ptr(residual), M, N, K,
                     a.stride(0), w.stride(0), out.stride(0), act, _stream())
    return out


def gemm_nt_supported(N: int, K: int) -> bool:
    return N % 128 == 0 and K % 64 == 0


# ------------------------------------------------------- decode GEMM (M<=256) --
_SK_WS: dict = {}        # (device, stream) -> (slabs fp32, tickets int32)
SPLITK_MAX_M = 256


def splitk_splits(N: int, K: int, target_blocks: int = 256) -> int:
    """K-split so that (N/64) * splits ~ one workgroup per CU (guide: 'Projection
    GEMM at M = 256', decomposition first)."""
    tiles = N // 64
    s = max(1, min(8, round(target_blocks / max(1, tiles))))
    while s > 1 and K % (s * 64) != 0:
        s -= 1
    return s


def gemm_splitk_supported(M: int, N: int, K: int) -> bool:
    return 0 < M <= SPLITK_MAX_M and N % 64 == 0 and K % 64 == 0


# workspaces a larger request replaced: kept alive for the process lifetime,
# because decode graphs captured earlier have their addresses baked in (a
# freed buffer could be handed to another tensor while a graph still writes
# its slabs there)
_RETIRED_WS: list = []


def _retire_ws(ws) -> None:
    if ws is not None:
        _RETIRED_WS.append(ws)


def _sk_workspace(dev: torch.device, n_floats: int, n_tickets: int):
    key = (dev.index, _stream())
    ws = _SK_WS.get(key)
    if ws is None or ws[0].numel() < n_floats or ws[1].numel() < n_tickets:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("gemm_splitk workspace must be allocated before graph capture "
                               "(run the shape once eagerly)")
        n_floats = max(n_floats, ws[0].numel() if ws else 0)
        n_tickets = max(n_tickets, 4096, ws[1].numel() if ws else 0)
        ws = (torch.empty(n_floats, dtype=torch.float32, device=dev),
              torch.zeros(n_tickets, dtype=torch.int32, device=dev))
        _retire_ws(_SK_WS.get(key))
        _SK_WS[key] = ws
    return ws


def gemm_splitk(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
                splits: int | None = None) -> torch.Tensor:
    """a @ w^T for decode-sized M (<= 256) on the split-K MFMA kernel."""
    M, K = a.shape
    N = w.shape[0]
    if not a.is_cuda:
        y = ref.gemm_nt(a, w, None, 0, None)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(a, "a"); _bf16(w, "w")
    _chk(gemm_splitk_supported(M, N, K), f"gemm_splitk shape M={M} N={N} K={K}")
    _chk(w.shape[1] == K and a.stride(1) == 1 and w.stride(1) == 1, "gemm_splitk layout")
    _chk(a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0
         and w.data_ptr() % 16 == 0, "gemm_splitk operands need 16-B aligned rows")
    s = splits or splitk_splits(N, K)
    _chk(K % (s * 64) == 0, "K must split into 64-multiples")
    if out is None:
        out = torch.empty((M, N), dtype=a.dtype, device=a.device)
    _chk(out.shape == (M, N) and out.stride(1) == 1 and out.stride(0) % 4 == 0
         and out.data_ptr() % 8 == 0, "gemm_splitk output layout")
    slabs, tickets = (None, None)
    if s > 1:
        slabs, tickets = _sk_workspace(a.device, s * M * N, N // 64)
    native().gemm_splitk(_ptr(out), _ptr(a), _ptr(w), _ptr(slabs), _ptr(tickets), M, N, K,
                         a.stride(0), w.stride(0), out.stride(0), s, _stream())
    return out


def splitk_preferred(M: int, N: int, K: int) -> bool:
    """Measured dispatch (profiles/r1_splitk_gemm.md, cold weights on MI355X,
    Llama-3-8B and -70B shapes): the split-K kernel beats hipBLASLt for wide
    d=4096 gate/up projections at M <= 32, for long-K down projections
    (K >= 16384 at 48 <= M <= 256, K 8192-16384 at 48 <= M <= 160) and for
    d=4096 square projections at M <= 16; hipBLASLt wins elsewhere (incl. the
    70B QKV / O projections at K = 8192)."""
    if not gemm_splitk_supported(M, N, K):
        return False
    if N >= 16384 and K <= 4096:
        return M <= 32
    if K >= 16384:
        return 48 <= M <= 256
    if K > 8192:
        return 48 <= M <= 160
    if N == K and K <= 4096:
        return M <= 16
    return False


# decode batches above the decode kernels' 256 rows: K13's 256 x 256 tiles
# leave most of the CUs idle on the narrow projections (a 512-row step has 32
# tiles for O / down at d = 4096: 237 us for the down projection, 6x its
# 256-row K14 time), so such a product runs as equal row pieces of <= 256 rows
# on the decode kernels instead (profiles/r6_serving.md "512 streams")
ROWS_SPLIT_MAX = int(os.environ.get("LMX_ROWS_SPLIT_MAX", "1024"))   # largest batch split this way
ROWS_SPLIT_TILES = 128     # K13 tiles below which the product is split


def rows_split(M: int, N: int, K: int | None = None, epi: int = 0,
               w: torch.Tensor | None = None) -> int:
    """Row-piece size for an M-row product with N output columns, or 0 (one
    product): 256 < M <= ROWS_SPLIT_MAX, fewer than ROWS_SPLIT_TILES 256 x 256
    tiles and (given K) a packed-only weight, whose only other form is K13 with
    packed W (K14 then serves the pieces).  A row-major weight takes hipBLASLt
    there instead (``large_gemm_backend``: 1.1-1.9x faster than these pieces,
    profiles/r6_lab/rows_split_probe.log)."""
    if not (DGEMM_MAX_M < M <= ROWS_SPLIT_MAX) or -(-M // 256) * (N // 256) >= ROWS_SPLIT_TILES:
        return 0
    if K is not None and not (w is not None and is_packed_only(w)):
        return 0
    n = -(-M // DGEMM_MAX_M)
    return -(-M // n)


def _by_rows(x: torch.Tensor, piece: int, ncols: int, fn) -> torch.Tensor:
    """fn(rows, out) over row pieces of x, each written in place into its rows
    of one [M, ncols] result (no concatenation pass)."""
    y = torch.empty((x.shape[0], ncols), dtype=x.dtype, device=x.device)
    for i in range(0, x.shape[0], piece):
        fn(x[i:i + piece], y[i:i + piece])
    return y


def _into(out: torch.Tensor | None, y: torch.Tensor) -> torch.Tensor:
    if out is None or y.data_ptr() == out.data_ptr():
        return y
    return out.copy_(y)


def linear(x: torch.Tensor, w: torch.Tensor, defer: bool = False,
           bias: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """x @ w^T (+ bias): the decode GEMM (K11) where the measured table picks
    it, the older split-K kernel where it was measured faster, the large-M
    GEMM (K13) for prefill-sized M where ``large_gemm_backend`` picks it, else
    hipBLASLt (bias in its epilogue).  ``defer``: the caller feeds the result to
    ``rms_norm(..., residual=)``, so a table entry for the partials-only form
    (epi 2) may return ``Partials`` and leave the K reduction to the norm.
    ``out``: a bf16 [M, N] destination (plain products only, not with defer)."""
    _chk(out is None or not defer, "linear: out= is for the plain product")
    if x.is_cuda and x.dim() == 2 and (piece := rows_split(x.shape[0], w.shape[0], w.shape[1], 0, w)):
        return _by_rows(x, piece, w.shape[0], lambda xs, o: linear(xs, w, bias=bias, out=o))
    if is_packed_only(w):
        _chk(bias is None and x.is_cuda and x.dim() == 2, "packed-only weight: plain CUDA product")
        return _packed_product(x, w, 2 if defer and x.shape[0] <= 256 else 0, out=out)
    if x.is_cuda and x.dim() == 2:
        M, N, K = x.shape[0], w.shape[0], w.shape[1]
        if bias is None:
            rc = rs_choice(M, N, K, epi=2 if defer else 0, w=w)
            if rc is not None and rsgemm_operands_ok(x, w):
                return rsgemm(x, w, rc[0], rc[1], epi=2 if defer else 0, out=out)
        if defer and bias is None:
            s = sk_choice(M, N, K, epi=2)
            if s is not None and pgemm_operands_ok(x, w):
                return pgemm_sk(x, w, s, epi=2)
            ch = dgemm_choice(M, N, K, epi=2)
            if ch is not None:
                return dgemm_partials(x, w, ch[0], ch[1])
        s = sk_choice(M, N, K) if bias is None else None
        if s is not None and pgemm_operands_ok(x, w):
            return pgemm_sk(x, w, s, out=out)
        ch = dgemm_choice(M, N, K)
        y = None
        if ch is not None:
            y = dgemm(x, w, ch[0], ch[1], out=out)
        elif splitk_preferred(M, N, K):
            y = _into(out, gemm_splitk(x, w))
        if y is not None:
            if bias is not None:
                y += bias
            return y
        if (large_gemm_backend(M, N, K, 0, bias is not None) == "k13"
                and pgemm_operands_ok(x, w) and pgemm_bias_ok(bias, N)):
            return pgemm(x, w, bias=bias, out=out)
    return _into(out, torch.nn.functional.linear(x, w, bias))


def linear_swiglu(x: torch.Tensor, w: torch.Tensor, block: int,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """silu(gate) * up of x @ w^T for gate|up weights interleaved per
    ``block`` channels: the fused-epilogue decode GEMM where the table picks
    it, K13 with its SwiGLU epilogue for prefill-sized M (block 16), else the
    library GEMM + the GLU kernel.  block 16: the in-register
    epilogue over 16-column gate/up pairs (epi 3, any tile width); otherwise
    the LDS hand-off form (epi 1, tile BN = 2 * block)."""
    if x.is_cuda and x.dim() == 2 and (piece := rows_split(
            x.shape[0], w.shape[0], w.shape[1], 3 if block == SWIGLU16 else 1, w)):
        return _by_rows(x, piece, w.shape[0] // 2, lambda xs, o: linear_swiglu(xs, w, block, out=o))
    if is_packed_only(w):
        _chk(block == SWIGLU16 and x.is_cuda and x.dim() == 2,
             "packed-only gate/up: the SwiGLU16 interleave on CUDA")
        return _packed_product(x, w, 3, out=out)
    if x.is_cuda and x.dim() == 2:
        if block == SWIGLU16:
            rc = rs_choice(x.shape[0], w.shape[0], w.shape[1], epi=3, w=w)
            if rc is not None and rsgemm_operands_ok(x, w):
                return rsgemm(x, w, rc[0], rc[1], epi=3, out=out)     # K14, SwiGLU epilogue
            s = sk_choice(x.shape[0], w.shape[0], w.shape[1], epi=3)
            if s is not None and pgemm_operands_ok(x, w):
                return pgemm_sk(x, w, s, act=ACT_SWIGLU, out=out)   # K13-SK, SwiGLU epilogue
            ch = dgemm_choice(x.shape[0], w.shape[0], w.shape[1], epi=3)
            if ch is not None:
                return dgemm(x, w, ch[0], ch[1], epi=3, out=out)
            if (large_gemm_backend(x.shape[0], w.shape[0], w.shape[1], ACT_SWIGLU) == "k13"
                    and pgemm_operands_ok(x, w)):
                return pgemm(x, w, act=ACT_SWIGLU, out=out)     # K13 with the SwiGLU epilogue
        else:
            ch = dgemm_choice(x.shape[0], w.shape[0], w.shape[1], epi=1)
            if ch is not None and DGEMM_CONFIGS[ch[0] & DGEMM_CFG_MASK][1] == 2 * block:
                return dgemm(x, w, ch[0], ch[1], epi=1, out=out)
    return _into(out, silu_mul(linear(x, w), block=block))


def swiglu_block(N: int, K: int) -> int:
    """Interleave block of the gate|up weights for the fused decode GEMM of
    this shape: 16 when the table has in-register-epilogue (epi 3) entries,
    else BN/2 of the measured epi-1 configurations; 0 = not fused."""
    if (any(cfg >= 0 for m, cfg, s in _dg_table().get((N, K, 3), ())) or _sk_table().get((N, K, 3))
            or _rs_table().get((N, K, 3))):
        return SWIGLU16
    # one interleave serves every batch size, so take the tile width of the
    # largest-batch bucket the fused kernel won: buckets measured with another
    # width fall back to library + GLU (Llama-3-70B TP=1: 64-row buckets at BN
    # 128, the 128-row bucket at BN 256 -- the old smallest-width pick sent the
    # 128-row decode steps to the library + GLU, 228 vs 160 us per layer)
    best = max(((m, cfg) for m, cfg, s in _dg_table().get((N, K, 1), ()) if cfg >= 0),
               default=None)
    return DGEMM_CONFIGS[best[1] & DGEMM_CFG_MASK][1] // 2 if best else 0


def swiglu16_ok(cfg: int) -> bool:
    """Configuration can run the epi-3 (16-column pair) SwiGLU epilogue."""
    c = cfg & DGEMM_CFG_MASK
    return (DGEMM_CONFIGS[c][1] * DGEMM_WM[c] // 8) % 32 == 0


# ---------------------------------------------------------------------------
# K11: decode-shape projection GEMM (csrc/kernels/dgemm.hip)
# ---------------------------------------------------------------------------
# (BM, BN) of each kernel configuration id, in the order of kDgCfgs
DGEMM_CONFIGS = [(256, 128), (128, 128), (64, 128), (256, 64), (128, 64), (64, 64), (128, 256),
                 (64, 64), (128, 64), (64, 128), (128, 128), (128, 256), (256, 128), (256, 256),
                 (64, 64), (128, 64), (64, 128), (128, 128), (128, 256),
                 (64, 96), (128, 64), (64, 64), (128, 128), (256, 64), (64, 128),  # 19-25:
                 (64, 64),                                                          # 128-deep K
                 (64, 96), (64, 96), (64, 96),                       # 26-28: 64 x 96 tiles
                 (64, 96), (64, 96),                                 # 29-30: the same, 128-deep K
                 (64, 128)]                                          # 31: 64 x 128, 128-deep K
# waves along M of each configuration (dgemm.hip kDgCfgs): the fused SwiGLU on
# 16-column gate/up pairs (epi 3) needs a wave tile width BN*WM/8 divisible by 32
DGEMM_WM = [4, 2, 2, 8, 4, 2, 2, 2, 4, 2, 2, 2, 4, 4, 2, 4, 2, 2, 2,
            4, 4, 2, 2, 8, 2, 2,
            4, 4, 4, 4, 4, 2]
SWIGLU16 = 16              # gate/up interleave block of the epi-3 form
DGEMM_BK128 = (19, 20, 21, 22, 23, 24, 25, 29, 30, 31)  # configurations with 128-deep K-steps (K % (128 S) == 0)
DGEMM_MAX_M = 256
# a configuration id with bit 5 set (cfg | DGEMM_NT) streams the weights
# non-temporal (dgemm.hip NT): the low bits select the tile
DGEMM_NT, DGEMM_CFG_MASK = 32, 31
# cfg | DGEMM_SK: the stream-K form (dgemm.hip dgemm_sk_kernel + its reduction):
# ``splits`` is then the workgroup count G (0: one per CU), plain epilogue only
DGEMM_SK = 64
_DG_WS: dict = {}          # (device, stream) -> (slabs fp32, tickets uint32)
_DG_TICKETS = 8192
DGEMM_TABLE: dict | None = None
DGEMM_CALLS = [0]          # host-side launch count (tests: the K11 path really ran)


def _dg_table() -> dict:
    """Measured dispatch: {(N, K, epi): [(M_max, cfg, splits), ...]} from
    config/dgemm_gfx950.json (bench/dgemm_bench.py --write).  A shape or M
    absent from the table stays on hipBLASLt.  LMX_DGEMM=0 disables."""
    global DGEMM_TABLE
    if DGEMM_TABLE is None:
        import json
        import os
        DGEMM_TABLE = {}
        path = os.environ.get("LMX_DGEMM_TABLE") or os.path.join(
            os.path.dirname(os.path.dirname(__file__)), "config", "dgemm_gfx950.json")
        if os.environ.get("LMX_DGEMM", "1") == "1" and os.path.exists(path):
            with open(path) as f:
                raw = json.load(f)
            for e in raw.get("entries", []):
                key = (int(e["N"]), int(e["K"]), int(e.get("epi", 0)))
                DGEMM_TABLE.setdefault(key, []).append(
                    (int(e["m_max"]), int(e["cfg"]), int(e["splits"])))
            for v in DGEMM_TABLE.values():
                v.sort()
    return DGEMM_TABLE


_ENC_TABLE: dict | None = None


def _enc_table() -> dict:
    """{(N, K): encoder-table entry} (config dgemm_gfx950.json "encoder",
    bench/dgemm_bench.py --encoder: TF/s of K11's best tile, gemm_nt and
    hipBLASLt on prefill / encoder shapes at the largest M measured)."""
    global _ENC_TABLE
    if _ENC_TABLE is None:
        _ENC_TABLE = {}
        import json
        import os
        path = os.environ.get("LMX_DGEMM_TABLE") or os.path.join(
            os.path.dirname(os.path.dirname(__file__)), "config", "dgemm_gfx950.json")
        if os.environ.get("LMX_DGEMM", "1") == "1" and os.path.exists(path):
            with open(path) as f:
                for e in json.load(f).get("encoder", []):
                    _ENC_TABLE[(int(e["N"]), int(e["K"]))] = e
    return _ENC_TABLE


def encoder_choice(N: int, K: int) -> int | None:
    """K11 tile for a fused-epilogue encoder GEMM of this (N, K) (the SwiGLU
    gate/up projection), where K11 was measured faster than the older
    hand-written gemm_nt; None keeps gemm_nt."""
    e = _enc_table().get((N, K))
    if e is None or e.get("tflops") is None or e.get("cfg") is None:
        return None
    if e.get("gemm_nt_tflops") is None or e["tflops"] > e["gemm_nt_tflops"]:
        return int(e["cfg"])
    return None


def encoder_backend(N: int, K: int, act: int = 0,
                    bias: bool = False) -> tuple[str, int | None]:
    """Backend of an encoder projection of this (N, K) (+ bias / activation
    epilogue): the large-M hand-written GEMM K13 (("k13", None)) for every
    shape it takes.  LMX_ENCODER_LIBRARY=1 lets hipBLASLt (("lib", None))
    take the shapes where the encoder table (bench/dgemm_bench.py --encoder)
    measured it faster than K13.  Shapes K13 does not take: the faster
    measured of K11 (("k11", cfg)) and gemm_nt, gemm_nt when unmeasured."""
    import os
    e = _enc_table().get((N, K))
    if pgemm_supported(N, K, act, bias):
        if (os.environ.get("LMX_ENCODER_LIBRARY", "0") == "1" and e is not None
                and e.get("lib_tflops") and e.get("k13_tflops")
                and e["lib_tflops"] > e["k13_tflops"]):
            return ("lib", None)
        return ("k13", None)
    if e is None or e.get("tflops") is None or e.get("cfg") is None:
        return ("gemm_nt", None)
    cands = [(e["tflops"], "k11")]
    if e.get("gemm_nt_tflops") is not None:
        cands.append((e["gemm_nt_tflops"], "gemm_nt"))
    if e.get("lib_tflops") is not None and os.environ.get("LMX_ENCODER_LIBRARY", "0") == "1":
        cands.append((e["lib_tflops"], "lib"))
    best = max(cands)[1]
    return (best, int(e["cfg"]) if best == "k11" else None)


PGEMM_MIN_M = 512          # below: the decode-sized paths (K11 / split-K / library)
PGEMM_LIB_MARGIN = 0.05    # "auto": hipBLASLt only where measured > 5 % faster than K13
# K13 is persistent over 256 x 256 tiles on the 256 CUs, so a product of fewer
# tiles than about 1.5 waves takes a whole wave's time: at 512-1536 rows the
# narrow Llama-3-8B projections ran 1.1-2.6x slower on K13 than on hipBLASLt
# (QKV / O flat at ~72 / ~67 us from 512 to 1536 rows; tools/rows_split_probe.py,
# profiles/r6_lab/rows_split_probe.log).  Below this fraction of its last
# tile wave filled (first two waves only) a decode-sized product (<=
# ROWS_SPLIT_MAX rows, the captured decode-graph buckets) goes to the library;
# eager prefill / mixed steps of arbitrary row counts keep K13 (no per-shape
# library heuristics on the step path).
PGEMM_NUM_CUS = 256
PGEMM_MIN_FILL = float(os.environ.get("LMX_K13_MIN_FILL", "0.6"))


def k13_wave_fill(M: int, N: int) -> float:
    """Fraction of K13's last 256-CU tile wave an M x N product fills (1.0
    from two waves of tiles on: the rule only governs the first two)."""
    t = -(-M // 256) * -(-N // 256)
    if t >= 2 * PGEMM_NUM_CUS:
        return 1.0
    return t / (PGEMM_NUM_CUS * -(-t // PGEMM_NUM_CUS))


def large_gemm_backend(M: int, N: int, K: int, act: int = 0, bias: bool = False) -> str:
    """"k13" or "lib" for a large-M (prefill) projection.  LMX_LARGE_GEMM:
    "k13" / "lib" force one; "auto" (default) takes the faster of the two in
    the encoder table (config/dgemm_gfx950.json "encoder": k13_tflops vs
    lib_tflops, or k13_swiglu_tflops vs lib_glu_tflops for the fused SwiGLU
    form) -- the library only where it is more than PGEMM_LIB_MARGIN faster,
    since K13 also removes the neighbouring elementwise passes (a whole
    headline bench with every prefill projection on K13 measured 16,142 vs
    15,995 tok/s all-library, profiles/r3_k13_and_decode_sk.md) -- and K13 for
    unmeasured shapes."""
    import os
    if M < PGEMM_MIN_M or not pgemm_supported(N, K, act, bias):
        return "lib"
    mode = os.environ.get("LMX_LARGE_GEMM", "auto")
    if mode in ("k13", "lib"):
        return mode
    if M <= ROWS_SPLIT_MAX and k13_wave_fill(M, N) < PGEMM_MIN_FILL:
        return "lib"          # decode-sized batches only: prefill / mixed steps keep K13
    e = _enc_table().get((N, K))
    if e is None:
        return "k13"
    mine, lib = (("k13_swiglu_tflops", "lib_glu_tflops") if act == ACT_SWIGLU
                 else ("k13_tflops", "lib_tflops"))
    if e.get(mine) is None or e.get(lib) is None:
        return "k13"
    return "k13" if e[mine] >= (1.0 - PGEMM_LIB_MARGIN) * e[lib] else "lib"


_SK_TABLE: dict | None = None


def _sk_table() -> dict:
    """Measured K13-SK dispatch: {(N, K, epi): [(m_min, m_max, splits), ...]}
    from config/dgemm_gfx950.json "sk" (tools/pgemm_sk_probe.py: shapes and
    batch ranges where the split-K 256x256 tile beat K11 / hipBLASLt).  epi 0
    plain, 2 partials for the residual-add RMSNorm, 3 SwiGLU (16-row gate/up
    interleave).  LMX_DGEMM=0 or LMX_SK=0 disables."""
    global _SK_TABLE
    if _SK_TABLE is None:
        import json
        import os
        _SK_TABLE = {}
        path = os.environ.get("LMX_DGEMM_TABLE") or os.path.join(
            os.path.dirname(os.path.dirname(__file__)), "config", "dgemm_gfx950.json")
        if (os.environ.get("LMX_DGEMM", "1") == "1" and os.environ.get("LMX_SK", "1") == "1"
                and os.path.exists(path)):
            with open(path) as f:
                for e in json.load(f).get("sk", []):
                    _SK_TABLE.setdefault((int(e["N"]), int(e["K"]), int(e.get("epi", 0))), []).append(
                        (int(e["m_min"]), int(e["m_max"]), int(e["splits"])))
    return _SK_TABLE


def sk_choice(M: int, N: int, K: int, epi: int = 0) -> int | None:
    """Split count of K13-SK for this decode GEMM, or None."""
    for m_min, m_max, s in _sk_table().get((N, K, epi), ()):
        if (m_min <= M <= m_max and pgemm_sk_supported(M, N, K, s)
                and (epi != 2 or s in (1, 2, 4, 8, 16))):     # rmsnorm_slabs' S
            return s
    return None


def dgemm_choice(M: int, N: int, K: int, epi: int = 0) -> tuple[int, int] | None:
    """(cfg, splits) for this decode GEMM, or None (use the library)."""
    if not 0 < M <= DGEMM_MAX_M:
        return None
    for m_max, cfg, s in _dg_table().get((N, K, epi), ()):
        if M <= m_max:
            return (cfg, s) if cfg >= 0 else None   # cfg -1: the library won this bucket
    return None


def _dg_workspace(dev: torch.device, n_floats: int):
    key = (dev.index, _stream())
    ws = _DG_WS.get(key)
    if ws is None or ws[0].numel() < n_floats:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dgemm workspace must be allocated before graph capture "
                               "(run the shape once eagerly)")
        n_floats = max(n_floats, ws[0].numel() if ws else 0, 1 << 20)
        tickets = ws[1] if ws else torch.zeros(_DG_TICKETS, dtype=torch.int32, device=dev)
        ws = (torch.empty(n_floats, dtype=torch.float32, device=dev), tickets)
        _retire_ws(_DG_WS.get(key))
        _DG_WS[key] = ws
    return ws


def dgemm(a: torch.Tensor, w: torch.Tensor, cfg: int, splits: int, epi: int = 0,
          out: torch.Tensor | None = None) -> torch.Tensor:
    """a @ w^T for decode-sized M on the K11 kernel; epi=1: ``w`` interleaved
    per BN-column tile as [BN/2 gate | BN/2 up] rows (``interleave_gate_up``
    with ``block=BN/2``) and the result is silu(gate) * up (N/2 columns);
    epi=3: the same with ``w`` interleaved per 16 rows (block 16, any tile
    whose wave tile width is a multiple of 32, ``swiglu16_ok``)."""
    M, K = a.shape
    N = w.shape[0]
    bm, bn = DGEMM_CONFIGS[cfg & DGEMM_CFG_MASK]
    ncols = N // 2 if epi in (1, 3) else N
    sk = bool(cfg & DGEMM_SK)
    _chk(epi != 3 or swiglu16_ok(cfg), f"dgemm cfg {cfg} cannot run the epi-3 epilogue")
    _chk(not sk or epi == 0, "the stream-K form has the plain epilogue only")
    if not a.is_cuda:
        y = a.float() @ w.float().t()
        if epi in (1, 3):
            blk = SWIGLU16 if epi == 3 else bn // 2
            y = y.view(M, N // (2 * blk), 2, blk)
            y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, ncols)
        y = y.to(a.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(a, "a"); _bf16(w, "w")
    bk = 128 if (cfg & DGEMM_CFG_MASK) in DGEMM_BK128 else 64
    _chk(M > 0 and N % bn == 0 and K % (bk * (1 if sk else splits)) == 0 and splits >= 0,
         f"dgemm shape M={M} N={N} K={K} cfg={cfg} splits={splits}")
    _chk(w.shape[1] == K and a.stride(1) == 1 and w.stride(1) == 1, "dgemm layout")
    _chk(a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0
         and w.data_ptr() % 16 == 0, "dgemm operands need 16-B aligned rows")
    if out is None:
        out = torch.empty((M, ncols), dtype=a.dtype, device=a.device)
    _chk(out.shape == (M, ncols) and out.stride(1) == 1 and out.stride(0) % 4 == 0
         and out.data_ptr() % 8 == 0, "dgemm output layout")
    slabs = tickets = None
    if sk:
        slabs, tickets = _dg_workspace(a.device, native().dgemm_sk_pieces(M, N, K, cfg, splits)
                                       * M * N)
    elif splits > 1:
        _chk(-(-M // bm) * (N // bn) <= _DG_TICKETS, "dgemm tile count")
        slabs, tickets = _dg_workspace(a.device, splits * M * N)
    native().dgemm(_ptr(out), _ptr(a), _ptr(w), _ptr(slabs), _ptr(tickets), _DG_TICKETS, M, N, K,
                   a.stride(0), w.stride(0), out.stride(0), cfg, splits, epi, _stream())
    DGEMM_CALLS[0] += 1
    return out


def dgemm_partials(a: torch.Tensor, w: torch.Tensor, cfg: int, splits: int) -> Partials:
    """K11 with the partials-only epilogue: S fp32 slabs, no reduction pass
    (the consumer -- ``rms_norm`` -- sums them)."""
    M, K = a.shape
    N = w.shape[0]
    bm, bn = DGEMM_CONFIGS[cfg & DGEMM_CFG_MASK]
    _bf16(a, "a"); _bf16(w, "w")
    bk = 128 if (cfg & DGEMM_CFG_MASK) in DGEMM_BK128 else 64
    _chk(0 < M <= DGEMM_MAX_M and N % bn == 0 and K % (bk * splits) == 0,
         f"dgemm_partials shape M={M} N={N} K={K} cfg={cfg} splits={splits}")
    _chk(w.shape[1] == K and a.stride(1) == 1 and w.stride(1) == 1, "dgemm layout")
    _chk(a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0
         and w.data_ptr() % 16 == 0, "dgemm operands need 16-B aligned rows")
    slabs, tickets = _dg_workspace(a.device, splits * M * N)
    native().dgemm(0, _ptr(a), _ptr(w), _ptr(slabs), _ptr(tickets), _DG_TICKETS, M, N, K,
                   a.stride(0), w.stride(0), N, cfg, splits, 2, _stream())
    DGEMM_CALLS[0] += 1
    return Partials(slabs[:splits * M * N].view(splits, M, N), splits, M, N)


# ---------------------------------------------------------------------------
# K14: register-streamed decode GEMM, 129..256 rows (csrc/kernels/rsgemm.hip)
# ---------------------------------------------------------------------------
RS_BN = 256
RS_ROWMAJOR, RS_NT, RS_BM128, RS_BM64 = 64, 32, 4, 8   # cfg bits: row-major W, nt, 128 / 64-row tiles
RS_U = {0: 3, 2: 2}               # cfg & 3 -> K64 steps per ring block (D6 / D4)
RSGEMM_CALLS = [0]                # host-side launch count (tests: the K14 path ran)
_RS_TABLE: dict | None = None
_RS_WS: dict = {}
_RS_CNT = 4096


def _rs_table() -> dict:
    """Measured K14 dispatch: {(N, K, epi): [(m_min, m_max, cfg, splits)]} from
    config/dgemm_gfx950.json "rs" (tools/rsgemm_lab.cpp, cold weights, against
    K11 and the in-bench hipBLASLt times).  LMX_DGEMM=0 or LMX_RS=0 disables."""
    global _RS_TABLE
    if _RS_TABLE is None:
        import json
        import os
        _RS_TABLE = {}
        path = os.environ.get("LMX_DGEMM_TABLE") or os.path.join(
            os.path.dirname(os.path.dirname(__file__)), "config", "dgemm_gfx950.json")
        if (os.environ.get("LMX_DGEMM", "1") == "1" and os.environ.get("LMX_RS", "1") == "1"
                and os.path.exists(path)):
            with open(path) as f:
                for e in json.load(f).get("rs", []):
                    key = (int(e["N"]), int(e["K"]), int(e.get("epi", 0)))
                    ent = (int(e["m_min"]), int(e["m_max"]), int(e["cfg"]), int(e["splits"]))
                    _RS_TABLE.setdefault(key, []).append(ent)
                    # entries measured slower than K11 exist to serve packed-only
                    # weights (one copy: K11 cannot read the packed layout)
                    pts = [(v, e["k11_" + k]) for k, v in e.items()
                           if k.startswith("us_m") and isinstance(v, (int, float))
                           and isinstance(e.get("k11_" + k), (int, float))]
                    if pts and sum(a for a, _ in pts) > sum(b for _, b in pts):
                        _RS_PACKED_ONLY_ENTRIES.add(key + ent)
    return _RS_TABLE


_RS_PACKED_ONLY_ENTRIES: set = set()


def rsgemm_supported(M: int, N: int, K: int, cfg: int, splits: int, epi: int = 0) -> bool:
    """Shapes K14 takes: <= 256 rows, 256-column tiles, a K slice that is a
    whole number of the configuration's ring blocks; all-rows tiles (no 64 /
    128-row bit) only with the partials epilogue (the others spill there and
    are not built: rsgemm.hip, build.py ASM_RING_KERNELS)."""
    u = RS_U.get(cfg & 3)
    if u is None or not (0 < M <= 256 and N % RS_BN == 0 and splits in (1, 2, 4, 8, 16)
                         and K % (64 * splits) == 0):
        return False
    if not (cfg & (RS_BM64 | RS_BM128)) and epi != 2:
        return False
    nk = K // splits // 64
    return nk >= u and nk % u == 0


def rs_choice(M: int, N: int, K: int, epi: int = 0,
              w: torch.Tensor | None = None) -> tuple[int, int] | None:
    """(cfg, splits) of K14 for this decode GEMM, or None.  An entry on packed
    weights applies only when ``w`` has its packed copy (rs_prepare)."""
    for m_min, m_max, cfg, s in _rs_table().get((N, K, epi), ()):
        if (m_min <= M <= m_max and rsgemm_supported(M, N, K, cfg, s, epi)
                and (epi != 2 or s in (1, 2, 4, 8, 16))):     # rmsnorm_slabs' S
            if not (cfg & RS_ROWMAJOR) and _rs_packed_of(w) is None:
                continue
            # K11 is faster here and can read this weight's row-major copy
            if ((N, K, epi, m_min, m_max, cfg, s) in _RS_PACKED_ONLY_ENTRIES
                    and w is not None and not is_packed_only(w)):
                continue
            return cfg, s
    return None


def rsgemm_operands_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """Row-major layouts K14 reads directly (16-B aligned unit-stride rows)."""
    return (a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and a.stride(1) == 1
            and w.stride(1) == 1 and a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def _rs_workspace(dev: torch.device, n_floats: int):
    key = (dev.index, _stream())
    ws = _RS_WS.get(key)
    if ws is None or ws[0].numel() < n_floats:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("rsgemm workspace must be allocated before graph capture "
                               "(run the shape once eagerly)")
        n_floats = max(n_floats, ws[0].numel() if ws else 0, 1 << 20)
        cnt = ws[1] if ws else torch.zeros(_RS_CNT, dtype=torch.int32, device=dev)
        ws = (torch.empty(n_floats, dtype=torch.float32, device=dev), cnt)
        _retire_ws(_RS_WS.get(key))
        _RS_WS[key] = ws
    return ws


_RS_PACKED_BYTES = [0]             # live packed copies (a finalizer subtracts)


def _rs_packed_of(w: torch.Tensor | None) -> torch.Tensor | None:
    """The packed copy rs_prepare attached to this weight tensor object (the
    copy lives and dies with the weight: a freed weight's address reused by
    another tensor can never find a stale copy); a packed-only weight
    (rs_pack_only) is its own."""
    if w is None:
        return None
    if getattr(w, "_lmx_packed_only", False):
        return w
    return getattr(w, "_lmx_rs_packed", None)


# ---- one copy of the MLP weights (round 5) ---------------------------------
# A weight whose every consumer reads K14's packed layout is stored ONLY
# packed: decode batches (M <= 256) run K14 on it (the measured "rs" entry of
# the batch size, else rs_default's), prefill-sized M runs K13 with packed W
# (pgemm.hip WP).  No row-major copy is kept, so the model takes its own size
# in HBM and the KV pool gets the rest.  LMX_RS_SINGLE: 1 always, 0 never
# (row-major + packed copies), auto (default): one copy only when the model's
# weights take more than RS_SINGLE_FRACTION of the GPU's memory -- a small
# model keeps its row-major copy because K11 on it is faster than K14 below
# 129 rows (Llama-3-8B, +11.3 GB = 4 % of HBM: decode step 5.23 -> 4.72 ms at
# 64 rows, 6.70 -> 6.34 at 128, level at 256; profiles/r6_serving.md), while
# Llama-3-70B at TP = 1 (141 GB) stays on one copy.
RS_SINGLE_MODE = os.environ.get("LMX_RS_SINGLE", "auto")
RS_SINGLE_FRACTION = 0.25
RS_SINGLE = RS_SINGLE_MODE != "0"


def rs_single_wanted(weight_bytes: int, device: torch.device) -> bool:
    """Store the MLP weights packed-only (one copy) for a model of this size."""
    if RS_SINGLE_MODE in ("0", "1"):
        return RS_SINGLE_MODE == "1"
    if device.type != "cuda":
        return True
    total = torch.cuda.get_device_properties(device).total_memory
    return weight_bytes > RS_SINGLE_FRACTION * total


def is_packed_only(w: torch.Tensor | None) -> bool:
    return bool(getattr(w, "_lmx_packed_only", False))


def rs_single_ok(w: torch.Tensor, swiglu: bool = False) -> bool:
    """``w`` can be stored packed-only: a CUDA bf16 [N, K] weight of a shape
    the K14 table runs on packed weights, with K13 (packed W) taking its
    prefill-sized products -- the plain / residual product, or SwiGLU for a
    gate/up weight in the 16-row interleave (``swiglu``)."""
    if not (RS_SINGLE and w.is_cuda and w.dim() == 2 and w.dtype == torch.bfloat16
            and w.is_contiguous()):
        return False
    N, K = w.shape
    return (_rs_wants_packed(w) and pgemm_supported(N, K, ACT_SWIGLU if swiglu else 0)
            and rs_default(1, N, K, 3 if swiglu else 0) is not None)


def rs_pack_only(w: torch.Tensor) -> torch.Tensor:
    """The packed-only form of ``w`` (a new tensor; drop the row-major one)."""
    p = rsgemm_pack(w)
    p._lmx_packed_only = True
    return p


def rs_unpack(p: torch.Tensor) -> torch.Tensor:
    """Row-major [N, K] of a packed weight (references, export): packed is
    [N/256][8 waves][K/32][2 halves][4 k-chunks][16 rows][8]."""
    N, K = p.shape
    v = p.reshape(N // RS_BN, 8, K // 32, 2, 4, 16, 8)
    return v.permute(0, 1, 3, 5, 2, 4, 6).reshape(N, K)


def dense_weight(w: torch.Tensor) -> torch.Tensor:
    """``w`` row-major, whatever form the model keeps it in."""
    return rs_unpack(w) if is_packed_only(w) else w


def rs_default(M: int, N: int, K: int, epi: int) -> tuple[int, int] | None:
    """K14 configuration of a packed-only weight at a batch size the table
    has no entry for: 64-row tiles up to 64 rows, else 128-row; the fewest
    K slices that give >= 192 workgroups (K-slice partials: S <= 16)."""
    cfg = RS_NT | 2 | (RS_BM64 if M <= 64 else RS_BM128)
    tiles = -(-M // (64 if M <= 64 else 128)) * (N // RS_BN)
    ok = [s for s in (1, 2, 4, 8, 16) if rsgemm_supported(M, N, K, cfg, s, epi)]
    if not ok:
        return None
    for s in ok:
        if tiles * s >= 192:
            return cfg, s
    return cfg, ok[-1]


def _packed_product(x: torch.Tensor, w: torch.Tensor, epi: int,
                    out: torch.Tensor | None = None) -> torch.Tensor | Partials:
    """x @ w^T for a packed-only ``w``: K14 at decode batch sizes (epi 0 / 2
    partials / 3 SwiGLU16), K13 with packed W above 256 rows."""
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    if M <= 256:
        rc = rs_choice(M, N, K, epi=epi, w=w) or rs_default(M, N, K, epi)
        _chk(rc is not None and rsgemm_operands_ok(x, w),
             f"packed-only weight {tuple(w.shape)}: no K14 form for M={M} epi={epi}")
        return rsgemm(x, w, rc[0], rc[1], epi=epi, out=out)
    if not x.is_contiguous():
        x = x.contiguous()
    return pgemm(x, w, act=ACT_SWIGLU if epi == 3 else ACT_NONE, packed=True, out=out)


def _rs_wants_packed(w: torch.Tensor) -> bool:
    if not w.is_cuda or w.dim() != 2:
        return False
    N, K = w.shape
    if N % RS_BN or K % 32:
        return False
    return any(not (cfg & RS_ROWMAJOR) for ep in (0, 2, 3)
               for _, _, cfg, _ in _rs_table().get((N, K, ep), ()))


def _rs_attach_packed(w: torch.Tensor) -> None:
    import weakref
    nbytes = w.numel() * w.element_size()
    w._lmx_rs_packed = rsgemm_pack(w)
    _RS_PACKED_BYTES[0] += nbytes
    weakref.finalize(w, _rs_unpacked, nbytes)


def rs_prepare(w: torch.Tensor) -> bool:
    """One weight alone (tests, single layers): ``rs_prepare_all([w])``."""
    return bool(rs_prepare_all([w]).get(tuple(w.shape), False))


def rs_prepare_all(weights: list, budget_gb: float | None = None) -> dict:
    """Called once at model load with every decode weight: when the K14 table
    runs a weight shape on PACKED weights (an entry whose cfg lacks
    RS_ROWMAJOR), build the packed copies (rsgemm_pack) and attach them to the
    weight tensors, where ``rs_choice`` / ``rsgemm`` find them.

    The copies sit beside the row-major weights prefill reads, so they are
    bounded by ``LMX_RS_PACK_GB`` (default 24) -- decided per SHAPE, all or
    nothing: the bytes of every weight of a shape are summed and the shape is
    packed only if all of them fit (a running per-weight test would pack the
    first layers of a big model and leave the rest on another kernel, taking
    HBM from the KV cache for a mixed setup).  Returns {(N, K): packed}."""
    import logging
    import os
    if budget_gb is None:
        budget_gb = float(os.environ.get("LMX_RS_PACK_GB", "24"))
    budget = budget_gb * (1 << 30)
    groups: dict = {}
    for w in weights:
        if w is None or is_packed_only(w) or not _rs_wants_packed(w):
            continue
        groups.setdefault(tuple(w.shape), []).append(w)
    out = {}
    for shape, ws in groups.items():
        todo = [w for w in ws if _rs_packed_of(w) is None]
        need = sum(w.numel() * w.element_size() for w in todo)
        ok = _RS_PACKED_BYTES[0] + need <= budget
        if ok:
            for w in todo:
                _rs_attach_packed(w)
        out[shape] = ok
        logging.getLogger("lmx.ops").info(
            "K14 packed weights %s: %d tensors, %.2f GB -> %s (LMX_RS_PACK_GB=%g)", shape,
            len(ws), need / 2**30, "packed" if ok else "row-major (over budget)", budget_gb)
    return out


def _rs_unpacked(nbytes: int) -> None:
    _RS_PACKED_BYTES[0] -= nbytes


def rsgemm_pack(w: torch.Tensor) -> torch.Tensor:
    """``w`` [N, K] in K14's packed layout (each (tile, wave, K32 block,
    16-row half) one 1-KB run in MFMA fragment order).  Same element count."""
    _bf16(w, "w")
    N, K = w.shape
    _chk(N % RS_BN == 0 and K % 32 == 0 and w.stride(1) == 1 and w.stride(0) % 8 == 0,
         f"rsgemm_pack shape N={N} K={K}")
    out = torch.empty((N, K), dtype=w.dtype, device=w.device)
    native().rsgemm_pack(_ptr(out), _ptr(w), N, K, w.stride(0), _stream())
    return out


def rsgemm(a: torch.Tensor, w: torch.Tensor, cfg: int, splits: int, epi: int = 0,
           out: torch.Tensor | None = None, packed: bool = False):
    """a @ w^T on K14 (M <= 256).  epi 0: bf16 [M, N]; 2: fp32 ``Partials``
    [splits, M, N] for ``rms_norm(..., residual=)``; 3: SwiGLU over gate/up
    rows interleaved per 16 (``interleave_gate_up(w, 16)``), bf16 [M, N/2].
    ``w`` row-major (cfg | RS_ROWMAJOR) or from ``rsgemm_pack`` (``packed``)."""
    M, K = a.shape
    N = w.shape[0]
    if not packed and not (cfg & RS_ROWMAJOR) and a.is_cuda:
        # a table entry on packed weights: the copy rs_prepare built, else
        # the row-major form of the same ring shape
        wp = _rs_packed_of(w)
        if wp is not None:
            w, packed = wp, True
    if is_packed_only(w):
        packed = True           # the only copy there is, whatever the entry said
    cfg = (cfg & ~RS_ROWMAJOR) | (0 if packed else RS_ROWMAJOR)
    _chk(rsgemm_supported(M, N, K, cfg, splits, epi), f"rsgemm shape M={M} N={N} K={K} "
                                                 f"cfg={cfg} S={splits}")
    if not a.is_cuda:
        _chk(not packed, "rsgemm: the CPU reference takes row-major weights")
        y = a.float() @ w.float().t()
        if epi == 2:
            p = torch.cat([y.unsqueeze(0)] + [torch.zeros_like(y).unsqueeze(0)] * (splits - 1))
            return Partials(p, splits, M, N)
        if epi == 3:
            y = y.view(M, N // 32, 2, 16)
            y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, N // 2)
        y = y.to(a.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(a, "a"); _bf16(w, "w")
    _chk(w.shape[1] == K and rsgemm_operands_ok(a, w), "rsgemm operands need 16-B aligned rows")
    RSGEMM_CALLS[0] += 1
    if epi == 2:
        slabs, cnt = _rs_workspace(a.device, splits * M * N)
        native().rsgemm(0, _ptr(a), _ptr(w), _ptr(slabs), _ptr(cnt), _RS_CNT, M, N, K,
                        a.stride(0), w.stride(0), N, cfg, splits, 2, _stream())
        return Partials(slabs[:splits * M * N].view(splits, M, N), splits, M, N)
    ncols = N // 2 if epi == 3 else N
    if out is None:
        out = torch.empty((M, ncols), dtype=a.dtype, device=a.device)
    _chk(out.shape == (M, ncols) and out.stride(1) == 1 and out.stride(0) % 4 == 0
         and out.data_ptr() % 8 == 0, "rsgemm output layout")
    slabs = cnt = None
    if splits > 1:
        bm = 64 if cfg & RS_BM64 else 128 if cfg & RS_BM128 else 256
        _chk(-(-M // bm) * (N // RS_BN) <= _RS_CNT, "rsgemm tile count")
        slabs, cnt = _rs_workspace(a.device, splits * M * N)
    native().rsgemm(_ptr(out), _ptr(a), _ptr(w), _ptr(slabs), _ptr(cnt), _RS_CNT, M, N, K,
                    a.stride(0), w.stride(0), out.stride(0), cfg, splits, epi, _stream())
    return out


# ---------------------------------------------------------------------------
# K13: large-M GEMM (csrc/kernels/pgemm.hip): prefill chunks, encoder batches
# ---------------------------------------------------------------------------
PGEMM_MAX_BIAS = 8192
PGEMM_CALLS = [0]          # host-side launch count (tests: the K13 path really ran)
RESIDUAL_EPILOGUE = os.environ.get("LMX_RESIDUAL_EPILOGUE", "1") != "0"


def pgemm_supported(N: int, K: int, act: int = 0, bias: bool = False) -> bool:
    """Shapes K13 takes: 256-column tiles, 64-deep K-steps, >= 3 of them;
    a bias row fits its LDS slot; the SwiGLU form takes no bias."""
    return (N % 256 == 0 and K % 64 == 0 and K >= 192 and act in (0, 1, 2, 3, 4)
            and not (bias and (N > PGEMM_MAX_BIAS or act == ACT_SWIGLU)))


def pgemm_operands_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """Layouts K13 reads directly: unit-stride 16-B aligned rows."""
    return (a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and a.stride(1) == 1
            and w.stride(1) == 1 and a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def pgemm_bias_ok(bias: torch.Tensor | None, N: int) -> bool:
    """A bias K13 reads directly (else the caller keeps the library path)."""
    return bias is None or (bias.dtype == torch.bfloat16 and bias.numel() == N
                            and bias.is_contiguous() and bias.data_ptr() % 16 == 0)


def pgemm(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: int = 0,
          out: torch.Tensor | None = None, grid: int = 0,
          residual: torch.Tensor | None = None, packed: bool = False,
          row_scale: torch.Tensor | None = None,
          ssq: torch.Tensor | None = None) -> torch.Tensor:
    """act(a @ w^T + bias) on the persistent 256x256 MFMA GEMM (any M).
    act: ACT_NONE / ACT_GELU (tanh) / ACT_SILU / ACT_GELU_ERF, or ACT_SWIGLU
    with ``w`` from ``interleave_gate_up(w, 16)`` (result [M, N/2]).
    ``grid``: workgroups (0 = one per CU).  ``residual`` (bf16 [M, N], no
    bias / act): the product is added into it in the epilogue, in place, with
    the rounding of the separate pass it replaces -- residual = bf16(residual
    + bf16(a @ w^T)) -- and it is returned.  The losing design points of
    the kernel (tools/lab_kernels/pgemm_lab.hip) are lab-only."""
    M, K = a.shape
    N = w.shape[0]
    if not packed and bias is None and act in (ACT_NONE, ACT_SWIGLU) and a.is_cuda:
        # a row-major weight with K14's packed copy beside it (two copies):
        # prefill reads the packed one, as a packed-only weight would (WP)
        wp = _rs_packed_of(w)
        if wp is not None:
            w, packed = wp, True
    packed = packed or is_packed_only(w)
    _chk(not packed or (bias is None and act in (ACT_NONE, ACT_SWIGLU) and a.is_cuda),
         "pgemm on packed W: plain / residual / SwiGLU products on CUDA")
    ncols = N // 2 if act == ACT_SWIGLU else N
    if residual is not None:
        _chk(act == ACT_NONE and bias is None and out is None, "pgemm residual: plain product only")
        _chk(residual.shape == (M, N) and residual.dtype == a.dtype, "pgemm residual shape")
    if not a.is_cuda:
        if residual is not None:
            y = ref.gemm_nt(a, w, None, ACT_NONE, None)
            residual.copy_((residual.float() + y.float()).to(residual.dtype))
            if ssq is not None:
                ssq.copy_(residual.float().pow(2).view(M, N // 64, 64).sum(-1))
            return residual
        if row_scale is not None:
            y = (a.float() @ w.float().t()) * row_scale.float()[:, None]
            if act == ACT_SWIGLU:
                y = y.view(M, N // 32, 2, 16)
                y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, ncols)
            y = y.to(a.dtype)
            if out is not None:
                out.copy_(y)
                return out
            return y
        if act == ACT_SWIGLU:
            y = (a.float() @ w.float().t()).view(M, N // 32, 2, 16)
            y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, ncols).to(a.dtype)
        else:
            y = ref.gemm_nt(a, w, bias, act, None)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _bf16(a, "a"); _bf16(w, "w")
    _chk(pgemm_supported(N, K, act, bias is not None),
         f"pgemm shape N={N} K={K} act={act} bias={bias is not None}")
    _chk(w.shape[1] == K and a.stride(1) == 1 and w.stride(1) == 1 and a.stride(0) % 8 == 0
         and w.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0,
         "pgemm operands need 16-B aligned rows")
    if bias is not None:
        _bf16(bias, "bias")
        _chk(bias.numel() == N and bias.is_contiguous() and bias.data_ptr() % 16 == 0,
             "pgemm bias")
    if residual is not None:
        _chk(residual_gemm_layout_ok(residual), "pgemm residual layout (16-B rows)")
        out = residual
    nrm = None
    if ssq is not None:
        # the RMSNorm folded into the projections: the new residual rows' sums
        # of squares per 64-column block, for row_scale
        _chk(residual is not None and ssq.dtype == torch.float32 and ssq.is_contiguous()
             and ssq.shape == (M, N // 64), "pgemm ssq: fp32 [M, N/64] with the residual epilogue")
        nrm = ssq
    if row_scale is not None:
        _chk(residual is None and bias is None and row_scale.dtype == torch.float32
             and row_scale.is_contiguous() and row_scale.numel() == M,
             "pgemm row_scale: fp32 [M], plain product or SwiGLU")
        _chk(nrm is None, "pgemm: row_scale and ssq are exclusive")
        nrm = row_scale
    if out is None:
        out = torch.empty((M, ncols), dtype=a.dtype, device=a.device)
    _chk(out.shape == (M, ncols) and out.stride(1) == 1 and out.stride(0) % 4 == 0
         and out.data_ptr() % 8 == 0, "pgemm output layout")
    PGEMM_CALLS[0] += 1
    native().pgemm(_ptr(out), _ptr(a), _ptr(w), _ptr(bias), M, N, K, a.stride(0), w.stride(0),
                   out.stride(0), act, grid, int(residual is not None), int(packed), _ptr(nrm),
                   _stream())
    return out


def row_scale(eps: float, part: torch.Tensor | None = None,
              x: torch.Tensor | None = None, cols: int | None = None) -> torch.Tensor:
    """RMSNorm row scales rsqrt(mean(x^2) + eps), fp32 [M]: from the fixed
    per-64-column partial sums a residual epilogue wrote (``part`` [M, P],
    summed in slot order; ``cols`` = the row length), or from the bf16 rows of
    ``x`` (the first layer's input)."""
    if part is not None:
        M, P = part.shape
        cols = cols or 64 * P
        if not part.is_cuda:
            return torch.rsqrt(part.float().sum(-1) / cols + eps)
        s = torch.empty(M, dtype=torch.float32, device=part.device)
        native().row_scale(_ptr(s), _ptr(part), P, 0, 0, M, cols, float(eps), _stream())
        return s
    _chk(x is not None and x.dim() == 2, "row_scale: partials or rows")
    M, cols = x.shape
    if not x.is_cuda:
        return torch.rsqrt(x.float().pow(2).mean(-1) + eps)
    _bf16(x, "x")
    _chk(x.stride(1) == 1 and cols % 8 == 0, "row_scale rows")
    s = torch.empty(M, dtype=torch.float32, device=x.device)
    native().row_scale(_ptr(s), 0, 0, _ptr(x), x.stride(0), M, cols, float(eps), _stream())
    return s


def residual_gemm_layout_ok(residual: torch.Tensor) -> bool:
    """A residual stream K13's epilogue reads and writes in 16-B runs."""
    return (residual.dtype == torch.bfloat16 and residual.stride(1) == 1
            and residual.stride(0) % 8 == 0 and residual.data_ptr() % 16 == 0)


def residual_gemm_ok(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None) -> bool:
    """``residual += x @ w^T`` can run as K13 with the residual epilogue:
    the prefill-sized shapes ``linear`` sends to K13 (no decode-table kernel
    claims them), operands and the residual stream in K13's layouts.
    LMX_RESIDUAL_EPILOGUE=0 keeps the separate residual-add pass."""
    if residual is None or not x.is_cuda or x.dim() != 2 or not RESIDUAL_EPILOGUE:
        return False
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    if residual.shape != (M, N) or not residual_gemm_layout_ok(residual):
        return False
    if rows_split(M, N, K, 0, w):
        return False          # row pieces on the decode kernels (linear), not one K13 product
    if is_packed_only(w):
        return M > 256 and pgemm_operands_ok(x, w)
    if (rs_choice(M, N, K, epi=2, w=w) is not None or rs_choice(M, N, K, w=w) is not None
            or sk_choice(M, N, K, epi=2) is not None or sk_choice(M, N, K) is not None
            or dgemm_choice(M, N, K, epi=2) is not None or dgemm_choice(M, N, K) is not None
            or splitk_preferred(M, N, K)):
        return False
    return (large_gemm_backend(M, N, K, 0, False) == "k13" and pgemm_supported(N, K)
            and pgemm_operands_ok(x, w))


_PG_WS: dict = {}
_PG_CNT = 4096


def _pg_workspace(dev: torch.device, n_floats: int):
    key = (dev.index, _stream())
    ws = _PG_WS.get(key)
    if ws is None or ws[0].numel() < n_floats:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("pgemm_sk workspace must be allocated before graph capture "
                               "(run the shape once eagerly)")
        n_floats = max(n_floats, ws[0].numel() if ws else 0, 1 << 20)
        cnt = ws[1] if ws else torch.zeros(_PG_CNT, dtype=torch.int32, device=dev)
        ws = (torch.empty(n_floats, dtype=torch.float32, device=dev), cnt)
        _retire_ws(_PG_WS.get(key))
        _PG_WS[key] = ws
    return ws


def pgemm_sk_supported(M: int, N: int, K: int, splits: int) -> bool:
    """Shapes K13-SK takes: 256-column tiles, >= 2 64-deep K-steps per slice."""
    return (0 < M and N % 256 == 0 and splits >= 1 and K % (64 * splits) == 0
            and K // (64 * splits) >= 2 and 2 * (-(-M // 256)) * (N // 256) <= _PG_CNT)


def pgemm_sk(a: torch.Tensor, w: torch.Tensor, splits: int, act: int = 0, epi: int = 0,
             out: torch.Tensor | None = None):
    """act(a @ w^T) on K13-SK (the 256x256 ping-pong tile, split-K over
    ``splits`` slices, one workgroup per (slice, tile)): the decode-batch form
    (M <= 256).  epi 0: bf16 [M, N] ([M, N/2] for ACT_SWIGLU with ``w`` from
    ``interleave_gate_up(w, 16)``), slices combined in-kernel; epi 2: fp32
    ``Partials`` [splits, M, N] summed by ``rms_norm(..., residual=)``."""
    M, K = a.shape
    N = w.shape[0]
    _chk(pgemm_sk_supported(M, N, K, splits), f"pgemm_sk shape M={M} N={N} K={K} S={splits}")
    if not a.is_cuda:
        if epi == 2:
            y = (a.float() @ w.float().t()).unsqueeze(0)
            p = torch.cat([y] + [torch.zeros_like(y)] * (splits - 1))
            return Partials(p, splits, M, N)
        return pgemm(a, w, act=act, out=out)
    _bf16(a, "a"); _bf16(w, "w")
    _chk(w.shape[1] == K and pgemm_operands_ok(a, w), "pgemm_sk operands need 16-B aligned rows")
    tiles = -(-M // 256) * (N // 256)
    PGEMM_CALLS[0] += 1
    if epi == 2:
        slabs, cnt = _pg_workspace(a.device, splits * M * N)
        native().pgemm_sk(0, _ptr(a), _ptr(w), _ptr(slabs), _ptr(cnt), _PG_CNT, M, N, K,
                          a.stride(0), w.stride(0), N, 0, splits, 2, _stream())
        return Partials(slabs[:splits * M * N].view(splits, M, N), splits, M, N)
    ncols = N // 2 if act == ACT_SWIGLU else N
    if out is None:
        out = torch.empty((M, ncols), dtype=a.dtype, device=a.device)
    _chk(out.shape == (M, ncols) and out.stride(1) == 1 and out.stride(0) % 8 == 0
         and out.data_ptr() % 16 == 0, "pgemm_sk output layout")
    slabs = cnt = None
    if splits > 1:
        slabs, cnt = _pg_workspace(a.device, tiles * splits * 65536)
    native().pgemm_sk(_ptr(out), _ptr(a), _ptr(w), _ptr(slabs), _ptr(cnt), _PG_CNT, M, N, K,
                      a.stride(0), w.stride(0), out.stride(0), act, splits, 0, _stream())
    return out
