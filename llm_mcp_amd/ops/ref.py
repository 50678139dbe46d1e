"""Plain PyTorch (fp32-accumulating) reference implementations of every HIP
kernel in ``csrc/kernels``.

They serve two purposes:
* numerics oracle for the kernel parity tests (``tests/test_kernels_gpu.py``);
* the CPU execution path of the ops (tests, CPU-only plumbing configs).  A
  CUDA/HIP tensor never takes this path: ``ops.kernels`` dispatches device
  tensors to the native kernels and raises if the extension is missing.

Cache layouts match the kernels: k_cache [NB, Hkv, BS, D], v_cache [NB, Hkv, BS/4, D, 4]
(key-quad: v_cache[blk, h, key // 4, d, key % 4]).
"""
from __future__ import annotations

import math

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float,
             residual: torch.Tensor | None = None) -> torch.Tensor:
    if residual is not None:
        h = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(h)
        x = h
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def layer_norm(x, w, b, eps, residual=None):
    if residual is not None:
        x = (x.float() + residual.float()).to(x.dtype)
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(),
                                          eps).to(x.dtype)


def rope_cos_sin(max_pos: int, dim: int, theta: float, device=None,
                 scaling: dict | None = None) -> torch.Tensor:
    """[max_pos, dim] fp32 table: cos in [:, :dim/2], sin in [:, dim/2:]."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    if scaling and scaling.get("rope_type") == "llama3":
        # Llama-3.1 frequency-dependent scaling
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_wl, inv / factor, inv)
        mid = (wavelen <= lo_wl) & (wavelen >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] -> rotated (rotate-half form)."""
    D = x.shape[-1]
    cs = cos_sin[positions.long()]
    cos, sin = cs[:, None, : D // 2], cs[:, None, D // 2:]
    x1, x2 = x[..., : D // 2].float(), x[..., D // 2:].float()
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def head_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """Per-head RMSNorm over the last dim, kept in fp32 (Qwen3 q_norm/k_norm)."""
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, rotate_k_inplace,
               q_norm=None, k_norm=None, eps=1e-6):
    T = qkv.shape[0]
    v3 = qkv.view(T, -1, D)
    qh, kh = v3[:, :Hq], v3[:, Hq:Hq + Hkv]
    if q_norm is not None:
        qh, kh = head_norm(qh, q_norm, eps), head_norm(kh, k_norm, eps)
    q = apply_rope(qh, positions, cos_sin).to(qkv.dtype)
    k = apply_rope(kh, positions, cos_sin).to(qkv.dtype)
    v = v3[:, Hq + Hkv:Hq + 2 * Hkv]
    v3[:, :Hq] = q
    if rotate_k_inplace or k_cache is None:
        v3[:, Hq:Hq + Hkv] = k
    if k_cache is not None and slots is not None:
        write_cache(k, v, slots, k_cache, v_cache)


def write_cache(k, v, slots, k_cache, v_cache):
    BS = k_cache.shape[2]
    s = slots.long()
    keep = s >= 0
    s, k, v = s[keep], k[keep], v[keep]
    blk, off = s // BS, s % BS
    k_cache[blk, :, off, :] = k.to(k_cache.dtype)
    v_cache[blk, :, off // 4, :, off % 4] = v.to(v_cache.dtype)


def gather_kv(k_cache, v_cache, block_table, n):
    """Dense K, V [n, Hkv, D] of one sequence from the paged cache."""
    BS = k_cache.shape[2]
    idx = torch.arange(n, device=k_cache.device)
    blk = block_table.long()[idx // BS]
    off = idx % BS
    k = k_cache[blk, :, off, :]           # [n, Hkv, D]
    v = v_cache[blk, :, off // 4, :, off % 4]   # [n, Hkv, D]
    return k, v


def attention_dense(q, k, v, scale, causal_offset: int | None):
    """q [Tq, Hq, D], k/v [Tk, Hkv, D]; query i sees keys <= causal_offset + i."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    kf = k.float().repeat_interleave(G, dim=1)
    vf = v.float().repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal_offset is not None:
        Tq, Tk = q.shape[0], k.shape[0]
        qi = torch.arange(Tq, device=q.device)[:, None] + causal_offset
        ki = torch.arange(Tk, device=q.device)[None, :]
        s = s.masked_fill((ki > qi)[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf)


def paged_decode(q, k_cache, v_cache, block_tables, context_lens, scale):
    """q [B, Hq, D] -> [B, Hq, D] (one query per sequence at position ctx-1)."""
    out = torch.empty_like(q)
    for b in range(q.shape[0]):
        n = int(context_lens[b])
        k, v = gather_kv(k_cache, v_cache, block_tables[b], n)
        out[b] = attention_dense(q[b:b + 1], k, v, scale, None)[0].to(q.dtype)
    return out


def paged_prefill(q, k_cache, v_cache, block_tables, cu_q, context_lens, scale, causal=True):
    """q [T, Hq, D] for a varlen batch; keys come from the paged cache."""
    out = torch.empty_like(q)
    for s in range(len(context_lens)):
        a, b = int(cu_q[s]), int(cu_q[s + 1])
        n = int(context_lens[s])
        k, v = gather_kv(k_cache, v_cache, block_tables[s], n)
        off = (n - (b - a)) if causal else None
        out[a:b] = attention_dense(q[a:b], k, v, scale, off).to(q.dtype)
    return out


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    I = x.shape[-1] // 2
    g, u = x[..., :I].float(), x[..., I:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def gelu_mul(x: torch.Tensor) -> torch.Tensor:
    I = x.shape[-1] // 2
    g, u = x[..., :I].float(), x[..., I:].float()
    return (torch.nn.functional.gelu(g, approximate="tanh") * u).to(x.dtype)


def mean_pool_l2(h, cu, dims, normalize=True):
    outs = []
    for s in range(len(cu) - 1):
        a, b = int(cu[s]), int(cu[s + 1])
        m = h[a:b].float().mean(0)[:dims] if b > a else \
            torch.zeros(dims, dtype=torch.float32, device=h.device)
        if normalize:
            m = m / m.norm().clamp_min(1e-12)
        outs.append(m)
    return torch.stack(outs)


def gemm_nt(a, w, bias=None, act=0, residual=None):
    y = a.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if act == 1:
        y = torch.nn.functional.gelu(y, approximate="tanh")
    elif act == 2:
        y = torch.nn.functional.silu(y)
    elif act == 4:
        y = torch.nn.functional.gelu(y)
    if residual is not None:
        y = y + residual.float()
    return y.to(a.dtype)


def _uniform(seed: int, off: int, idx: torch.Tensor) -> torch.Tensor:
    # host-side mirror of the kernel's counter-based hash is not needed for the
    # CPU path; a seeded torch generator gives the same *distribution*.
    g = torch.Generator().manual_seed((seed * 1000003 + off) & 0x7FFFFFFFFFFFFFFF)
    return torch.rand(idx.shape, generator=g)


def sample(logits, temperature, top_k, top_p, seeds, offsets):
    """Greedy when temperature <= 0, else softmax(logits / T) truncated by
    top-k / top-p.  Returns (tokens int32 [B], logprobs fp32 [B])."""
    B, V = logits.shape
    toks = torch.empty(B, dtype=torch.int32)
    lps = torch.empty(B, dtype=torch.float32)
    for b in range(B):
        x = logits[b].float().cpu()
        t = float(temperature[b])
        k = int(top_k[b]) if top_k is not None else 0
        if t <= 0 or k == 1:
            j = int(torch.argmax(x))
            toks[b] = j
            lps[b] = float(torch.log_softmax(x, -1)[j])
            continue
        z = x / t
        logp = torch.log_softmax(z, -1)
        p = logp.exp()
        keep = torch.ones(V, dtype=torch.bool)
        if k > 0 and k < V:
            kth = torch.topk(z, k).values[-1]
            keep &= z >= kth
        tp = float(top_p[b]) if top_p is not None else 1.0
        if tp < 1.0:
            sp, si = torch.sort(p, descending=True)
            above = torch.cumsum(sp, 0) - sp
            nucleus = torch.zeros(V, dtype=torch.bool)
            nucleus[si[above < tp]] = True
            keep &= nucleus
        pk = torch.where(keep, p, torch.zeros_like(p))
        u = _uniform(int(seeds[b]) if seeds is not None else 0,
                     int(offsets[b]) if offsets is not None else 0, torch.zeros(1))
        c = torch.cumsum(pk / pk.sum(), 0)
        j = int(torch.searchsorted(c, u.clamp(max=float(c[-1]) - 1e-7)))
        toks[b] = j
        lps[b] = float(logp[j])
    return toks, lps


_M32 = 0xFFFFFFFF


def _lowbias32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def _mix64(z: int) -> int:
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _row_key(seed: int, off: int, rnd: int) -> tuple[int, int]:
    m = (1 << 64) - 1
    h = _mix64((seed & m) ^ _mix64((off * 0x9E3779B97F4A7C15 + rnd) & m))
    return h & _M32, h >> 32


def race_gumbel(seed: int, off: int, rnd: int, idx: torch.Tensor) -> torch.Tensor:
    """The race kernel's per-element noise G_i = -log(-log U_i), U_i a hash of
    (seed, offset, round, global index i)."""
    k0, k1 = _row_key(seed, off, rnd)
    h = _lowbias32((_lowbias32(idx.to(torch.int64) ^ k0) + k1) & _M32)
    u = ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)
    return -torch.log(-torch.log(u))


def sample_race(logits, temperature, top_k, top_p, seeds, offsets, exchange, v0, V,
                max_rounds):
    """CPU mirror of ops.sample_race (race_kernel's phases, same records and
    exchanges -- one per round, the next round raced speculatively with each
    mass pass): exact race winners, so every rank -- and a one-shard run
    over the whole row -- picks the same tokens."""
    B, Vs = logits.shape
    x = logits.float()
    idx = torch.arange(v0, v0 + Vs, dtype=torch.int64)
    temp = [float(t) for t in temperature[:B]]
    kk = [int(k) for k in top_k[:B]] if top_k is not None else [0] * B
    tp = [float(p) for p in top_p[:B]] if top_p is not None else [1.0] * B
    sd = [int(s) for s in seeds[:B]] if seeds is not None else [0x1234] * B
    of = [int(o) for o in offsets[:B]] if offsets is not None else [0] * B
    greedy = [not (t > 0) or k == 1 for t, k in zip(temp, kk)]
    inv_t = [1.0 if g else 1.0 / t for g, t in zip(greedy, temp)]
    trunc = [not g and (p < 1.0 or 0 < k < V) for g, p, k in zip(greedy, tp, kk)]
    NONE = (-math.inf, 0x7FFFFFFF, -math.inf)

    def race(b, rnd, pivot):
        keep = x[b] > pivot
        if not bool(keep.any()):
            return NONE
        key = x[b] * inv_t[b] + race_gumbel(sd[b], of[b], rnd, idx)
        key = torch.where(keep, key, torch.full_like(key, -math.inf))
        j = int(torch.argmax(key))          # first maximum: the lowest index
        return float(key[j]), v0 + j, float(x[b, j])

    rec = torch.zeros(B, 8)
    for b in range(B):                       # phase 0
        m = float(x[b].max())
        s_ = float(torch.exp((x[b] - m) * inv_t[b]).sum())
        j = int(torch.argmax(x[b]))
        c = race(b, 0, -math.inf) if not greedy[b] else NONE
        # indices travel as floats here (exact below 2^24)
        rec[b] = torch.tensor([m, s_, float(x[b, j]), float(v0 + j), c[0], float(c[1]), c[2], 0])
    g = exchange(rec)
    W = g.shape[0]
    xmax, S = [0.0] * B, [0.0] * B
    am = [(0.0, 0)] * B
    done = [False] * B
    tok, lp = [0] * B, [0.0] * B
    cand = [(0, 0.0)] * B

    def finish(b, t, x_):
        done[b], tok[b], lp[b] = True, t, (x_ - xmax[b]) * inv_t[b] - math.log(S[b])

    for rnd in range(max_rounds + 1):        # phase 1 rounds, then phase 2
        last = rnd == max_rounds
        rec = torch.zeros(B, 8)
        rec[:, 4] = -math.inf
        for b in range(B):
            if rnd == 0:
                xmax[b] = max(float(g[q, b, 0]) for q in range(W))
                S[b] = sum(float(g[q, b, 1]) * math.exp((float(g[q, b, 0]) - xmax[b]) * inv_t[b])
                           for q in range(W) if float(g[q, b, 0]) != -math.inf)
                best = (-math.inf, 0x7FFFFFFF)
                for q in range(W):
                    v, j = float(g[q, b, 2]), int(g[q, b, 3])
                    if v > best[0] or (v == best[0] and j < best[1]):
                        best = (v, j)
                am[b] = best
                if greedy[b]:
                    done[b], tok[b] = True, best[1]
                    lp[b] = best[0] - xmax[b] - math.log(S[b])
            elif not done[b]:
                mass = sum(float(g[q, b, 0]) for q in range(W)) / S[b]
                cnt = sum(float(g[q, b, 1]) for q in range(W))
                if mass < tp[b] and (kk[b] <= 0 or cnt < kk[b]):
                    finish(b, cand[b][0], cand[b][1])
                elif last:
                    finish(b, am[b][1], am[b][0])
            if last or done[b]:
                continue
            best = NONE
            for q in range(W):
                k_, j_, x_ = float(g[q, b, 4]), int(g[q, b, 5]), float(g[q, b, 6])
                if k_ > best[0] or (k_ == best[0] and j_ < best[1]):
                    best = (k_, j_, x_)
            if best[0] == -math.inf:
                finish(b, am[b][1], am[b][0])
                continue
            if not trunc[b]:
                finish(b, best[1], best[2])
                continue
            cand[b] = (best[1], best[2])
            above = x[b] > best[2]
            rec[b, 0] = float(torch.exp((x[b][above] - xmax[b]) * inv_t[b]).sum())
            rec[b, 1] = float(above.sum())
            if rnd + 1 < max_rounds:
                k_, j_, x_ = race(b, rnd + 1, best[2])
                rec[b, 4], rec[b, 5], rec[b, 6] = k_, float(j_), x_
        if not last:
            g = exchange(rec)
    return torch.tensor(tok, dtype=torch.int32), torch.tensor(lp, dtype=torch.float32)


def apply_penalties(logits, window, ngen, pen, v0: int = 0):
    """In place: repetition (every window token), presence / frequency (counts
    over the generated tail of the right-aligned window)."""
    B, W = window.shape
    for b in range(B):
        ids = window[b].tolist()
        g0 = W - int(ngen[b])
        rep, pres, freq = (float(v) for v in pen[b])
        seen = set()
        for i, t in enumerate(ids):
            if t < 0 or t in seen:
                continue
            seen.add(t)
            if not v0 <= t < v0 + logits.shape[1]:     # another rank's vocabulary shard
                continue
            cnt = sum(1 for j in range(max(i, g0), W) if ids[j] == t)
            x = float(logits[b, t - v0])
            if rep != 1.0:
                x = x / rep if x > 0 else x * rep
            x -= freq * cnt + (pres if cnt > 0 else 0.0)
            logits[b, t - v0] = x
    return logits
