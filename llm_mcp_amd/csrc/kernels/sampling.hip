// K6: fused sampling over the vocabulary: temperature, top-k, top-p (nucleus),
// greedy, seeded and batch-composition independent, plus the chosen token's
// log-probability (for OpenAI `logprobs` / usage accounting).
//
// One 1024-thread workgroup per row; the row (128256 logits for Llama-3) is
// streamed from L2 once per pass, no sort.  Sampling is inverse-CDF in a
// fixed element order (one uniform per row and round, see the pass structure
// below); truncation uses rejection
// with a pivot: draw j from the distribution restricted to {z > pivot}; accept
// iff j is inside both the nucleus (mass strictly above j < top_p) and the
// top-k set (count strictly above j < k); otherwise pivot = z_j.  Every
// rejection removes j and everything less likely, the nucleus always survives,
// and conditional on acceptance the draw is exactly the renormalised truncated
// distribution.  Rounds are capped; the fallback is the argmax (always inside).
//
// The reference forwards only `temperature` to Ollama and drops top_p /
// max_tokens / stop (core/internal/api/handlers.go:2333-2340); this engine
// honours all of them.
#include "common.h"

namespace lmx {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// A 64-bit (seed, offset, round) key mixed once per row-round.
struct RowKey { uint32_t k0, k1; };

__device__ __forceinline__ RowKey row_key(uint64_t seed, uint64_t off, int round) {
  const uint64_t h = mix64(seed ^ mix64(off * 0x9E3779B97F4A7C15ULL + (uint64_t)round));
  return RowKey{(uint32_t)h, (uint32_t)(h >> 32)};
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, int i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int i) { return bf2f(p[i]); }

// Visit every element of a row: 16-B vector loads (8 bf16 / 4 fp32 per lane
// and iteration) when the row is 16-B aligned, scalar tail / fallback.
template <typename T, typename F>
__device__ __forceinline__ void scan_row(const T* __restrict__ x, int V, F&& f) {
  constexpr int VEC = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(VEC)));
  int done = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int nv = V / VEC;
    const vec_t* xv = reinterpret_cast<const vec_t*>(x);
    for (int b = threadIdx.x; b < nv; b += blockDim.x) {
      const vec_t w = xv[b];
#pragma unroll
      for (int j = 0; j < VEC; ++j) f(b * VEC + j, ld<T>(reinterpret_cast<const T*>(&w), j));
    }
    done = nv * VEC;
  }
  for (int i = done + threadIdx.x; i < V; i += blockDim.x) f(i, ld<T>(x, i));
}

// scan_row already visits only the calling thread's elements, in a fixed
// order; the inverse-CDF walk re-reads them in that same order
template <typename T, typename F>
__device__ __forceinline__ void scan_row_own(const T* __restrict__ x, int V, F&& f) {
  scan_row(x, V, static_cast<F&&>(f));
}

struct ArgMax { float v; int i; };

__device__ __forceinline__ ArgMax argmax_combine(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ __forceinline__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = argmax_combine(a, b);
  }
  __syncthreads();
  if (lane == 0) { sv[wid] = a.v; si[wid] = a.i; }
  __syncthreads();
  ArgMax r{-INFINITY, 0x7fffffff};
  if (lane < nw) r = ArgMax{sv[lane], si[lane]};
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(r.v, o, 64), __shfl_xor(r.i, o, 64)};
    r = argmax_combine(r, b);
  }
  return r;
}

// online (max, sum exp((x - max) * inv_t)) pair
struct MaxSum { float m, s; };

__device__ __forceinline__ MaxSum ms_combine(MaxSum a, MaxSum b, float inv_t) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return MaxSum{m, 0.f};
  return MaxSum{m, a.s * __expf((a.m - m) * inv_t) + b.s * __expf((b.m - m) * inv_t)};
}

__device__ __forceinline__ MaxSum block_maxsum(MaxSum a, float inv_t, float* sv, float* sv2) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    a = ms_combine(a, MaxSum{__shfl_xor(a.m, o, 64), __shfl_xor(a.s, o, 64)}, inv_t);
  __syncthreads();
  if (lane == 0) { sv[wid] = a.m; sv2[wid] = a.s; }
  __syncthreads();
  MaxSum r{-INFINITY, 0.f};
  if (lane < nw) r = MaxSum{sv[lane], sv2[lane]};
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    r = ms_combine(r, MaxSum{__shfl_xor(r.m, o, 64), __shfl_xor(r.s, o, 64)}, inv_t);
  return r;
}

// Pass structure (the row is 128256 logits = 256 KB in bf16; B rows do not
// fit the L2s, so passes are the cost, and per-element VALU work decides each
// pass's time -- the round-1 Gumbel-max draw spent two logs and a 64-bit-free
// hash per element):
//   pass 1: online max + softmax normaliser S (one exp per element);
//   draw:   inverse CDF in the threads' element order: every thread's sum of
//           the p_i = exp((x_i - xmax) / T) of its own elements (the scan_row
//           order: coalesced; for the first draw it is the thread's pass-1
//           online normaliser rescaled to the row max, so no extra pass), a
//           block scan of the 1024 sums places one
//           uniform u * total in one thread, which walks its own elements
//           again to the index (exact sampling from the restricted
//           distribution for any fixed element order);
//   check:  (top-k / top-p only) mass and count strictly above the draw ->
//           accept (~1 - top_p rejections) or pivot on it and redraw.
// Seeded per (seed, offset, round): batch-composition independent.
__device__ __forceinline__ float row_uniform(uint64_t seed, uint64_t off, int round) {
  const RowKey k = row_key(seed, off, round);
  return ((float)(k.k0 >> 8) + 0.5f) * (1.0f / 16777216.0f);   // (0, 1)
}

// exclusive block scan of one float per thread (1024 threads); also the total
__device__ __forceinline__ float block_excl_scan(float v, float* sv, float* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  __syncthreads();
  if (lane == 63) sv[wid] = inc;
  __syncthreads();
  float wbase = 0.f, tot = 0.f;
  for (int w2 = 0; w2 < nw; ++w2) {
    const float t = sv[w2];
    if (w2 < wid) wbase += t;
    tot += t;
  }
  *total = tot;
  return wbase + inc - v;
}

// One draw restricted to {x > pivot_x} (pivot_x = -inf: the full row).
// Returns the index (every thread), or -1 when rounding left the target past
// the total (probability ~2^-24; the caller falls back to the argmax).
// loc_in >= 0: this thread's sum is already known (the first draw reuses the
// thread's pass-1 online normaliser, rescaled to the row max: no extra pass).
template <typename T>
__device__ __forceinline__ int icdf_draw(const T* __restrict__ x, int V, float xmax, float inv_t,
                                         float pivot_x, float u, float* sv, int* sel,
                                         float loc_in = -1.f) {
  float loc = loc_in;
  if (loc < 0.f) {
    loc = 0.f;
    scan_row(x, V, [&](int i, float v) {
      if (v > pivot_x) loc += __expf((v - xmax) * inv_t);
    });
  }
  float tot;
  const float pre = block_excl_scan(loc, sv, &tot);
  const float target = u * tot;
  if (threadIdx.x == 0) *sel = -1;
  __syncthreads();
  if (loc > 0.f && target >= pre && target < pre + loc) {
    // this thread's elements hold the target: walk them in the same order
    float acc = pre;
    int j = -1, last = -1;
    scan_row_own(x, V, [&](int i, float v) {
      if (j < 0 && v > pivot_x) {
        acc += __expf((v - xmax) * inv_t);
        last = i;
        if (acc > target) j = i;
      }
    });
    *sel = j >= 0 ? j : last;
  }
  __syncthreads();
  const int r = *sel;
  __syncthreads();   // sel is rewritten by the next draw
  return r;
}

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(
    const T* __restrict__ logits, long stride, int V, const float* __restrict__ temperature,
    const int* __restrict__ top_k, const float* __restrict__ top_p,
    const uint64_t* __restrict__ seeds, const int* __restrict__ offsets, int* __restrict__ out_tok,
    float* __restrict__ out_logprob, int max_rounds) {
  __shared__ float sv[16], sv2[16];
  __shared__ int si[16];
  __shared__ int sel;
  const int row = blockIdx.x;
  const T* x = logits + (long)row * stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const int kk = top_k ? top_k[row] : 0;
  if (!(temp > 0.f) || kk == 1) {
    // greedy: argmax (+ log-softmax of the winner at T = 1)
    ArgMax am{-INFINITY, 0x7fffffff};
    MaxSum ms{-INFINITY, 0.f};
    const bool want_lp = out_logprob != nullptr;
    scan_row(x, V, [&](int i, float v) {
      if (v > am.v) { am.v = v; am.i = i; }
      if (want_lp) {
        if (v > ms.m) { ms.s = ms.s * __expf(ms.m - v) + 1.f; ms.m = v; }
        else ms.s += __expf(v - ms.m);
      }
    });
    am = block_argmax(am, sv, si);
    if (out_logprob) ms = block_maxsum(ms, 1.f, sv, sv2);
    if (threadIdx.x == 0) {
      out_tok[row] = am.i;
      if (out_logprob) out_logprob[row] = am.v - ms.m - __logf(ms.s);
    }
    return;
  }
  const float inv_t = 1.f / temp;
  const uint64_t seed = seeds ? seeds[row] : 0x1234ULL;
  const uint64_t off = offsets ? (uint64_t)offsets[row] : 0ULL;
  // pass 1: max and normaliser
  MaxSum ms{-INFINITY, 0.f};
  scan_row(x, V, [&](int i, float v) {
    if (v > ms.m) { ms.s = ms.s * __expf((ms.m - v) * inv_t) + 1.f; ms.m = v; }
    else ms.s += __expf((v - ms.m) * inv_t);
  });
  const MaxSum mine = ms;
  ms = block_maxsum(ms, inv_t, sv, sv2);
  const float xmax = ms.m, S = ms.s;        // z_i = (x_i - xmax) / T, S = sum exp(z)
  // this thread's share of S: the first (unrestricted) draw needs no pass
  const float loc0 = mine.m == -INFINITY ? 0.f : mine.s * __expf((mine.m - xmax) * inv_t);
  const float tp = top_p ? top_p[row] : 1.f;
  const bool truncate = (tp < 1.f) || (kk > 0 && kk < V);
  int chosen = -1;
  float pivot_x = -INFINITY;
  float loc = loc0;       // this thread's mass above the pivot, for the next draw
  for (int round = 0; round < (truncate ? max_rounds : 1); ++round) {
    const int j = icdf_draw(x, V, xmax, inv_t, pivot_x, row_uniform(seed, off, round), sv, &sel,
                            loc);
    if (j < 0) break;
    if (!truncate) { chosen = j; break; }
    float mass = 0.f, cnt = 0.f;
    // z > zj  <=>  x > xj (T > 0): compare raw logits, exp only above
    const float xj = ld<T>(x, j);
    scan_row(x, V, [&](int i, float v) {
      if (v > xj) { mass += __expf((v - xmax) * inv_t); cnt += 1.f; }
    });
    // on rejection the pivot becomes xj, and this thread's mass above xj is
    // exactly its share of the restricted distribution: the redraw needs no
    // pass of its own (one pass per rejection round)
    loc = mass;
    mass = block_sum(mass, sv) / S;
    cnt = block_sum(cnt, sv);
    const bool in_p = mass < tp;
    const bool in_k = (kk <= 0) || (cnt < (float)kk);
    if (in_p && in_k) { chosen = j; break; }
    pivot_x = xj;
  }
  if (chosen < 0) {   // fallback: the argmax is inside every truncation
    ArgMax am{-INFINITY, 0x7fffffff};
    scan_row(x, V, [&](int i, float v) {
      if (v > am.v) { am.v = v; am.i = i; }
    });
    chosen = block_argmax(am, sv, si).i;
  }
  if (threadIdx.x == 0) {
    out_tok[row] = chosen;
    if (out_logprob) out_logprob[row] = (ld<T>(x, chosen) - xmax) * inv_t - __logf(S);
  }
}

int sample(const void* logits, int logits_bf16, long stride, int B, int V, const float* temperature,
           const int* top_k, const float* top_p, const uint64_t* seeds, const int* offsets,
           int* out_tok, float* out_logprob, int max_rounds, hipStream_t stream) {
  if (B <= 0) return 0;
  if (logits_bf16)
    sample_kernel<bf16_t><<<dim3(B), dim3(1024), 0, stream>>>(
        (const bf16_t*)logits, stride, V, temperature, top_k, top_p, seeds, offsets, out_tok,
        out_logprob, max_rounds);
  else
    sample_kernel<float><<<dim3(B), dim3(1024), 0, stream>>>(
        (const float*)logits, stride, V, temperature, top_k, top_p, seeds, offsets, out_tok,
        out_logprob, max_rounds);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------------
// K6-R: the same truncated sampler in exponential-race form, decomposable
// over vocabulary shards (vocab-parallel LM head under TP: every rank holds
// logits [B, V/TP] and NO rank gathers the full rows).
//
// A draw from softmax(x / T) restricted to {x > pivot} is
//     j = argmax over {x_i > pivot} of  x_i / T + G_i,   G_i = -log(-log U_i)
// (Gumbel-max / exponential race) with U_i a hash of (seed, offset, round,
// GLOBAL vocabulary index i): the key of element i does not depend on which
// rank holds it, so the argmax over the shards' local argmaxes is bitwise the
// argmax over the whole row.  Truncation is the same pivot rejection as
// sample_kernel: accept j iff the mass strictly above x_j is < top_p and the
// count strictly above x_j is < top_k, else pivot on x_j and race again with
// fresh noise (round + 1).  Rounds are capped; the fallback is the argmax.
//
// Per row and rank a phase writes an 8-float record; the caller exchanges the
// records (one all-gather of B x 32 B per rank: the peer slots under TP, an
// alias at W = 1) and every rank combines them in rank order into the same
// row state, so every rank ends with the same token.  Each mass pass also
// races the NEXT round over {x > x_j} speculatively (its winner is used only
// when x_j is rejected), so a round costs one exchange:
//   0  local max / normaliser / argmax and the round-0 race winner;
//   1  (round r) r = 0: the row state from the statistics (greedy rows
//      finish); r > 0: accept round r-1's candidate or pivot on it.  Then
//      combine round r's winners (untruncated rows finish) -> local mass and
//      count above x_j + the round r+1 race over {x > x_j};
//   2  (round = max_rounds) accept the last candidate or take the argmax;
//      write the tokens.
// Records: phase 0 {m, s, ax, aj, key, j, xj}, phase 1 {mass, cnt, -, -, key,
// j, xj}.  Every thread reads the exchanged records before any block-level
// barrier and thread 0 writes the record after one, so at W = 1 the record
// may be its own exchange.
namespace {
constexpr int RACE_REC = 8, RACE_ST = 12;
enum { ST_XMAX, ST_S, ST_CJ, ST_CX, ST_DONE, ST_AX, ST_AJ, ST_TOK, ST_LP };

__device__ __forceinline__ float race_gumbel(RowKey k, uint32_t gi) {
  const uint32_t h = lowbias32(lowbias32(gi ^ k.k0) + k.k1);
  const float u = ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}
}  // namespace

template <typename T>
__global__ void __launch_bounds__(1024) race_kernel(
    int phase, int round, int max_rounds, const T* __restrict__ logits, long stride, int Vs,
    int v0, int V, const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const uint64_t* __restrict__ seeds,
    const int* __restrict__ offsets, const float* __restrict__ gath, int W,
    float* __restrict__ rec, float* __restrict__ st, int* __restrict__ out_tok,
    float* __restrict__ out_lp) {
  __shared__ float sv[16], sv2[16];
  __shared__ int si[16];
  const int row = blockIdx.x, B = gridDim.x;
  const T* x = logits + (long)row * stride;
  float* s = st + (long)row * RACE_ST;
  float* r = rec + (long)row * RACE_REC;
  const float temp = temperature[row];
  const int kk = top_k ? top_k[row] : 0;
  const bool greedy = !(temp > 0.f) || kk == 1;
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const float tp = top_p ? top_p[row] : 1.f;
  const bool truncate = !greedy && ((tp < 1.f) || (kk > 0 && kk < V));
  const uint64_t seed = seeds ? seeds[row] : 0x1234ULL;
  const uint64_t off = offsets ? (uint64_t)offsets[row] : 0ULL;
  auto g = [&](int q, int slot) { return gath[((long)q * B + row) * RACE_REC + slot]; };
  // race over {x > pivot} with round `rnd`'s noise: (key, global index, x)
  auto race = [&](int rnd, float pivot, float* out3) {
    const RowKey key = row_key(seed, off, rnd);
    ArgMax c{-INFINITY, 0x7fffffff};
    scan_row(x, Vs, [&](int i, float v) {
      if (v > pivot) {
        const float k = v * inv_t + race_gumbel(key, (uint32_t)(v0 + i));
        if (k > c.v) { c.v = k; c.i = v0 + i; }   // ascending i per thread: ties keep the lowest
      }
    });
    c = block_argmax(c, sv, si);
    out3[0] = c.v;
    out3[1] = __int_as_float(c.i);
    out3[2] = c.v == -INFINITY ? -INFINITY : ld<T>(x, c.i - v0);
  };

  if (phase == 0) {
    MaxSum ms{-INFINITY, 0.f};
    ArgMax am{-INFINITY, 0x7fffffff};
    scan_row(x, Vs, [&](int i, float v) {
      if (v > ms.m) { ms.s = ms.s * __expf((ms.m - v) * inv_t) + 1.f; ms.m = v; }
      else ms.s += __expf((v - ms.m) * inv_t);
      if (v > am.v) { am.v = v; am.i = v0 + i; }
    });
    ms = block_maxsum(ms, inv_t, sv, sv2);
    am = block_argmax(am, sv, si);
    float c3[3] = {-INFINITY, __int_as_float(0x7fffffff), -INFINITY};
    if (!greedy) race(0, -INFINITY, c3);
    if (threadIdx.x == 0) {
      r[0] = ms.m; r[1] = ms.s; r[2] = am.v; r[3] = __int_as_float(am.i);
      r[4] = c3[0]; r[5] = c3[1]; r[6] = c3[2]; r[7] = 0.f;
    }
    return;
  }

  // ---- every read of the exchanged records and of the row state first ----
  float xmax, S, ax;
  int aj;
  bool done;
  float mass_in = 0.f, cnt_in = 0.f;
  if (round == 0) {
    xmax = -INFINITY;
    for (int q = 0; q < W; ++q) xmax = fmaxf(xmax, g(q, 0));
    S = 0.f;
    ArgMax am{-INFINITY, 0x7fffffff};
    for (int q = 0; q < W; ++q) {
      if (g(q, 0) != -INFINITY) S += g(q, 1) * __expf((g(q, 0) - xmax) * inv_t);
      am = argmax_combine(am, ArgMax{g(q, 2), __float_as_int(g(q, 3))});
    }
    ax = am.v;
    aj = am.i;
    done = false;
  } else {
    xmax = s[ST_XMAX]; S = s[ST_S]; ax = s[ST_AX]; aj = __float_as_int(s[ST_AJ]);
    done = s[ST_DONE] != 0.f;
    for (int q = 0; q < W; ++q) { mass_in += g(q, 0); cnt_in += g(q, 1); }
  }
  ArgMax c{-INFINITY, 0x7fffffff};
  float cx = -INFINITY;
  if (phase == 1) {
    for (int q = 0; q < W; ++q) {
      const ArgMax b{g(q, 4), __float_as_int(g(q, 5))};
      if (b.v > c.v || (b.v == c.v && b.i < c.i)) { c = b; cx = g(q, 6); }
    }
  }
  const int prev_j = __float_as_int(s[ST_CJ]);
  const float prev_x = s[ST_CX];
  __syncthreads();    // nothing below writes before every thread has read

  int tok = 0;
  float lp = 0.f;
  const float logS = __logf(S);
  if (round == 0 && greedy) {
    done = true; tok = aj; lp = ax - xmax - logS;
  } else if (round > 0 && !done) {
    // round - 1's candidate: accepted, or the pivot of this round's race
    if (mass_in / S < tp && (kk <= 0 || cnt_in < (float)kk)) {
      done = true; tok = prev_j; lp = (prev_x - xmax) * inv_t - logS;
    } else if (phase == 2) {
      done = true; tok = aj; lp = (ax - xmax) * inv_t - logS;   // rounds used up: the argmax
    }
  }
  if (phase == 1 && !done) {
    if (c.v == -INFINITY) {                   // nothing above the pivot: the argmax
      done = true; tok = aj; lp = (ax - xmax) * inv_t - logS;
    } else if (!truncate) {
      done = true; tok = c.i; lp = (cx - xmax) * inv_t - logS;
    }
  }
  float mass = 0.f, cnt = 0.f;
  float c3[3] = {-INFINITY, __int_as_float(0x7fffffff), -INFINITY};
  if (phase == 1 && !done) {
    scan_row(x, Vs, [&](int i, float v) {
      if (v > cx) { mass += __expf((v - xmax) * inv_t); cnt += 1.f; }
    });
    mass = block_sum(mass, sv);
    cnt = block_sum(cnt, sv);
    // the next round's race over {x > x_j}, used only if x_j is rejected
    if (round + 1 < max_rounds) race(round + 1, cx, c3);
  }
  if (threadIdx.x == 0) {
    const bool was_done = round > 0 && s[ST_DONE] != 0.f;   // (round 0: last call's state)
    if (round == 0) {
      s[ST_XMAX] = xmax; s[ST_S] = S; s[ST_AX] = ax; s[ST_AJ] = __int_as_float(aj);
    }
    if (phase == 1 && !done) { s[ST_CJ] = __int_as_float(c.i); s[ST_CX] = cx; }
    if (done && !was_done) { s[ST_TOK] = __int_as_float(tok); s[ST_LP] = lp; }
    s[ST_DONE] = done ? 1.f : 0.f;
    r[0] = mass; r[1] = cnt; r[4] = c3[0]; r[5] = c3[1]; r[6] = c3[2];
    if (phase == 2) {
      out_tok[row] = __float_as_int(s[ST_TOK]);
      if (out_lp) out_lp[row] = s[ST_LP];
    }
  }
}

int race_sample_phase(int phase, int round, int max_rounds, const void* logits, int logits_bf16,
                      long stride, int B, int Vs, int v0, int V, const float* temperature,
                      const int* top_k, const float* top_p, const uint64_t* seeds,
                      const int* offsets, const float* gath, int W, float* rec, float* st,
                      int* out_tok, float* out_lp, hipStream_t stream) {
  if (B <= 0) return 0;
  if (phase < 0 || phase > 2 || W < 1 || Vs < 1 || max_rounds < 1) return -1;
  const int threads = Vs > 32768 ? 1024 : 256;
  if (logits_bf16)
    race_kernel<bf16_t><<<dim3(B), dim3(threads), 0, stream>>>(
        phase, round, max_rounds, (const bf16_t*)logits, stride, Vs, v0, V, temperature, top_k,
        top_p, seeds, offsets, gath, W, rec, st, out_tok, out_lp);
  else
    race_kernel<float><<<dim3(B), dim3(threads), 0, stream>>>(
        phase, round, max_rounds, (const float*)logits, stride, Vs, v0, V, temperature, top_k,
        top_p, seeds, offsets, gath, W, rec, st, out_tok, out_lp);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------------
// Repetition / presence / frequency penalties applied to the logits in place,
// before sampling.  One wave per sampled row, lane i owns entry i of the row's
// right-aligned window of the last W (<= 64) context tokens (-1 = empty); the
// last ngen entries are generated tokens.  The lane holding the FIRST
// occurrence of a token applies, once:
//   repetition (HF / Ollama repeat_penalty, over every window token):
//       l = l > 0 ? l / r : l * r
//   presence / frequency (OpenAI, over the generated part of the window):
//       l -= frequency * count + presence * (count > 0)
// `on` (device flag, may be null) lets a captured graph skip the kernel for
// steps without penalised rows.
__global__ void __launch_bounds__(64) penalty_kernel(bf16_t* __restrict__ logits, long ld, int V,
                                                     const int* __restrict__ win,
                                                     const int* __restrict__ ngen,
                                                     const float* __restrict__ pen,
                                                     const int* __restrict__ on, int W, int v0) {
  if (on != nullptr && on[0] == 0) return;
  __shared__ int ids[64];
  const int row = blockIdx.x, lane = threadIdx.x;
  const int t = lane < W ? win[(long)row * W + lane] : -1;
  ids[lane] = t;
  __syncthreads();
  if (t < v0 || t >= v0 + V) return;           // another rank's vocabulary shard
  for (int j = 0; j < lane; ++j)
    if (ids[j] == t) return;                   // not the first occurrence
  const int g0 = W - ngen[row];
  int cnt = 0;
  for (int j = lane > g0 ? lane : g0; j < W; ++j) cnt += ids[j] == t;
  const float rep = pen[3 * row], pres = pen[3 * row + 1], freq = pen[3 * row + 2];
  bf16_t* p = logits + (long)row * ld + (t - v0);
  float l = bf2f(*p);
  if (rep != 1.f) l = l > 0.f ? l / rep : l * rep;
  l -= freq * (float)cnt + (cnt > 0 ? pres : 0.f);
  *p = f2bf(l);
}

int apply_penalties(void* logits, long ld, int B, int V, const int* win, const int* ngen,
                    const float* pen, const int* on, int W, int v0, hipStream_t stream) {
  if (B <= 0) return 0;
  if (W <= 0 || W > 64) return -1;
  penalty_kernel<<<dim3(B), dim3(64), 0, stream>>>((bf16_t*)logits, ld, V, win, ngen, pen, on, W,
                                                    v0);
  return (int)hipGetLastError();
}

}  // namespace lmx
