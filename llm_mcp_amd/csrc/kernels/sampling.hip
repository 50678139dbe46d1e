// K6: fused sampling over the vocabulary: temperature, top-k, top-p (nucleus),
// greedy, seeded and batch-composition independent, plus the chosen token's
// log-probability (for OpenAI `logprobs` / usage accounting).
//
// One 1024-thread workgroup per row; the row (128256 logits for Llama-3) is
// streamed from L2 once per pass, no sort.  Sampling is Gumbel-max
// (argmax z_i + G_i == a draw from softmax(z)); truncation uses rejection
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

// uniform in (0,1) from (seed, offset, round, index)
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t off, int i) {
  const uint64_t h = mix64(seed ^ mix64(off * 0x9E3779B97F4A7C15ULL + (uint64_t)i));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, int i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int i) { return bf2f(p[i]); }

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

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(
    const T* __restrict__ logits, long stride, int V, const float* __restrict__ temperature,
    const int* __restrict__ top_k, const float* __restrict__ top_p,
    const uint64_t* __restrict__ seeds, const int* __restrict__ offsets, int* __restrict__ out_tok,
    float* __restrict__ out_logprob, int max_rounds) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const T* x = logits + (long)row * stride;
  const float temp = temperature ? temperature[row] : 0.f;
  // pass 1: max (and argmax for greedy)
  ArgMax am{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = ld<T>(x, i);
    if (v > am.v) { am.v = v; am.i = i; }
  }
  am = block_argmax(am, sv, si);
  const float xmax = am.v;
  const int kk = top_k ? top_k[row] : 0;
  if (!(temp > 0.f) || kk == 1) {
    if (threadIdx.x == 0) {
      out_tok[row] = am.i;
      if (out_logprob) out_logprob[row] = 0.f;  // filled by pass 2 below when requested
    }
    if (!out_logprob) return;
    float s = 0.f;
    for (int i = threadIdx.x; i < V; i += blockDim.x) s += __expf(ld<T>(x, i) - xmax);
    s = block_sum(s, sv);
    if (threadIdx.x == 0) out_logprob[row] = -__logf(s);
    return;
  }
  const float inv_t = 1.f / temp;
  // pass 2: softmax normaliser of z = (x - max)/T
  float s = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) s += __expf((ld<T>(x, i) - xmax) * inv_t);
  const float S = block_sum(s, sv);
  const float tp = top_p ? top_p[row] : 1.f;
  const bool truncate = (tp < 1.f) || (kk > 0 && kk < V);
  const uint64_t seed = seeds ? seeds[row] : 0x1234ULL;
  const uint64_t off = offsets ? (uint64_t)offsets[row] : 0ULL;
  float pivot = -INFINITY;
  int chosen = -1;
  for (int round = 0; round < (truncate ? max_rounds : 1); ++round) {
    ArgMax g{-INFINITY, 0x7fffffff};
    const uint64_t roff = off * 64 + round;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float z = (ld<T>(x, i) - xmax) * inv_t;
      if (z > pivot) {
        const float u = uniform01(seed, roff, i);
        const float key = z - __logf(-__logf(u));
        if (key > g.v) { g.v = key; g.i = i; }
      }
    }
    g = block_argmax(g, sv, si);
    const int j = g.i;
    if (!truncate) { chosen = j; break; }
    const float zj = (ld<T>(x, j) - xmax) * inv_t;
    float mass = 0.f, cnt = 0.f;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float z = (ld<T>(x, i) - xmax) * inv_t;
      if (z > zj) { mass += __expf(z); cnt += 1.f; }
    }
    mass = block_sum(mass, sv) / S;
    cnt = block_sum(cnt, sv);
    const bool in_p = mass < tp;
    const bool in_k = (kk <= 0) || (cnt < (float)kk);
    if (in_p && in_k) { chosen = j; break; }
    pivot = zj;
  }
  if (chosen < 0) chosen = am.i;
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

}  // namespace lmx
