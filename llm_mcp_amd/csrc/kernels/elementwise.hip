// K8 / K9 / K10: fused element-wise and pooling ops.
//   silu_mul      SwiGLU activation: out[t, i] = silu(x[t, i]) * x[t, I + i]
//                 (x = fused gate|up projection output)
//   gelu_mul      GeGLU variant, same layout
//   embed_gather  token-embedding row gather, vocab-parallel aware: rows
//                 outside [vocab_start, vocab_start + vocab_rows) are zeroed
//                 (the TP all-reduce then sums the shards)
//   mean_pool_l2  masked mean over each sequence's token rows (varlen,
//                 cu_seqlens), optional Matryoshka truncation to `dims`, L2
//                 normalisation, fp32 output -- the nomic-embed-text head.
// All bf16 traffic is 16 B per lane.
#include "common.h"

namespace lmx {

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// grid (rows, ceil(I/8 / 256)), block 256: one 16-byte chunk of gate and up
// per thread.  2-D grid, so no per-element 64-bit division (multi-instruction
// on CDNA); a 256-row decode step launches 256 x 14 workgroups for Llama-3-8B.
// ``block`` > 0: the gate|up columns are interleaved per block (the layout of
// the fused-SwiGLU decode GEMM weights, dgemm.hip): gate channel i sits at
// column (i / block) * 2 * block + i % block and its up partner block later.
template <int ACT>
__global__ void __launch_bounds__(256) glu_kernel(bf16_t* __restrict__ out,
                                                  const bf16_t* __restrict__ x, int I,
                                                  int block) {
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= I / 8) return;
  const long r = blockIdx.x;
  const bf16_t* xr = x + r * (2L * I);
  const int gi = c * 8;
  const int go = block > 0 ? (gi / block) * 2 * block + gi % block : gi;
  const int uo = block > 0 ? go + block : I + gi;
  const u16x8 g = *reinterpret_cast<const u16x8*>(xr + go);
  const u16x8 u = *reinterpret_cast<const u16x8*>(xr + uo);
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gv = bf2f(g.v[j]);
    const float a = ACT == 0 ? silu(gv) : gelu_tanh(gv);
    o.v[j] = f2bf(a * bf2f(u.v[j]));
  }
  *reinterpret_cast<u16x8*>(out + r * I + c * 8) = o;
}

int glu(void* out, const void* x, long rows, int I, int act, int block, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (I % 8 != 0 || rows > 0x7fffffffL || block < 0 || block % 8 != 0 ||
      (block > 0 && I % block != 0))
    return -1;
  const dim3 grid((unsigned)rows, (unsigned)((I / 8 + 255) / 256));
  if (act == 0)
    glu_kernel<0><<<grid, dim3(256), 0, stream>>>((bf16_t*)out, (const bf16_t*)x, I, block);
  else
    glu_kernel<1><<<grid, dim3(256), 0, stream>>>((bf16_t*)out, (const bf16_t*)x, I, block);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) embed_gather_kernel(bf16_t* __restrict__ out,
                                                           const bf16_t* __restrict__ table,
                                                           const int* __restrict__ ids, int d,
                                                           int vocab_start, int vocab_rows) {
  const int t = blockIdx.x;
  const int id = ids[t] - vocab_start;
  const bool own = id >= 0 && id < vocab_rows;
  const bf16_t* src = table + (long)(own ? id : 0) * d;
  bf16_t* dst = out + (long)t * d;
  for (int c = threadIdx.x; c < d / 8; c += blockDim.x) {
    u16x8 v;
    if (own) v = *reinterpret_cast<const u16x8*>(src + c * 8);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v.v[j] = 0;
    }
    *reinterpret_cast<u16x8*>(dst + c * 8) = v;
  }
}

int embed_gather(void* out, const void* table, const int* ids, int T, int d, int vocab_start,
                 int vocab_rows, hipStream_t stream) {
  if (T <= 0) return 0;
  if (d % 8 != 0) return -1;
  embed_gather_kernel<<<dim3(T), dim3(256), 0, stream>>>((bf16_t*)out, (const bf16_t*)table, ids,
                                                         d, vocab_start, vocab_rows);
  return (int)hipGetLastError();
}

// Lookahead decode (engine "async" stepping): step n+1 is launched before the
// host has read step n's sampled tokens, so the rows whose input token is still
// on the device name it by its sample index (src >= 0) and take it from the
// previous step's token buffer here, in stream order ahead of the embedding.
__global__ void __launch_bounds__(256) ids_from_prev_kernel(int* __restrict__ ids,
                                                            const int* __restrict__ src,
                                                            const int* __restrict__ prev, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int s = src[i];
    if (s >= 0) ids[i] = prev[s];
  }
}

int ids_from_prev(int* ids, const int* src, const int* prev, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  ids_from_prev_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(ids, src, prev, n);
  return (int)hipGetLastError();
}

// grid (nseq), block 256; d <= 256 * 8
__global__ void __launch_bounds__(256) mean_pool_l2_kernel(float* __restrict__ out,
                                                           const bf16_t* __restrict__ h,
                                                           const int* __restrict__ cu, int d,
                                                           int dims, int normalize) {
  __shared__ float scratch[16];
  const int s = blockIdx.x;
  const int t0 = cu[s], t1 = cu[s + 1];
  const int c = threadIdx.x;  // 8-element chunk
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool active = c < d / 8;
  if (active) {
    for (int t = t0; t < t1; ++t) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(h + (long)t * d + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v.v[j]);
    }
  }
  const float inv_n = t1 > t0 ? 1.f / (float)(t1 - t0) : 0.f;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[j] *= inv_n;
    if (active && c * 8 + j < dims) ss += acc[j] * acc[j];
  }
  ss = block_sum(ss, scratch);
  const float inv = normalize ? rsqrtf(fmaxf(ss, 1e-24f)) : 1.f;
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      if (col < dims) out[(long)s * dims + col] = acc[j] * inv;
    }
  }
}

// Two-stage varlen pooling.  Stage 1 spreads the token rows over
// ceil(T / POOL_ROWS) blocks (one 16 B chunk of a row per lane) and adds each
// block's per-sequence partial sums into an fp32 accumulator [nseq, d] with
// global atomics; stage 2 (one block per sequence) scales by 1/len, truncates
// to `dims` and L2-normalises.  The one-block-per-sequence kernel above walked
// all rows of a sequence on one CU and was latency-bound (311 us for a
// 64 x 512-token batch) -- it is kept for batches of many short sequences,
// where one block per sequence already fills the chip without atomics.
constexpr int POOL_ROWS = 32;

__device__ __forceinline__ void pool_flush(float* __restrict__ dst, float (&a)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    atomicAdd(dst + j, a[j]);
    a[j] = 0.f;
  }
}

// grid (ceil(T / POOL_ROWS)), block = d/8 lanes rounded up to a wave
__global__ void __launch_bounds__(256) pool_partial_kernel(float* __restrict__ acc,
                                                           const bf16_t* __restrict__ h,
                                                           const int* __restrict__ cu, int nseq,
                                                           int T, int d) {
  const int c = threadIdx.x;
  if (c >= d / 8) return;
  const int tend = min(T, cu[nseq]);  // rows past the last sequence are padding
  const int r0 = blockIdx.x * POOL_ROWS;
  const int r1 = min(r0 + POOL_ROWS, tend);
  if (r0 >= r1) return;
  int lo = 0, hi = nseq - 1;  // last sequence starting at or before r0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cu[mid] <= r0) lo = mid;
    else hi = mid - 1;
  }
  int s = lo, end = cu[s + 1], n = 0;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = r0; t < r1; ++t) {
    while (t >= end) {  // t < tend <= cu[nseq] keeps s < nseq
      if (n) pool_flush(acc + (long)s * d + c * 8, a);
      n = 0;
      ++s;
      end = cu[s + 1];
    }
    const u16x8 v = *reinterpret_cast<const u16x8*>(h + (long)t * d + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += bf2f(v.v[j]);
    ++n;
  }
  if (n) pool_flush(acc + (long)s * d + c * 8, a);
}

// grid (nseq), block 256; d <= 2048
__global__ void __launch_bounds__(256) pool_finish_kernel(float* __restrict__ out,
                                                          const float* __restrict__ acc,
                                                          const int* __restrict__ cu, int d,
                                                          int dims, int normalize) {
  __shared__ float scratch[16];
  const int s = blockIdx.x;
  const int len = cu[s + 1] - cu[s];
  const float inv_n = len > 0 ? 1.f / (float)len : 0.f;
  float v[8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = threadIdx.x + j * 256;
    v[j] = col < dims ? acc[(long)s * d + col] * inv_n : 0.f;
    ss += v[j] * v[j];
  }
  ss = block_sum(ss, scratch);
  const float inv = normalize ? rsqrtf(fmaxf(ss, 1e-24f)) : 1.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = threadIdx.x + j * 256;
    if (col < dims) out[(long)s * dims + col] = v[j] * inv;
  }
}

// acc: fp32 workspace [nseq, d] (zeroed here, on the stream).  Batches of few
// sequences (fewer than one block's worth of rows per CU) keep the one-pass
// kernel, which needs no atomics.
int mean_pool_l2(float* out, float* acc, const void* h, const int* cu, int nseq, int T, int d,
                 int dims, int normalize, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (d % 8 != 0 || d > 2048 || dims > d || dims <= 0 || T < 0) return -1;
  if (acc == nullptr) {
    mean_pool_l2_kernel<<<dim3(nseq), dim3(256), 0, stream>>>(out, (const bf16_t*)h, cu, d, dims,
                                                              normalize);
    return (int)hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(acc, 0, sizeof(float) * (size_t)nseq * d, stream);
  if (e != hipSuccess) return (int)e;
  if (T > 0) {
    const int lanes = ((d / 8 + 63) / 64) * 64;
    pool_partial_kernel<<<dim3((T + POOL_ROWS - 1) / POOL_ROWS), dim3(lanes), 0, stream>>>(
        acc, (const bf16_t*)h, cu, nseq, T, d);
  }
  pool_finish_kernel<<<dim3(nseq), dim3(256), 0, stream>>>(out, acc, cu, d, dims, normalize);
  return (int)hipGetLastError();
}

// bias add (+ optional GELU/SiLU) in place on [rows, n] bf16 (used after
// library GEMMs that do not fuse an epilogue)
__global__ void __launch_bounds__(256) bias_act_kernel(bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ bias, int n,
                                                       long rows, int act) {
  const long nchunk = rows * (n / 8);
  const int cpr = n / 8;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < nchunk;
       e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % cpr);
    u16x8 v = *reinterpret_cast<u16x8*>(x + e * 8);
    const u16x8 b = *reinterpret_cast<const u16x8*>(bias + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = bf2f(v.v[j]) + bf2f(b.v[j]);
      if (act == 1) f = gelu_tanh(f);
      else if (act == 2) f = silu(f);
      v.v[j] = f2bf(f);
    }
    *reinterpret_cast<u16x8*>(x + e * 8) = v;
  }
}

int bias_act(void* x, const void* bias, long rows, int n, int act, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (n % 8 != 0) return -1;
  long blocks = (rows * (n / 8) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  bias_act_kernel<<<dim3((unsigned)blocks), dim3(256), 0, stream>>>((bf16_t*)x, (const bf16_t*)bias, n,
                                                                 rows, act);
  return (int)hipGetLastError();
}

}  // namespace lmx
