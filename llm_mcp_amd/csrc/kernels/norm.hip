// K1: RMSNorm (+ fused residual add) and LayerNorm (+ fused residual add, for
// the post-norm nomic-bert encoder).  One workgroup per row, bf16 in/out, fp32
// statistics, 16-byte vector loads, the whole row kept in registers so the
// input is read from HBM exactly once.
//
// Replaces the normalisation Ollama/llama.cpp runs behind /api/chat and
// /api/embed (reference: worker/llm_worker/main.py:222-261,
// core/internal/api/handlers.go:1942-2015 only *call* it over HTTP).
#include "common.h"

namespace lmx {

// VPT = 8-element chunks per thread. Row length = cols, multiple of 8.
template <int VPT>
__global__ void __launch_bounds__(256) rmsnorm_kernel(
    bf16_t* __restrict__ out, bf16_t* __restrict__ residual,  // residual may be null
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
    int cols, long in_stride, long out_stride, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (long)row * in_stride;
  bf16_t* orow = out + (long)row * out_stride;
  bf16_t* rr = residual ? residual + (long)row * cols : nullptr;
  const int nchunk = cols >> 3;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      u16x8 a = *reinterpret_cast<const u16x8*>(xr + c * 8);
      if (rr) {
        u16x8 b = *reinterpret_cast<const u16x8*>(rr + c * 8);
        u16x8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // residual stream is kept in bf16 (as the model's hidden state is)
          const uint16_t hb = f2bf(bf2f(a.v[j]) + bf2f(b.v[j]));
          h.v[j] = hb;
          v[i][j] = bf2f(hb);
        }
        *reinterpret_cast<u16x8*>(rr + c * 8) = h;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a.v[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  // gain loads issued before the reduction: their latency overlaps it
  u16x8 wvs[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) wvs[i] = *reinterpret_cast<const u16x8*>(w + c * 8);
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)cols + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      const u16x8 wv = wvs[i];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = f2bf(v[i][j] * inv * bf2f(wv.v[j]));
      *reinterpret_cast<u16x8*>(orow + c * 8) = o;
    }
  }
}

// RMSNorm whose input is the S fp32 split-K partial slabs of the preceding
// projection (dgemm.hip epi 2, "partials only"): the K-split reduction, the
// residual add and the norm in one pass, so the projection needs neither a
// reduction pass nor a bf16 output round trip.  residual += sum_s slab[s]
// (rounded to bf16 once, as the bf16 hidden state), out = rms_norm(residual).
// S is a template parameter so the S x 2 slab loads of a chunk are all issued
// before the first add (a runtime trip count serialised them: S dependent
// memory latencies per chunk, ~8 us per 256-row call at S = 4).
template <int VPT, int S>
__global__ void __launch_bounds__(512) rmsnorm_slabs_kernel(
    bf16_t* __restrict__ out, bf16_t* __restrict__ residual, const float* __restrict__ slabs,
    long slab_stride, const bf16_t* __restrict__ w, int cols, long out_stride,
    float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const float* xr = slabs + (long)row * cols;
  bf16_t* orow = out + (long)row * out_stride;
  bf16_t* rr = residual + (long)row * cols;
  const int nchunk = cols >> 3;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      f32x4_t p0[S], p1[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        p0[s] = *reinterpret_cast<const f32x4_t*>(xr + s * slab_stride + c * 8);
        p1[s] = *reinterpret_cast<const f32x4_t*>(xr + s * slab_stride + c * 8 + 4);
      }
      const u16x8 b = *reinterpret_cast<const u16x8*>(rr + c * 8);
      f32x4_t a0 = p0[0], a1 = p1[0];
#pragma unroll
      for (int s = 1; s < S; ++s) {
        a0 += p0[s];
        a1 += p1[s];
      }
      u16x8 h;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint16_t hb = f2bf((j < 4 ? a0[j] : a1[j - 4]) + bf2f(b.v[j]));
        h.v[j] = hb;
        v[i][j] = bf2f(hb);
        ss += v[i][j] * v[i][j];
      }
      *reinterpret_cast<u16x8*>(rr + c * 8) = h;
    }
  }
  u16x8 wvs[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) wvs[i] = *reinterpret_cast<const u16x8*>(w + c * 8);
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)cols + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      const u16x8 wv = wvs[i];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = f2bf(v[i][j] * inv * bf2f(wv.v[j]));
      *reinterpret_cast<u16x8*>(orow + c * 8) = o;
    }
  }
}

template <int VPT>
__global__ void __launch_bounds__(256) layernorm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ x, const bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ b, int cols, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (long)row * cols;
  const bf16_t* rr = residual ? residual + (long)row * cols : nullptr;
  bf16_t* orow = out + (long)row * cols;
  const int nchunk = cols >> 3;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      u16x8 a = *reinterpret_cast<const u16x8*>(xr + c * 8);
      u16x8 r;
      if (rr) r = *reinterpret_cast<const u16x8*>(rr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = bf2f(a.v[j]);
        if (rr) t = bf2f(f2bf(t + bf2f(r.v[j])));
        v[i][j] = t;
        s += t;
      }
    }
  }
  const float mean = block_sum(s, scratch) / (float)cols;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; sq += d * d; }
    }
  }
  const float inv = rsqrtf(block_sum(sq, scratch) / (float)cols + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      u16x8 wv = *reinterpret_cast<const u16x8*>(w + c * 8);
      u16x8 bv = *reinterpret_cast<const u16x8*>(b + c * 8);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = f2bf((v[i][j] - mean) * inv * bf2f(wv.v[j]) + bf2f(bv.v[j]));
      *reinterpret_cast<u16x8*>(orow + c * 8) = o;
    }
  }
}

static int pick_threads(int nchunk) {
  int t = ((nchunk + 63) / 64) * 64;
  return t > 256 ? 256 : (t < 64 ? 64 : t);
}

int rmsnorm(void* out, void* residual, const void* x, const void* w, int rows, int cols,
            long in_stride, long out_stride, float eps, hipStream_t stream) {
  if (cols % 8 != 0 || rows <= 0) return -1;
  const int nchunk = cols / 8;
  const int threads = pick_threads(nchunk);
  const int vpt = (nchunk + threads - 1) / threads;
  dim3 g(rows), b(threads);
#define LMX_RMS(V)                                                                      \
  rmsnorm_kernel<V><<<g, b, 0, stream>>>((bf16_t*)out, (bf16_t*)residual, (const bf16_t*)x, \
                                         (const bf16_t*)w, cols, in_stride, out_stride, eps)
  if (vpt <= 1) LMX_RMS(1);
  else if (vpt <= 2) LMX_RMS(2);
  else if (vpt <= 4) LMX_RMS(4);
  else if (vpt <= 8) LMX_RMS(8);
  else return -2;
#undef LMX_RMS
  return (int)hipGetLastError();
}

// Row scales of the RMSNorm folded into the projections (pgemm.hip NRM, prefill):
//   s[r] = rsqrt(sum_j part[r][j] / cols + eps)
// from the producing residual GEMM's fixed per-64-column partials (P per row,
// summed in slot order: deterministic), or -- part == null -- from the bf16
// rows of x themselves (the first layer's input: the embedding rows).
__global__ void __launch_bounds__(256) row_scale_part_kernel(float* __restrict__ s,
                                                             const float* __restrict__ part,
                                                             int M, int P, float inv_cols,
                                                             float eps) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  const float4* p = reinterpret_cast<const float4*>(part + (long)r * P);
  float acc = 0.f;
  for (int j = 0; j < P / 4; ++j) {
    const float4 v = p[j];
    acc += v.x;
    acc += v.y;
    acc += v.z;
    acc += v.w;
  }
  s[r] = rsqrtf(acc * inv_cols + eps);
}

template <int VPT>
__global__ void __launch_bounds__(256) row_scale_x_kernel(float* __restrict__ s,
                                                          const bf16_t* __restrict__ x,
                                                          long stride, int cols, float eps) {
  __shared__ float scratch[16];
  const bf16_t* xr = x + (long)blockIdx.x * stride;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < cols / 8) {
      const u16x8 a = *reinterpret_cast<const u16x8*>(xr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = bf2f(a.v[j]);
        ss += v * v;
      }
    }
  }
  ss = block_sum(ss, scratch);
  if (threadIdx.x == 0) s[blockIdx.x] = rsqrtf(ss / (float)cols + eps);
}

int row_scale(float* s, const float* part, int P, const void* x, long x_stride, int M, int cols,
              float eps, hipStream_t stream) {
  if (M <= 0) return 0;
  if (cols % 8 != 0) return -1;
  if (part) {
    if (P % 4 != 0 || P <= 0) return -1;
    row_scale_part_kernel<<<dim3((M + 255) / 256), dim3(256), 0, stream>>>(s, part, M, P,
                                                                          1.f / (float)cols, eps);
  } else {
    const int nchunk = cols / 8, threads = pick_threads(nchunk);
    const int vpt = (nchunk + threads - 1) / threads;
#define LMX_RSX(V)                                                                      \
  row_scale_x_kernel<V><<<dim3(M), dim3(threads), 0, stream>>>(s, (const bf16_t*)x, x_stride, \
                                                               cols, eps)
    if (vpt <= 1) LMX_RSX(1);
    else if (vpt <= 2) LMX_RSX(2);
    else if (vpt <= 4) LMX_RSX(4);
    else if (vpt <= 8) LMX_RSX(8);
    else return -2;
#undef LMX_RSX
  }
  return (int)hipGetLastError();
}

// workgroup cap of the slab norm (probe knob: tools/slab_norm_probe.py)
static int g_slab_threads = 512;
void set_slab_norm_threads(int t) { g_slab_threads = t < 64 ? 64 : (t > 512 ? 512 : t); }

int rmsnorm_slabs(void* out, void* residual, const float* slabs, int S, long slab_stride,
                  const void* w, int rows, int cols, long out_stride, float eps,
                  hipStream_t stream) {
  if (cols % 8 != 0 || rows <= 0 || S < 1 || residual == nullptr) return -1;
  const int nchunk = cols / 8;
  // up to 512 threads (one 8-column chunk per thread at hidden 4096): a
  // decode step has one workgroup per row (~one per CU), so the S slabs'
  // loads of a row are spread over twice the waves of the plain norm
  int threads = ((nchunk + 63) / 64) * 64;
  threads = threads > g_slab_threads ? g_slab_threads : (threads < 64 ? 64 : threads);
  const int vpt = (nchunk + threads - 1) / threads;
  dim3 g(rows), b(threads);
#define LMX_RMSS(V, SS)                                                                     \
  rmsnorm_slabs_kernel<V, SS><<<g, b, 0, stream>>>((bf16_t*)out, (bf16_t*)residual, slabs,  \
                                                   slab_stride, (const bf16_t*)w, cols,     \
                                                   out_stride, eps)
#define LMX_RMSS_S(V)                                                                       \
  switch (S) {                                                                              \
    case 1: LMX_RMSS(V, 1); break;                                                          \
    case 2: LMX_RMSS(V, 2); break;                                                          \
    case 4: LMX_RMSS(V, 4); break;                                                          \
    case 8: LMX_RMSS(V, 8); break;                                                          \
    case 16: LMX_RMSS(V, 16); break;                                                        \
    default: return -3;                                                                     \
  }
  if (vpt <= 1) { LMX_RMSS_S(1) }
  else if (vpt <= 2) { LMX_RMSS_S(2) }
  else if (vpt <= 4) { LMX_RMSS_S(4) }
  else return -2;
#undef LMX_RMSS_S
#undef LMX_RMSS
  return (int)hipGetLastError();
}

int layernorm(void* out, const void* x, const void* residual, const void* w, const void* b,
              int rows, int cols, float eps, hipStream_t stream) {
  if (cols % 8 != 0 || rows <= 0) return -1;
  const int nchunk = cols / 8;
  const int threads = pick_threads(nchunk);
  const int vpt = (nchunk + threads - 1) / threads;
  dim3 g(rows), bl(threads);
#define LMX_LN(V)                                                                    \
  layernorm_kernel<V><<<g, bl, 0, stream>>>((bf16_t*)out, (const bf16_t*)x,           \
                                            (const bf16_t*)residual, (const bf16_t*)w, \
                                            (const bf16_t*)b, cols, eps)
  if (vpt <= 1) LMX_LN(1);
  else if (vpt <= 2) LMX_LN(2);
  else if (vpt <= 4) LMX_LN(4);
  else if (vpt <= 8) LMX_LN(8);
  else return -2;
#undef LMX_LN
  return (int)hipGetLastError();
}

}  // namespace lmx
