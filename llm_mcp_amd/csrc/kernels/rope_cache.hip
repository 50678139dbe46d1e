// K2 + K5: rotary embedding (neox / rotate-half form, as Llama-3 and
// nomic-bert use) applied in place to the q and k heads of the fused QKV
// projection output, fused with the scatter of k and v into the paged KV cache.
//
// KV-cache layout (MI355X-first, chosen for the MFMA operand maps of the
// attention kernels, see decode_attn.hip):
//   k_cache [num_blocks][Hkv][BS][D]   token-major: a K row is the 16-B A/B
//                                      fragment source of S = K.Q^T
//   v_cache [num_blocks][Hkv][BS/4][D][4]   key-quad: the 4 consecutive
//                                      tokens of one d are the contiguous 8-B
//                                      fragment run of O^T = V^T.P^T, and one
//                                      token's D values share D/16 128-B lines
//                                      (a d-major page [D][BS] spread a token
//                                      over D/2 lines: 17-20 us per decode
//                                      call of partial-line writes)
// cos/sin come from a host-precomputed fp32 table [max_pos][D] (cos | sin),
// so no transcendental runs on the device (guide App. B, element-wise).
#include "common.h"

namespace lmx {

// Optional per-head RMSNorm of q and k before the rotation (Qwen3's q_norm /
// k_norm).  The 16 lanes that own one head (tph = D/8 lanes x 8 elements)
// are consecutive and 16-aligned in every loop below, so the head's sum of
// squares is a 16-wide xor-shuffle reduction; normalisation stays in fp32
// through the rotation (one bf16 rounding).
__device__ __forceinline__ void qk_norm(float (&a)[4], float (&b)[4], const bf16_t* w, int i,
                                        int half, int D, float eps) {
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) ss += a[j] * a[j] + b[j] * b[j];
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
  const float r = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] *= r * bf2f(w[i + j]);
    b[j] *= r * bf2f(w[half + i + j]);
  }
}

// Decode rows: one workgroup per token.  A thread owns up to IT rotation
// items (4 pairs of one head each); all of its q/k and cos/sin loads are
// issued before the first use (IT is a template parameter: a runtime-bounded
// loop re-serialised them into IT dependent memory latencies), then the V row
// goes to the transposed page 4 elements (one 8-B load) per thread.
template <int IT>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    bf16_t* __restrict__ qkv, long qkv_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int Hq, int Hkv, int D,
    const int* __restrict__ slot_mapping, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, int BS, int rotate_k_inplace,
    const bf16_t* __restrict__ q_norm, const bf16_t* __restrict__ k_norm, float eps) {
  const int t = blockIdx.x;
  const int half = D >> 1;
  const int tph = half >> 2;  // threads per head, each owns 4 rotation pairs
  bf16_t* row = qkv + (long)t * qkv_stride;
  const int pos = positions[t];
  const float* cs = cos_sin + (long)pos * D;
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const int blk = slot >= 0 ? slot / BS : 0, off = slot >= 0 ? slot % BS : 0;
  const int nrot = (Hq + Hkv) * tph;

  bf16x4_t x1[IT], x2[IT];
  float4 c[IT], sn[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int it = threadIdx.x + k * 256;
    if (it < nrot) {
      const int h = it / tph, i = (it % tph) * 4;
      const bf16_t* hp = row + (long)h * D;
      x1[k] = *reinterpret_cast<const bf16x4_t*>(hp + i);
      x2[k] = *reinterpret_cast<const bf16x4_t*>(hp + half + i);
      c[k] = *reinterpret_cast<const float4*>(cs + i);
      sn[k] = *reinterpret_cast<const float4*>(cs + half + i);
    }
  }
  // V row loads issued with the rest (4 elements per thread per pass)
  const bf16_t* vrow = row + (long)(Hq + Hkv) * D;
  const int nv = Hkv * D;
  constexpr int VP = 2;                       // V passes held in registers (nv <= 2048)
  bf16x4_t vv[VP];
#pragma unroll
  for (int k = 0; k < VP; ++k) {
    const int e = (threadIdx.x + k * 256) * 4;
    if (slot >= 0 && v_cache && e < nv) vv[k] = *reinterpret_cast<const bf16x4_t*>(vrow + e);
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int it = threadIdx.x + k * 256;
    if (it >= nrot) continue;
    const int h = it / tph, i = (it % tph) * 4;
    bf16_t* hp = row + (long)h * D;
    const float cc[4] = {c[k].x, c[k].y, c[k].z, c[k].w};
    const float ss[4] = {sn[k].x, sn[k].y, sn[k].z, sn[k].w};
    const bool is_k = h >= Hq;
    float a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = bf2f((uint16_t)x1[k][j]), b[j] = bf2f((uint16_t)x2[k][j]);
    if (q_norm) qk_norm(a, b, is_k ? k_norm : q_norm, i, half, D, eps);
    bf16x4_t o1, o2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o1[j] = (short)f2bf(a[j] * cc[j] - b[j] * ss[j]);
      o2[j] = (short)f2bf(b[j] * cc[j] + a[j] * ss[j]);
    }
    if (!is_k || rotate_k_inplace || slot < 0) {
      *reinterpret_cast<bf16x4_t*>(hp + i) = o1;
      *reinterpret_cast<bf16x4_t*>(hp + half + i) = o2;
    }
    if (is_k && slot >= 0 && k_cache) {
      bf16_t* kp = k_cache + (((long)blk * Hkv + (h - Hq)) * BS + off) * D;
      *reinterpret_cast<bf16x4_t*>(kp + i) = o1;
      *reinterpret_cast<bf16x4_t*>(kp + half + i) = o2;
    }
  }
  if (slot < 0 || !v_cache) return;
  // v -> key-quad cache page (2-B stores 8 B apart: one token's D values
  // share D/16 lines of its page)
#pragma unroll
  for (int k = 0; k < VP; ++k) {
    const int e = (threadIdx.x + k * 256) * 4;
    if (e >= nv) continue;
    const int h = e / D, d = e % D;
    bf16_t* vp = v_cache + ((long)blk * Hkv + h) * BS * D + vq_off(d, off, D);
#pragma unroll
    for (int j = 0; j < 4; ++j) vp[4 * j] = (bf16_t)vv[k][j];
  }
}

// Prefill rows: 32 consecutive tokens per workgroup.  Rotation and the K
// write as above; V goes through an LDS tile so that the key-quad cache page
// ([BS/4][D][4]) is written in 16-B pieces -- a thread stores 4 consecutive
// tokens of 2 d whenever their slots are consecutive and 4-aligned (always
// true inside a prefill chunk), and a wave covers 8 whole 128-B lines.
// The per-token kernel's 2-B stores remain for decode rows (one token per
// page per step, nothing to coalesce).
constexpr int RT = 32;
constexpr int RT_VCOLS = 1024;   // V staging columns per LDS pass

// bytes of the tiled kernel's dynamic LDS (the V staging tile)
static size_t rope_tile_smem(int Hkv, int D) {
  const int hg = RT_VCOLS / D < Hkv ? RT_VCOLS / D : Hkv;
  return (size_t)RT * (hg * D + 8) * sizeof(bf16_t);
}

__global__ void __launch_bounds__(256) rope_cache_tiled_kernel(
    bf16_t* __restrict__ qkv, long qkv_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int row0, int T, int Hq, int Hkv, int D,
    const int* __restrict__ slot_mapping, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, int BS, int rotate_k_inplace,
    const bf16_t* __restrict__ q_norm, const bf16_t* __restrict__ k_norm, float eps, int skip_q) {
  // V staging tile (dynamic LDS, sized by the launcher): HG = min(RT_VCOLS / D,
  // Hkv) whole heads of 32 tokens, rows of HG * D + 8 elements -- a TP rank's
  // single kv head takes 8.7 KB instead of a fixed 66 KB (more workgroups per
  // CU; and the 64 KB static limit of older parts is not crossed)
  extern __shared__ __attribute__((aligned(16))) bf16_t vt[];
  __shared__ int sslot[RT];
  const int t0 = row0 + blockIdx.x * RT;
  const int nt = min(RT, T - t0);
  const int half = D >> 1, tph = half >> 3;   // 8-pair chunks per head
  if (threadIdx.x < RT)
    sslot[threadIdx.x] = (threadIdx.x < nt && slot_mapping) ? slot_mapping[t0 + threadIdx.x] : -1;
  __syncthreads();
  // a thread owns one (token, 4-pair chunk) and walks every q / k head of the
  // token: the cos/sin chunk is loaded once per item instead of once per
  // head, and HU heads' loads are issued before their arithmetic
  const int H = Hq + Hkv;
  constexpr int HU = 4;
  for (int it = threadIdx.x; it < nt * tph; it += blockDim.x) {
    const int tt = it / tph, i = (it % tph) * 8;
    bf16_t* row = qkv + (long)(t0 + tt) * qkv_stride;
    const float* cs = cos_sin + (long)positions[t0 + tt] * D;
    const int slot = sslot[tt];
    float cc[8], ss[8];
#pragma unroll
    for (int q4 = 0; q4 < 2; ++q4) {
      const float4 c = *reinterpret_cast<const float4*>(cs + i + 4 * q4);
      const float4 sn = *reinterpret_cast<const float4*>(cs + half + i + 4 * q4);
      cc[4 * q4] = c.x; cc[4 * q4 + 1] = c.y; cc[4 * q4 + 2] = c.z; cc[4 * q4 + 3] = c.w;
      ss[4 * q4] = sn.x; ss[4 * q4 + 1] = sn.y; ss[4 * q4 + 2] = sn.z; ss[4 * q4 + 3] = sn.w;
    }
    // skip_q: the prefill attention rotates q itself (paged_prefill rope_cs)
    for (int h0 = skip_q ? Hq : 0; h0 < H; h0 += HU) {
      u16x8 x1[HU], x2[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        if (h0 + u < H) {
          const bf16_t* hp = row + (long)(h0 + u) * D;
          x1[u] = *reinterpret_cast<const u16x8*>(hp + i);
          x2[u] = *reinterpret_cast<const u16x8*>(hp + half + i);
        }
      }
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int h = h0 + u;
        if (h >= H) break;
        bf16_t* hp = row + (long)h * D;
        const bool is_k = h >= Hq;
        float a[8], b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = bf2f(x1[u].v[j]), b[j] = bf2f(x2[u].v[j]);
        if (q_norm) {
          // per-head RMSNorm of q / k (Qwen3): the head's D values are spread
          // over the 8 consecutive lanes of this (token, head)
          float sq = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) sq += a[j] * a[j] + b[j] * b[j];
#pragma unroll
          for (int o = 4; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 8);
          const float r = rsqrtf(sq / (float)D + eps);
          const bf16_t* w = is_k ? k_norm : q_norm;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            a[j] *= r * bf2f(w[i + j]);
            b[j] *= r * bf2f(w[half + i + j]);
          }
        }
        u16x8 o1, o2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o1.v[j] = f2bf(a[j] * cc[j] - b[j] * ss[j]);
          o2.v[j] = f2bf(b[j] * cc[j] + a[j] * ss[j]);
        }
        if (!is_k || rotate_k_inplace || slot < 0) {
          *reinterpret_cast<u16x8*>(hp + i) = o1;
          *reinterpret_cast<u16x8*>(hp + half + i) = o2;
        }
        if (is_k && slot >= 0 && k_cache) {
          bf16_t* kp = k_cache + (((long)(slot / BS) * Hkv + (h - Hq)) * BS + slot % BS) * D;
          *reinterpret_cast<u16x8*>(kp + i) = o1;
          *reinterpret_cast<u16x8*>(kp + half + i) = o2;
        }
      }
    }
  }
  if (!v_cache || !slot_mapping) return;
  // HG heads per LDS pass (all 8 of Llama-3 at D 128): two barriers per pass
  // instead of two per head
  const int HG = RT_VCOLS / D < Hkv ? RT_VCOLS / D : Hkv;
  const int LD = HG * D + 8, chunks = HG * D / 8;
  for (int h0 = 0; h0 < Hkv; h0 += HG) {
    const int hg = Hkv - h0 < HG ? Hkv - h0 : HG;
    for (int it = threadIdx.x; it < nt * chunks; it += blockDim.x) {
      const int tt = it / chunks, c = it - tt * chunks;
      if (8 * c >= hg * D) continue;
      const bf16_t* src = qkv + (long)(t0 + tt) * qkv_stride + (long)(Hq + Hkv + h0) * D + 8 * c;
      *reinterpret_cast<u16x8*>(&vt[tt * LD + 8 * c]) = *reinterpret_cast<const u16x8*>(src);
    }
    __syncthreads();
    // one 16-B store per (head, key quad, d pair): 4 tokens x 2 d of the
    // key-quad page, whenever the quad's 4 slots are consecutive and
    // 4-aligned (always, inside a prefill chunk's whole pages)
    const int per_h = (D / 2) * (RT / 4);
    for (int it = threadIdx.x; it < hg * per_h; it += blockDim.x) {
      const int hl = it / per_h, r = it - hl * per_h;
      const int d = 2 * (r % (D / 2)), tt0 = (r / (D / 2)) * 4, h = h0 + hl;
      if (tt0 >= nt) continue;
      const int col = hl * D + d;
      const int s0 = sslot[tt0];
      bool vec = tt0 + 4 <= nt && s0 >= 0 && (s0 % 4) == 0;
#pragma unroll
      for (int j = 1; j < 4; ++j) vec = vec && sslot[tt0 + j] == s0 + j;
      if (vec) {
        u16x8 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          w.v[j] = vt[(tt0 + j) * LD + col];
          w.v[4 + j] = vt[(tt0 + j) * LD + col + 1];
        }
        *reinterpret_cast<u16x8*>(v_cache + ((long)(s0 / BS) * Hkv + h) * BS * D +
                                  vq_off(d, s0 % BS, D)) = w;
      } else {
        for (int j = 0; j < 4 && tt0 + j < nt; ++j) {
          const int sl = sslot[tt0 + j];
          if (sl < 0) continue;
          bf16_t* vp = v_cache + ((long)(sl / BS) * Hkv + h) * BS * D + vq_off(d, sl % BS, D);
          vp[0] = vt[(tt0 + j) * LD + col];
          vp[4] = vt[(tt0 + j) * LD + col + 1];
        }
      }
    }
    __syncthreads();
  }
}

int rope_cache(void* qkv, long qkv_stride, const int* positions, const float* cos_sin, int T,
               int Hq, int Hkv, int D, const int* slot_mapping, void* k_cache, void* v_cache,
               int BS, int rotate_k_inplace, int tile_from, const void* q_norm,
               const void* k_norm, float eps, int skip_q, hipStream_t stream) {
  if (T <= 0) return 0;
  // skip_q only for the tiled (prefill) rows and without q/k norms
  if (skip_q && (tile_from > 0 || q_norm != nullptr)) return -1;
  if (D % 16 != 0 || D > 256) return -1;       // 8-pair rotation chunks
  if ((q_norm == nullptr) != (k_norm == nullptr) || (q_norm && D != 128)) return -1;
  const int n1 = tile_from < 0 ? 0 : (tile_from > T ? T : tile_from);
  if (n1 > 0) {
    const int nrot = (Hq + Hkv) * (D / 8);
    if (Hkv * D > 2048 || nrot > 6 * 256) return -1;
#define LMX_RC(IT)                                                                            \
    rope_cache_kernel<IT><<<dim3(n1), dim3(256), 0, stream>>>(                                 \
        (bf16_t*)qkv, qkv_stride, positions, cos_sin, Hq, Hkv, D, slot_mapping,               \
        (bf16_t*)k_cache, (bf16_t*)v_cache, BS, rotate_k_inplace, (const bf16_t*)q_norm,      \
        (const bf16_t*)k_norm, eps)
    if (nrot <= 256) LMX_RC(1);
    else if (nrot <= 512) LMX_RC(2);
    else if (nrot <= 768) LMX_RC(3);
    else if (nrot <= 1024) LMX_RC(4);
    else LMX_RC(6);
#undef LMX_RC
  }
  if (T > n1) {
    const size_t smem = v_cache && slot_mapping ? rope_tile_smem(Hkv, D) : 0;
    static size_t attr = 0;
    if (smem > 65536 && smem > attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)rope_cache_tiled_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)smem);
      if (e != hipSuccess) return (int)e;
      attr = smem;
    }
    rope_cache_tiled_kernel<<<dim3((T - n1 + RT - 1) / RT), dim3(256), smem, stream>>>(
        (bf16_t*)qkv, qkv_stride, positions, cos_sin, n1, T, Hq, Hkv, D, slot_mapping,
        (bf16_t*)k_cache, (bf16_t*)v_cache, BS, rotate_k_inplace, (const bf16_t*)q_norm,
        (const bf16_t*)k_norm, eps, skip_q);
  }
  return (int)hipGetLastError();
}

// Plain cache write (no rotation), used by the paged-cache tests and by
// models without rotary embeddings.
__global__ void kv_write_kernel(const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                long kv_stride, const int* __restrict__ slot_mapping, int Hkv,
                                int D, bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                int BS) {
  const int t = blockIdx.x;
  const int slot = slot_mapping[t];
  if (slot < 0) return;
  const int blk = slot / BS, off = slot % BS;
  for (int it = threadIdx.x; it < Hkv * D; it += blockDim.x) {
    const int h = it / D, d = it % D;
    k_cache[(((long)blk * Hkv + h) * BS + off) * D + d] = k[(long)t * kv_stride + it];
    v_cache[((long)blk * Hkv + h) * BS * D + vq_off(d, off, D)] = v[(long)t * kv_stride + it];
  }
}

int kv_write(const void* k, const void* v, long kv_stride, const int* slot_mapping, int T, int Hkv,
             int D, void* k_cache, void* v_cache, int BS, hipStream_t stream) {
  if (T <= 0) return 0;
  kv_write_kernel<<<dim3(T), dim3(256), 0, stream>>>((const bf16_t*)k, (const bf16_t*)v,
                                                     kv_stride, slot_mapping, Hkv, D,
                                                     (bf16_t*)k_cache, (bf16_t*)v_cache, BS);
  return (int)hipGetLastError();
}

}  // namespace lmx
