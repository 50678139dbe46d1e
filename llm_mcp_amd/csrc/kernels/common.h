// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of llm_mcp_amd.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes (hard-coded, never warpSize arithmetic on 32);
//   * bf16 tensors are passed as raw uint16 storage and moved 16 B per lane
//     (8 elements) wherever the row length allows (Guideline 13);
//   * accumulation is always fp32;
//   * every launch function takes an explicit hipStream_t so the caller can
//     capture it in a hipGraph (no allocation / sync inside launchers).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define LMX_WAVE 64

typedef uint16_t bf16_t;
typedef short bf16x8_t __attribute__((ext_vector_type(8)));   // MFMA A/B fragment (4 VGPRs)
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));    // 16x16 MFMA accumulator
typedef float f32x16_t __attribute__((ext_vector_type(16)));  // 32x32 MFMA accumulator

struct __attribute__((aligned(16))) u16x8 { uint16_t v[8]; };

__device__ __forceinline__ float bf2f(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  // hipcc lowers this to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950.
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

// 2^x as the bare v_exp_f32 (exp2f adds a denormal range fix-up -- v_cmp,
// two v_cndmask and a v_ldexp per call, 4 of the ~7 VALU per softmax element
// of the attention kernels).  Results below 2^-126 flush to 0, -inf -> 0:
// what a softmax weight needs.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of up to 1024 threads. `scratch` needs >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? scratch[lane] : 0.f;
  return wave_sum(t);
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? scratch[lane] : -INFINITY;
  return wave_max(t);
}

// 16x16x32 bf16 MFMA: D = A(16x32) * B(32x16) + C.
//   lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15] (j = 0..7);
//   C/D: col = l&15, row = 4(l>>4) + reg.
__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 32x32x16 bf16 MFMA: lane l holds A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31];
//   C/D: col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5).
__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t load_frag16B(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// Two 8-byte halves -> one fragment (used for permuted-k operands).
// V-cache page layout [BS/4][D][4] ("key-quad"): the 4 consecutive keys of
// one d are 8 contiguous bytes (the 8-B V^T fragment run of the PV MFMA), and
// one token's D values lie in one D x 8-B span, so a decode step's per-token
// write touches D/16 128-B lines instead of D/2 (profiles/r2_decode_attention.md)
__device__ __forceinline__ long vq_off(int d, int key, int D) {
  return ((long)(key >> 2) * D + d) * 4 + (key & 3);
}

__device__ __forceinline__ bf16x8_t load_frag_2x8B(const bf16_t* p0, const bf16_t* p1) {
  bf16x4_t a = *reinterpret_cast<const bf16x4_t*>(p0);
  bf16x4_t b = *reinterpret_cast<const bf16x4_t*>(p1);
  bf16x8_t r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// XCD-aware bijective remap of a linear workgroup id (cdna guide §5, T1):
// consecutive logical tiles land on the same XCD so neighbouring tiles share L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

#define LMX_CHECK_LAUNCH() (hipGetLastError())
