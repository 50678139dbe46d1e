// K7: bf16 "NT" GEMM on gfx950 MFMA with a fused epilogue:
//     C[M,N] = act(A[M,K] . W[N,K]^T + bias[N])      (fp32 accumulate)
// W is the PyTorch nn.Linear layout, so both operands are K-contiguous and
// feed the 16x16x32 MFMA A/B fragments as 16-B reads.
//
// Structure (cdna guide §5, 'minimum 2-phase' recipe):
//   * 128x128 output tile, BK = 64, 256 threads = 4 waves (2 x 2), each wave
//     64x64 = 4 x 4 MFMA tiles, 64 fp32 accumulators per lane;
//   * global -> LDS by global_load_lds 16 B per lane (LDS-DMA, no VGPR hop),
//     two LDS buffers (64 KiB), stage t+1 issued before the MFMAs of tile t,
//     one vmcnt(0) + barrier per K-tile;
//   * LDS image is lane-linear (DMA writes base + 16*lane), so the bank
//     swizzle is applied to the per-lane GLOBAL source chunk and undone on the
//     ds_read: LDS(row r, chunk c) holds global chunk c ^ ((r >> 1) & 7),
//     which makes every ds_read_b128 lane group of the fragment read hit 16
//     distinct 16-B slots (conflict-free);
//   * XCD-aware bijective tile remap (T1) so tiles sharing A rows share an L2.
// Requirements (checked on the host): N % 128 == 0, K % 64 == 0; M arbitrary.
#include "common.h"

namespace lmx {

constexpr int GBM = 128, GBN = 128, GBK = 64;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// stage a 128 x 64 bf16 tile (row-major, K-contiguous in global) into LDS
__device__ __forceinline__ void stage_tile(bf16_t* lds_tile, const bf16_t* __restrict__ g,
                                           long ld, int row0, int rows_valid, int k0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;        // 16 pieces of 8 rows each
    const int r = piece * 8 + (lane >> 3); // tile row
    const int c = lane & 7;                // LDS chunk
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;  // clamp (masked on store)
    const bf16_t* src = g + (long)gr * ld + k0 + 8 * (c ^ swz(r));
    glds16(src, lds_tile + piece * 8 * GBK);
  }
}

__device__ __forceinline__ bf16x8_t lds_frag(const bf16_t* lds_tile, int r, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(lds_tile + r * GBK + 8 * (chunk ^ swz(r)));
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) {
    const float k0 = 0.7978845608f, k1 = 0.044715f;
    return 0.5f * v * (1.f + tanhf(k0 * (v + k1 * v * v * v)));
  }
  if (act == 2) return v / (1.f + __expf(-v));
  return v;
}

__global__ void __launch_bounds__(256, 2) gemm_nt_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ bias, const bf16_t* __restrict__ residual, int M, int N, int K,
    long lda, long ldw, long ldc, int act) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // buffer b: A tile at smem + b*32K, B tile at smem + b*32K + 16K
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);

  const int tiles_m = (M + GBM - 1) / GBM, tiles_n = N / GBN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  // group 8 M-tiles: walk N within a group so W panels are reused in L2
  const int GROUP = 8;
  const int group_sz = GROUP * tiles_n;
  const int gid = wg / group_sz, first_m = gid * GROUP;
  const int gm = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wg % group_sz) % gm, tn = (wg % group_sz) / gm;
  const int m0 = tm * GBM, n0 = tn * GBN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  stage_tile(lds, A, lda, m0, M, 0);
  stage_tile(lds + GBM * GBK, W, ldw, n0, N, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      bf16_t* nb = lds + (cur ^ 1) * 2 * GBM * GBK;
      stage_tile(nb, A, lda, m0, M, (t + 1) * GBK);
      stage_tile(nb + GBM * GBK, W, ldw, n0, N, (t + 1) * GBK);
    }
    const bf16_t* a_t = lds + cur * 2 * GBM * GBK;
    const bf16_t* b_t = a_t + GBM * GBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(a_t, wr * 64 + i * 16 + fr, ks * 4 + fg);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(b_t, wc * 64 + j * 16 + fr, ks * 4 + fg);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: acc[i][j] is the 16x16 tile with S^T-free standard map
  //   row = m0 + wr*64 + 16i + 4fg + r, col = n0 + wc*64 + 16j + fr
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wc * 64 + 16 * j + fr;
    const float bv = bias ? bf2f(bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 64 + 16 * i + 4 * fg + r;
        if (row < M) {
          float v = apply_act(acc[i][j][r] + bv, act);
          if (residual) v += bf2f(residual[(long)row * ldc + col]);
          C[(long)row * ldc + col] = f2bf(v);
        }
      }
    }
  }
}

int gemm_nt(void* C, const void* A, const void* W, const void* bias, const void* residual, int M,
            int N, int K, long lda, long ldw, long ldc, int act, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % GBN != 0 || K % GBK != 0) return -1;
  const int tiles = ((M + GBM - 1) / GBM) * (N / GBN);
  const size_t smem = 4 * GBM * GBK * sizeof(bf16_t);  // 64 KiB
  gemm_nt_kernel<<<dim3(tiles), dim3(256), smem, stream>>>(
      (bf16_t*)C, (const bf16_t*)A, (const bf16_t*)W, (const bf16_t*)bias,
      (const bf16_t*)residual, M, N, K, lda, ldw, ldc, act);
  return (int)hipGetLastError();
}

}  // namespace lmx
