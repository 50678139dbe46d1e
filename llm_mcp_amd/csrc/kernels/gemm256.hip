// K7 (large-M path): bf16 "NT" GEMM with a fused epilogue on gfx950 MFMA,
//     C[M,N] = act(A[M,K] . W[N,K]^T + bias[N]) (+ residual)      fp32 accumulate
// for the token-parallel shapes (encoder batches, prefill chunks): M >= 256.
//
// Why a second GEMM next to gemm_nt (gemm.hip): the 128x128 two-buffer loop
// tops out near 0.4-0.9 PFLOP/s on the nomic shapes (profiles/r1_embed_engine.md),
// the structure ceiling the guide measures for it (§5 'step-3 structure').
// This kernel is built the way the guide says breaks that ceiling:
//   * 256 x TN output tile (TN = 256 or 128), 512 threads = 8 waves as
//     2 (M) x 4 (N); a wave owns 128 x TN/4 -> 8 x TN/64 MFMA 16x16x32 tiles,
//     so every fragment read from LDS feeds 4-8 MFMAs;
//   * one workgroup per CU with a 4-deep LDS ring of BK = 32 stages filled by
//     global_load_lds (16 B per lane, no VGPR hop), THREE stages in flight
//     across the raw s_barrier of each K-step, retired by a counted
//     `s_waitcnt vmcnt(N)` -- never vmcnt(0) inside the loop;
//   * all LDS in ONE dynamic array (the second-__shared__-object trap);
//   * lane-linear LDS image (what LDS-DMA writes) with the bank swizzle
//     applied to the per-lane GLOBAL source chunk and undone on the
//     ds_read_b128: 64-B rows, chunk c of row r holds global chunk
//     c ^ (3 * ((r >> 3) & 1)), which spreads each 16-lane group of a 16x32
//     fragment read over 16 distinct 16-B slots (conflict-free);
//   * MFMA operands swapped (D = W_tile . A_tile^T) so a lane's 4 accumulator
//     registers are 4 consecutive output columns: 8-B epilogue stores;
//   * XCD-aware bijective tile remap + 8-row-tile groups (T1).
// Epilogues: bias, GELU(tanh) / SiLU, residual add, and SwiGLU over
// interleaved [64 gate | 64 up] weight rows (ops.interleave_gate_up), where
// the "up" waves hand their values to the "gate" waves through the drained
// LDS ring and C gets N/2 columns.
// Host requirements (checked): N % TN == 0, K % 32 == 0, M >= 1.
#include "common.h"

namespace lmx {
namespace g256 {

constexpr int TM = 256, TK = 32;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ int swz(int r) { return ((r >> 3) & 1) * 3; }

template <int CNT>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// rows x 32 bf16 tile -> LDS [rows][32]; each wave instruction moves 16 rows
// (1 KiB: lane l -> row l >> 2, chunk l & 3).
template <int ROWS, int NW>
__device__ __forceinline__ void stage(bf16_t* lds, const bf16_t* __restrict__ g, long ld,
                                      int row0, int rows_valid, int k0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int PER_WAVE = ROWS / 16 / NW;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    const int r = piece * 16 + (lane >> 2), c = lane & 3;
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;   // clamped rows are masked at the store
    glds16(g + (long)gr * ld + k0 + 8 * (c ^ swz(r)), lds + piece * 16 * TK);
  }
}

__device__ __forceinline__ bf16x8_t frag(const bf16_t* tile, int r, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(tile + r * TK + 8 * (chunk ^ swz(r)));
}

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) {
    const float k0 = 0.7978845608f, k1 = 0.044715f;
    return 0.5f * v * (1.f + tanhf(k0 * (v + k1 * v * v * v)));
  }
  if (act == 2) return v / (1.f + __expf(-v));
  return v;
}

// NW waves as 2 (M) x NW/2 (N); NST ring slots.  <256, 8, 4>: one 512-thread
// workgroup per CU; <128, 4, 3>: two 256-thread workgroups per CU (72 KiB of
// LDS each), so one workgroup's MFMAs run while the other waits on its fills.
template <int TN, int NW, int NST>
__global__ void __launch_bounds__(NW * 64, 8 / NW) gemm256_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ bias, const bf16_t* __restrict__ residual, int M, int N, int K,
    long lda, long ldw, long ldc, int act) {
  constexpr int WCOLS = TN / (NW / 2);   // columns per wave
  constexpr int NJ = WCOLS / 16;         // MFMA column tiles per wave (4 or 2)
  constexpr int LPS = (TM + TN) / 16 / NW;   // glds per thread per stage
  constexpr int STAGE = (TM + TN) * TK;  // elements per ring slot
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);

  const int tiles_m = (M + TM - 1) / TM, tiles_n = N / TN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;   // walk N inside a group of 8 row tiles: W panels reused in L2
  const int group_sz = GROUP * tiles_n;
  const int gid = wg / group_sz, first_m = gid * GROUP;
  const int gm = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wg % group_sz) % gm, tn = (wg % group_sz) / gm;
  const int m0 = tm * TM, n0 = tn * TN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / (NW / 2), wc = wave % (NW / 2);
  const int fr = lane & 15, fg = lane >> 4;

  f32x4_t acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TK;
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) {
      bf16_t* s = lds + p * STAGE;
      stage<TM, NW>(s, A, lda, m0, M, p * TK);
      stage<TN, NW>(s + TM * TK, W, ldw, n0, N, p * TK);
    }
  for (int t = 0; t < nk; ++t) {
    // stage t has landed once at most the later-issued stages remain in flight
    if (NST == 4 && t + 2 < nk) vm_wait<(NST - 2) * LPS>();
    else if (t + 1 < nk) vm_wait<LPS>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // raw: __syncthreads() would drain the ring (vmcnt(0))
    if (t + NST - 1 < nk) {         // refill the slot every wave finished reading at t-1
      bf16_t* s = lds + ((t + NST - 1) % NST) * STAGE;
      stage<TM, NW>(s, A, lda, m0, M, (t + NST - 1) * TK);
      stage<TN, NW>(s + TM * TK, W, ldw, n0, N, (t + NST - 1) * TK);
    }
    const bf16_t* a_t = lds + (t % NST) * STAGE;
    const bf16_t* w_t = a_t + TM * TK;
    bf16x8_t af[8], bw[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bw[j] = frag(w_t, wc * WCOLS + j * 16 + fr, fg);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag(a_t, wr * 128 + i * 16 + fr, fg);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bw[j], af[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  }

  // epilogue: acc[i][j][r] = C[m0 + wr*128 + 16i + fr][n0 + wc*WCOLS + 16j + 4fg + r]
  if (act == 3) {
    vm_wait<0>();
    __syncthreads();   // every wave is done with the ring: reuse it for the hand-off
    constexpr int ULD = TN / 2 + 4;   // fp32 [256 rows][TN/2 up cols + pad]: 16-B row skew
    float* up = reinterpret_cast<float*>(smem);
    const int col0 = wc * WCOLS;              // wave's first column inside the tile
    const int grp = col0 >> 7, within = col0 & 127;
    const bool is_up = within >= 64;
    if (is_up) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          *reinterpret_cast<f32x4_t*>(up + (wr * 128 + 16 * i + fr) * ULD + grp * 64 +
                                      (within - 64) + 16 * j + 4 * fg) = acc[i][j];
    }
    __syncthreads();
    if (is_up) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int lrow = wr * 128 + 16 * i + fr, row = m0 + lrow;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int uc = grp * 64 + within + 16 * j + 4 * fg;
        const f32x4_t u = *reinterpret_cast<const f32x4_t*>(up + lrow * ULD + uc);
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = acc[i][j][r];
          o[r] = (short)f2bf(g / (1.f + __expf(-g)) * u[r]);
        }
        *reinterpret_cast<bf16x4_t*>(C + (long)row * ldc + (n0 >> 1) + uc) = o;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + 16 * i + fr;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + wc * WCOLS + 16 * j + 4 * fg;
      bf16x4_t bv4 = {0, 0, 0, 0}, rv4 = {0, 0, 0, 0};
      if (bias) bv4 = *reinterpret_cast<const bf16x4_t*>(bias + col);
      if (residual) rv4 = *reinterpret_cast<const bf16x4_t*>(residual + (long)row * ldc + col);
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = act_fn(acc[i][j][r] + (bias ? bf2f((uint16_t)bv4[r]) : 0.f), act);
        if (residual) v += bf2f((uint16_t)rv4[r]);
        o[r] = (short)f2bf(v);
      }
      *reinterpret_cast<bf16x4_t*>(C + (long)row * ldc + col) = o;
    }
  }
}

}  // namespace g256

// variant: 1 = 256x256 tile, 8 waves, 4-slot ring (1 workgroup / CU)
//          2 = 256x128 tile, 8 waves, 4-slot ring (1 workgroup / CU)
//          3 = 256x128 tile, 4 waves, 3-slot ring (2 workgroups / CU)
int gemm_nt256(void* C, const void* A, const void* W, const void* bias, const void* residual,
               int M, int N, int K, long lda, long ldw, long ldc, int act, int variant,
               hipStream_t stream) {
  using namespace g256;
  if (M <= 0) return 0;
  if (K % TK != 0 || N % 128 != 0) return -1;
  if (variant == 0) variant = 3;
  const int tn = variant == 1 ? 256 : 128;
  if (N % tn != 0) return -1;
  const int tiles = ((M + TM - 1) / TM) * (N / tn);
  const int nst = variant == 3 ? 3 : 4;
  const size_t ring = (size_t)nst * (TM + tn) * TK * sizeof(bf16_t);
  const size_t hand = act == 3 ? (size_t)TM * (tn / 2 + 4) * sizeof(float) : 0;
  const size_t smem = ring > hand ? ring : hand;
  static bool attr[4] = {false, false, false, false};
#define LMX_G256(V, TNV, NWV, NSTV)                                                           \
  if (variant == V) {                                                                        \
    if (!attr[V]) {                                                                          \
      (void)hipFuncSetAttribute((const void*)gemm256_kernel<TNV, NWV, NSTV>,                  \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);     \
      attr[V] = true;                                                                        \
    }                                                                                        \
    gemm256_kernel<TNV, NWV, NSTV><<<dim3(tiles), dim3(NWV * 64), smem, stream>>>(           \
        (bf16_t*)C, (const bf16_t*)A, (const bf16_t*)W, (const bf16_t*)bias,                 \
        (const bf16_t*)residual, M, N, K, lda, ldw, ldc, act);                               \
  }
  LMX_G256(1, 256, 8, 4)
  LMX_G256(2, 128, 8, 4)
  LMX_G256(3, 128, 4, 3)
#undef LMX_G256
  return (int)hipGetLastError();
}

}  // namespace lmx
