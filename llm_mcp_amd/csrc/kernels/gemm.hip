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
  if (act == 4) return 0.5f * v * (1.f + erff(v * 0.70710678118f));   // exact GELU (BERT)
  return v;
}

// Two-buffer loop (vmcnt(0) + barrier per K-step); 2-3 workgroups per CU
// hide the latency.  A 3-slot counted-vmcnt ring at 1 workgroup per CU was
// measured 1.4-1.6x SLOWER on the nomic shapes (K = 768 / 3072), as the
// guide predicts for the 128^2 structure.
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
  constexpr int STAGE = 2 * GBM * GBK;     // A + B tile elements
  auto compute = [&](const bf16_t* a_t) {
    const bf16_t* b_t = a_t + GBM * GBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(a_t, wr * 64 + i * 16 + fr, ks * 4 + fg);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(b_t, wc * 64 + j * 16 + fr, ks * 4 + fg);
      // operands swapped (D = W_tile . A_tile^T): a lane's 4 accumulator
      // registers are 4 consecutive output COLUMNS of one row, so the
      // epilogue stores 8 B per lane instead of four scattered 2-B stores
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  stage_tile(lds, A, lda, m0, M, 0);
  stage_tile(lds + GBM * GBK, W, ldw, n0, N, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      bf16_t* nb = lds + (cur ^ 1) * STAGE;
      stage_tile(nb, A, lda, m0, M, (t + 1) * GBK);
      stage_tile(nb + GBM * GBK, W, ldw, n0, N, (t + 1) * GBK);
    }
    compute(lds + cur * STAGE);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: acc[i][j][r] = C[row][col + r] with
  //   row = m0 + wr*64 + 16i + fr, col = n0 + wc*64 + 16j + 4fg
  if (act == 3) {
    // fused SwiGLU (K8): W rows are interleaved per 128-column tile as
    // [64 gate | 64 up] of the same 64 channels (host: ops.interleave_gate_up),
    // so the wc = 1 waves hand their up values to the wc = 0 waves through
    // the (now idle) LDS and C has N/2 columns: silu(gate) * up.
    float* up = reinterpret_cast<float*>(smem);   // [128 rows][64 + 4] fp32
    constexpr int ULD = 68;
    if (wc == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4_t*>(up + (wr * 64 + 16 * i + fr) * ULD + 16 * j + 4 * fg) =
              acc[i][j];
    }
    __syncthreads();
    if (wc == 1) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wr * 64 + 16 * i + fr;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t u = *reinterpret_cast<const f32x4_t*>(
            up + (wr * 64 + 16 * i + fr) * ULD + 16 * j + 4 * fg);
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = acc[i][j][r];
          o[r] = (short)f2bf(g / (1.f + __expf(-g)) * u[r]);
        }
        *reinterpret_cast<bf16x4_t*>(C + (long)row * ldc + (n0 >> 1) + 16 * j + 4 * fg) = o;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + wr * 64 + 16 * i + fr;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + 16 * j + 4 * fg;
      bf16x4_t bv4 = {0, 0, 0, 0}, rv4 = {0, 0, 0, 0};
      if (bias) bv4 = *reinterpret_cast<const bf16x4_t*>(bias + col);
      if (residual) rv4 = *reinterpret_cast<const bf16x4_t*>(residual + (long)row * ldc + col);
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = apply_act(acc[i][j][r] + (bias ? bf2f((uint16_t)bv4[r]) : 0.f), act);
        if (residual) v += bf2f((uint16_t)rv4[r]);
        o[r] = (short)f2bf(v);
      }
      *reinterpret_cast<bf16x4_t*>(C + (long)row * ldc + col) = o;
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

// --------------------------------------------------------------------------
// Decode-shape GEMM (M <= 256):  C[M,N] = A[M,K] . W[N,K]^T, bf16 out.
//
// hipBLASLt picks 48-96 workgroup tilings for the QKV / O projections at
// M = 256 (a fifth of the 256 CUs) and the in-graph step runs them 2-4x off
// the weight-streaming roofline (profiles/r1_gemm_decode_shapes.md).  This
// kernel follows the guide's M = 256 projection recipe instead:
//   * one workgroup = all BM rows x 64 columns, K split S ways so that
//     (N/64) * S ~ one workgroup per CU;
//   * 512 threads = 8 waves; BM = 256: 8 x 1 waves of 32 rows; BM = 128:
//     4 x 2; BM = 64: 2 x 4 (wave tile 32 x 64/WN, 16x16x32 MFMA);
//   * A (activations, L2-resident, re-read by every column tile) and W (read
//     once from HBM) move by global_load_lds into an XOR-swizzled [row][64]
//     image, double-buffered (BK = 64);
//   * split-K partials: fp32 slabs + arrival ticket; the last-arriving slice
//     sums the slabs and writes the bf16 tile (agent-scope release/acquire,
//     counters zeroed by the launcher's memset node).
// --------------------------------------------------------------------------
constexpr int SK_BN = 64, SK_BK = 64, SK_THREADS = 512;

template <int BM>
__device__ __forceinline__ void sk_stage(bf16_t* lds_a, bf16_t* lds_w,
                                         const bf16_t* __restrict__ A, long lda, int M,
                                         const bf16_t* __restrict__ W, long ldw, int n0, int k0) {
  const int t = threadIdx.x, wave = t >> 6;
  // 512 threads x 16 B = 64 rows x 64 bf16 per instruction
#pragma unroll
  for (int i = 0; i < BM / 64; ++i) {
    const int r = i * 64 + (t >> 3), c = t & 7;
    const int gr = r < M ? r : M - 1;   // clamped rows are masked at the store
    glds16(A + (long)gr * lda + k0 + 8 * (c ^ swz(r)), lds_a + i * 64 * SK_BK + wave * 8 * SK_BK);
  }
  const int r = t >> 3, c = t & 7;
  glds16(W + (long)(n0 + r) * ldw + k0 + 8 * (c ^ swz(r)), lds_w + wave * 8 * SK_BK);
}

template <int CNT>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// stages in the LDS ring: enough K-steps in flight to cover HBM latency with
// one workgroup per CU (a 2-stage ring leaves one in flight: latency-bound)
template <int BM> struct SkCfg;
template <> struct SkCfg<64> { static constexpr int NST = 6; };
template <> struct SkCfg<128> { static constexpr int NST = 4; };
template <> struct SkCfg<256> { static constexpr int NST = 3; };

template <int BM>
__global__ void __launch_bounds__(SK_THREADS, 1) gemm_splitk_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    float* __restrict__ slabs, int* __restrict__ tickets, int M, int N, int K, long lda,
    long ldw, long ldc, int splits) {
  constexpr int WM = BM / 32, WN = 8 / WM, NJ = 4 / WN;   // waves along M / N, col tiles
  constexpr int NST = SkCfg<BM>::NST;
  constexpr int LPS = BM / 64 + 1;                         // glds per thread per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);
  constexpr int STAGE = (BM + SK_BN) * SK_BK;              // elements per stage

  const int tiles_n = N / SK_BN;
  const int nwg = tiles_n * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  // the K slices of one column tile get neighbouring ids (same XCD after the
  // remap), so the last arriver reads its partner slabs from its own L2
  const int tn = wg / splits, ks = wg % splits;
  const int n0 = tn * SK_BN;
  const int kc = K / splits, kbeg = ks * kc;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fg = lane >> 4;

  f32x4_t acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = kc / SK_BK;
  // prologue: NST-1 stages in flight
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) {
      bf16_t* b = lds + p * STAGE;
      sk_stage<BM>(b, b + BM * SK_BK, A, lda, M, W, ldw, n0, kbeg + p * SK_BK);
    }
  for (int t = 0; t < nk; ++t) {
    // stage t landed when at most (stages issued after it) x LPS loads remain
    if (t + NST - 2 < nk) vm_wait<(NST - 2) * LPS>(); else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();      // raw: __syncthreads would drain the ring
    if (t + NST - 1 < nk) {            // refill the slot every wave finished at t-1
      bf16_t* b = lds + ((t + NST - 1) % NST) * STAGE;
      sk_stage<BM>(b, b + BM * SK_BK, A, lda, M, W, ldw, n0, kbeg + (t + NST - 1) * SK_BK);
    }
    const bf16_t* a_t = lds + (t % NST) * STAGE;
    const bf16_t* w_t = a_t + BM * SK_BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[2], bw[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lds_frag(a_t, wr * 32 + i * 16 + fr, kk * 4 + fg);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bw[j] = lds_frag(w_t, wc * (SK_BN / WN) + j * 16 + fr, kk * 4 + fg);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af[i], bw[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // acc[i][j]: row = wr*32 + 16i + 4fg + r, col = n0 + wc*(64/WN) + 16j + fr
  if (splits == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wc * (SK_BN / WN) + 16 * j + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 32 + 16 * i + 4 * fg + r;
          if (row < M) C[(long)row * ldc + col] = f2bf(acc[i][j][r]);
        }
      }
    return;
  }
  // split-K: publish this slice's fp32 partial tile
  float* slab = slabs + (long)ks * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + wc * (SK_BN / WN) + 16 * j + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + 16 * i + 4 * fg + r;
        if (row < M) slab[(long)row * N + col] = acc[i][j][r];
      }
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);   // reuse the one LDS array (no 2nd __shared__)
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(&tickets[tn], 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    *flag = (old == splits - 1);
  }
  __syncthreads();
  if (!*flag) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tickets[tn] = 0;   // re-armed for the next call (the memset node also zeroes it)
  }
  __syncthreads();
  // last arriver: C[:, n0:n0+64] = sum_s slab[s]   (float4 per thread, 16 per row)
  for (int e = threadIdx.x; e < M * (SK_BN / 4); e += SK_THREADS) {
    const int row = e / (SK_BN / 4), c4 = (e % (SK_BN / 4)) * 4;
    float4 sum = {0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < splits; ++s2) {
      const float4 v = *reinterpret_cast<const float4*>(slabs + (long)s2 * M * N +
                                                        (long)row * N + n0 + c4);
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    bf16x4_t o;
    o[0] = (short)f2bf(sum.x); o[1] = (short)f2bf(sum.y);
    o[2] = (short)f2bf(sum.z); o[3] = (short)f2bf(sum.w);
    *reinterpret_cast<bf16x4_t*>(C + (long)row * ldc + n0 + c4) = o;
  }
}

int gemm_splitk(void* C, const void* A, const void* W, float* slabs, int* tickets, int M, int N,
                int K, long lda, long ldw, long ldc, int splits, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 256 || N % SK_BN != 0 || splits < 1 || K % (splits * SK_BK) != 0) return -1;
  if (splits > 1 && (slabs == nullptr || tickets == nullptr)) return -2;
  const int BM = M <= 64 ? 64 : (M <= 128 ? 128 : 256);
  const int nwg = (N / SK_BN) * splits;
  const int nst = BM == 64 ? SkCfg<64>::NST : (BM == 128 ? SkCfg<128>::NST : SkCfg<256>::NST);
  const size_t smem = (size_t)nst * (BM + SK_BN) * SK_BK * sizeof(bf16_t);
  if (splits > 1) {
    const hipError_t e = hipMemsetAsync(tickets, 0, sizeof(int) * (N / SK_BN), stream);
    if (e != hipSuccess) return (int)e;
  }
  static bool attr_set[3] = {false, false, false};   // > 64 KiB dynamic LDS (BM = 256)
#define LMX_SK(BMV)                                                                          \
  if (!attr_set[BMV / 128]) {                                                                \
    (void)hipFuncSetAttribute((const void*)gemm_splitk_kernel<BMV>,                                 \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);               \
    attr_set[BMV / 128] = true;                                                              \
  }                                                                                          \
  gemm_splitk_kernel<BMV><<<dim3(nwg), dim3(SK_THREADS), smem, stream>>>(                    \
      (bf16_t*)C, (const bf16_t*)A, (const bf16_t*)W, slabs, tickets, M, N, K, lda, ldw, ldc,  \
      splits);
  if (BM == 64) { LMX_SK(64) } else if (BM == 128) { LMX_SK(128) } else { LMX_SK(256) }
#undef LMX_SK
  return (int)hipGetLastError();
}

}  // namespace lmx
