// K11: decoder projection GEMM for decode-sized M (1..256 rows):
//     C[M, N] = A[M, K] . W[N, K]^T        (bf16 in, fp32 accumulate, bf16 out)
// with an optional fused SwiGLU epilogue (gate/up weights interleaved per
// BN-column tile as [BN/2 gate | BN/2 up] rows; C = silu(gate) * up, N/2 cols).
//
// Why a separate kernel from gemm.hip's gemm_nt: at decode M the problem is a
// weight stream (the W bytes dominate HBM traffic) plus an activation operand
// that is re-read from L2 by every column tile.  hipBLASLt picks 48-112
// workgroup tilings for the Llama-3-8B QKV / O / down projections at M = 256
// and runs them at 1.2-2.5 TB/s effective (profiles/r1_gemm_decode_shapes.md).
// Here the decomposition is chosen per shape (bench/dgemm_bench.py, measured
// table in ops.DGEMM_TABLE):
//   * a workgroup owns a BM x BN output tile (BM in {64,128,256}, BN in
//     {64,128,256}) over K/S of the reduction; the grid (M/BM) x (N/BN) x S is
//     sized to ~ one workgroup per CU (256 CUs);
//   * 512 threads = 8 waves laid out WM x WN over the tile, 16x16x32 bf16
//     MFMA with the operands swapped (D = W_tile . A_tile^T) so each lane's
//     4 accumulator registers are 4 consecutive output COLUMNS of one row
//     (8-B bf16 / 16-B fp32 stores);
//   * both operands move global -> LDS by LDS-DMA (global_load_lds 16 B per
//     lane), NST-deep ring, counted vmcnt and raw s_barrier (a
//     __syncthreads would drain the ring: cdna guide §5 "Pipelining across
//     barriers"); XOR-swizzled [row][64] images (swizzle on the global source
//     chunk, undone on the ds_read) for conflict-free ds_read_b128;
//   * workgroup -> (tile, slice) mapping puts the slices and the M-tiles of
//     one column tile on one XCD after the bijective remap (the M-tiles share
//     the W panel in that L2, the last arriver reads its partners' slabs
//     there);
//   * NT (cfg id bit 5): the W stream is loaded non-temporal (LDS-DMA aux 2):
//     a decode step reads each weight once, 15 GB apart, so keeping its lines
//     in L2 / MALL only delays the next tile's misses (microarch guide,
//     "nt-weights"); the activation operand keeps the default policy (every
//     column tile re-reads it);
//   * split-K partials go to fp32 slabs; arrival tickets (agent-scope
//     release / acquire, guide "Projection GEMM at M = 256" item 2) elect the
//     last slice, which adds the other slices' slabs into its accumulators
//     and runs the epilogue.  Tickets are
//     zero-initialised once and re-armed by the last arriver, so a captured
//     decode graph needs no memset node per GEMM.
#include "common.h"

#include <algorithm>

namespace lmx {
namespace {

constexpr int DTHREADS = 512;

typedef __attribute__((address_space(3))) void lds_void_t;

template <int AUX = 0>
__device__ __forceinline__ void dg_glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void_t*)lds_base, 16, 0, AUX);
}

// XOR swizzle of the 16-B chunk index in row r of a [row][BK] image, chosen
// so that the 16-lane groups of a ds_read_b128 (lanes {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... : 16 rows x chunk fg) hit 16 distinct 16-B slots
// of the 256-B bank row.  BK 128 (256-B rows): chunk ^ (r mod 16).  BK 64
// (128-B rows): chunk ^ (r/2 mod 8).  BK 32 (64-B rows, 4 rows per bank
// row): chunk ^ {0,2,3,1}[r/4 mod 4].
template <int BK>
__device__ __forceinline__ int dg_swz(int r) {
  if constexpr (BK == 128) return r & 15;     // 256-B rows: one row per bank row
  else if constexpr (BK == 64) return (r >> 1) & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;
}

template <int BK>
__device__ __forceinline__ bf16x8_t dg_frag(const bf16_t* tile, int r, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(tile + r * BK + 8 * (chunk ^ dg_swz<BK>(r)));
}

template <int CNT>
__device__ __forceinline__ void dg_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// One K-step (BK deep) of the A rows [m0, m0+BM) and W rows [n0, n0+BN).
// 512 lanes x 16 B per instruction = RPI rows x BK; wave w fills rows
// (64/CPR)w .. of each RPI-row slab (lane-linear LDS destination, swizzle on
// the global source chunk).
template <int BM, int BN, int NT, int BK>
__device__ __forceinline__ void dg_stage(bf16_t* lds_a, bf16_t* lds_w, const bf16_t* __restrict__ A,
                                         long lda, int m0, int M, const bf16_t* __restrict__ W,
                                         long ldw, int n0, int k0) {
  constexpr int CPR = BK / 8, RPI = DTHREADS / CPR, RPW = 64 / CPR;
  const int t = threadIdx.x, wave = t >> 6;
  const int rr = t / CPR, c = t % CPR;
#pragma unroll
  for (int i = 0; i < BM / RPI; ++i) {
    const int r = i * RPI + rr;
    int gr = m0 + r;
    gr = gr < M ? gr : M - 1;            // padded rows re-read row M-1; never stored
    dg_glds16(A + (long)gr * lda + k0 + 8 * (c ^ dg_swz<BK>(r)),
              lds_a + (i * RPI + wave * RPW) * BK);
  }
#pragma unroll
  for (int i = 0; i < BN / RPI; ++i) {
    const int r = i * RPI + rr;
    dg_glds16<NT ? 2 : 0>(W + (long)(n0 + r) * ldw + k0 + 8 * (c ^ dg_swz<BK>(r)),
                          lds_w + (i * RPI + wave * RPW) * BK);
  }
  if constexpr (BN % RPI != 0) {
    // a tile width that is not a multiple of RPI rows (e.g. BN = 224): the
    // waves below (BN % RPI) / RPW issue one more instruction (wave-uniform;
    // the kernel's counted waits use per-wave counts)
    constexpr int i = BN / RPI;
    if (wave < (BN % RPI) / RPW) {
      const int r = i * RPI + rr;
      dg_glds16<NT ? 2 : 0>(W + (long)(n0 + r) * ldw + k0 + 8 * (c ^ dg_swz<BK>(r)),
                            lds_w + (i * RPI + wave * RPW) * BK);
    }
  }
}

__device__ __forceinline__ float dg_silu(float g) { return g / (1.f + __expf(-g)); }

// The K loop of one output tile over nk K-steps starting at kbeg (rotated by
// rot steps): NST-deep LDS-DMA ring, counted vmcnt, raw s_barrier; returns
// with the ring drained and every wave past its last ds_read, so the caller
// may restage the ring or reuse the LDS for an epilogue.
template <int BM, int BN, int WM, int NST, int NT, int BK, int TM, int TN>
__device__ __forceinline__ void dg_kloop(f32x4_t (&acc)[TM][TN], bf16_t* lds,
                                         const bf16_t* __restrict__ A, long lda, int m0, int M,
                                         const bf16_t* __restrict__ W, long ldw, int n0, int kbeg,
                                         int nk, int rot) {
  constexpr int WN = 8 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RPI = DTHREADS * 8 / BK, RPW = RPI / 8;
  // LDS-DMA instructions per thread per stage: LPS_F for the waves that stage
  // the partial last W slab of a BN % RPI != 0 tile, LPS_P for the others
  constexpr int LPS_P = BM / RPI + BN / RPI, LPS_F = LPS_P + (BN % RPI != 0);
  constexpr int WFULL = BN % RPI == 0 ? 8 : (BN % RPI) / RPW;
  constexpr int STAGE = (BM + BN) * BK;             // bf16 elements per ring slot
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) {
      bf16_t* b = lds + p * STAGE;
      dg_stage<BM, BN, NT, BK>(b, b + BM * BK, A, lda, m0, M, W, ldw, n0,
                               kbeg + ((p + rot) % nk) * BK);
    }
  for (int t = 0; t < nk; ++t) {
    if (t + NST - 2 < nk) {
      if (wave < WFULL) dg_vmwait<(NST - 2) * LPS_F>(); else dg_vmwait<(NST - 2) * LPS_P>();
    } else {
      dg_vmwait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NST - 1 < nk) {       // refill the slot every wave finished reading at t-1
      bf16_t* b = lds + ((t + NST - 1) % NST) * STAGE;
      dg_stage<BM, BN, NT, BK>(b, b + BM * BK, A, lda, m0, M, W, ldw, n0,
                               kbeg + ((t + NST - 1 + rot) % nk) * BK);
    }
    const bf16_t* a_t = lds + (t % NST) * STAGE;
    const bf16_t* w_t = a_t + BM * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = dg_frag<BK>(a_t, wr * WTM + i * 16 + fr, kk * 4 + fg);
#pragma unroll
      for (int j = 0; j < TN; ++j) bw[j] = dg_frag<BK>(w_t, wc * WTN + j * 16 + fr, kk * 4 + fg);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bw[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  dg_vmwait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

}  // namespace

template <int BM, int BN, int WM, int NST, int EPI, int ROT, int NT, int BK>
__global__ void __launch_bounds__(DTHREADS, 2) dgemm_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    float* __restrict__ slabs, unsigned* __restrict__ tickets, int M, int N, int K, long lda,
    long ldw, long ldc, int splits) {
  constexpr int WN = 8 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;       // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;       // 16x16 MFMA tiles per wave
  constexpr int RPI = DTHREADS * 8 / BK, RPW = RPI / 8;  // rows per glds instruction / per wave
  static_assert(WM * WN == 8 && TM >= 1 && TN >= 1 && WTM % 16 == 0 && WTN % 16 == 0, "tile");
  static_assert(BK == 32 || BK == 64 || BK == 128, "BK");
  static_assert(BM % RPI == 0 && BN % RPW == 0, "stage rows");
  static_assert(EPI != 1 || (WN % 2 == 0 || WN == 1), "swiglu wave split");
  static_assert(EPI != 3 || WTN % 32 == 0, "swiglu16: gate/up 16-column pairs inside a wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);

  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int ks = wg % splits, rest = wg / splits;
  const int tm = rest % tiles_m, tn = rest / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kc = K / splits, kbeg = ks * kc, nk = kc / BK;
  // K-step order rotated per column tile: the workgroups of an XCD start at
  // different k-offsets, so their concurrent reads of the shared activation
  // rows (and of their W rows, all at the same 8-KB-strided offsets
  // otherwise) spread over the L2 / HBM channels instead of camping on one.
  // ROT 2 also staggers the M-tiles that share a W panel by 2 K-steps: the
  // leader's W reads miss to HBM, its followers re-read those lines from the
  // XCD's L2 two steps later (short latency) instead of merging into the same
  // in-flight misses -- per-CU throughput is bounded by the L1's outstanding
  // misses x their latency (profiles/r2_pmc_kernels.md)
  const int rot = ROT == 0 ? 0 : ((tn * 5 + (ROT == 2 ? 2 * tm : 0)) % nk);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fg = lane >> 4;

  f32x4_t acc[TM][TN];
  dg_kloop<BM, BN, WM, NST, NT, BK>(acc, lds, A, lda, m0, M, W, ldw, n0, kbeg, nk, rot);

  // acc[i][j][r] = C[m][n]:  m = m0 + wr*WTM + 16i + fr,  n = n0 + wc*WTN + 16j + 4fg + r
  if (splits > 1 || EPI == 2) {
    // ---- split-K: publish this slice's fp32 partial tile ------------------
    float* slab = slabs + (long)ks * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * WTN + 16 * j + 4 * fg;
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + n) = acc[i][j];
      }
    }
    if (EPI == 2) return;   // partials only: the consumer kernel sums the S slabs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);       // the one LDS array (no 2nd __shared__)
    const int tile = tn * tiles_m + tm;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(&tickets[tile], 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      *flag = (old == (unsigned)(splits - 1));
    }
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tickets[tile] = 0u;     // re-armed: every slice of this call has arrived
    }
    __syncthreads();
    // last arriver: add the OTHER slices' partials into its own accumulators
    // (its own slab is never read back), in the canonical order
    // ((p0 + p1) + ...) + p(S-1) whichever slice arrives last, so a call's
    // result is bitwise reproducible
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      const long row = (long)(m < M ? m : M - 1) * N;   // load unconditionally (guide §5 item 4c)
      if (ks > 0) {
        f32x4_t pre[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j)
          pre[j] = *reinterpret_cast<const f32x4_t*>(slabs + row + n0 + wc * WTN + 16 * j + 4 * fg);
        for (int s2 = 1; s2 < ks; ++s2) {
          const float* o = slabs + (long)s2 * M * N + row;
#pragma unroll
          for (int j = 0; j < TN; ++j)
            pre[j] += *reinterpret_cast<const f32x4_t*>(o + n0 + wc * WTN + 16 * j + 4 * fg);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = pre[j] + acc[i][j];
      }
      for (int s2 = ks + 1; s2 < splits; ++s2) {
        const float* o = slabs + (long)s2 * M * N + row;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4_t*>(o + n0 + wc * WTN + 16 * j + 4 * fg);
      }
    }
    __syncthreads();            // the SwiGLU hand-off below reuses the LDS word of the flag
  }

  if (EPI == 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * WTN + 16 * j + 4 * fg;
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[i][j][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + n) = o;
      }
    }
    return;
  }
  if constexpr (EPI == 3) {
    // SwiGLU on 16-column pairs (ops.interleave_gate_up(w, 16): W rows
    // [16 gate | 16 up] per 16 channels): tiles 2j and 2j+1 of a wave are the
    // gate and up values of the same 16 channels in the same lane registers,
    // so the epilogue needs no LDS hand-off and any BN with WTN % 32 == 0 works
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN / 2; ++j) {
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = (short)f2bf(dg_silu(acc[i][2 * j][r]) * acc[i][2 * j + 1][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + ((n0 + wc * WTN) >> 1) + 16 * j +
                                     4 * fg) = o;
      }
    }
    return;
  }
  constexpr int HALF = BN / 2, ULD = HALF + 4;
  if constexpr (WN == 1) {
    // one wave column holds both halves: gate tiles j < TN/2, up tiles j + TN/2
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN / 2; ++j) {
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = (short)f2bf(dg_silu(acc[i][j][r]) * acc[i][j + TN / 2][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + (n0 >> 1) + 16 * j + 4 * fg) = o;
      }
    }
    return;
  }
  // fused SwiGLU: the up half of the tile (waves wc >= WN/2) hands its
  // values to the gate half through the idle LDS ring
  float* up = reinterpret_cast<float*>(smem);
  const bool is_up = (wc * WTN) >= HALF;
  if (is_up) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4_t*>(up + (wr * WTM + 16 * i + fr) * ULD +
                                    (wc * WTN - HALF) + 16 * j + 4 * fg) = acc[i][j];
  }
  __syncthreads();
  if (is_up) return;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wr * WTM + 16 * i + fr, m = m0 + ml;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nl = wc * WTN + 16 * j + 4 * fg;
      const f32x4_t u = *reinterpret_cast<const f32x4_t*>(up + ml * ULD + nl);
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(dg_silu(acc[i][j][r]) * u[r]);
      *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + (n0 >> 1) + nl) = o;
    }
  }
}

// ---- stream-K form (cfg bit 6) ------------------------------------------------
// Split-K with S slices runs tiles x S workgroups: for a shape with few column
// tiles (the Llama-3-70B QKV at 128 rows: 40 tiles of 128 x 256) no S fills the
// 256 CUs evenly (S 4 = 160 workgroups, S 8 = 320 = 1.25 rounds), and the last
// arriver then reads S-1 partial tiles alone.  Here the (tile, K-step) space is
// cut into G equal runs of `per` steps, one workgroup each, so every CU streams
// the same bytes; a run that crosses a tile boundary finishes one tile's piece
// and starts the next.  Piece p of tile t (p = g - first workgroup of t) goes to
// slab p; dg_sk_reduce_kernel then sums each tile's pieces in piece order
// (bitwise reproducible) and writes bf16 -- the reduction is spread over the
// whole grid instead of one workgroup per tile.
template <int BM, int BN, int WM, int NST, int NT, int BK>
__global__ void __launch_bounds__(DTHREADS, 2) dgemm_sk_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, float* __restrict__ slabs, int M,
    int N, int K, long lda, long ldw, int per) {
  constexpr int WN = 8 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);
  const int tiles_m = (M + BM - 1) / BM, nk = K / BK;
  const int total = tiles_m * (N / BN) * nk;
  const int g = blockIdx.x;
  const int end = min(g * per + per, total);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fg = lane >> 4;
  for (int it = g * per; it < end;) {
    const int t = it / nk, kb = it - t * nk, n_it = min(nk - kb, end - it);
    const int tm = t % tiles_m, tn = t / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    f32x4_t acc[TM][TN];
    dg_kloop<BM, BN, WM, NST, NT, BK>(acc, lds, A, lda, m0, M, W, ldw, n0, kb * BK, n_it, 0);
    float* slab = slabs + (long)(g - t * nk / per) * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + n0 + wc * WTN + 16 * j + 4 * fg) = acc[i][j];
    }
    it += n_it;
  }
}

// C[m][n..n+3] = sum over tile(m, n)'s pieces, 4 columns per thread
__global__ void __launch_bounds__(256) dg_sk_reduce_kernel(bf16_t* __restrict__ C,
                                                           const float* __restrict__ slabs, int M,
                                                           int N, long ldc, int BM, int BN, int nk,
                                                           int per) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = N >> 2;
  if (i >= (long)M * q) return;
  const int m = (int)(i / q), n = (int)(i - (long)m * q) * 4;
  const int t = (n / BN) * ((M + BM - 1) / BM) + m / BM;
  const int np = (t * nk + nk - 1) / per - t * nk / per + 1;
  const float* src = slabs + (long)m * N + n;
  f32x4_t s = *reinterpret_cast<const f32x4_t*>(src);
  for (int p = 1; p < np; ++p) s += *reinterpret_cast<const f32x4_t*>(src + (long)p * M * N);
  bf16x4_t o;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(s[r]);
  *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + n) = o;
}

// ---- launcher ---------------------------------------------------------------
// cfg ids (BM, BN, WM, NST, ROT, BK); kept in sync with ops.DGEMM_CONFIGS
struct DgCfg { int bm, bn, wm, nst, rot, bk; };
static const DgCfg kDgCfgs[] = {
    {256, 128, 4, 3, 0, 64},   // 0
    {128, 128, 2, 4, 0, 64},   // 1
    {64, 128, 2, 5, 0, 64},    // 2
    {256, 64, 8, 3, 0, 64},    // 3
    {128, 64, 4, 4, 0, 64},    // 4
    {64, 64, 2, 6, 0, 64},     // 5
    {128, 256, 2, 3, 0, 64},   // 6
    // the same tiles with the per-column-tile K rotation
    {64, 64, 2, 6, 1, 64},     // 7
    {128, 64, 4, 4, 1, 64},    // 8
    {64, 128, 2, 5, 1, 64},    // 9
    {128, 128, 2, 4, 1, 64},   // 10
    {128, 256, 2, 3, 1, 64},   // 11
    {256, 128, 4, 3, 1, 64},   // 12
    {256, 256, 4, 2, 1, 64},   // 13
    // M-tile stagger (ROT 2)
    {64, 64, 2, 6, 2, 64},     // 14
    {128, 64, 4, 4, 2, 64},    // 15
    {64, 128, 2, 5, 2, 64},    // 16
    {128, 128, 2, 4, 2, 64},   // 17
    {128, 256, 2, 3, 2, 64},   // 18
    // 128-deep K-steps (256-B LDS rows): half the ring barriers and counted
    // waits per weight byte of the 64-deep forms (ids 19-25 held 32-deep and
    // 224-column tiles until round 4; those lost every measured shape)
    {64, 96, 4, 4, 1, 128},    // 19
    {128, 64, 4, 3, 1, 128},   // 20
    {64, 64, 2, 4, 1, 128},    // 21
    {128, 128, 2, 2, 1, 128},  // 22
    {256, 64, 8, 2, 1, 128},   // 23
    {64, 128, 2, 3, 0, 128},   // 24
    {64, 64, 2, 5, 1, 128},    // 25
    // 64 x 96 tiles, 4 x 2 waves: 4 x 64 = 256 workgroups at M = 256 for the
    // 6144-column QKV without split-K (hipBLASLt's decomposition of that shape)
    {64, 96, 4, 4, 0, 64},     // 26
    {64, 96, 4, 6, 0, 64},     // 27
    {64, 96, 4, 4, 1, 64},     // 28
    // the same tile with 128-deep K-steps (256-B LDS rows): half the ring
    // barriers and waits per weight byte of the 64-deep form
    {64, 96, 4, 3, 0, 128},    // 29
    {64, 96, 4, 3, 1, 128},    // 30
    {64, 128, 2, 3, 1, 128},   // 31: 64 x 128, 128-deep (the last id below the NT bit)
};
constexpr int kNumDgCfgs = sizeof(kDgCfgs) / sizeof(kDgCfgs[0]);

int dgemm_num_configs() { return kNumDgCfgs; }

int dgemm_config(int cfg, int* bm, int* bn) {
  if (cfg < 0 || cfg >= kNumDgCfgs) return -1;
  *bm = kDgCfgs[cfg].bm;
  *bn = kDgCfgs[cfg].bn;
  return 0;
}

// K-steps per workgroup of the stream-K form and its slab count (the most
// pieces any tile is cut into): ops sizes the workspace as pieces x M x N
int dgemm_sk_per(int M, int N, int K, int bm, int bn, int bk, int groups) {
  const long total = (long)((M + bm - 1) / bm) * (N / bn) * (K / bk);
  const int G = groups > 0 ? groups : 256;
  return (int)std::max<long>(1, (total + G - 1) / G);
}

int dgemm_sk_pieces(int M, int N, int K, int cfg, int groups) {
  cfg &= 31;
  if (cfg < 0 || cfg >= kNumDgCfgs) return -1;
  const DgCfg c = kDgCfgs[cfg];
  const int nk = K / c.bk, per = dgemm_sk_per(M, N, K, c.bm, c.bn, c.bk, groups);
  return (nk + per - 1) / per + 1;
}

template <int BM, int BN, int WM, int NST, int EPI, int ROT, int NT, int BK>
static int dg_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, float* slabs,
                     unsigned* tickets, int M, int N, int K, long lda, long ldw, long ldc,
                     int splits, hipStream_t stream) {
  constexpr size_t ring = (size_t)NST * (BM + BN) * BK * sizeof(bf16_t);
  constexpr size_t xchg = EPI == 1 ? (size_t)BM * (BN / 2 + 4) * 4 : 0;   // SwiGLU hand-off
  constexpr size_t smem = ring > xchg ? ring : xchg;
  static_assert(smem <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(
        (const void*)dgemm_kernel<BM, BN, WM, NST, EPI, ROT, NT, BK>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int nwg = ((M + BM - 1) / BM) * (N / BN) * splits;
  dgemm_kernel<BM, BN, WM, NST, EPI, ROT, NT, BK><<<dim3(nwg), dim3(DTHREADS), smem, stream>>>(
      C, A, W, slabs, tickets, M, N, K, lda, ldw, ldc, splits);
  return (int)hipGetLastError();
}

// stream-K launch: G = `groups` workgroups (0: one per CU), then the reduction
template <int BM, int BN, int WM, int NST, int NT, int BK>
static int dg_sk_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, float* slabs, int M, int N,
                        int K, long lda, long ldw, long ldc, int groups, hipStream_t stream) {
  constexpr size_t smem = (size_t)NST * (BM + BN) * BK * sizeof(bf16_t);
  static_assert(smem <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)dgemm_sk_kernel<BM, BN, WM, NST, NT, BK>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int nk = K / BK, total = ((M + BM - 1) / BM) * (N / BN) * nk;
  const int per = dgemm_sk_per(M, N, K, BM, BN, BK, groups);
  const int G = (total + per - 1) / per;
  dgemm_sk_kernel<BM, BN, WM, NST, NT, BK><<<dim3(G), dim3(DTHREADS), smem, stream>>>(
      A, W, slabs, M, N, K, lda, ldw, per);
  const long n4 = (long)M * (N / 4);
  dg_sk_reduce_kernel<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream>>>(
      C, slabs, M, N, ldc, BM, BN, nk, per);
  return (int)hipGetLastError();
}

int dgemm(void* C, const void* A, const void* W, float* slabs, unsigned* tickets, int n_tickets,
          int M, int N, int K, long lda, long ldw, long ldc, int cfg, int splits, int epi,
          hipStream_t stream) {
  if (M <= 0) return 0;
  const int nt = (cfg >> 5) & 1;      // bit 5: non-temporal weight stream
  const int sk = (cfg >> 6) & 1;      // bit 6: stream-K, `splits` = workgroups (0: 256)
  cfg &= 31;
  if (cfg < 0 || cfg >= kNumDgCfgs || splits < 0 || epi < 0 || epi > 3) return -1;
  const DgCfg c = kDgCfgs[cfg];
  if (sk) {
    if (epi != 0 || N % c.bn != 0 || K % c.bk != 0) return -1;
    if (slabs == nullptr) return -2;
  } else if (splits < 1 || N % c.bn != 0 || K % (splits * c.bk) != 0) {
    return -1;
  }
  if (epi == 2 && slabs == nullptr) return -2;
  if (!sk && splits > 1 && epi != 2) {
    if (slabs == nullptr || tickets == nullptr) return -2;
    if (((M + c.bm - 1) / c.bm) * (N / c.bn) > n_tickets) return -3;
  }
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
#define LMX_DG_E(BM, BN, WM, NST, ROT, NT, BK)                                                 \
  if (sk)                                                                                     \
    return dg_sk_launch<BM, BN, WM, NST, NT, BK>(C_, A_, W_, slabs, M, N, K, lda, ldw, ldc,   \
                                                 splits, stream);                             \
  if (epi == 3) {                                                                             \
    if constexpr ((BN / (8 / WM)) % 32 == 0)                                                  \
      return dg_launch<BM, BN, WM, NST, 3, ROT, NT, BK>(C_, A_, W_, slabs, tickets, M, N, K, \
                                                        lda, ldw, ldc, splits, stream);       \
    return -1;                                                                                \
  }                                                                                           \
  if (epi == 1)                                                                               \
    return dg_launch<BM, BN, WM, NST, 1, ROT, NT, BK>(C_, A_, W_, slabs, tickets, M, N, K, lda, \
                                                      ldw, ldc, splits, stream);              \
  if (epi == 2)                                                                               \
    return dg_launch<BM, BN, WM, NST, 2, ROT, NT, BK>(C_, A_, W_, slabs, tickets, M, N, K, lda, \
                                                      ldw, ldc, splits, stream);              \
  return dg_launch<BM, BN, WM, NST, 0, ROT, NT, BK>(C_, A_, W_, slabs, tickets, M, N, K, lda,   \
                                                    ldw, ldc, splits, stream);
#define LMX_DG(ID, BM, BN, WM, NST, ROT, BK)                                                  \
  case ID:                                                                                    \
    if (nt) { LMX_DG_E(BM, BN, WM, NST, ROT, 1, BK) }                                         \
    LMX_DG_E(BM, BN, WM, NST, ROT, 0, BK)
  switch (cfg) {
    LMX_DG(0, 256, 128, 4, 3, 0, 64)
    LMX_DG(1, 128, 128, 2, 4, 0, 64)
    LMX_DG(2, 64, 128, 2, 5, 0, 64)
    LMX_DG(3, 256, 64, 8, 3, 0, 64)
    LMX_DG(4, 128, 64, 4, 4, 0, 64)
    LMX_DG(5, 64, 64, 2, 6, 0, 64)
    LMX_DG(6, 128, 256, 2, 3, 0, 64)
    LMX_DG(7, 64, 64, 2, 6, 1, 64)
    LMX_DG(8, 128, 64, 4, 4, 1, 64)
    LMX_DG(9, 64, 128, 2, 5, 1, 64)
    LMX_DG(10, 128, 128, 2, 4, 1, 64)
    LMX_DG(11, 128, 256, 2, 3, 1, 64)
    LMX_DG(12, 256, 128, 4, 3, 1, 64)
    LMX_DG(13, 256, 256, 4, 2, 1, 64)
    LMX_DG(14, 64, 64, 2, 6, 2, 64)
    LMX_DG(15, 128, 64, 4, 4, 2, 64)
    LMX_DG(16, 64, 128, 2, 5, 2, 64)
    LMX_DG(17, 128, 128, 2, 4, 2, 64)
    LMX_DG(18, 128, 256, 2, 3, 2, 64)
    LMX_DG(19, 64, 96, 4, 4, 1, 128)
    LMX_DG(20, 128, 64, 4, 3, 1, 128)
    LMX_DG(21, 64, 64, 2, 4, 1, 128)
    LMX_DG(22, 128, 128, 2, 2, 1, 128)
    LMX_DG(23, 256, 64, 8, 2, 1, 128)
    LMX_DG(24, 64, 128, 2, 3, 0, 128)
    LMX_DG(25, 64, 64, 2, 5, 1, 128)
    LMX_DG(26, 64, 96, 4, 4, 0, 64)
    LMX_DG(27, 64, 96, 4, 6, 0, 64)
    LMX_DG(28, 64, 96, 4, 4, 1, 64)
    LMX_DG(29, 64, 96, 4, 3, 0, 128)
    LMX_DG(30, 64, 96, 4, 3, 1, 128)
    LMX_DG(31, 64, 128, 2, 3, 1, 128)
  }
#undef LMX_DG
#undef LMX_DG_E
  return -1;
}

}  // namespace lmx
