// K13 design points that lost to the shipped 2-phase ping-pong kernel
// (llm_mcp_amd/csrc/kernels/pgemm.hip, variant 2) and are kept for the lab only:
//   variant 1: 8-wave ping-pong with 4 phases per 64-deep K-step (one quadrant
//              of 16 MFMAs per barrier interval): 0.60 MFMA util on l8b o;
//   variant 3: the 2-phase ping-pong with the DMA split 4/4 over the phases;
//   variant 0: 4 waves (one per SIMD), 192 x 256 tiles, register double-buffered
//              fragments (profiles/r3_k13_and_decode_sk.md).
// Included into tools/pgemm_lab.cpp (single translation unit with pgemm.hip).
#include "pgemm.hip"

namespace lmx {
namespace {

struct PgRegs {
  f32x4_t acc[2][2][4][2];       // [quadrant m][quadrant n][16-row tile][16-col tile]
  bf16x8_t a[4][2];              // A fragments of the current M-half: [16-row tile][k32]
  bf16x8_t w[2][2];              // W fragments of the current N-half: [16-col tile][k32]
};


template <int QM, int QN, bool ZERO>
__device__ __forceinline__ void pg_mma(PgRegs& R) {
  const bf16x8_t(&a)[4][2] = R.a;
  const bf16x8_t(&w)[2][2] = R.w;
  const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        R.acc[QM][QN][i][j] =
            mfma16(w[j][kk], a[i][kk], (ZERO && kk == 0) ? z : R.acc[QM][QN][i][j]);
}

// quadrant (QM, QN) of the tile described by O: NS stores per wave, always
// issued (rows >= M are out of the buffer range and dropped)

// DMA issue schedule (one half-tile per phase; a half is refilled in the
// phase after its last ds_read): phase 0 of K-step s issues W N-half 0 of
// s+1, phases 1-3 A M-half 0, W N-half 1, A M-half 1 of s+2.  Fragment reads
// (same phase as their MFMAs): phase 0 A0 + W0, 1 W1, 2 A1, 3 W0 again.
//
// vmcnt at the end of phase Q's read half: the youngest DMA the next phase
// reads was issued D phases back (Q 0/1: 6 -- W1 / A1 of this K-step; Q 3: 3 --
// W0 of the next K-step; Q 2: the next phase reads nothing new, no wait);
// every vector-memory op issued after it counts -- 2 DMA per phase plus the
// epilogue stores of the window (NS per store phase; the store phases are the
// 4 phases of a tile's first K-step S, so the windows of K-steps S, S+1 and
// S+2 hold some of them).  Returns -1 for "no wait".
template <int Q, int MODE, int ACT>
constexpr int pg_vmcnt() {
  if constexpr (Q == 2) return -1;
  constexpr int base = Q == 3 ? 6 : 12;
  constexpr int ns = pg_ns<ACT>();
  if constexpr (MODE == MODE_K0) return base + ns * (Q == 0 ? 1 : Q == 1 ? 2 : 3);
  else if constexpr (MODE == MODE_K1) return base + ns * (Q == 3 ? 0 : 4);
  else if constexpr (MODE == MODE_K2) return base + ns * (Q == 0 ? 1 : 0);
  else return base;
}

template <int Q, int MODE, int ACT, int BIAS>
__device__ __forceinline__ void pg_phase(PgRegs& R, char* smem, int stage, const PgLoad& L1,
                                         const PgLoad& L2, const PgOut& O, const PgThr& T) {
  constexpr int QM = (Q == 2 || Q == 3) ? 1 : 0;
  constexpr int QN = (Q == 1 || Q == 2) ? 1 : 0;
  // ---- read half: epilogue of the previous tile's quadrant, fragments, DMA
  if constexpr (MODE == MODE_K0) pg_store<QM, QN, ACT, BIAS>(R, O, T, smem);
  if constexpr (Q == 0) {
    pg_read_a<HA0>(R.a, smem, stage, T);
    pg_read_w<0>(R.w, smem, stage, T);
    pg_issue<HW0>(smem, stage ^ 1, L1, T);
  } else if constexpr (Q == 1) {
    pg_read_w<1>(R.w, smem, stage, T);
    pg_issue<HA0>(smem, stage, L2, T);
  } else if constexpr (Q == 2) {
    pg_read_a<HA1>(R.a, smem, stage, T);
    pg_issue<HW1>(smem, stage, L2, T);
  } else {
    pg_read_w<0>(R.w, smem, stage, T);
    pg_issue<HA1>(smem, stage, L2, T);
  }
  constexpr int vm = pg_vmcnt<Q, MODE, ACT>();
  if constexpr (vm >= 0) pg_vmwait<vm>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pg_barrier();
  // ---- MFMA half
  __builtin_amdgcn_s_setprio(1);
  pg_mma<QM, QN, MODE == MODE_K0 || MODE == MODE_FIRST>(R);
  __builtin_amdgcn_s_setprio(0);
  pg_barrier();
}

template <int MODE, int ACT, int BIAS>
__device__ __forceinline__ void pg_step(PgRegs& R, char* smem, int stage, const PgLoad& L1,
                                        const PgLoad& L2, const PgOut& O, const PgThr& T) {
  pg_phase<0, MODE, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
  pg_phase<1, MODE, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
  pg_phase<2, MODE, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
  pg_phase<3, MODE, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
}

}  // namespace


template <int ACT, int BIAS>
__global__ void __launch_bounds__(PG_THREADS, 1) pgemm_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ bias, int M, int N, int K, int lda, int ldw, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int r = xcd_remap(blockIdx.x, G);
  const int my_tiles = (ntiles - r + G - 1) / G;
  const int nk = K / 64;

  PgThr T;
  const int lane = threadIdx.x & 63;
  T.wave = threadIdx.x >> 6;
  T.wm = T.wave >> 2;
  T.wn = T.wave & 3;
  T.fr = lane & 15;
  T.fg = lane >> 4;
  T.ldc = ldc;
  {
    // DMA: instr i of a half covers image rows [64i, 64i+64); this lane's row
    // 64i + 8 wave + lane/8, chunk lane%8 read from source chunk ^ swizzle
    const int sc = (lane & 7) ^ ((4 * T.wave + (lane >> 4)) & 7);
    const int rr = 8 * T.wave + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) T.a_voff[h][i] = (128 * i + 64 * h + rr) * lda * 2 + sc * 16;
    // W image row lr = 64i + rr -> tile column (2i + wave/4) * 64 + 32h + 8 (wave%4) + lane/8
    T.w_voff = ((T.wave >> 2) * 64 + 8 * (T.wave & 3) + (lane >> 3)) * ldw * 2 + sc * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) T.w_uoff[h][i] = (128 * i + 32 * h) * ldw * 2;
    T.ra_off = (T.wm * 64 + T.fr) * 128;
    T.rw_off = (T.wn * 32 + T.fr) * 128;
    const int s = (T.fr >> 1) & 7;
    T.co[0] = 16 * (T.fg ^ s);
    T.co[1] = 16 * ((4 + T.fg) ^ s);
  }

  if constexpr (BIAS) {
    // bias row staged once (no DMA in flight yet)
    for (int c = threadIdx.x * 8; c < N; c += PG_THREADS * 8)
      *reinterpret_cast<bf16x8_t*>(smem + PG_RING_B + c * 2) =
          *reinterpret_cast<const bf16x8_t*>(bias + c);
    __syncthreads();
  }

  auto set_tile = [&](PgLoad& L, int t) {
    int tm, tn;
    pg_tile_coords(t * G + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const long rows = M - m0;
    const long abytes = rows * (long)lda * 2;
    L.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)m0 * lda), (short)0,
                                             (int)(abytes < 0x7fffffffL ? abytes : 0x7fffffffL),
                                             0x00020000);
    const long wbytes = 256L * ldw * 2;
    L.rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (long)n0 * ldw), (short)0, (int)wbytes,
                                             0x00020000);
  };
  auto set_out = [&](PgOut& O, int t) {
    int tm, tn;
    pg_tile_coords(t * G + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256;
    const long cbytes = (long)(M - m0) * ldc * 2;
    O.rc = __builtin_amdgcn_make_buffer_rsrc((void*)(C + (long)m0 * ldc), (short)0,
                                             (int)(cbytes < 0x7fffffffL ? cbytes : 0x7fffffffL),
                                             0x00020000);
    O.n0 = tn * 256;
  };
  auto advance = [&](PgLoad& L) {
    if (L.done) return;
    if (++L.k == nk) {
      if (L.tile + 1 >= my_tiles) {
        L.done = true;            // keep re-issuing the last K-step into free halves
        L.k = nk - 1;
        return;
      }
      L.k = 0;
      ++L.tile;
      set_tile(L, L.tile);
    }
    L.kbyte = L.k * 128;
  };

  PgRegs R;
  PgLoad L1, L2;                    // K-steps s+1 and s+2 of the running K-step s
  L2.k = 0;
  L2.tile = 0;
  L2.kbyte = 0;
  L2.done = false;
  set_tile(L2, 0);
  PgOut O;
  set_out(O, 0);

  // ---- prologue: the DMA of the phases before K-step 0, in loop order
  pg_issue<HA0>(smem, 0, L2, T);
  pg_issue<HW1>(smem, 0, L2, T);
  pg_issue<HA1>(smem, 0, L2, T);
  pg_issue<HW0>(smem, 0, L2, T);
  advance(L2);
  pg_issue<HA0>(smem, 1, L2, T);
  pg_issue<HW1>(smem, 1, L2, T);
  pg_issue<HA1>(smem, 1, L2, T);
  L1 = L2;
  advance(L2);
  pg_vmwait<6>();                   // A0, W0 of K-step 0
  pg_barrier();
  if (T.wm == 1) pg_barrier();      // waves 4-7 run one barrier behind

  int stage = 0;
  auto next = [&]() {
    L1 = L2;
    advance(L2);
    stage ^= 1;
  };
  for (int t = 0; t < my_tiles; ++t) {
    if (t == 0) {
      pg_step<MODE_FIRST, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
      next();
      pg_step<MODE_PLAIN, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
      next();
      pg_step<MODE_PLAIN, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
    } else {
      pg_step<MODE_K0, ACT, BIAS>(R, smem, stage, L1, L2, O, T);   // stores tile t-1
      next();
      set_out(O, t);
      pg_step<MODE_K1, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
      next();
      pg_step<MODE_K2, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
    }
    next();
    for (int k = 3; k < nk; ++k) {
      pg_step<MODE_PLAIN, ACT, BIAS>(R, smem, stage, L1, L2, O, T);
      next();
    }
  }
  if (T.wm == 0) pg_barrier();
  pg_vmwait<0>();                   // trailing (re-issued) DMA lands before the LDS is released
  pg_store<0, 0, ACT, BIAS>(R, O, T, smem);
  pg_store<0, 1, ACT, BIAS>(R, O, T, smem);
  pg_store<1, 1, ACT, BIAS>(R, O, T, smem);
  pg_store<1, 0, ACT, BIAS>(R, O, T, smem);
}


// ============================================================================
// K13 variant 0 (default): 4 waves, one per SIMD, (16 TM) x 128 wave tiles
// ============================================================================
// The ping-pong form above keeps a quadrant's 16 MFMAs (256 cycles) per
// barrier-delimited interval and re-reads the fragments of every quadrant
// (8 waves x 28 ds_read_b128 per 64-deep K-step); measured (l8b o, M 32768):
// 0.60 MFMA utilisation with ~35 % of the wave cycles parked at barriers /
// waits.  This variant gives each SIMD ONE wave with a (16 TM) x 128 tile
// (TM x 8 accumulator tiles in the AGPR half of the 512-register budget of
// one wave per SIMD): per 32-deep K-step a wave reads TM A + 8 W fragments for
// 8 TM MFMAs, and the next K-step's fragments are read into a second register
// set while the current MFMAs issue (explicit sched_group_barrier
// interleave: per 8 MFMAs about 2 ds_read_b128 + 1 LDS-DMA), so there is one
// barrier per K-step and no exposed LDS latency.  TM = 6 (a 192 x 256
// workgroup tile, 192 accumulator AGPRs) is the default: at TM = 8 the 256
// accumulator registers fill the AGPR file exactly and hipcc rotates ~7
// accumulator tiles through VGPRs (v_accvgpr copies + s_nop MFMA hazards in
// the loop).
//   * LDS: 4 stages x (A (32 TM) x 32 + W 256 x 32) bf16; the DMA issued in
//     K-step s fills K-step s+4 into the stage whose fragments were read in
//     s-1 (every wave passed the barrier of s after reading them); the wait
//     at the top of K-step s retires the batch of s-3 (the stage read in s):
//     two younger batches in flight, ~2 K-steps (~2k cycles) per DMA;
//   * persistent tile walk and one load stream across tiles as above; the
//     epilogue (after a tile's last K-step) widens each lane's 4-column runs
//     to 8 columns with v_permlane16_swap (lanes l and l+16 trade the two
//     tiles of a 16-column pair) and stores 16 B per lane (4 TM stores per
//     wave), counted by the waits of the next three K-steps; the accumulators
//     are zeroed before the next tile's first K-step (one loop body for every
//     K-step keeps them in fixed registers).
namespace {

constexpr int P4_THREADS = 256;
constexpr int P4_NST = 4;
constexpr int P4_WOPB = 256 * 32 * 2;           // W image per stage: 16 KB

template <int TM> struct P4Geo {
  static constexpr int BM = 32 * TM;             // workgroup tile rows
  static constexpr int AOPB = BM * 32 * 2;       // A image per stage
  static constexpr int STAGE = AOPB + P4_WOPB;
  static constexpr int RING = P4_NST * STAGE;
  static constexpr int NA = TM / 2;              // A DMA per wave per K-step (16 rows x 64 B each)
  static constexpr int ND = NA + 4;              // + 4 W DMA
  static constexpr int NS = 4 * TM;              // epilogue stores per wave
  static_assert(TM % 2 == 0 && TM <= 8, "TM");
};

// 64-B rows (32 bf16): XOR of the 16-B chunk with {0,2,3,1}[(r/4) mod 4], so the
// four 16-lane groups of a ds_read_b128 (16 rows x chunk fg) hit 16 distinct
// 16-B slots of the 256-B bank row (the BK 32 image of dgemm.hip)
__device__ __forceinline__ int p4_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int TM>
struct P4Frag {
  bf16x8_t a[TM], w[8];
};

struct P4Thr {
  int a_voff[4];        // A source offset of this lane for A DMA d (row part + chunk)
  int w_voff;           // W source offset (thread part); W DMA d adds 64 d rows (uniform)
  int w_row64;          // 64 W rows in bytes
  int rd_a, rd_w;       // fragment read offsets in a stage's A / W image (bytes)
  int wave, wm, wn, fr, fg;
  int ldc;
};

struct P4Load {
  __amdgpu_buffer_rsrc_t ra, rw;
  int kbyte, k, tile;
  bool done;
};

struct P4Out {
  __amdgpu_buffer_rsrc_t rc;
  int n0;
};

// DMA d of a K-step: d < NA: A rows (4 d + wave) * 16 ..+16; else W rows (4 (d-NA) + wave) * 16
template <int TM, int D>
__device__ __forceinline__ void p4_issue(char* smem, int stage, const P4Load& L, const P4Thr& T) {
  using G = P4Geo<TM>;
  if constexpr (D < G::NA) {
    char* dst = smem + stage * G::STAGE + ((4 * D + T.wave) * 16) * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(L.ra, (lds_void_t*)dst, 16, T.a_voff[D], L.kbyte, 0,
                                             0);
  } else {
    constexpr int E = D - G::NA;
    char* dst = smem + stage * G::STAGE + G::AOPB + ((4 * E + T.wave) * 16) * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(L.rw, (lds_void_t*)dst, 16, T.w_voff,
                                             L.kbyte + E * T.w_row64, 0, 0);
  }
}

template <int TM>
__device__ __forceinline__ void p4_issue_all(char* smem, int stage, const P4Load& L,
                                             const P4Thr& T) {
  p4_issue<TM, 0>(smem, stage, L, T);
  p4_issue<TM, 1>(smem, stage, L, T);
  p4_issue<TM, 2>(smem, stage, L, T);
  p4_issue<TM, 3>(smem, stage, L, T);
  p4_issue<TM, 4>(smem, stage, L, T);
  p4_issue<TM, 5>(smem, stage, L, T);
  p4_issue<TM, 6>(smem, stage, L, T);
  if constexpr (P4Geo<TM>::ND > 7) p4_issue<TM, 7>(smem, stage, L, T);
  static_assert(P4Geo<TM>::ND == 7 || P4Geo<TM>::ND == 8, "DMA count");
}

template <int TM>
__device__ __forceinline__ void p4_read_a(P4Frag<TM>& F, int i, const char* smem, int stage,
                                          const P4Thr& T) {
  F.a[i] = *reinterpret_cast<const bf16x8_t*>(smem + stage * P4Geo<TM>::STAGE + T.rd_a + i * 1024);
}

template <int TM>
__device__ __forceinline__ void p4_read_w(P4Frag<TM>& F, int j, const char* smem, int stage,
                                          const P4Thr& T) {
  F.w[j] = *reinterpret_cast<const bf16x8_t*>(smem + stage * P4Geo<TM>::STAGE + P4Geo<TM>::AOPB +
                                              T.rd_w + j * 1024);
}

// group I of a K-step: the 8 MFMAs of accumulator row I, the reads of the next
// K-step's A[I] and W[I] (and W[TM + I] for the first 8 - TM groups), DMA I
// (and DMA TM + I for the first ND - TM groups), in a fixed order pinned by
// sched_barrier (hipcc's sched_group_barrier solver clustered every read and
// DMA ahead of the MFMAs here): 2 MFMA | read A | 2 MFMA | DMA | 2 MFMA | read W
// (| DMA) | 2 MFMA
template <int TM, int I>
__device__ __forceinline__ void p4_group(f32x4_t (&acc)[TM][8], const P4Frag<TM>& F,
                                         P4Frag<TM>& G, char* smem, int rstage, int wstage,
                                         const P4Load& L, const P4Thr& T) {
  acc[I][0] = mfma16(F.w[0], F.a[I], acc[I][0]);
  acc[I][1] = mfma16(F.w[1], F.a[I], acc[I][1]);
  __builtin_amdgcn_sched_barrier(0);
  p4_read_a<TM>(G, I, smem, rstage, T);
  __builtin_amdgcn_sched_barrier(0);
  acc[I][2] = mfma16(F.w[2], F.a[I], acc[I][2]);
  acc[I][3] = mfma16(F.w[3], F.a[I], acc[I][3]);
  __builtin_amdgcn_sched_barrier(0);
  p4_issue<TM, I>(smem, wstage, L, T);
  __builtin_amdgcn_sched_barrier(0);
  acc[I][4] = mfma16(F.w[4], F.a[I], acc[I][4]);
  acc[I][5] = mfma16(F.w[5], F.a[I], acc[I][5]);
  __builtin_amdgcn_sched_barrier(0);
  p4_read_w<TM>(G, I, smem, rstage, T);
  if constexpr (I < 8 - TM) p4_read_w<TM>(G, TM + I, smem, rstage, T);
  if constexpr (I < P4Geo<TM>::ND - TM) p4_issue<TM, TM + I>(smem, wstage, L, T);
  __builtin_amdgcn_sched_barrier(0);
  acc[I][6] = mfma16(F.w[6], F.a[I], acc[I][6]);
  acc[I][7] = mfma16(F.w[7], F.a[I], acc[I][7]);
  __builtin_amdgcn_sched_barrier(0);
}

// `after_store`: one of the three K-steps after a tile epilogue, whose stores
// are younger than the batch this wait retires
template <int TM>
__device__ __forceinline__ void p4_step(f32x4_t (&acc)[TM][8], const P4Frag<TM>& F,
                                        P4Frag<TM>& G, char* smem, int s, bool after_store,
                                        const P4Load& L, const P4Thr& T) {
  constexpr int base = 2 * P4Geo<TM>::ND, post = base + P4Geo<TM>::NS;
  static_assert(post < 64, "vmcnt");
  if (after_store)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(post) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(base) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  const int rstage = (s + 1) & 3, wstage = s & 3;
  p4_group<TM, 0>(acc, F, G, smem, rstage, wstage, L, T);
  p4_group<TM, 1>(acc, F, G, smem, rstage, wstage, L, T);
  p4_group<TM, 2>(acc, F, G, smem, rstage, wstage, L, T);
  p4_group<TM, 3>(acc, F, G, smem, rstage, wstage, L, T);
  p4_group<TM, 4>(acc, F, G, smem, rstage, wstage, L, T);
  p4_group<TM, 5>(acc, F, G, smem, rstage, wstage, L, T);
  if constexpr (TM > 6) {
    p4_group<TM, 6>(acc, F, G, smem, rstage, wstage, L, T);
    p4_group<TM, 7>(acc, F, G, smem, rstage, wstage, L, T);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// tile epilogue: 4 TM stores per wave (16-B after the permlane16 widening; 8-B
// SwiGLU outputs), always issued -- rows >= M are outside the buffer range
template <int TM, int ACT, int BIAS>
__device__ __forceinline__ void p4_store(const f32x4_t (&acc)[TM][8], const P4Out& O,
                                         const P4Thr& T, const char* smem) {
  // byte offsets: the row part stays in the VGPR offset (the buffer range check
  // drops rows >= M), the tile column n0 goes to the SGPR offset, the 16-col
  // pair jp to the instruction offset
  if constexpr (ACT == 3) {
    int cthr = (T.wm * 16 * TM + T.fr) * T.ldc * 2 + (T.wn * 64 + 4 * T.fg) * 2;
    asm volatile("" : "+v"(cthr));
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int voff = cthr + 16 * i * T.ldc * 2;
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const f32x4_t g = acc[i][2 * jp], u = acc[i][2 * jp + 1];
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(g[r] / (1.f + __expf(-g[r])) * u[r]);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o), O.rc,
                                              voff + jp * 32, O.n0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    f32x4_t b[8];
    if constexpr (BIAS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bf16x4_t bb = *reinterpret_cast<const bf16x4_t*>(
            smem + P4Geo<TM>::RING + (O.n0 + T.wn * 128 + 16 * j + 4 * T.fg) * 2);
#pragma unroll
        for (int r = 0; r < 4; ++r) b[j][r] = bf2f((uint16_t)bb[r]);
      }
    }
    const int odd = T.fg & 1;
    int cthr = (T.wm * 16 * TM + T.fr) * T.ldc * 2 +
               (T.wn * 128 + 16 * odd + 8 * (T.fg >> 1)) * 2;
    // laundered: the per-store offsets are recomputed here, not hoisted out of
    // the tile loop into live (spilled) registers
    asm volatile("" : "+v"(cthr));
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int voff = cthr + 16 * i * T.ldc * 2;
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        unsigned d[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4_t v = acc[i][2 * jp + h];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            float x0 = v[2 * q], x1 = v[2 * q + 1];
            if constexpr (BIAS) {
              x0 += b[2 * jp + h][2 * q];
              x1 += b[2 * jp + h][2 * q + 1];
            }
            d[h][q] = pack_bf16x2(pg_act<ACT>(x0), pg_act<ACT>(x1));
          }
        }
        // lanes of 16-lane rows 0/2 keep tile 2jp and take columns 4-7 from the
        // row above; rows 1/3 take tile 2jp+1 columns 0-3 from the row below
        const auto p = __builtin_amdgcn_permlane16_swap(d[0][0], d[1][0], false, false);
        const auto q = __builtin_amdgcn_permlane16_swap(d[0][1], d[1][1], false, false);
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t o = {p[0], q[0], p[1], q[1]};
        __builtin_amdgcn_raw_buffer_store_b128(o, O.rc, voff + jp * 64, O.n0 * 2, 0);
        __builtin_amdgcn_sched_barrier(0);   // one tile pair at a time (no hoisted acc reads)
      }
    }
  }
}

}  // namespace

template <int TM, int ACT, int BIAS>
__global__ void __launch_bounds__(P4_THREADS, 1) pgemm4_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ bias, int M, int N, int K, int lda, int ldw, int ldc) {
  using Geo = P4Geo<TM>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_m = (M + Geo::BM - 1) / Geo::BM, tiles_n = N / 256, ntiles = tiles_m * tiles_n;
  const int Gd = gridDim.x;
  const int r = xcd_remap(blockIdx.x, Gd);
  const int my_tiles = (ntiles - r + Gd - 1) / Gd;
  const int nk = K / 32;

  P4Thr T;
  const int lane = threadIdx.x & 63;
  T.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: SGPR math
  T.wm = T.wave >> 1;
  T.wn = T.wave & 1;
  T.fr = lane & 15;
  T.fg = lane >> 4;
  T.ldc = ldc;
  {
    // DMA of wave w: image rows (4 d + w) * 16 + lane / 4, chunk lane % 4
    const int rr = lane >> 2;
    const int sc = (lane & 3) ^ p4_swz(rr);
#pragma unroll
    for (int d = 0; d < 4; ++d) T.a_voff[d] = ((4 * d + T.wave) * 16 + rr) * lda * 2 + sc * 16;
    T.w_voff = (T.wave * 16 + rr) * ldw * 2 + sc * 16;
    T.w_row64 = 64 * ldw * 2;
    const int ch = 16 * (T.fg ^ p4_swz(T.fr));
    T.rd_a = (T.wm * 16 * TM + T.fr) * 64 + ch;
    T.rd_w = (T.wn * 128 + T.fr) * 64 + ch;
  }

  if constexpr (BIAS) {
    for (int c = threadIdx.x * 8; c < N; c += P4_THREADS * 8)
      *reinterpret_cast<bf16x8_t*>(smem + Geo::RING + c * 2) =
          *reinterpret_cast<const bf16x8_t*>(bias + c);
    __syncthreads();
  }

  auto set_tile = [&](P4Load& L, int t) {
    int tm, tn;
    pg_tile_coords(t * Gd + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * Geo::BM, n0 = tn * 256;
    const long abytes = (long)(M - m0) * lda * 2;
    L.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)m0 * lda), (short)0,
                                             (int)(abytes < 0x7fffffffL ? abytes : 0x7fffffffL),
                                             0x00020000);
    L.rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (long)n0 * ldw), (short)0,
                                             (int)(256L * ldw * 2), 0x00020000);
  };
  auto set_out = [&](P4Out& O, int t) {
    int tm, tn;
    pg_tile_coords(t * Gd + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * Geo::BM;
    const long cbytes = (long)(M - m0) * ldc * 2;
    O.rc = __builtin_amdgcn_make_buffer_rsrc((void*)(C + (long)m0 * ldc), (short)0,
                                             (int)(cbytes < 0x7fffffffL ? cbytes : 0x7fffffffL),
                                             0x00020000);
    O.n0 = tn * 256;
  };
  auto advance = [&](P4Load& L) {
    if (L.done) return;
    if (++L.k == nk) {
      if (L.tile + 1 >= my_tiles) {
        L.done = true;            // keep re-issuing the last K-step into free stages
        L.k = nk - 1;
        return;
      }
      L.k = 0;
      ++L.tile;
      set_tile(L, L.tile);
    }
    L.kbyte = L.k * 64;
  };

  f32x4_t acc[TM][8];
  P4Frag<TM> F0, F1;
  P4Load L;
  L.k = 0;
  L.tile = 0;
  L.kbyte = 0;
  L.done = false;
  set_tile(L, 0);
  P4Out O;
  set_out(O, 0);

  // ---- prologue: K-steps 0..3 into stages 0..3, fragments of K-step 0
#pragma unroll
  for (int st = 0; st < P4_NST; ++st) {
    p4_issue_all<TM>(smem, st, L, T);
    advance(L);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * Geo::ND) : "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < TM; ++i) p4_read_a<TM>(F0, i, smem, 0, T);
#pragma unroll
  for (int j = 0; j < 8; ++j) p4_read_w<TM>(F0, j, smem, 0, T);

  int s = 0;
  for (int t = 0; t < my_tiles; ++t) {
    // acc lives within one tile (zeroed here, stored at the end): no
    // accumulator value is carried around the tile loop
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nk; k += 2) {
      const bool after = t > 0 && k < 3;
      p4_step<TM>(acc, F0, F1, smem, s, after, L, T);
      advance(L); ++s;
      p4_step<TM>(acc, F1, F0, smem, s, after && k + 1 < 3, L, T);
      advance(L); ++s;
    }
    set_out(O, t);
    p4_store<TM, ACT, BIAS>(acc, O, T, smem);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing DMA lands before the LDS is released
}

constexpr int P4_TM = 6;

template <int ACT, int BIAS>
static int pg_lab_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, const bf16_t* bias, int M,
                         int N, int K, int lda, int ldw, int ldc, int grid, int variant,
                         hipStream_t stream) {
  constexpr size_t ring = P4Geo<P4_TM>::RING > PG_RING_B ? P4Geo<P4_TM>::RING : PG_RING_B;
  constexpr size_t smem = ring + (BIAS ? PG_MAX_BIAS * 2 : 0);
  static_assert(smem <= 160 * 1024, "LDS");
  const void* fn = variant == 1   ? (const void*)pgemm_kernel<ACT, BIAS>
                   : variant == 2 ? (const void*)pgemm_pp2_kernel<ACT, BIAS, 0>
                   : variant == 3 ? (const void*)pgemm_pp2_kernel<ACT, BIAS, 1>
                                  : (const void*)pgemm4_kernel<P4_TM, ACT, BIAS>;
  const hipError_t e =
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return (int)e;
  if (variant == 1)
    pgemm_kernel<ACT, BIAS><<<dim3(grid), dim3(PG_THREADS), smem, stream>>>(C, A, W, bias, M, N,
                                                                          K, lda, ldw, ldc);
  else if (variant == 2)
    pgemm_pp2_kernel<ACT, BIAS, 0><<<dim3(grid), dim3(PG_THREADS), smem, stream>>>(
        C, A, W, bias, M, N, K, lda, ldw, ldc);
  else if (variant == 3)
    pgemm_pp2_kernel<ACT, BIAS, 1><<<dim3(grid), dim3(PG_THREADS), smem, stream>>>(
        C, A, W, bias, M, N, K, lda, ldw, ldc);
  else
    pgemm4_kernel<P4_TM, ACT, BIAS><<<dim3(grid), dim3(P4_THREADS), smem, stream>>>(
        C, A, W, bias, M, N, K, lda, ldw, ldc);
  return (int)hipGetLastError();
}

// plain / SiLU epilogues of any variant (same operand rules as pgemm())
int pgemm_lab(void* C, const void* A, const void* W, int M, int N, int K, int act, int grid,
              int variant, hipStream_t stream) {
  if (variant < 0 || variant > 3 || N % 256 || K % 64 || K < 192 || (act != 0 && act != 2))
    return -1;
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
  if (act == 2)
    return pg_lab_launch<2, 0>(C_, A_, W_, nullptr, M, N, K, K, K, N, grid, variant, stream);
  return pg_lab_launch<0, 0>(C_, A_, W_, nullptr, M, N, K, K, K, N, grid, variant, stream);
}

}  // namespace lmx
