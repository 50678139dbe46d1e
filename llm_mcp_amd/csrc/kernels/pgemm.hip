// K13: large-M projection GEMM (prefill chunks, embedding-model batches) --
// the projections behind the chat and embedding requests that the reference
// proxies to Ollama (reference core/internal/api/handlers.go:1942 proxyOllamaEmbed,
// :2427 streamOllamaChat); K13-SK below serves decode batches:
//     C[M, N] = epi(A[M, K] . W[N, K]^T)     bf16 in, fp32 accumulate, bf16 out
// epi: optional bias (staged in LDS), then none / GELU(tanh) / SiLU / GELU(erf),
// or SwiGLU over 16-row gate/up pairs (W from ops.interleave_gate_up(w, 16);
// C then has N/2 columns).
//
// The structure is chosen for one 512-thread workgroup per CU holding a
// 256 x 256 output tile (cdna guide §5 "the 256² 8-phase template", MI355X
// microarch guide §LDS / MFMA):
//   * persistent: gridDim = min(tiles, CUs); a workgroup walks its tiles
//     (linear id i * grid + xcd_remap(block), grouped 8 M-tiles x N so one XCD's
//     32 concurrent tiles share 8 A panels and 4 W panels in its L2) and the
//     k-steps of consecutive tiles form ONE load stream: the next tile's first
//     K-steps are already in LDS when the current tile's last MFMA retires, so
//     there is no per-tile prologue bubble (what a fresh workgroup per tile
//     pays: the short-K encoder shapes, K = 768-1024, run 12-16 K-steps a tile);
//   * 8 waves: 2 (M) x 4 (N), wave tile 128 x 64 = 2 x 2 quadrants of 64 x 32
//     (16x16x32 bf16 MFMA, operands swapped so each lane's 4 accumulators are
//     4 consecutive output columns); one K-step (64 deep) is 2 phases, one
//     M-half (two quadrants, 32 MFMAs) per phase (details at the kernel);
//   * ping-pong: waves 4-7 run one barrier behind waves 0-3, so on every SIMD
//     one wave issues its 32 MFMAs while the other reads its next fragments
//     and issues its LDS-DMA (s_setprio(1) around the MFMA cluster);
//   * LDS: two K-step stages of four 16-KB half-tile images (A rows of M-half
//     0/1 of every wave, W columns of N-half 0/1 of every wave) filled by
//     buffer_load ... lds (16 B per lane, XOR-swizzled on the global source
//     chunk, undone on the ds_read_b128); a half is refilled in the phase
//     after its last ds_read and waited for two phases later with a counted
//     vmcnt -- never 0 in the loop;
//   * epilogue: the previous tile's quadrants are converted and stored (raw
//     buffer stores: rows >= M fall outside the buffer and are dropped, so the
//     instruction count per wave is fixed) in the read intervals of the next
//     tile's first K-step, just before their first (zero-input) MFMAs; the
//     counted waits of that K-step and the next include the stores.
// The other measured design points (4-phase ping-pong, 4/4 DMA split, 4-wave
// 192 x 256 tiles) live in tools/lab_kernels/pgemm_lab.hip, out of the extension.
//
// WP (packed weights): W is K14's packed layout (rsgemm.hip rsgemm_pack: each
// (256-column tile, 32-column wave block, K32 block, 16-column half) one 1-KB
// run in MFMA fragment order) instead of row-major -- one copy of a weight
// serves the K14 decode GEMM and this prefill GEMM.  K14's wave block 2 wn + H
// is exactly this kernel's W half-image H of wave column wn, so a half-image
// of one K-step is 16 such runs (4 KB contiguous per wn); the DMA copies them
// 1 KB per wave-instruction and the fragment reads are linear (lane x 16 B,
// conflict-free without the XOR swizzle).
//
// Requirements (checked by the launcher): N % 256 == 0, K % 64 == 0, K >= 192,
// lda / ldw / ldc multiples of 8 elements, 16-B aligned operands; bias (if
// any) N <= 8192.
#include "common.h"

namespace lmx {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));

constexpr int PG_THREADS = 512;
constexpr int PG_HALF_B = 128 * 64 * 2;       // one half-tile image: 128 rows x 64 bf16
constexpr int PG_STAGE_B = 4 * PG_HALF_B;     // A0 A1 W0 W1
constexpr int PG_RING_B = 2 * PG_STAGE_B;     // 128 KB
constexpr int PG_MAX_BIAS = 8192;
constexpr int PG_GROUP_M = 8;                 // M-tiles per tile group (L2 reuse)
constexpr int HA0 = 0, HA1 = 1, HW0 = 2, HW1 = 3;

// step modes: plain K-step / first K-step of a tile after another tile (stores
// the previous tile's quadrants) / the two K-steps after that (their vmcnt
// windows still hold some of those stores) / first K-step of the first tile
constexpr int MODE_PLAIN = 0, MODE_K0 = 1, MODE_K1 = 2, MODE_K2 = 3, MODE_FIRST = 4;

template <int CNT>
__device__ __forceinline__ void pg_vmwait() {
  static_assert(CNT >= 0 && CNT < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

__device__ __forceinline__ void pg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int ACT>
__device__ __forceinline__ float pg_act(float v) {
  if constexpr (ACT == 1) {
    const float u = 0.7978845608f * (v + 0.044715f * v * v * v);
    return 0.5f * v * (1.f + tanhf(u));
  } else if constexpr (ACT == 2) {
    return v / (1.f + __expf(-v));
  } else if constexpr (ACT == 4) {
    return 0.5f * v * (1.f + erff(v * 0.70710678118f));
  } else {
    return v;
  }
}

// load cursor: the K-step whose half-tiles the current K-step's phases issue
struct PgLoad {
  __amdgpu_buffer_rsrc_t ra;     // A rows [m0, M) of the cursor's tile
  __amdgpu_buffer_rsrc_t rw;     // W rows [n0, N)
  int kbyte;                     // k * 128
  int k, tile;                   // K-step in the tile, tile index of this workgroup
  bool done;                     // past the last step: re-issue the last one (free halves)
};

// output side of the tile whose quadrants are stored
struct PgOut {
  __amdgpu_buffer_rsrc_t rc;     // C rows [m0, M)
  __amdgpu_buffer_rsrc_t rn;     // NRM 1: row scales [m0, M); NRM 2: ssq partials of rows [m0, M)
  int n0;
};

// thread constants
struct PgThr {
  int a_voff[2][2];              // [half][instr]: A source offset (bytes, from the tile's row 0)
  int w_voff;                    // W source offset of this thread (instr / half parts uniform)
  int w_uoff[2][2];              // [half][instr]: uniform W row offset (bytes)
  int ra_off, rw_off;            // fragment row offsets in a half image (bytes)
  int wp_voff[2][2];             // WP: [half][instr] packed-run source offset (bytes, + lane)
  int rwp_off;                   // WP: this lane's fragment offset in a half image
  int co[2];                     // fragment chunk offsets for k32 step 0 / 1 (bytes)
  int wave, wm, wn, fr, fg;
  int ldc;
};

__device__ __forceinline__ void pg_tile_coords(int lin, int tiles_m, int tiles_n, int& tm,
                                               int& tn) {
  const int per_group = PG_GROUP_M * tiles_n;
  const int g = lin / per_group, r = lin % per_group;
  const int first = g * PG_GROUP_M;
  const int gsize = min(PG_GROUP_M, tiles_m - first);
  tm = first + r % gsize;
  tn = r / gsize;
}

template <int H, int WP = 0>
__device__ __forceinline__ void pg_issue(char* smem, int stage, const PgLoad& L, const PgThr& T) {
  char* dst = smem + stage * PG_STAGE_B + H * PG_HALF_B + T.wave * 1024;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (H == HA0 || H == HA1) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(L.ra, (lds_void_t*)(dst + i * 8192), 16,
                                               T.a_voff[H][i], L.kbyte, 0, 0);
    } else if constexpr (WP) {
      // K-step s of a packed tile starts at s * 4 KB of every wave block
      __builtin_amdgcn_raw_ptr_buffer_load_lds(L.rw, (lds_void_t*)(dst + i * 8192), 16,
                                               T.wp_voff[H - HW0][i], L.kbyte * 32, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(L.rw, (lds_void_t*)(dst + i * 8192), 16,
                                               T.w_voff, L.kbyte + T.w_uoff[H - HW0][i], 0, 0);
    }
  }
}

__device__ __forceinline__ bf16x8_t pg_frag(const char* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// A fragments of M-half H from stage `stage`
template <int H>
__device__ __forceinline__ void pg_read_a(bf16x8_t (&a)[4][2], const char* smem, int stage,
                                          const PgThr& T) {
  const char* b = smem + stage * PG_STAGE_B + H * PG_HALF_B + T.ra_off;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) a[i][kk] = pg_frag(b + i * 2048 + T.co[kk]);
}

template <int H, int WP = 0>
__device__ __forceinline__ void pg_read_w(bf16x8_t (&w)[2][2], const char* smem, int stage,
                                          const PgThr& T) {
  if constexpr (WP) {
    // run (wn, kk, j) at wn * 4 KB + kk * 2 KB + j * 1 KB of the half image
    const char* b = smem + stage * PG_STAGE_B + (HW0 + H) * PG_HALF_B + T.rwp_off;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) w[j][kk] = pg_frag(b + kk * 2048 + j * 1024);
  } else {
    const char* b = smem + stage * PG_STAGE_B + (HW0 + H) * PG_HALF_B + T.rw_off;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) w[j][kk] = pg_frag(b + j * 2048 + T.co[kk]);
  }
}

// NRM (the RMSNorm folded into the projections, prefill):
//   1  consumer: the rows of A are the raw residual stream and the norm gain is
//      folded into W; every output row is scaled by its rsqrt(mean(x^2) + eps)
//      (O.rn: fp32 [M], ops.row_scale) before bias / activation / SwiGLU;
//   2  producer (residual epilogue): the sum of squares of each new residual
//      row over this wave's 64 columns goes to O.rn [M][N / 64] (fixed
//      slots, summed in order by the row-scale kernel: no float atomics).
template <int QM, int QN, int ACT, int BIAS, int NRM = 0, class RT>
__device__ __forceinline__ void pg_store(RT& R, const PgOut& O, const PgThr& T,
                                         const char* smem, int N = 0) {
  float rs[4];
  if constexpr (NRM == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      rs[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          O.rn, (T.wm * 128 + QM * 64 + 16 * i + T.fr) * 4, 0, 0));
  }
  if constexpr (ACT == 3) {
    // SwiGLU: 16-col tiles 0 (gate) and 1 (up) of the quadrant are one pair
    const int col = (O.n0 >> 1) + T.wn * 32 + QN * 16 + 4 * T.fg;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = T.wm * 128 + QM * 64 + 16 * i + T.fr;
      if constexpr (NRM == 1) {       // in place: no second copy of the quadrant live
        R.acc[QM][QN][i][0] *= rs[i];
        R.acc[QM][QN][i][1] *= rs[i];
      }
      const f32x4_t g = R.acc[QM][QN][i][0], u = R.acc[QM][QN][i][1];
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(g[r] / (1.f + __expf(-g[r])) * u[r]);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o), O.rc,
                                            (row * T.ldc + col) * 2, 0, 0);
    }
  } else {
    // the quadrant's two 16-column tiles as one 16-B store per lane: lanes of
    // 16-lane rows 0/2 keep tile 0 and take its columns 4-7 from the row
    // above, rows 1/3 take tile 1's columns 0-3 from the row below
    // (v_permlane16_swap), so 4 stores per quadrant instead of 8
    f32x4_t b[2];
    if constexpr (BIAS == 1) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int bc = O.n0 + T.wn * 64 + QN * 32 + 16 * j + 4 * T.fg;
        const bf16x4_t bb = *reinterpret_cast<const bf16x4_t*>(smem + PG_RING_B + bc * 2);
#pragma unroll
        for (int r = 0; r < 4; ++r) b[j][r] = bf2f((uint16_t)bb[r]);
      }
    }
    const int col = O.n0 + T.wn * 64 + QN * 32 + 16 * (T.fg & 1) + 8 * (T.fg >> 1);
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    // BIAS 2: residual epilogue -- C is the bf16 residual stream, updated in
    // place: C = bf16(C + bf16(acc)), the rounding order of the separate
    // residual-add pass it replaces.  The quadrant's residual rows are loaded
    // (16 B per lane, rows >= M read as 0 and their stores dropped) before the
    // conversions; the compiler waits for them at their first use.
    u32x4_t res[4];
    if constexpr (BIAS == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        res[i] = __builtin_amdgcn_raw_buffer_load_b128(
            O.rc, ((T.wm * 128 + QM * 64 + 16 * i + T.fr) * T.ldc + col) * 2, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = T.wm * 128 + QM * 64 + 16 * i + T.fr;
      unsigned d[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (NRM == 1) R.acc[QM][QN][i][j] *= rs[i];
        const f32x4_t v = R.acc[QM][QN][i][j];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float x0 = v[2 * q], x1 = v[2 * q + 1];
          if constexpr (BIAS == 1) {
            x0 += b[j][2 * q];
            x1 += b[j][2 * q + 1];
          }
          d[j][q] = pack_bf16x2(pg_act<ACT>(x0), pg_act<ACT>(x1));
        }
      }
      const auto p = __builtin_amdgcn_permlane16_swap(d[0][0], d[1][0], false, false);
      const auto q = __builtin_amdgcn_permlane16_swap(d[0][1], d[1][1], false, false);
      u32x4_t o = {p[0], q[0], p[1], q[1]};
      if constexpr (BIAS == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = bf2f((uint16_t)(o[e] & 0xffff)) + bf2f((uint16_t)(res[i][e] & 0xffff));
          const float hi = bf2f((uint16_t)(o[e] >> 16)) + bf2f((uint16_t)(res[i][e] >> 16));
          o[e] = pack_bf16x2(lo, hi);
        }
        if constexpr (NRM == 2) {
          // squares of the bf16 residual values the next norm would read
          float sq = QN == 0 ? 0.f : R.ssq[i];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = bf2f((uint16_t)(o[e] & 0xffff)), hi = bf2f((uint16_t)(o[e] >> 16));
            sq += lo * lo + hi * hi;
          }
          R.ssq[i] = sq;
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(o, O.rc, (row * T.ldc + col) * 2, 0, 0);
    }
    if constexpr (BIAS == 2 && NRM == 2 && QN == 1) {
      // the wave's 64 columns of each row: the 4 lanes c, c+16, c+32, c+48, then
      // one fp32 per (row, wave column block); every lane stores (the 4 lanes of
      // a row write the same value to the same slot), so the store count is fixed
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = R.ssq[i];
        const unsigned u0 = __float_as_uint(x);
        const auto a = __builtin_amdgcn_permlane16_swap(u0, u0, false, false);
        x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
        const unsigned u1 = __float_as_uint(x);
        const auto b2 = __builtin_amdgcn_permlane32_swap(u1, u1, false, false);
        x = __uint_as_float(b2[0]) + __uint_as_float(b2[1]);
        const int row = T.wm * 128 + QM * 64 + 16 * i + T.fr;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), O.rn,
                                              (row * (N / 64) + (O.n0 >> 6) + T.wn) * 4, 0, 0);
      }
    }
  }
}

// stores per quadrant per wave
template <int ACT>
constexpr int pg_ns() { return 4; }   // 16-B (8-B SwiGLU) stores of 16 rows each

}  // namespace
// ============================================================================
// K13 kernel: the ping-pong form with 2 phases per 64-deep K-step
// ============================================================================
// The 4-phase form (one 16-MFMA quadrant per barrier interval, 8 intervals per
// K-step; kept with the other losing design points in
// tools/lab_kernels/pgemm_lab.hip) measured 0.60 MFMA utilisation (l8b o), the read intervals
// (fragment reads + LDS-DMA issue + their latency) longer than the 256-cycle
// MFMA intervals.  Here one phase runs the 32 MFMAs of a wave's M-half
// (two quadrants, 512 cycles) and its read interval has that long to cover:
//   phase 0: read A0, W0, W1 of K-step s (16 ds_read_b128), DMA A1 of s+1;
//            MFMA (0,0) (0,1)
//   phase 1: read A1 of s (8), DMA A0 W0 W1 of s+2; MFMA (1,0) (1,1)
// (fragment registers: one A half + both W halves = 64 VGPRs).  Each half is
// refilled in a phase after its last read and waited for 2 phases later
// (vmcnt 8 in both phases: 6 + 2 DMA issued after the one retired); the
// epilogue of the previous tile is stored in the read intervals of the next
// tile's first K-step (quadrant pair of phase q, before its zero-input
// MFMAs), and those stores are counted by the waits of that K-step and the
// next one.
namespace {

struct PpRegs {
  f32x4_t acc[2][2][4][2];
  bf16x8_t a[4][2];
  bf16x8_t w0[2][2], w1[2][2];
  float ssq[4];                   // NRM 2: a quadrant pair's row sums of squares
};

template <int ACT, int NRM = 0>
constexpr int pp_nsp() {   // stores per phase (two quadrants; + the 4 ssq partials of NRM 2)
  return 2 * pg_ns<ACT>() + (NRM == 2 ? 4 : 0);
}

// SCHED 0: phase 0 issues A1 of s+1, phase 1 A0 W0 W1 of s+2 (2 / 6 DMA per
// wave); SCHED 1: phase 0 A1 and W1 of s+1, phase 1 A0 W0 of s+2 (4 / 4; W1 then
// has one phase less to land)
template <int Q, int MODE, int ACT, int SCHED, int NRM = 0>
constexpr int pp_vmcnt() {
  constexpr int ns = pp_nsp<ACT, NRM>();
  constexpr int b0 = SCHED == 0 ? 8 : 10, b1 = SCHED == 0 ? 8 : 4;
  if constexpr (MODE == MODE_K0) return Q == 0 ? b0 + ns : (SCHED == 0 ? b1 + 2 * ns : b1 + ns);
  else if constexpr (MODE == MODE_K1) return Q == 0 ? b0 + ns : b1;
  else return Q == 0 ? b0 : b1;
}

template <int QM, bool ZERO>
__device__ __forceinline__ void pp_mma(PpRegs& R) {
  const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int qn = 0; qn < 2; ++qn) {
    const bf16x8_t(&w)[2][2] = qn == 0 ? R.w0 : R.w1;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          R.acc[QM][qn][i][j] =
              mfma16(w[j][kk], R.a[i][kk], (ZERO && kk == 0) ? z : R.acc[QM][qn][i][j]);
  }
}

template <int Q, int MODE, int ACT, int BIAS, int SCHED, int WP = 0, int NRM = 0>
__device__ __forceinline__ void pp_phase(PpRegs& R, char* smem, int stage, const PgLoad& L1,
                                         const PgLoad& L2, const PgOut& O, const PgThr& T,
                                         int N = 0) {
  if constexpr (MODE == MODE_K0) {
    pg_store<Q, 0, ACT, BIAS, NRM>(R, O, T, smem, N);
    __builtin_amdgcn_sched_barrier(0);
    pg_store<Q, 1, ACT, BIAS, NRM>(R, O, T, smem, N);
    __builtin_amdgcn_sched_barrier(0);   // epilogue temporaries die before the fragment reads
  }
  if constexpr (Q == 0) {
    pg_read_a<HA0>(R.a, smem, stage, T);
    pg_read_w<0, WP>(R.w0, smem, stage, T);
    pg_read_w<1, WP>(R.w1, smem, stage, T);
    pg_issue<HA1>(smem, stage ^ 1, L1, T);
    if constexpr (SCHED == 1) pg_issue<HW1, WP>(smem, stage ^ 1, L1, T);
  } else {
    pg_read_a<HA1>(R.a, smem, stage, T);
    pg_issue<HA0>(smem, stage, L2, T);
    pg_issue<HW0, WP>(smem, stage, L2, T);
    if constexpr (SCHED == 0) pg_issue<HW1, WP>(smem, stage, L2, T);
  }
  pg_vmwait<pp_vmcnt<Q, MODE, ACT, SCHED, NRM>()>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pg_barrier();
  __builtin_amdgcn_s_setprio(1);
  pp_mma<Q, MODE == MODE_K0 || MODE == MODE_FIRST>(R);
  __builtin_amdgcn_s_setprio(0);
  pg_barrier();
}

template <int MODE, int ACT, int BIAS, int SCHED, int WP = 0, int NRM = 0>
__device__ __forceinline__ void pp_step(PpRegs& R, char* smem, int stage, const PgLoad& L1,
                                        const PgLoad& L2, const PgOut& O, const PgThr& T,
                                        int N = 0) {
  pp_phase<0, MODE, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
  pp_phase<1, MODE, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
}

}  // namespace

template <int ACT, int BIAS, int SCHED, int WP = 0, int NRM = 0>
__global__ void __launch_bounds__(PG_THREADS, 1) pgemm_pp2_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ bias, int M, int N, int K, int lda, int ldw, int ldc,
    float* __restrict__ nrm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int r = xcd_remap(blockIdx.x, G);
  const int my_tiles = (ntiles - r + G - 1) / G;
  const int nk = K / 64;

  PgThr T;
  const int lane = threadIdx.x & 63;
  T.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T.wm = T.wave >> 2;
  T.wn = T.wave & 3;
  T.fr = lane & 15;
  T.fg = lane >> 4;
  T.ldc = ldc;
  {
    const int sc = (lane & 7) ^ ((4 * T.wave + (lane >> 4)) & 7);
    const int rr = 8 * T.wave + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) T.a_voff[h][i] = (128 * i + 64 * h + rr) * lda * 2 + sc * 16;
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
    if constexpr (WP) {
      // instruction i of wave v fills run r = 8 i + v of a half image: (wn, kk, j) =
      // (r / 4, r / 2 % 2, r % 2), K14 wave block 2 wn + H, K32 block 2 s + kk, half j
      const int kb = K / 32;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = 8 * i + T.wave, wn = r >> 2, kk = (r >> 1) & 1, j = r & 1;
          T.wp_voff[h][i] = (2 * wn + h) * kb * 2048 + kk * 2048 + j * 1024 + lane * 16;
        }
      T.rwp_off = T.wn * 4096 + lane * 16;
    }
  }

  if constexpr (BIAS == 1) {
    for (int c = threadIdx.x * 8; c < N; c += PG_THREADS * 8)
      *reinterpret_cast<bf16x8_t*>(smem + PG_RING_B + c * 2) =
          *reinterpret_cast<const bf16x8_t*>(bias + c);
    __syncthreads();
  }

  auto set_tile = [&](PgLoad& L, int t) {
    int tm, tn;
    pg_tile_coords(t * G + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const long abytes = (long)(M - m0) * lda * 2;
    L.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)m0 * lda), (short)0,
                                             (int)(abytes < 0x7fffffffL ? abytes : 0x7fffffffL),
                                             0x00020000);
    L.rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (long)n0 * ldw), (short)0,
                                             (int)(256L * ldw * 2), 0x00020000);
  };
  auto set_out = [&](PgOut& O, int t) {
    int tm, tn;
    pg_tile_coords(t * G + r, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256;
    const long cbytes = (long)(M - m0) * ldc * 2;
    O.rc = __builtin_amdgcn_make_buffer_rsrc((void*)(C + (long)m0 * ldc), (short)0,
                                             (int)(cbytes < 0x7fffffffL ? cbytes : 0x7fffffffL),
                                             0x00020000);
    if constexpr (NRM == 1)
      O.rn = __builtin_amdgcn_make_buffer_rsrc((void*)(nrm + m0), (short)0, (M - m0) * 4,
                                               0x00020000);
    if constexpr (NRM == 2)
      O.rn = __builtin_amdgcn_make_buffer_rsrc((void*)(nrm + (long)m0 * (N / 64)), (short)0,
                                               (M - m0) * (N / 64) * 4, 0x00020000);
    O.n0 = tn * 256;
  };
  auto advance = [&](PgLoad& L) {
    if (L.done) return;
    if (++L.k == nk) {
      if (L.tile + 1 >= my_tiles) {
        L.done = true;
        L.k = nk - 1;
        return;
      }
      L.k = 0;
      ++L.tile;
      set_tile(L, L.tile);
    }
    L.kbyte = L.k * 128;
  };

  PpRegs R;
  PgLoad L1, L2;                    // K-steps s+1 and s+2 of the running K-step s
  L2.k = 0;
  L2.tile = 0;
  L2.kbyte = 0;
  L2.done = false;
  set_tile(L2, 0);
  PgOut O;
  set_out(O, 0);

  // ---- prologue: the DMA of the phases before K-step 0, in loop order
  if constexpr (SCHED == 0) {
    pg_issue<HA0>(smem, 0, L2, T);
    pg_issue<HW0, WP>(smem, 0, L2, T);
    pg_issue<HW1, WP>(smem, 0, L2, T);
    pg_issue<HA1>(smem, 0, L2, T);
    advance(L2);
    pg_issue<HA0>(smem, 1, L2, T);
    pg_issue<HW0, WP>(smem, 1, L2, T);
    pg_issue<HW1, WP>(smem, 1, L2, T);
    L1 = L2;
    advance(L2);
    pg_vmwait<8>();                 // A0, W0, W1 of K-step 0
  } else {
    pg_issue<HA0>(smem, 0, L2, T);
    pg_issue<HW0, WP>(smem, 0, L2, T);
    pg_issue<HA1>(smem, 0, L2, T);
    pg_issue<HW1, WP>(smem, 0, L2, T);
    advance(L2);
    pg_issue<HA0>(smem, 1, L2, T);
    pg_issue<HW0, WP>(smem, 1, L2, T);
    L1 = L2;
    advance(L2);
    pg_vmwait<4>();                 // A0, W0, W1 of K-step 0
  }
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
      pp_step<MODE_FIRST, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
      next();
      pp_step<MODE_PLAIN, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
    } else {
      pp_step<MODE_K0, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);   // stores tile t-1
      next();
      set_out(O, t);
      pp_step<MODE_K1, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
    }
    next();
    for (int k = 2; k < nk; ++k) {
      pp_step<MODE_PLAIN, ACT, BIAS, SCHED, WP, NRM>(R, smem, stage, L1, L2, O, T, N);
      next();
    }
  }
  if (T.wm == 0) pg_barrier();
  pg_vmwait<0>();
  pg_store<0, 0, ACT, BIAS, NRM>(R, O, T, smem, N);
  pg_store<0, 1, ACT, BIAS, NRM>(R, O, T, smem, N);
  pg_store<1, 0, ACT, BIAS, NRM>(R, O, T, smem, N);
  pg_store<1, 1, ACT, BIAS, NRM>(R, O, T, smem, N);
}

// ============================================================================
// K13-SK: the 2-phase ping-pong 256 x 256 tile with split-K, for decode batches
// ============================================================================
// At decode batch sizes (M <= 256) one 256-row tile covers the batch, and every
// column tile re-reads the whole 256 x K activation panel from L2: at the
// 128-column tiles of K11 / hipBLASLt each CU moves 2 bytes of activations
// through its vector L1 per byte of weights, and the L1's outstanding-miss
// capacity bounds those kernels (profiles/r3_decode_gemm_study.md).  A
// 256-column tile halves that ratio; split-K over S slices gives the N / 256
// tiles enough workgroups to fill the CUs (Llama-3-8B gate/up: 112 tiles x 2).
// One workgroup per (slice, tile), slice-major (the workgroups of one XCD read
// the same K-slice of the activations from its L2); the main loop is the
// pgemm_pp2 one with a single tile.  Combine:
//   EPI 0: ticketed, in-kernel -- the first S-1 arrivals publish their fp32
//          accumulators write-through (sc1) in the lane-native order (32
//          coalesced 16-B stores per lane, no index math) and leave; the last
//          adds them in slice order (deterministic) and runs the bf16 epilogue
//          of pg_store, incl. the SwiGLU form;  counters re-armed by the last;
//   EPI 2: every slice writes its fp32 partial tile to slab [S][M][N] and the
//          residual-add RMSNorm that consumes the result sums the slabs
//          (rmsnorm_slabs), so no combine at all.
template <int ACT, int EPI>
__global__ void __launch_bounds__(PG_THREADS, 1) pgemm_sk_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    float* __restrict__ slabs, unsigned* __restrict__ cnt, int M, int N, int K, int lda, int ldw,
    int ldc, int splits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256, ntiles = tiles_m * tiles_n;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int ks = wid / ntiles, tile = wid - ks * ntiles;
  const int nk = K / 64 / splits;
  const int k0 = ks * nk * 64;

  PgThr T;
  const int lane = threadIdx.x & 63;
  T.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T.wm = T.wave >> 2;
  T.wn = T.wave & 3;
  T.fr = lane & 15;
  T.fg = lane >> 4;
  T.ldc = ldc;
  {
    const int sc = (lane & 7) ^ ((4 * T.wave + (lane >> 4)) & 7);
    const int rr = 8 * T.wave + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) T.a_voff[h][i] = (128 * i + 64 * h + rr) * lda * 2 + sc * 16;
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

  int tm, tn;
  pg_tile_coords(tile, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  PgLoad L1, L2;
  {
    // the slice's K range starts at k0: base pointers moved there, byte
    // ranges shortened by as much (rows >= M still fall outside the range)
    const long abytes = (long)(M - m0) * lda * 2 - (long)k0 * 2;
    L2.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)m0 * lda + k0), (short)0,
                                              (int)(abytes < 0x7fffffffL ? abytes : 0x7fffffffL),
                                              0x00020000);
    L2.rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (long)n0 * ldw + k0), (short)0,
                                              (int)(256L * ldw * 2 - (long)k0 * 2), 0x00020000);
  }
  L2.k = 0;
  L2.tile = 0;
  L2.kbyte = 0;
  L2.done = false;
  PgOut O;
  {
    const long cbytes = (long)(M - m0) * ldc * 2;
    O.rc = __builtin_amdgcn_make_buffer_rsrc((void*)(C + (long)m0 * ldc), (short)0,
                                             (int)(cbytes < 0x7fffffffL ? cbytes : 0x7fffffffL),
                                             0x00020000);
    O.n0 = n0;
  }
  auto advance = [&](PgLoad& L) {
    if (L.done) return;
    if (++L.k == nk) {
      L.done = true;                // re-issue the last K-step into free halves
      L.k = nk - 1;
      return;
    }
    L.kbyte = L.k * 128;
  };

  PpRegs R;
  pg_issue<HA0>(smem, 0, L2, T);
  pg_issue<HW0>(smem, 0, L2, T);
  pg_issue<HW1>(smem, 0, L2, T);
  pg_issue<HA1>(smem, 0, L2, T);
  advance(L2);
  pg_issue<HA0>(smem, 1, L2, T);
  pg_issue<HW0>(smem, 1, L2, T);
  pg_issue<HW1>(smem, 1, L2, T);
  L1 = L2;
  advance(L2);
  pg_vmwait<8>();                   // A0, W0, W1 of K-step 0
  pg_barrier();
  if (T.wm == 1) pg_barrier();      // waves 4-7 run one barrier behind

  int stage = 0;
  auto next = [&]() {
    L1 = L2;
    advance(L2);
    stage ^= 1;
  };
  pp_step<MODE_FIRST, ACT, 0, 0>(R, smem, stage, L1, L2, O, T);
  next();
  for (int k = 1; k < nk; ++k) {
    pp_step<MODE_PLAIN, ACT, 0, 0>(R, smem, stage, L1, L2, O, T);
    next();
  }
  if (T.wm == 0) pg_barrier();
  pg_vmwait<0>();

  if constexpr (EPI == 2) {
    // fp32 partial tile -> slab ks [M][N]; rows >= M fall outside the range
    const long sbytes = (long)M * N * 4;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(
        slabs + (long)ks * M * N, (short)0, (int)(sbytes < 0x7fffffffL ? sbytes : 0x7fffffffL),
        0x00020000);
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int row = m0 + T.wm * 128 + qm * 64 + 16 * i + T.fr;
            const int col = n0 + T.wn * 64 + qn * 32 + 16 * j + 4 * T.fg;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, R.acc[qm][qn][i][j]),
                                                   rs, (row * N + col) * 4, 0, 0);
          }
    return;
  } else {
    if (splits > 1) {
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      constexpr int TSLAB = PG_THREADS * 128;        // floats of one slice's tile
      unsigned* word = reinterpret_cast<unsigned*>(smem + PG_RING_B);
      __syncthreads();                               // every wave's DMA has landed
      if (threadIdx.x == 0)
        word[0] = __hip_atomic_fetch_add(&cnt[2 * tile], 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const unsigned order = word[0];
      float* tslab = slabs + (long)tile * splits * TSLAB;
      // accumulator r = ((qm * 2 + qn) * 4 + i) * 2 + j of every lane is float4
      // r * PG_THREADS + tid of a slice's slab
#define PG_FOR_ACC(BODY)                                   \
  _Pragma("unroll") for (int qm = 0; qm < 2; ++qm)         \
  _Pragma("unroll") for (int qn = 0; qn < 2; ++qn)         \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)            \
  _Pragma("unroll") for (int j = 0; j < 2; ++j) {          \
    const int r = ((qm * 2 + qn) * 4 + i) * 2 + j;         \
    f32x4_t& a = R.acc[qm][qn][i][j];                      \
    BODY                                                   \
  }
      if (order + 1 < (unsigned)splits) {
        // publish write-through (sc1): no L2 write-back fence (wgemm.hip)
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(tslab + (long)ks * TSLAB, (short)0,
                                                          TSLAB * 4, 0x00020000);
        PG_FOR_ACC(__builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4_t, a), rs, (r * PG_THREADS + (int)threadIdx.x) * 16, 0, 16);)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
          __hip_atomic_fetch_add(&cnt[2 * tile + 1], 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      if (threadIdx.x == 0) {
        while (__hip_atomic_load(&cnt[2 * tile + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               (unsigned)(splits - 1))
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&cnt[2 * tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&cnt[2 * tile + 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      // ((p0 + p1) + ...) + p(S-1), own partial at its slice position
      const f32x4_t* tin = reinterpret_cast<const f32x4_t*>(tslab) + threadIdx.x;
      PG_FOR_ACC({
        f32x4_t v;
        if (ks > 0) {
          v = tin[r * PG_THREADS];
          for (int s = 1; s < ks; ++s) v += tin[(long)s * (TSLAB / 4) + r * PG_THREADS];
          v += a;
        } else {
          v = a;
        }
        for (int s = ks + 1; s < splits; ++s) v += tin[(long)s * (TSLAB / 4) + r * PG_THREADS];
        a = v;
      })
#undef PG_FOR_ACC
    }
    pg_store<0, 0, ACT, 0>(R, O, T, smem);
    pg_store<0, 1, ACT, 0>(R, O, T, smem);
    pg_store<1, 0, ACT, 0>(R, O, T, smem);
    pg_store<1, 1, ACT, 0>(R, O, T, smem);
  }
}


// ---- launcher ---------------------------------------------------------------
static int g_pg_cus = 0;

template <int ACT, int BIAS, int WP = 0, int NRM = 0>
static int pg_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, const bf16_t* bias, int M,
                     int N, int K, int lda, int ldw, int ldc, int grid, hipStream_t stream,
                     float* nrm = nullptr) {
  constexpr size_t smem = PG_RING_B + (BIAS == 1 ? PG_MAX_BIAS * 2 : 0);
  static_assert(smem <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)pgemm_pp2_kernel<ACT, BIAS, 0, WP, NRM>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  pgemm_pp2_kernel<ACT, BIAS, 0, WP, NRM><<<dim3(grid), dim3(PG_THREADS), smem, stream>>>(
      C, A, W, bias, M, N, K, lda, ldw, ldc, nrm);
  return (int)hipGetLastError();
}

// res 1: C is read as well -- C = bf16(C + bf16(A . W^T)) (the residual
// stream of a pre-norm block, updated in place; act 0, no bias)
// wpacked 1: W is rsgemm_pack's layout of the [N][K] weight (ldw == K); the
// plain product, the residual epilogue and SwiGLU (no bias, no other act)
// nrm (the RMSNorm folded into the projections): with res, the new residual
// rows' sums of squares per 64-column block go to nrm [M][N / 64]; without,
// the output rows are scaled by nrm [M] (plain product or SwiGLU, no bias)
int pgemm(void* C, const void* A, const void* W, const void* bias, int M, int N, int K, long lda,
          long ldw, long ldc, int act, int grid, int res, int wpacked, float* nrm,
          hipStream_t stream) {
  if (M <= 0) return 0;
  if (wpacked && (bias != nullptr || ldw != K || (act != 0 && act != 3) || (res && act != 0)))
    return -1;
  if (nrm && (bias != nullptr || (act != 0 && act != 3) || (res && act != 0))) return -1;
  if (res && (act != 0 || bias != nullptr)) return -1;
  if (N % 256 != 0 || K % 64 != 0 || K < 192) return -1;
  if (lda % 8 || ldw % 8 || ldc % 4) return -1;
  if (act < 0 || act > 4 || (act == 3 && bias != nullptr)) return -1;
  if (bias != nullptr && N > PG_MAX_BIAS) return -1;
  // byte offsets of one tile's rows are 32-bit
  if (256L * lda * 2 > 0x7fffffffL || 256L * ldw * 2 > 0x7fffffffL || 256L * ldc * 2 > 0x7fffffffL)
    return -1;
  if (g_pg_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -2;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return -2;
    g_pg_cus = p.multiProcessorCount;
  }
  const long tiles = (long)((M + 255) / 256) * (N / 256);
  if (grid <= 0) grid = g_pg_cus;
  if (grid > tiles) grid = (int)tiles;
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
  auto b_ = (const bf16_t*)bias;
  const int ia = (int)lda, iw = (int)ldw, ic = (int)ldc;
  if (bias != nullptr) {
    switch (act) {
      case 0: return pg_launch<0, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
      case 1: return pg_launch<1, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
      case 2: return pg_launch<2, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
      case 4: return pg_launch<4, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    }
    return -1;
  }
  if (nrm) {
    // the folded-norm forms: producer (residual) and consumers (QKV plain,
    // gate/up SwiGLU), row-major or packed W
#define LMX_PG_N(WPV)                                                                        \
    if (res) return pg_launch<0, 2, WPV, 2>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream, nrm); \
    if (act == 3) return pg_launch<3, 0, WPV, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream, nrm); \
    return pg_launch<0, 0, WPV, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream, nrm);
    if (wpacked) { LMX_PG_N(1) } else { LMX_PG_N(0) }
#undef LMX_PG_N
  }
  if (wpacked) {
    if (res) return pg_launch<0, 2, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    if (act == 3) return pg_launch<3, 0, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    return pg_launch<0, 0, 1>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
  }
  if (res) return pg_launch<0, 2>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
  switch (act) {
    case 0: return pg_launch<0, 0>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    case 1: return pg_launch<1, 0>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    case 2: return pg_launch<2, 0>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    case 3: return pg_launch<3, 0>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
    case 4: return pg_launch<4, 0>(C_, A_, W_, b_, M, N, K, ia, iw, ic, grid, stream);
  }
  return -1;
}

// ---- K13-SK launcher --------------------------------------------------------
template <int ACT, int EPI>
static int pg_sk_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, float* slabs, unsigned* cnt,
                        int M, int N, int K, int lda, int ldw, int ldc, int splits, int grid,
                        hipStream_t stream) {
  constexpr size_t smem = PG_RING_B + 16;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)pgemm_sk_kernel<ACT, EPI>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  pgemm_sk_kernel<ACT, EPI><<<dim3(grid), dim3(PG_THREADS), smem, stream>>>(
      C, A, W, slabs, cnt, M, N, K, lda, ldw, ldc, splits);
  return (int)hipGetLastError();
}

// epi 0: C = act(A . W^T) bf16 ([M, N/2] for the SwiGLU act 3); splits > 1
// needs `slabs` >= tiles * splits * 65536 floats and `cnt` >= 2 * tiles zeroed
// counters (re-armed by the kernel).  epi 2: fp32 partials [splits][M][N] in
// `slabs` (C unused).
int pgemm_sk(void* C, const void* A, const void* W, void* slabs, void* cnt, int ncnt, int M,
             int N, int K, long lda, long ldw, long ldc, int act, int splits, int epi,
             hipStream_t stream) {
  if (M <= 0) return 0;
  if (splits < 1 || N % 256 != 0 || K % (64 * splits) != 0 || K / (64 * splits) < 2) return -1;
  if (lda % 8 || ldw % 8 || ldc % 4) return -1;
  if (epi != 0 && epi != 2) return -1;
  if (act < 0 || act > 4) return -1;
  if (256L * lda * 2 > 0x7fffffffL || 256L * ldw * 2 > 0x7fffffffL || 256L * ldc * 2 > 0x7fffffffL)
    return -1;
  const long tiles = (long)((M + 255) / 256) * (N / 256);
  if (epi == 2 && (slabs == nullptr || (long)M * N * 4 > 0x7fffffffL)) return -1;
  if (epi == 0 && splits > 1 && (slabs == nullptr || cnt == nullptr || 2 * tiles > ncnt)) return -1;
  const int grid = (int)(tiles * splits);
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
  auto s_ = (float*)slabs;
  auto c_ = (unsigned*)cnt;
  const int ia = (int)lda, iw = (int)ldw, ic = (int)ldc;
  if (epi == 2) return pg_sk_launch<0, 2>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
  switch (act) {
    case 0: return pg_sk_launch<0, 0>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
    case 1: return pg_sk_launch<1, 0>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
    case 2: return pg_sk_launch<2, 0>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
    case 3: return pg_sk_launch<3, 0>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
    case 4: return pg_sk_launch<4, 0>(C_, A_, W_, s_, c_, M, N, K, ia, iw, ic, splits, grid, stream);
  }
  return -1;
}

}  // namespace lmx
