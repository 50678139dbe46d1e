// K12: weight-streaming projection GEMM for decode batches of 129..256 rows
//     C[M, N] = A[M, K] . W[N, K]^T      (bf16 in, fp32 accumulate)
//
// Why a second decode GEMM next to dgemm.hip (K11): at M = 256 every column
// tile of a projection re-reads the whole 256-row activation panel from L2,
// so the bytes a CU moves per weight byte are (1 + 256 / BN) with the whole
// 256-row panel in one workgroup.  K11's 8-wave 64..128-column tiles move 2-3x
// the weight bytes per CU and are bound by the per-CU load path
// (profiles/r2_pmc_kernels.md); hipBLASLt's 256x128 tile sits at the same
// ~45 GB/s per CU (gate/up 69.7 us, profiles/r2_final_timeline.md).  This
// kernel is built around the two quantities that bound the M = 256 case:
//
//   * per-CU bytes: ONE workgroup per CU owns all 256 rows and a 96..256-column
//     tile, 4 waves in a 2 x 2 (or 4 x 1) layout, each wave a 128 x 112 (or
//     64 x 224) output block, its accumulators in the AGPR half of a
//     512-register budget (1 wave per SIMD).  Split-K (S slices of the
//     reduction) fills the 256 CUs when N / BN < 256;
//   * bytes in flight: the weight tile streams from HBM (~2 us under load)
//     while the activation panel is an L2 hit, so the two operands get
//     separate LDS rings -- a deep one for W (NW slots, loads issued NW-1
//     K-steps ahead) and a shallow one for A (NX slots) -- both filled by
//     LDS-DMA (global_load_lds, 16 B per lane) into XOR-swizzled [row][BK]
//     images, with counted vmcnt waits and raw s_barriers (a __syncthreads
//     would drain the W ring: cdna guide §5 "Pipelining across barriers").
//     Per K-step the A loads are issued before the W loads, so the counted
//     wait for A(t) leaves the younger W loads in flight.
//
// Split-K combine (S > 1) without a second launch and without every slice
// writing a slab: each slice takes an arrival ticket when its main loop ends;
// the first S-1 arrivals publish their fp32 partial tile (write-through sc1
// stores, publish counter) and leave, the last arrival waits for the S-1 publishes
// (it only waits for workgroups that are already running: no residency
// assumption), acquires, and adds the partials in slice order, so a call's
// result does not depend on which slice arrived last.  Counters are re-armed
// by the last arrival (graph replays need no memset node).
//
// Epilogues: EPI 0 bf16 C; EPI 2 fp32 partials only (slab per slice, summed by
// the residual-add RMSNorm that consumes them: rmsnorm_slabs); EPI 3 SwiGLU on
// gate/up weights interleaved in 4-row blocks ([4 gate | 4 up] per 4
// channels, ops.interleave_gate_up(w, 4)): a lane's 4 accumulator columns
// are 4 gate or 4 up values of the same 4 channels as the lane 16 above it,
// and one v_permlane16_swap per register over the tile pair (i, i+1) hands
// every lane a matching (gate, up) set.
#include "common.h"

#include <algorithm>

namespace lmx {
namespace {

typedef __attribute__((address_space(3))) void wg_lds_void_t;

template <int AUX>
__device__ __forceinline__ void wg_glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (wg_lds_void_t*)lds_base, 16, 0, AUX);
}

// 16-B chunk swizzle of row r of a [row][BK] image, conflict-free for the
// ds_read_b128 lane groups (same as K11: dgemm.hip dg_swz)
template <int BK>
__device__ __forceinline__ int wg_swz(int r) {
  if constexpr (BK == 64) return (r >> 1) & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;
}

template <int BK>
__device__ __forceinline__ bf16x8_t wg_frag(const bf16_t* img, int r, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(img + r * BK + 8 * (chunk ^ wg_swz<BK>(r)));
}

template <int CNT>
__device__ __forceinline__ void wg_vmwait_c() {
  static_assert(CNT >= 0 && CNT < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// run-time count (the last K-steps, where fewer loads follow): a scalar
// switch over the counts a configuration can produce
__device__ __forceinline__ void wg_vmwait(int n) {
#define WG_VC(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
  switch (n) {
    WG_VC(1) WG_VC(2) WG_VC(3) WG_VC(4) WG_VC(5) WG_VC(6) WG_VC(7) WG_VC(8) WG_VC(9)
    WG_VC(10) WG_VC(11) WG_VC(12) WG_VC(13) WG_VC(14) WG_VC(15) WG_VC(16) WG_VC(17)
    WG_VC(18) WG_VC(19) WG_VC(20) WG_VC(21) WG_VC(22) WG_VC(23) WG_VC(24) WG_VC(25)
    WG_VC(26) WG_VC(27) WG_VC(28) WG_VC(29) WG_VC(30) WG_VC(31) WG_VC(32) WG_VC(33)
    WG_VC(34) WG_VC(35) WG_VC(36) WG_VC(37) WG_VC(38) WG_VC(39) WG_VC(40)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef WG_VC
}

__device__ __forceinline__ float wg_silu(float g) { return g / (1.f + __expf(-g)); }

}  // namespace

// BN: column tile; WM x WN waves over the 256 x BN tile; BK: K-step;
// NX / NW: A / W ring slots; EPI: 0 bf16, 2 partial slabs, 3 SwiGLU;
// NT: non-temporal weight stream; MMA: 1 = compute, 0 = data movement only,
// 2 / 3 = data movement without the A / W loads (lab probes)
template <int BN, int WM, int WN, int BK, int NX, int NW, int EPI, int NT, int MMA, int PK>
__global__ void __launch_bounds__(WM * WN * 64, 1)
wgemm_kernel(bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
             float* __restrict__ slabs, unsigned* __restrict__ cnt, int M, int N, int K, long lda,
             long ldw, long ldc, int splits) {
  constexpr int BM = 256;
  constexpr int NWAVE = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;       // wave output block
  constexpr int TM = WTM / 16, TN = WTN / 16;       // 16x16 MFMA tiles per wave
  constexpr int CPR = BK / 8;                       // 16-B chunks per image row
  constexpr int RPW = 64 / CPR;                     // rows per wave-instruction
  constexpr int RPR = NWAVE * RPW;                  // rows per workgroup round
  constexpr int XI = BM / RPR;                      // A loads per wave per K-step
  constexpr int WIF = BN / RPR;                     // full W rounds
  constexpr int WREM_WAVES = (BN % RPR) / RPW;      // waves issuing one more W load
  constexpr int XSLOT = BM * BK, WSLOT = BN * BK;   // bf16 elements per slot
  static_assert(WM * WN >= 4 && WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(BM % RPR == 0 && (BN % RPR) % RPW == 0, "staging rounds");
  static_assert(NX >= 2 && NW >= NX, "rings");
  static_assert(EPI != 3 || TM % 2 == 0, "SwiGLU pairs tiles (i, i+1)");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* const wsm = xs + NX * XSLOT;

  const int tiles_n = N / BN, nwg = tiles_n * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tile = wg / splits, ks = wg % splits;   // a tile's slices: one XCD
  const int n0 = tile * BN;
  const int nk_all = K / BK;
  const int kb = (int)((long)ks * nk_all / splits);
  const int nk = (int)((long)(ks + 1) * nk_all / splits) - kb;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fg = lane >> 4;
  const int srow = lane / CPR, sc = lane % CPR;     // staging: row / chunk of this lane
  const bool wextra = wave < WREM_WAVES;

  auto stage_x = [&](int slot, int kstep) {
    bf16_t* dst = xs + slot * XSLOT;
    const long k0 = (long)kstep * BK;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = i * RPR + wave * RPW + srow;
      const int gr = r < M ? r : M - 1;   // padded rows re-read row M-1; never stored
      wg_glds16<0>(A + (long)gr * lda + k0 + 8 * (sc ^ wg_swz<BK>(r)),
                   dst + (i * RPR + wave * RPW) * BK);
    }
  };
  auto stage_w = [&](int slot, int kstep) {
    bf16_t* dst = wsm + slot * WSLOT;
    if constexpr (PK) {
      // packed weights (wgemm_pack): the [BN][BK] LDS image of (tile, kstep)
      // is one contiguous run, read lane-linearly; PK 1: tiles outermost
      // (a workgroup streams one contiguous region), PK 2: K-steps outermost
      // (the workgroups of a K-step read adjacent images)
      const long blk = PK == 1 ? (long)tile * nk_all + kstep : (long)kstep * tiles_n + tile;
      const bf16_t* src = W + blk * WSLOT + lane * 8;
#pragma unroll
      for (int i = 0; i < WIF; ++i)
        wg_glds16<NT ? 2 : 0>(src + (i * RPR + wave * RPW) * BK, dst + (i * RPR + wave * RPW) * BK);
      if constexpr (WREM_WAVES > 0)
        if (wextra)
          wg_glds16<NT ? 2 : 0>(src + (WIF * RPR + wave * RPW) * BK,
                                dst + (WIF * RPR + wave * RPW) * BK);
      return;
    }
    const bf16_t* src = W + (long)n0 * ldw + (long)kstep * BK;
#pragma unroll
    for (int i = 0; i < WIF; ++i) {
      const int r = i * RPR + wave * RPW + srow;
      wg_glds16<NT ? 2 : 0>(src + (long)r * ldw + 8 * (sc ^ wg_swz<BK>(r)),
                            dst + (i * RPR + wave * RPW) * BK);
    }
    if constexpr (WREM_WAVES > 0) {
      if (wextra) {
        const int r = WIF * RPR + wave * RPW + srow;
        wg_glds16<NT ? 2 : 0>(src + (long)r * ldw + 8 * (sc ^ wg_swz<BK>(r)),
                              dst + (WIF * RPR + wave * RPW) * BK);
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // issue order: virtual K-iteration v loads A(v + NX - 1), then W(v + NW - 1)
#pragma unroll
  for (int v = -(NW - 1); v < 0; ++v) {
    const int tx = v + NX - 1, tw = v + NW - 1;
    if (MMA != 2 && tx >= 0 && tx < nk) stage_x(tx % NX, kb + tx);
    if (MMA != 3 && tw < nk) stage_w(tw % NW, kb + tw);
  }
  const int wi = WIF + (wextra ? 1 : 0);
  for (int t = 0; t < nk; ++t) {
    // A(t) was issued at v = t-NX+1; behind it: W(t+NW-NX) and the loads of
    // iterations t-NX+2 .. t-1.  W(t) is older than A(t).
    if constexpr (MMA >= 2) {
      // probes: one operand only; wait for the oldest outstanding stage of it
      constexpr int D = MMA == 2 ? NW : NX;
      const int per = MMA == 2 ? wi : XI;
      wg_vmwait(t + D - 2 < nk ? (D - 2) * per : 0);
    } else if (t + NW - 2 < nk) {
      // W(t+NW-NX), issued right after A(t), may stay in flight only when it
      // is a later K-step than t (NW > NX; with NW == NX it is W(t) itself)
      constexpr int LAG = NW > NX ? 1 : 0;
      if (wextra) wg_vmwait_c<LAG * (WIF + 1) + (NX - 2) * (XI + WIF + 1)>();
      else wg_vmwait_c<LAG * WIF + (NX - 2) * (XI + WIF)>();
    } else {
      int n = 0;
      for (int v = t - NX + 1; v <= t - 1; ++v) {
        if (v + NW - 1 < nk && (v > t - NX + 1 || NW > NX)) n += wi;
        if (v > t - NX + 1 && v + NX - 1 < nk) n += XI;
      }
      wg_vmwait(n);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      const int tx = t + NX - 1, tw = t + NW - 1;
      if (MMA != 2 && tx < nk) stage_x(tx % NX, kb + tx);
      if (MMA != 3 && tw < nk) stage_w(tw % NW, kb + tw);
    }
    const bf16_t* xt = xs + (t % NX) * XSLOT;
    const bf16_t* wt = wsm + (t % NW) * WSLOT;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = wg_frag<BK>(xt, wr * WTM + 16 * i + fr, kk * 4 + fg);
#pragma unroll
      for (int j = 0; j < TN; ++j) bw[j] = wg_frag<BK>(wt, wc * WTN + 16 * j + fr, kk * 4 + fg);
      if constexpr (MMA == 1) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bw[j], af[i], acc[i][j]);
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bw[j]));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // acc[i][j][r] = C[m][n]: m = wr*WTM + 16i + fr, n = n0 + wc*WTN + 16j + 4fg + r
  if constexpr (EPI == 2) {
    float* slab = slabs + (long)ks * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + n0 + wc * WTN + 16 * j + 4 * fg) =
            acc[i][j];
    }
    return;
  } else {
    if (splits > 1) {
      unsigned* word = reinterpret_cast<unsigned*>(smem);   // the one LDS array
      __syncthreads();                                      // every wave is out of the ring
      if (threadIdx.x == 0)
        word[0] = __hip_atomic_fetch_add(&cnt[2 * tile], 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const unsigned order = word[0];
      // slab of slice s of this tile: [256][BN] fp32, tile-major
      float* tslab = slabs + (long)tile * splits * BM * BN;
      if (order + 1 < (unsigned)splits) {
        // publish write-through (sc1 stores: no L2 write-back fence), every
        // storing wave drains, then one lane counts the publish (guide
        // Guideline 16 R1; a release fence here flushes the XCD's whole dirty
        // L2 and cost more than the main loop's tail)
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            tslab + (long)ks * BM * BN, 0, BM * BN * (int)sizeof(float), 0x00020000);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = wr * WTM + 16 * i + fr;
          if (m >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4_t, acc[i][j]), rsrc,
                (m * BN + wc * WTN + 16 * j + 4 * fg) * (int)sizeof(float), 0, 16);
          }
        }
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
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int m = wr * WTM + 16 * i + fr;
        m = m < M ? m : M - 1;              // load unconditionally (guide §5 item 4c)
        if (ks > 0) {
          f32x4_t pre[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j)
            pre[j] = *reinterpret_cast<const f32x4_t*>(tslab + m * BN + wc * WTN + 16 * j + 4 * fg);
          for (int s = 1; s < ks; ++s) {
            const float* o = tslab + (long)s * BM * BN + m * BN + wc * WTN + 4 * fg;
#pragma unroll
            for (int j = 0; j < TN; ++j) pre[j] += *reinterpret_cast<const f32x4_t*>(o + 16 * j);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = pre[j] + acc[i][j];
        }
        for (int s = ks + 1; s < splits; ++s) {
          const float* o = tslab + (long)s * BM * BN + m * BN + wc * WTN + 4 * fg;
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] += *reinterpret_cast<const f32x4_t*>(o + 16 * j);
        }
      }
    }
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wr * WTM + 16 * i + fr;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[i][j][r]);
          *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + n0 + wc * WTN + 16 * j + 4 * fg) = o;
        }
      }
    } else {
      // SwiGLU.  Tile (i, j), lane group g = fg: columns 4g..4g+3 of the
      // 16-column block are gate (g even) or up (g odd) of channels
      // (n0 + wc*WTN + 16j)/2 + 4(g>>1) + r.  permlane16_swap(a = tile i,
      // b = tile i+1) leaves group g holding (gate, up) of: g=0 tile i set 0,
      // g=1 tile i+1 set 0, g=2 tile i set 1, g=3 tile i+1 set 1.
      const int sub = fg & 1, set = fg >> 1;
#pragma unroll
      for (int i = 0; i < TM; i += 2) {
        const int m = wr * WTM + 16 * (i + sub) + fr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto p = __builtin_amdgcn_permlane16_swap(
                __float_as_uint(acc[i][j][r]), __float_as_uint(acc[i + 1][j][r]), false, false);
            const float g = __uint_as_float(p[0]), u = __uint_as_float(p[1]);
            o[r] = (short)f2bf(wg_silu(g) * u);
          }
          if (m < M)
            *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + ((n0 + wc * WTN + 16 * j) >> 1) +
                                         4 * set) = o;
        }
      }
    }
  }
}

// Packed weight layout of a configuration (BN, BK): for every column tile and
// K-step the [BN][BK] swizzled LDS image, contiguous, tiles outermost:
//   P[((tile * K/BK + kstep) * BN + r) * BK + 8p .. +8] =
//       W[tile*BN + r][kstep*BK + 8 (p ^ swz(r)) .. +8]
template <int BK>
__global__ void wgemm_pack_kernel(bf16_t* __restrict__ P, const bf16_t* __restrict__ W, int N,
                                  int K, long ldw, int BN, int kmajor) {
  constexpr int CPR = BK / 8;
  const long chunks = (long)N * K / 8;
  const int nk = K / BK;
  for (long c = blockIdx.x * (long)blockDim.x + threadIdx.x; c < chunks;
       c += (long)gridDim.x * blockDim.x) {
    const int p = (int)(c % CPR);
    const long rowblk = c / CPR;                 // (tile * nk + kstep) * BN + r
    const int r = (int)(rowblk % BN);
    const long tk = rowblk / BN;
    const int tiles = N / BN;
    const int kstep = kmajor ? (int)(tk / tiles) : (int)(tk % nk);
    const int tile = kmajor ? (int)(tk % tiles) : (int)(tk / nk);
    const long src = (long)(tile * BN + r) * ldw + (long)kstep * BK + 8 * (p ^ wg_swz<BK>(r));
    *reinterpret_cast<u16x8*>(P + c * 8) = *reinterpret_cast<const u16x8*>(W + src);
  }
}

// ---- K12-RS: register-streamed weights ------------------------------------
// The LDS-DMA weight ring above tops out at 5.1-5.4 TB/s (44-46 us for the
// 235 MB gate/up stream), while a plain 16-B vector-load stream from the same
// one-workgroup-per-CU grid reaches 6.4-6.7 TB/s
// (profiles/r3_decode_gemm_study.md).  So here the weights never touch LDS:
// each of the 4 waves owns all 256 rows x BN/4 columns of the tile, loads its
// W fragments (the MFMA A operand of D = W . X^T) straight into a DW-deep
// register ring from a packed layout in which every wave-instruction's 1 KB
// is exactly one fragment, and only the activation panel -- shared by the 4
// waves, an L2 hit -- is staged through LDS (register-staged, issue early /
// write late, two slots).  Every load is an ordinary vector load, so the
// compiler counts the waits; the K loop is unrolled by DW so the register
// ring is statically indexed.
template <int BN, int DW, int EPI, int NT, int WMR>
__global__ void __launch_bounds__(256, 1)
wgemm_rs_kernel(bf16_t* __restrict__ C, const bf16_t* __restrict__ A,
                const bf16_t* __restrict__ Wp, float* __restrict__ slabs,
                unsigned* __restrict__ cnt, int M, int N, int K, long lda, long ldc, int splits) {
  // WMR waves along M share each W fragment (loaded by each of them: the
  // second request of a line hits the CU's L1), 4 / WMR along N
  constexpr int BM = 256, BK = 64, KK = BK / 32, NWAVE = 4, WNR = NWAVE / WMR;
  constexpr int WTM = BM / WMR, WTN = BN / WNR, TN = WTN / 16, TM = WTM / 16;
  constexpr int XI = BM * BK / (NWAVE * 64 * 8);   // 16-B activation loads per lane per K-step
  constexpr int XSLOT = BM * BK;
  constexpr int WFR = TN * KK;                     // W fragments per wave per K-step
  static_assert(WTN % 16 == 0 && DW % 2 == 0 && DW >= 2, "rs geometry");
  static_assert(EPI != 3 || TM % 2 == 0, "SwiGLU pairs tiles (i, i+1)");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const xs = reinterpret_cast<bf16_t*>(smem);

  const int tiles_n = N / BN, nwg = tiles_n * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tile = wg / splits, ks = wg % splits;
  const int n0 = tile * BN;
  const int nk_all = K / BK;
  const int kb = (int)((long)ks * nk_all / splits);
  const int nk = (int)((long)(ks + 1) * nk_all / splits) - kb;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  // activation staging: instruction i of wave w covers rows w*64 + 8i .. +8
  const int xrow = wave * (BM / NWAVE) + (lane >> 3), xc = lane & 7;
  const bf16_t* xsrc[XI];
  int xdst[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int r = xrow + 8 * i;
    xsrc[i] = A + (long)(r < M ? r : M - 1) * lda + 8 * xc;
    xdst[i] = r * BK + 8 * (xc ^ wg_swz<BK>(r));
  }
  const int wr = wave % WMR, wc = wave / WMR;
  // W fragments of (tile, kstep, wave column): WFR x 1 KB, lane-linear
  const bf16_t* wsrc = Wp + (((long)tile * nk_all + kb) * WNR + wc) * (WFR * 512) + lane * 8;
  constexpr long WSTEP = (long)WNR * WFR * 512;     // elements per K-step of one tile

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t wq[DW][WFR];
  bf16x8_t xg[XI];
  auto load_w = [&](bf16x8_t (&dst)[WFR], int t) {
    const bf16_t* p = wsrc + (long)t * WSTEP;
#pragma unroll
    for (int f = 0; f < WFR; ++f) {
      if constexpr (NT)
        dst[f] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(p + f * 512));
      else
        dst[f] = *reinterpret_cast<const bf16x8_t*>(p + f * 512);
    }
  };
  auto load_x = [&](int t) {
    const long k0 = (long)(kb + t) * BK;
#pragma unroll
    for (int i = 0; i < XI; ++i) xg[i] = *reinterpret_cast<const bf16x8_t*>(xsrc[i] + k0);
  };
  auto store_x = [&](int slot) {
    bf16_t* d = xs + slot * XSLOT;
#pragma unroll
    for (int i = 0; i < XI; ++i) *reinterpret_cast<bf16x8_t*>(d + xdst[i]) = xg[i];
  };

  // prologue: activation K-step 0 into slot 0, weights of K-steps 0 .. DW-2
  load_x(0);
#pragma unroll
  for (int u = 0; u < DW - 1; ++u)
    if (u < nk) load_w(wq[u], u);
  store_x(0);
  __syncthreads();
  for (int t0 = 0; t0 < nk; t0 += DW) {
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      const int t = t0 + u;
      if (t < nk) {
        if (t + 1 < nk) load_x(t + 1);            // issued before this step's W load
        if (t + DW - 1 < nk) load_w(wq[(u + DW - 1) % DW], t + DW - 1);
        const bf16_t* xt = xs + (u & 1) * XSLOT;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const bf16x8_t xf = wg_frag<BK>(xt, wr * WTM + 16 * i + fr, kk * 4 + fg);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = mfma16(wq[u][j * KK + kk], xf, acc[i][j]);
          }
        }
        if (t + 1 < nk) store_x((u + 1) & 1);
        __syncthreads();
      }
    }
  }

  // acc[i][j][r] = C[m][n]: m = wr*WTM + 16i + fr, n = n0 + wc*WTN + 16j + 4fg + r
  if constexpr (EPI == 2) {
    float* slab = slabs + (long)ks * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = wr * WTM + 16 * i + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + n0 + wc * WTN + 16 * j + 4 * fg) =
            acc[i][j];
    }
    return;
  } else {
    if (splits > 1) {
      unsigned* word = reinterpret_cast<unsigned*>(smem);
      __syncthreads();
      if (threadIdx.x == 0)
        word[0] = __hip_atomic_fetch_add(&cnt[2 * tile], 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const unsigned order = word[0];
      float* tslab = slabs + (long)tile * splits * BM * BN;
      if (order + 1 < (unsigned)splits) {
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            tslab + (long)ks * BM * BN, 0, BM * BN * (int)sizeof(float), 0x00020000);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = wr * WTM + 16 * i + fr;
          if (m >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4_t, acc[i][j]), rsrc,
                (m * BN + wc * WTN + 16 * j + 4 * fg) * (int)sizeof(float), 0, 16);
          }
        }
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
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int m = wr * WTM + 16 * i + fr;
        m = m < M ? m : M - 1;
        if (ks > 0) {
          f32x4_t pre[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j)
            pre[j] = *reinterpret_cast<const f32x4_t*>(tslab + m * BN + wc * WTN + 16 * j + 4 * fg);
          for (int s2 = 1; s2 < ks; ++s2) {
            const float* o = tslab + (long)s2 * BM * BN + m * BN + wc * WTN + 4 * fg;
#pragma unroll
            for (int j = 0; j < TN; ++j) pre[j] += *reinterpret_cast<const f32x4_t*>(o + 16 * j);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = pre[j] + acc[i][j];
        }
        for (int s2 = ks + 1; s2 < splits; ++s2) {
          const float* o = tslab + (long)s2 * BM * BN + m * BN + wc * WTN + 4 * fg;
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] += *reinterpret_cast<const f32x4_t*>(o + 16 * j);
        }
      }
    }
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wr * WTM + 16 * i + fr;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[i][j][r]);
          *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + n0 + wc * WTN + 16 * j + 4 * fg) = o;
        }
      }
    } else {
      const int sub = fg & 1, set = fg >> 1;
#pragma unroll
      for (int i = 0; i < TM; i += 2) {
        const int m = wr * WTM + 16 * (i + sub) + fr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto p = __builtin_amdgcn_permlane16_swap(
                __float_as_uint(acc[i][j][r]), __float_as_uint(acc[i + 1][j][r]), false, false);
            const float g = __uint_as_float(p[0]), u = __uint_as_float(p[1]);
            o[r] = (short)f2bf(wg_silu(g) * u);
          }
          if (m < M)
            *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + ((n0 + wc * WTN + 16 * j) >> 1) +
                                         4 * set) = o;
        }
      }
    }
  }
}

// packed weights of K12-RS (BN columns per tile): for tile, K-step, wave w,
// fragment f = j*2 + kk, lane l = (fg << 4) | fr:
//   P[((((tile*nk + kstep)*4 + w)*WFR + f)*64 + l)*8 .. +8] =
//       W[tile*BN + w*BN/4 + 16j + fr][kstep*64 + 32kk + 8fg .. +8]
__global__ void wgemm_rs_pack_kernel(bf16_t* __restrict__ P, const bf16_t* __restrict__ W, int N,
                                     int K, long ldw, int BN, int WNR) {
  const int TN = BN / WNR / 16, WFR = TN * 2, nk = K / 64;
  const long chunks = (long)N * K / 8;
  for (long c = blockIdx.x * (long)blockDim.x + threadIdx.x; c < chunks;
       c += (long)gridDim.x * blockDim.x) {
    const int l = (int)(c & 63);
    long q = c >> 6;
    const int f = (int)(q % WFR);
    q /= WFR;
    const int w = (int)(q % WNR);
    q /= WNR;
    const int kstep = (int)(q % nk), tile = (int)(q / nk);
    const int j = f >> 1, kk = f & 1, fr = l & 15, fg = l >> 4;
    const long row = (long)tile * BN + w * (BN / WNR) + 16 * j + fr;
    const long col = (long)kstep * 64 + 32 * kk + 8 * fg;
    *reinterpret_cast<u16x8*>(P + c * 8) = *reinterpret_cast<const u16x8*>(W + row * ldw + col);
  }
}

struct WgRsCfg { int bn, dw, wmr; };
static const WgRsCfg kWgRsCfgs[] = {{128, 6, 1}, {128, 4, 1}, {128, 8, 1}, {64, 6, 1},
                                    {64, 8, 1},  {128, 2, 1}, {128, 6, 2}, {128, 8, 2},
                                    {112, 2, 4}, {112, 4, 4}, {224, 2, 2}, {128, 4, 2}};
constexpr int kNumWgRsCfgs = sizeof(kWgRsCfgs) / sizeof(kWgRsCfgs[0]);

int wgemm_rs_config(int cfg, int* bn) {
  if (cfg < 0 || cfg >= kNumWgRsCfgs) return -1;
  *bn = kWgRsCfgs[cfg].bn;
  return 0;
}

template <int BN, int DW, int EPI, int NT, int WMR>
static int wg_rs_launch(bf16_t* C, const bf16_t* A, const bf16_t* Wp, float* slabs, unsigned* cnt,
                        int M, int N, int K, long lda, long ldc, int splits, hipStream_t stream) {
  constexpr size_t smem = 2 * 256 * 64 * sizeof(bf16_t);
  auto kern = wgemm_rs_kernel<BN, DW, EPI, NT, WMR>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  kern<<<dim3((N / BN) * splits), dim3(256), smem, stream>>>(C, A, Wp, slabs, cnt, M, N, K, lda,
                                                            ldc, splits);
  return (int)hipGetLastError();
}

// cfg: K12-RS configuration (kWgRsCfgs) | 32 for non-temporal weight loads;
// Wp in the wgemm_rs_pack layout of the configuration's BN
int wgemm_rs(void* C, const void* A, const void* Wp, float* slabs, unsigned* cnt, int n_cnt, int M,
             int N, int K, long lda, long ldc, int cfg, int splits, int epi, hipStream_t stream) {
  if (M <= 0) return 0;
  const int nt = (cfg >> 5) & 1;
  cfg &= 31;
  if (cfg >= kNumWgRsCfgs || splits < 1 || M > 256) return -1;
  const WgRsCfg c = kWgRsCfgs[cfg];
  if (N % c.bn != 0 || K % 64 != 0 || K / 64 < splits) return -1;
  if (epi != 0 && epi != 2 && epi != 3) return -1;
  if ((epi == 2 || splits > 1) && slabs == nullptr) return -2;
  if (epi != 2 && splits > 1 && (cnt == nullptr || 2 * (N / c.bn) > n_cnt)) return -3;
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)Wp;
#define LMX_WGRS_E(BN, DW, NT, WMR)                                                              \
  if (epi == 3) return wg_rs_launch<BN, DW, 3, NT, WMR>(C_, A_, W_, slabs, cnt, M, N, K, lda, ldc, \
                                                        splits, stream);                         \
  if (epi == 2) return wg_rs_launch<BN, DW, 2, NT, WMR>(C_, A_, W_, slabs, cnt, M, N, K, lda, ldc, \
                                                        splits, stream);                         \
  return wg_rs_launch<BN, DW, 0, NT, WMR>(C_, A_, W_, slabs, cnt, M, N, K, lda, ldc, splits,       \
                                          stream);
#define LMX_WGRS_CASE(ID, BN, DW, WMR)                                                           \
  case ID:                                                                                       \
    if (nt) { LMX_WGRS_E(BN, DW, 1, WMR) }                                                       \
    LMX_WGRS_E(BN, DW, 0, WMR)
  switch (cfg) {
    LMX_WGRS_CASE(0, 128, 6, 1)
    LMX_WGRS_CASE(1, 128, 4, 1)
    LMX_WGRS_CASE(2, 128, 8, 1)
    LMX_WGRS_CASE(3, 64, 6, 1)
    LMX_WGRS_CASE(4, 64, 8, 1)
    LMX_WGRS_CASE(5, 128, 2, 1)
    LMX_WGRS_CASE(6, 128, 6, 2)
    LMX_WGRS_CASE(7, 128, 8, 2)
    LMX_WGRS_CASE(8, 112, 2, 4)
    LMX_WGRS_CASE(9, 112, 4, 4)
    LMX_WGRS_CASE(10, 224, 2, 2)
    LMX_WGRS_CASE(11, 128, 4, 2)
  }
#undef LMX_WGRS_CASE
#undef LMX_WGRS_E
  return -1;
}

int wgemm_rs_pack(void* P, const void* W, int N, int K, long ldw, int cfg, hipStream_t stream) {
  cfg &= 31;
  if (cfg >= kNumWgRsCfgs) return -1;
  const int bn = kWgRsCfgs[cfg].bn, wnr = 4 / kWgRsCfgs[cfg].wmr;
  if (N % bn != 0 || K % 64 != 0 || ldw % 8 != 0) return -1;
  const long chunks = (long)N * K / 8;
  const int grid = (int)std::min<long>(8192, (chunks + 255) / 256);
  wgemm_rs_pack_kernel<<<grid, 256, 0, stream>>>((bf16_t*)P, (const bf16_t*)W, N, K, ldw, bn,
                                                 wnr);
  return (int)hipGetLastError();
}

// ---- launcher ---------------------------------------------------------------
// cfg ids (BN, WM, WN, BK, NX, NW); kept in sync with ops.WGEMM_CONFIGS
struct WgCfg { int bn, wm, wn, bk, nx, nw; };
#define LMX_WG_CONFIGS(X)           \
  X(0, 224, 2, 2, 64, 2, 3)         \
  X(1, 224, 2, 2, 32, 3, 7)         \
  X(2, 256, 2, 2, 32, 3, 6)         \
  X(3, 112, 4, 1, 64, 2, 6)         \
  X(4, 112, 4, 1, 32, 3, 12)        \
  X(5, 224, 4, 2, 64, 2, 3)         \
  X(6, 128, 2, 2, 64, 2, 4)         \
  X(7, 128, 2, 2, 32, 3, 8)         \
  X(8, 96, 2, 2, 64, 2, 5)          \
  X(9, 192, 2, 2, 64, 2, 3)         \
  X(10, 256, 2, 2, 64, 2, 2)        \
  X(11, 224, 4, 1, 64, 2, 3)        \
  X(12, 128, 4, 1, 64, 2, 4)        \
  X(13, 112, 4, 1, 64, 3, 4)        \
  X(14, 112, 4, 1, 32, 4, 12)       \
  X(15, 128, 4, 1, 64, 3, 3)        \
  X(16, 112, 4, 1, 32, 2, 18)

static const WgCfg kWgCfgs[] = {
#define LMX_WG_ROW(ID, BN, WM, WN, BK, NX, NW) {BN, WM, WN, BK, NX, NW},
    LMX_WG_CONFIGS(LMX_WG_ROW)
#undef LMX_WG_ROW
};
constexpr int kNumWgCfgs = sizeof(kWgCfgs) / sizeof(kWgCfgs[0]);

int wgemm_num_configs() { return kNumWgCfgs; }

int wgemm_config(int cfg, int* bn, int* bk) {
  if (cfg < 0 || cfg >= kNumWgCfgs) return -1;
  *bn = kWgCfgs[cfg].bn;
  *bk = kWgCfgs[cfg].bk;
  return 0;
}

template <int BN, int WM, int WN, int BK, int NX, int NW, int EPI, int NT, int MMA, int PK>
static int wg_launch(bf16_t* C, const bf16_t* A, const bf16_t* W, float* slabs, unsigned* cnt,
                     int M, int N, int K, long lda, long ldw, long ldc, int splits,
                     hipStream_t stream) {
  constexpr size_t smem = (size_t)(NX * 256 + NW * BN) * BK * sizeof(bf16_t);
  static_assert(smem <= 160 * 1024, "LDS");
  auto kern = wgemm_kernel<BN, WM, WN, BK, NX, NW, EPI, NT, MMA, PK>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int nwg = (N / BN) * splits;
  kern<<<dim3(nwg), dim3(WM * WN * 64), smem, stream>>>(C, A, W, slabs, cnt, M, N, K, lda, ldw,
                                                        ldc, splits);
  return (int)hipGetLastError();
}

// epi: 0 bf16, 2 partial slabs, 3 SwiGLU (4-row gate/up blocks); cfg bit 5:
// non-temporal weight stream; cfg bit 6: no MFMA (data-movement probe);
// cfg bit 7: W is in the packed layout of this configuration (wgemm_pack);
// bit 10 (with bit 7): the K-step-major packed layout
int wgemm(void* C, const void* A, const void* W, float* slabs, unsigned* cnt, int n_cnt, int M,
          int N, int K, long lda, long ldw, long ldc, int cfg, int splits, int epi,
          hipStream_t stream) {
  if (M <= 0) return 0;
  const int nt = (cfg >> 5) & 1, pk = (cfg >> 7) & 1 ? ((cfg >> 10) & 1 ? 2 : 1) : 0;
  // bit 6: no MFMA; bit 8 / 9 (with bit 6): also skip the A / W loads
  const int probe = (cfg >> 6) & 1 ? ((cfg >> 8) & 1 ? 2 : (cfg >> 9) & 1 ? 3 : 1) : 0;
  constexpr int nt_probe = 0;
  cfg &= 31;
  if (cfg >= kNumWgCfgs || splits < 1 || M > 256) return -1;
  const WgCfg c = kWgCfgs[cfg];
  if (N % c.bn != 0 || K % c.bk != 0 || K / c.bk < splits) return -1;
  if (epi != 0 && epi != 2 && epi != 3) return -1;
  if ((epi == 2 || splits > 1) && slabs == nullptr) return -2;
  if (epi != 2 && splits > 1 && (cnt == nullptr || 2 * (N / c.bn) > n_cnt)) return -3;
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
#define LMX_WG_P(BN, WM, WN, BK, NX, NW, NT, MMA, PK)                                          \
  if (epi == 3) {                                                                             \
    if constexpr ((256 / WM / 16) % 2 == 0)                                                   \
      return wg_launch<BN, WM, WN, BK, NX, NW, 3, NT, MMA, PK>(C_, A_, W_, slabs, cnt, M, N,  \
                                                               K, lda, ldw, ldc, splits,      \
                                                               stream);                       \
    return -1;                                                                                \
  }                                                                                           \
  if (epi == 2)                                                                               \
    return wg_launch<BN, WM, WN, BK, NX, NW, 2, NT, MMA, PK>(C_, A_, W_, slabs, cnt, M, N, K,  \
                                                             lda, ldw, ldc, splits, stream);  \
  return wg_launch<BN, WM, WN, BK, NX, NW, 0, NT, MMA, PK>(C_, A_, W_, slabs, cnt, M, N, K,    \
                                                           lda, ldw, ldc, splits, stream);
#define LMX_WG_E(BN, WM, WN, BK, NX, NW, NT, MMA)                                               \
  if (pk == 2) { LMX_WG_P(BN, WM, WN, BK, NX, NW, NT, MMA, 2) }                               \
  if (pk) { LMX_WG_P(BN, WM, WN, BK, NX, NW, NT, MMA, 1) }                                    \
  LMX_WG_P(BN, WM, WN, BK, NX, NW, NT, MMA, 0)
#ifdef LMX_WGEMM_LAB
#define LMX_WG_CASE(ID, BN, WM, WN, BK, NX, NW)                                               \
  case ID:                                                                                    \
    if (probe == 2) { LMX_WG_E(BN, WM, WN, BK, NX, NW, nt_probe, 2) }                         \
    if (probe == 3) { LMX_WG_E(BN, WM, WN, BK, NX, NW, nt_probe, 3) }                         \
    if (probe) { LMX_WG_E(BN, WM, WN, BK, NX, NW, 0, 0) }                                     \
    if (nt) { LMX_WG_E(BN, WM, WN, BK, NX, NW, 1, 1) }                                        \
    LMX_WG_E(BN, WM, WN, BK, NX, NW, 0, 1)
#else
  // the library keeps the configurations the measurements left standing
  // (profiles/r3_decode_gemm_study.md): the 4x1 / 2x2 single-workgroup tiles
  // and the partials form; packed layouts row-major or K-step-major
#define LMX_WG_CASE(ID, BN, WM, WN, BK, NX, NW)                                               \
  case ID:                                                                                    \
    if constexpr (ID == 3 || ID == 6 || ID == 8 || ID == 12 || ID == 13) {                    \
      if (probe || pk == 1) return -1;                                                        \
      if (nt) { LMX_WG_E(BN, WM, WN, BK, NX, NW, 1, 1) }                                      \
      LMX_WG_E(BN, WM, WN, BK, NX, NW, 0, 1)                                                  \
    }                                                                                         \
    return -1;
#endif
  switch (cfg) { LMX_WG_CONFIGS(LMX_WG_CASE) }
#undef LMX_WG_CASE
#undef LMX_WG_E
#undef LMX_WG_P
  return -1;
}

// Packs W [N][K] (row stride ldw) into P for configuration cfg (N*K elements)
int wgemm_pack(void* P, const void* W, int N, int K, long ldw, int cfg, hipStream_t stream) {
  const bool kmajor = (cfg >> 10) & 1;
  cfg &= 31;
  if (cfg >= kNumWgCfgs) return -1;
  const WgCfg c = kWgCfgs[cfg];
  if (N % c.bn != 0 || K % c.bk != 0 || ldw % 8 != 0) return -1;
  const long chunks = (long)N * K / 8;
  const int grid = (int)std::min<long>(8192, (chunks + 255) / 256);
  const int km = kmajor ? 1 : 0;
  if (c.bk == 64)
    wgemm_pack_kernel<64><<<grid, 256, 0, stream>>>((bf16_t*)P, (const bf16_t*)W, N, K, ldw, c.bn,
                                                    km);
  else
    wgemm_pack_kernel<32><<<grid, 256, 0, stream>>>((bf16_t*)P, (const bf16_t*)W, N, K, ldw, c.bn,
                                                    km);
  return (int)hipGetLastError();
}

}  // namespace lmx
