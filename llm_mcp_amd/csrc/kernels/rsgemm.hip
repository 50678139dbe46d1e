// K14: register-streamed weight GEMM for 129..256-row decode batches
//     C[M, N] = A[M, K] . W[N, K]^T        (bf16 in, fp32 accumulate)
//
// Why (profiles/r3_decode_gemm_study.md, r3_k13_and_decode_sk.md): at M = 256
// a decode projection is a weight stream that every CU must also feed with
// the whole activation panel; the LDS-DMA designs (K11, K12, K13-SK) reach
// 5.1-5.4 TB/s on the weight stream alone, while plain 16-B register loads of
// a linear stream reach 6.4-6.7 TB/s.  K12-RS moved the weights to registers
// but with one wave per SIMD and every wave owning 128 columns it exposed the
// ds_read -> MFMA chain.  K14 keeps the weights register-streamed and shapes
// the rest around the CDNA4 numbers:
//   * one 512-thread workgroup per CU: 8 waves, 2 per SIMD, so one wave's LDS
//     reads and waits overlap its partner's MFMAs;
//   * a workgroup owns ALL rows (<= 256) x a 256-column tile over a K slice
//     (split-K over S workgroups); wave w owns columns [32w, 32w + 32): two
//     16-column MFMA tiles (16x16x32 bf16, weights as the A operand), so each
//     activation fragment read from LDS feeds 2 MFMAs and a K32 step is 1024
//     MFMA cycles per SIMD against 512 LDS cycles per CU;
//   * weights pre-packed (rsgemm_pack): each (tile, wave, K32 block, 16-column
//     half) is one 1-KB run in MFMA fragment order, so a wave's whole K slice
//     is ONE linear stream of global_load_dwordx4 (1 KB per instruction, 8
//     full lines), D K32 steps (2 x D loads) in flight in a register ring;
//   * activations move L2 -> LDS by LDS-DMA (global_load_lds_dwordx4) into an
//     NA-slot ring of 256 x 64 XOR-swizzled images (conflict-free
//     ds_read_b128), one raw s_barrier per K64 step;
//   * the weight loads are inline asm and every vmcnt wait is hand-counted:
//     beside an LDS-DMA hipcc waits vmcnt(0) for any ordinary register load
//     (cdna guide §5 "Projection GEMM at M = 256" item 4b), which would drain
//     the ring every step.  Issue order per K64 step t:
//        [4 LDS-DMA: A(t + NA - 1)] [2 loads: W(2t + D)] [2 loads: W(2t + 1 + D)]
//     so A(t) is complete at vmcnt(4 + 8 (NA - 2)) and W(2t + 1) at
//     vmcnt(8 (U - 1) + 6) with U = D / 2 (the prologue issues the same
//     pattern for the virtual steps -U .. -1);
//   * split-K: fp32 slabs + arrival ticket (K11's recipe); epilogues: bf16,
//     fp32 partials for the residual-add RMSNorm, SwiGLU over [16 gate | 16 up]
//     weight rows (interleave_gate_up(w, 16): a wave's two 16-column tiles are
//     the gate and up values of the same 16 channels, in the same lanes).
#include "common.h"

// RS_LAB (tools/rsgemm_lab.cpp only, never in the extension): bit 0 drops the
// MFMAs, bit 1 points every weight load at the wave's first K32 step (L1 /
// L2-hot), bit 2 every activation DMA at the first K64 step -- the time each
// part adds to the kernel.  Results are garbage in these builds.
#ifndef RS_LAB
#define RS_LAB 0
#endif

namespace lmx {
namespace {

constexpr int RS_THREADS = 512, RS_BN = 256, RS_BK = 64;

typedef __attribute__((address_space(3))) void rs_lds_t;

__device__ __forceinline__ int rs_swz(int r) { return (r >> 1) & 7; }

// one K64 step of the activation panel (BM rows from m0, padded rows re-read
// row M-1) into an LDS slot: BM / 64 LDS-DMA instructions per thread
template <int BM>
__device__ __forceinline__ void rs_stage_a(bf16_t* slot, const bf16_t* __restrict__ A, long lda,
                                           int M, int m0, int k0) {
  const int t = threadIdx.x, wave = t >> 6;
  const int rr = t >> 3, c = t & 7;
#pragma unroll
  for (int i = 0; i < BM / 64; ++i) {
    const int r = i * 64 + rr;
    const int gr = m0 + r < M ? m0 + r : M - 1;
    if constexpr ((RS_LAB & 4) != 0) k0 = 0;
    __builtin_amdgcn_global_load_lds(A + (long)gr * lda + k0 + 8 * (c ^ rs_swz(r)),
                                     (rs_lds_t*)(slot + (i * 64 + wave * 8) * RS_BK), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8_t rs_afrag(const bf16_t* slot, int r, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(slot + r * RS_BK + 8 * (chunk ^ rs_swz(r)));
}

// weight fragment load (hand-counted: see the header): wave-uniform SGPR base
// + the lane's 16-B offset + an immediate (< 4 KB), so the ring costs no
// 64-bit address VGPRs
template <int NT, int IMM>
__device__ __forceinline__ void rs_ldw(bf16x8_t& r, const void* sbase, unsigned voff) {
  if constexpr (NT)
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3 nt"
                 : "=v"(r) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3"
                 : "=v"(r) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}

// the loop's ring refill overwrites registers the MFMAs just before it read
// as their A operand; hipcc pads no hazard for an asm instruction, so the
// first refill after a compute phase starts behind 20 wait states
__device__ __forceinline__ void rs_mfma_war_pad() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
}

template <int CNT>
__device__ __forceinline__ void rs_wait(bf16x8_t& a, bf16x8_t& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(CNT) : "memory");
}

__device__ __forceinline__ void rs_wait0(bf16x8_t& a, bf16x8_t& b) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b) :: "memory");
}

// the same for K14W's four loads per K32 step: every destination of the
// step is an operand, so none of them is touched before the wait
template <int CNT>
__device__ __forceinline__ void rs_wait4(bf16x8_t (&w)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3])
               : "n"(CNT) : "memory");
}

__device__ __forceinline__ float rs_silu(float g) { return g / (1.f + __expf(-g)); }

// split-K combine of the last arriving slice: acc[j][g] = sum over the S
// slabs in slice order, with at most 8 loads (32 VGPRs) in flight at a time
// beside the 128 accumulator registers
template <int S, int NG>
__device__ __forceinline__ void rs_combine(f32x4_t (&acc)[2][NG], const float* __restrict__ slabs,
                                           long MN, int M, int N, int nb, int m0, int fr) {
  constexpr int SB = S < 8 ? S : 8;              // slabs per batch
  constexpr int UN = 8 / SB;                     // (row group, half) units per batch
#pragma unroll
  for (int u0 = 0; u0 < 2 * NG; u0 += UN) {
    long off[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int m = m0 + 16 * ((u0 + u) >> 1) + fr;
      off[u] = (long)(m < M ? m : M - 1) * N + nb + 16 * ((u0 + u) & 1);
    }
    f32x4_t t[UN];
#pragma unroll
    for (int sb = 0; sb < S; sb += SB) {
      f32x4_t v[UN][SB];
#pragma unroll
      for (int u = 0; u < UN; ++u)
#pragma unroll
        for (int s = 0; s < SB; ++s)
          v[u][s] = *reinterpret_cast<const f32x4_t*>(slabs + (sb + s) * MN + off[u]);
#pragma unroll
      for (int u = 0; u < UN; ++u)
#pragma unroll
        for (int s = 0; s < SB; ++s) t[u] = (sb + s == 0) ? v[u][0] : t[u] + v[u][s];
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) acc[(u0 + u) & 1][(u0 + u) >> 1] = t[u];
  }
}

}  // namespace

// W packed: [N/256][8 waves][K/32][2 halves][64 lanes][8]: lane l of (wave w,
// half j, block kb) holds W[256 T + 32 w + 16 j + (l & 15)][32 kb + 8 (l >> 4) .. +8]
__global__ void rsgemm_pack_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ W,
                                   int N, int K, long ldw) {
  const long c = blockIdx.x * 256L + threadIdx.x;
  if (c >= (long)N * K / 8) return;
  const int KB = K / 32;
  const int lane = (int)(c & 63);
  long q = c >> 6;
  const int j = (int)(q & 1);
  q >>= 1;
  const int kb = (int)(q % KB);
  q /= KB;
  const int w = (int)(q & 7), T = (int)(q >> 3);
  const long n = (long)T * 256 + w * 32 + j * 16 + (lane & 15);
  const int k = kb * 32 + (lane >> 4) * 8;
  *reinterpret_cast<u16x8*>(out + c * 8) = *reinterpret_cast<const u16x8*>(W + n * ldw + k);
}

// EPI: 0 bf16 [M, N]; 2 fp32 partial slabs [S][M][N] (no combine); 3 SwiGLU16
// -> bf16 [M, N/2].  D: weight ring depth in K32 steps (even); NA: A slots.
// RM: 0 packed weights (rsgemm_pack); 1 the plain row-major [N][ldw] weights,
// read as fragment-shaped loads (16 rows x 64 B per instruction; a row's two
// 64-B halves of a 128-B line are read by consecutive K32 steps).
// BM: rows per workgroup (256: all rows, or 128: the two row tiles of a column
// tile run side by side, adjacent workgroup ids, and share its weight stream
// through the XCD's L2 -- split-K-free at 224 workgroups for gate/up)
template <int EPI, int D, int NA, int NT, int RM, int BM>
__global__ void __launch_bounds__(RS_THREADS, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) rsgemm_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ Wp,
    float* __restrict__ slabs, unsigned* __restrict__ tickets, int M, int N, int K, long lda,
    long ldw, long ldc, int splits, int rot_mul) {
  constexpr int U = D / 2;
  // NA = U + 1: the prologue then issues every A slot it counts on (with
  // fewer slots the early steps would see fewer ops behind a load than the
  // steady-state counts assume)
  static_assert(D % 2 == 0 && U >= 2 && NA == U + 1, "ring shape");
  static_assert(BM == 256 || BM == 128 || BM == 64, "row tile");
  constexpr int NG = BM / 16, G = BM / 64, OPS = G + 4;   // row groups; VMEM ops per step
  constexpr int SLOT = BM * RS_BK;                  // bf16 elements of one A ring slot
  // with NA = U + 1, A(t) is issued just before W(2t) (step t - U): waiting
  // for W(2t) covers it
  constexpr int WAIT_TOP = 2 + OPS * (U - 1);       // W(2t) landed, top of step t
  constexpr int WAIT_W1 = OPS * (U - 1) + G + 2;    // W(2t + 1) landed, mid step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);

  const int tiles_m = (M + BM - 1) / BM, tiles = N / RS_BN, nwg = tiles_m * tiles * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int ks = wg % splits, rest = wg / splits;
  const int tm = rest % tiles_m, tn = rest / tiles_m, m0 = tm * BM;
  const int kc = K / splits, k0 = ks * kc, nk64 = kc / RS_BK;
  // K-step order rotated per column tile (rot_mul > 0; the two row tiles of
  // a column tile keep the same order, so their weight reads still merge):
  // the workgroups of an XCD then read different activation k-slices and
  // weight offsets at any moment instead of all hitting the same L2 lines
  const int rot = (BM != 256 && rot_mul) ? (tn * rot_mul) % nk64 : 0;   // (all-rows tiles: none, registers)
  auto kofs = [&](int step) { return k0 + ((step + rot) % nk64) * RS_BK; };
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;

  // this wave's weight stream.  Packed: 2 x 1 KB per K32 step, contiguous
  // over the slice (K32 step k at wstream + 2 KB k, + 1 KB for the second
  // half).  Row-major: rows 256 tn + 32 wave + 16 j + (lane & 15), 64 B per
  // row and K32 step (K32 step k at wstream + 64 k).
  const char* wstream =
      RM ? reinterpret_cast<const char*>(Wp) + ((long)(tn * RS_BN + 32 * wave) * ldw + k0) * 2
         : reinterpret_cast<const char*>(Wp) +
               ((long)(tn * 8 + wave) * (K / 32) + k0 / 32) * 2048;
  constexpr long KSTEP = RM ? 64 : 2048;
  const unsigned voff0 = RM ? (unsigned)((lane & 15) * ldw * 2 + (lane >> 4) * 16) : lane * 16;
  const unsigned voff1 = RM ? (unsigned)(((lane & 15) + 16) * ldw * 2 + (lane >> 4) * 16)
                            : lane * 16;
  constexpr int I0 = 0, I1 = RM ? 0 : 1024, I2 = RM ? 64 : 2048, I3 = RM ? 64 : 3072;
  auto wsb = [&](int k) -> const void* {   // wave-uniform base of K32 step k
    if constexpr ((RS_LAB & 2) != 0) k = 0;
    if (rot) k = (k + 2 * rot) % (2 * nk64);   // even k: the step pair stays contiguous
    return (const void*)(wstream + (long)k * KSTEP);
  };

  f32x4_t acc[2][NG];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[j][g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t wr[D][2];

  // prologue: the steady-state issue pattern of the virtual steps -U .. -1
#pragma unroll
  for (int s = -U; s < 0; ++s) {
    if (s + NA - 1 >= 0) rs_stage_a<BM>(lds + ((s + NA - 1) % NA) * SLOT, A, lda, M, m0,
                                        kofs(s + NA - 1));
    {
      const int k = 2 * (s + U);                     // K32 steps 2s + D, 2s + D + 1
      const void* b = wsb(k);
      rs_ldw<NT, I0>(wr[k][0], b, voff0);
      rs_ldw<NT, I1>(wr[k][1], b, voff1);
      rs_ldw<NT, I2>(wr[k + 1][0], b, voff0);
      rs_ldw<NT, I3>(wr[k + 1][1], b, voff1);
    }
  }

  // one K32 sub-step: the NG row-group fragments read in pairs, the next
  // pair in flight while the current pair's 4 MFMAs run
  auto compute = [&](const bf16_t* slot, int kk, const bf16x8_t& w0, const bf16x8_t& w1) {
    bf16x8_t cur0 = rs_afrag(slot, fr, kk * 4 + fg);
    bf16x8_t cur1 = rs_afrag(slot, 16 + fr, kk * 4 + fg);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int p = 0; p < NG / 2; ++p) {
      bf16x8_t nx0 = cur0, nx1 = cur1;
      if (p < NG / 2 - 1) {
        nx0 = rs_afrag(slot, 32 * (p + 1) + fr, kk * 4 + fg);
        nx1 = rs_afrag(slot, 32 * (p + 1) + 16 + fr, kk * 4 + fg);
      }
      if constexpr ((RS_LAB & 1) == 0) {
        acc[0][2 * p] = mfma16(w0, cur0, acc[0][2 * p]);
        acc[1][2 * p] = mfma16(w1, cur0, acc[1][2 * p]);
        acc[0][2 * p + 1] = mfma16(w0, cur1, acc[0][2 * p + 1]);
        acc[1][2 * p + 1] = mfma16(w1, cur1, acc[1][2 * p + 1]);
      } else {   // keep the fragment reads live without the MFMAs
        asm volatile("" :: "v"(w0), "v"(w1), "v"(cur0), "v"(cur1));
      }
      cur0 = nx0;
      cur1 = nx1;
    }
    // hold that order against the scheduler's register-pressure heuristic
    // (it otherwise reuses one fragment pair and waits lgkmcnt(0) per pair)
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int p = 0; p < NG / 2 - 1; ++p) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // steady state: steps [0, nk64 - U), in blocks of U (the ring index of a
  // K32 step is static inside the block)
  int t0 = 0;
  for (; t0 + U <= nk64 - U; t0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u;
      rs_wait<WAIT_TOP>(wr[2 * u][0], wr[2 * u][1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      rs_stage_a<BM>(lds + ((t + NA - 1) % NA) * SLOT, A, lda, M, m0,
                     kofs(t + NA - 1));
      const bf16_t* slot = lds + (t % NA) * SLOT;
      const void* b = wsb(2 * t + D);
      compute(slot, 0, wr[2 * u][0], wr[2 * u][1]);
      __builtin_amdgcn_sched_barrier(0);
      rs_mfma_war_pad();
      rs_ldw<NT, I0>(wr[2 * u][0], b, voff0);
      rs_ldw<NT, I1>(wr[2 * u][1], b, voff1);
      rs_wait<WAIT_W1>(wr[2 * u + 1][0], wr[2 * u + 1][1]);
      compute(slot, 1, wr[2 * u + 1][0], wr[2 * u + 1][1]);
      __builtin_amdgcn_sched_barrier(0);
      rs_mfma_war_pad();
      rs_ldw<NT, I2>(wr[2 * u + 1][0], b, voff0);
      rs_ldw<NT, I3>(wr[2 * u + 1][1], b, voff1);
    }
  }
  // tail: the last U steps (no weight loads left to issue), conservative waits
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = t0 + u;
    if (t >= nk64) break;
    rs_wait0(wr[2 * u][0], wr[2 * u][1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NA - 1 < nk64)
      rs_stage_a<BM>(lds + ((t + NA - 1) % NA) * SLOT, A, lda, M, m0, kofs(t + NA - 1));
    const bf16_t* slot = lds + (t % NA) * SLOT;
    compute(slot, 0, wr[2 * u][0], wr[2 * u][1]);
    rs_wait0(wr[2 * u + 1][0], wr[2 * u + 1][1]);
    compute(slot, 1, wr[2 * u + 1][0], wr[2 * u + 1][1]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // acc[j][g][r] = C[m][n]: m = m0 + 16 g + fr, n = 256 tn + 32 wave + 16 j + 4 fg + r
  const int nb = tn * RS_BN + 32 * wave + 4 * fg;
  if (splits > 1 || EPI == 2) {
    float* slab = slabs + (long)ks * M * N;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + nb + 16 * j) = acc[j][g];
    }
    if (EPI == 2) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(&tickets[tn * tiles_m + tm], 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (old == (unsigned)(splits - 1));
    }
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tickets[tn * tiles_m + tm] = 0u;   // re-armed: every slice of this call has arrived
    }
    __syncthreads();
    // every slab, this slice's own included, summed in slice order: the
    // result is bitwise the same whichever slice arrives last, and the loads
    // carry no per-element condition (a runtime "own or load" select makes
    // hipcc wait vmcnt(0) per load: one L2 round trip each)
    switch (splits) {
      case 2: rs_combine<2, NG>(acc, slabs, (long)M * N, M, N, nb, m0, fr); break;
      case 4: rs_combine<4, NG>(acc, slabs, (long)M * N, M, N, nb, m0, fr); break;
      case 8: rs_combine<8, NG>(acc, slabs, (long)M * N, M, N, nb, m0, fr); break;
      default: rs_combine<16, NG>(acc, slabs, (long)M * N, M, N, nb, m0, fr); break;
    }
  }
  if constexpr (EPI == 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[j][g][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + nb + 16 * j) = o;
      }
    }
  } else if constexpr (EPI == 3) {
    const int ob = (tn * RS_BN + 32 * wave) / 2 + 4 * fg;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(rs_silu(acc[0][g][r]) * acc[1][g][r]);
      *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + ob) = o;
    }
  }
}

// ---- K14W: one wave per SIMD, 64 columns per wave ---------------------------
// Why (profiles/r6_decode_gemm.md, tools/rs_decomp.sh): K14 at 256 rows sits on
// two separate ceilings of about its own run time -- the weight stream alone
// (MFMAs removed: 67.7 us for gate/up) is latency-bound at ~64 KB in flight
// per CU (8 waves x a 4-step register ring), and the LDS fragment reads plus
// the MFMAs alone (memory made L1-hot: 62.6 us) serialise at 512 + 512 cycles
// per K32 step, because every one of the 8 waves re-reads the whole
// activation panel from LDS for its 32 columns.  Here a 256-thread workgroup
// (one wave per SIMD, up to 512 VGPRs incl. AGPRs) owns the same BM x 256
// tile: wave w owns columns [64 w, 64 w + 64) = K14 wave units 2w, 2w + 1
// (the packed layout is unchanged), so
//   * each activation fragment read from LDS feeds 4 MFMAs (LDS traffic per
//     CU halves: 256 cycles per K32 step against 512 MFMA cycles per SIMD);
//   * the weight ring is D = 8 K32 steps deep (32 KB per wave, 128 KB per CU
//     in flight, twice K14's);
//   * issue order per K64 step t: [GA LDS-DMA: A(t + NA - 1)] [4 loads:
//     W(2t + D)] [4 loads: W(2t + 1 + D)] with the same hand-counted waits.
// Epilogues: bf16, fp32 partials (split-K, no in-kernel combine) and SwiGLU16.
template <int EPI, int D, int NA, int NT, int BM>
__global__ void __launch_bounds__(256, 1) rsgemm4_kernel(
    bf16_t* __restrict__ C, const bf16_t* __restrict__ A, const bf16_t* __restrict__ Wp,
    float* __restrict__ slabs, int M, int N, int K, long lda, long ldc, int splits) {
  constexpr int U = D / 2;
  static_assert(D % 2 == 0 && U >= 2 && NA == U + 1, "ring shape");
  static_assert(BM == 128 || BM == 64, "row tile");
  constexpr int NG = BM / 16, GA = BM / 32, OPS = GA + 8;
  constexpr int SLOT = BM * RS_BK;
  constexpr int WAIT_TOP = 4 + OPS * (U - 1);       // W(2t) landed, top of step t
  constexpr int WAIT_W1 = OPS * (U - 1) + GA + 4;   // W(2t + 1) landed, mid step
  static_assert(WAIT_W1 < 64 && WAIT_TOP < 64, "vmcnt is 6 bits");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);

  const int tiles_m = (M + BM - 1) / BM, tiles = N / RS_BN, nwg = tiles_m * tiles * splits;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int ks = wg % splits, rest = wg / splits;
  const int tm = rest % tiles_m, tn = rest / tiles_m, m0 = tm * BM;
  const int kc = K / splits, k0 = ks * kc, nk64 = kc / RS_BK;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;

  // the two K14 wave units of this wave: 2 x 1 KB runs per K32 step each
  const char* ws0 = reinterpret_cast<const char*>(Wp) +
                    ((long)(tn * 8 + 2 * wave) * (K / 32) + k0 / 32) * 2048;
  const char* ws1 = ws0 + (long)(K / 32) * 2048;
  const unsigned voff = lane * 16;
  auto wsb = [&](const char* ws, int k) -> const void* {   // K32 step k
    if constexpr ((RS_LAB & 2) != 0) k = 0;
    return (const void*)(ws + (long)k * 2048);
  };
  // A: BM rows x 64 k per K64 step, 256 lanes x 16 B per instruction
  auto stage_a = [&](bf16_t* slot, int kk) {
    const int t = threadIdx.x, rr = t >> 3, c = t & 7;
    if constexpr ((RS_LAB & 4) != 0) kk = 0;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int r = i * 32 + rr;
      const int gr = m0 + r < M ? m0 + r : M - 1;
      __builtin_amdgcn_global_load_lds(A + (long)gr * lda + kk + 8 * (c ^ rs_swz(r)),
                                       (rs_lds_t*)(slot + (i * 32 + wave * 8) * RS_BK), 16, 0, 0);
    }
  };

  f32x4_t acc[4][NG];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[j][g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t wr[D][4];   // [K32 step][col tile 2u + j]

  auto issue_w = [&](int k, bf16x8_t (&dst)[4], int imm_half) {
    // imm_half 0: K32 step k at [base, +2 KB); 1: the step after it at [+2, +4 KB)
    const void* b0 = wsb(ws0, k - imm_half);
    const void* b1 = wsb(ws1, k - imm_half);
    if (imm_half == 0) {
      rs_ldw<NT, 0>(dst[0], b0, voff);
      rs_ldw<NT, 1024>(dst[1], b0, voff);
      rs_ldw<NT, 0>(dst[2], b1, voff);
      rs_ldw<NT, 1024>(dst[3], b1, voff);
    } else {
      rs_ldw<NT, 2048>(dst[0], b0, voff);
      rs_ldw<NT, 3072>(dst[1], b0, voff);
      rs_ldw<NT, 2048>(dst[2], b1, voff);
      rs_ldw<NT, 3072>(dst[3], b1, voff);
    }
  };

#pragma unroll
  for (int s = -U; s < 0; ++s) {
    stage_a(lds + ((s + NA - 1) % NA) * SLOT, k0 + (s + NA - 1) * RS_BK);
    const int k = 2 * (s + U);
    issue_w(k, wr[k], 0);
    issue_w(k + 1, wr[k + 1], 1);
  }

  // one K32 sub-step: row-group fragments in pairs, the next pair in flight
  // while the current pair's 8 MFMAs run
  auto compute = [&](const bf16_t* slot, int kk, const bf16x8_t (&w)[4]) {
    bf16x8_t cur0 = rs_afrag(slot, fr, kk * 4 + fg);
    bf16x8_t cur1 = rs_afrag(slot, 16 + fr, kk * 4 + fg);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int p = 0; p < NG / 2; ++p) {
      bf16x8_t nx0 = cur0, nx1 = cur1;
      if (p < NG / 2 - 1) {
        nx0 = rs_afrag(slot, 32 * (p + 1) + fr, kk * 4 + fg);
        nx1 = rs_afrag(slot, 32 * (p + 1) + 16 + fr, kk * 4 + fg);
      }
      if constexpr ((RS_LAB & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j][2 * p] = mfma16(w[j], cur0, acc[j][2 * p]);
          acc[j][2 * p + 1] = mfma16(w[j], cur1, acc[j][2 * p + 1]);
        }
      } else {
        asm volatile("" :: "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(cur0), "v"(cur1));
      }
      cur0 = nx0;
      cur1 = nx1;
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int p = 0; p < NG / 2 - 1; ++p) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // a do-while (the host guarantees nk64 >= 2U): a loop entered on a branch
  // gets phi copies of the ring registers at its entry, taken while their
  // loads are still in flight (tools/vmem_hazard_audit.py)
  int t0 = 0;
  do {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u;
      rs_wait4<WAIT_TOP>(wr[2 * u]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stage_a(lds + ((t + NA - 1) % NA) * SLOT, k0 + (t + NA - 1) * RS_BK);
      const bf16_t* slot = lds + (t % NA) * SLOT;
      compute(slot, 0, wr[2 * u]);
      __builtin_amdgcn_sched_barrier(0);
      rs_mfma_war_pad();
      issue_w(2 * t + D, wr[2 * u], 0);
      rs_wait4<WAIT_W1>(wr[2 * u + 1]);
      compute(slot, 1, wr[2 * u + 1]);
      __builtin_amdgcn_sched_barrier(0);
      rs_mfma_war_pad();
      issue_w(2 * t + 1 + D, wr[2 * u + 1], 1);
    }
    t0 += U;
  } while (t0 + U <= nk64 - U);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = t0 + u;
    if (t >= nk64) break;
    rs_wait4<0>(wr[2 * u]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NA - 1 < nk64) stage_a(lds + ((t + NA - 1) % NA) * SLOT, k0 + (t + NA - 1) * RS_BK);
    const bf16_t* slot = lds + (t % NA) * SLOT;
    compute(slot, 0, wr[2 * u]);
    rs_wait4<0>(wr[2 * u + 1]);
    compute(slot, 1, wr[2 * u + 1]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // acc[j][g][r] = C[m][n]: m = m0 + 16 g + fr, n = 256 tn + 64 wave + 16 j + 4 fg + r
  const int nb = tn * RS_BN + 64 * wave + 4 * fg;
  if constexpr (EPI == 2) {
    float* slab = slabs + (long)ks * M * N;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4_t*>(slab + (long)m * N + nb + 16 * j) = acc[j][g];
    }
  } else if constexpr (EPI == 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[j][g][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + nb + 16 * j) = o;
      }
    }
  } else {
    // SwiGLU16: unit u's tiles 2u (gate) and 2u + 1 (up) hold the same 16
    // channels; unit u of this wave is K14 wave unit 2 wave + u
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = m0 + 16 * g + fr;
      if (m >= M) continue;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = (short)f2bf(rs_silu(acc[2 * u][g][r]) * acc[2 * u + 1][g][r]);
        *reinterpret_cast<bf16x4_t*>(C + (long)m * ldc + (tn * RS_BN + 64 * wave + 32 * u) / 2 +
                                     4 * fg) = o;
      }
    }
  }
}

template <int EPI, int D, int NA, int NT, int BM>
static int rs4_launch(bf16_t* C, const bf16_t* A, const bf16_t* Wp, float* slabs, int M, int N,
                      int K, long lda, long ldc, int splits, hipStream_t stream) {
  constexpr size_t smem = (size_t)NA * BM * RS_BK * sizeof(bf16_t);
  static_assert(smem <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)rsgemm4_kernel<EPI, D, NA, NT, BM>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  rsgemm4_kernel<EPI, D, NA, NT, BM>
      <<<dim3(((M + BM - 1) / BM) * (N / RS_BN) * splits), dim3(256), smem, stream>>>(
          C, A, Wp, slabs, M, N, K, lda, ldc, splits);
  return (int)hipGetLastError();
}

// ---- host -------------------------------------------------------------------
int rsgemm_pack(void* out, const void* W, int N, int K, long ldw, hipStream_t stream) {
  if (N % RS_BN != 0 || K % 32 != 0) return -1;
  const long chunks = (long)N * K / 8;
  rsgemm_pack_kernel<<<dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, stream>>>(
      (bf16_t*)out, (const bf16_t*)W, N, K, ldw);
  return (int)hipGetLastError();
}

template <int EPI, int D, int NA, int NT, int RM, int BM>
static int rs_launch(bf16_t* C, const bf16_t* A, const bf16_t* Wp, float* slabs,
                     unsigned* tickets, int M, int N, int K, long lda, long ldw, long ldc,
                     int splits, int rot_mul, hipStream_t stream) {
  constexpr size_t smem = (size_t)NA * BM * RS_BK * sizeof(bf16_t);
  static_assert(smem <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)rsgemm_kernel<EPI, D, NA, NT, RM, BM>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  rsgemm_kernel<EPI, D, NA, NT, RM, BM>
      <<<dim3(((M + BM - 1) / BM) * (N / RS_BN) * splits), dim3(RS_THREADS), smem, stream>>>(
          C, A, Wp, slabs, tickets, M, N, K, lda, ldw, ldc, splits, rot_mul);
  return (int)hipGetLastError();
}

// cfg: bits 0-1 ring shape (0: D 6 / NA 4, 2: D 4 / NA 3), bit 2 128-row
// tiles, bit 3 64-row tiles (else all 256 rows), bit 5 non-temporal weight
// loads, bit 6 row-major
// weights (W [N][ldw] as stored; else W is rsgemm_pack's layout).  The K
// slice must be a multiple of U = D / 2 K64 steps.
int rsgemm(void* C, const void* A, const void* W, float* slabs, unsigned* tickets,
           int n_tickets, int M, int N, int K, long lda, long ldw, long ldc, int cfg, int splits,
           int epi, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 256 || N % RS_BN != 0 || splits < 1 || K % (splits * RS_BK) != 0) return -1;
  if ((cfg >> 4) & 1) {
    // K14W (bit 4): packed weights, non-temporal (bit 5), 128- or 64-row
    // tiles, ring D 8; split-K only with the partials epilogue.  Measured
    // against K14 and not used by the dispatch table (profiles/r6_decode_gemm.md).
    // All 256 rows do not fit: 256 accumulator rows x 64 columns per wave
    // spill even with a 4-step ring.
    const int shape = cfg & 3, bm64 = (cfg >> 3) & 1, nt = (cfg >> 5) & 1;
    if ((cfg >> 6) & 1 || !((cfg >> 2) & 1 || bm64) || shape != 0 || !nt) return -1;
    if (epi != 0 && epi != 2 && epi != 3) return -1;
    if (splits > 1 && epi != 2) return -1;
    if (epi == 2 && slabs == nullptr) return -2;
    const int U = 4;
    const int nk64 = (K / splits) / RS_BK;
    if (nk64 < 2 * U || nk64 % U != 0) return -1;
    auto C_ = (bf16_t*)C;
    auto A_ = (const bf16_t*)A;
    auto W_ = (const bf16_t*)W;
#define LMX_RS4_E(BM)                                                                           \
  if (epi == 3) return rs4_launch<3, 8, 5, 1, BM>(C_, A_, W_, slabs, M, N, K, lda, ldc, splits,   \
                                                  stream);                                       \
  if (epi == 2) return rs4_launch<2, 8, 5, 1, BM>(C_, A_, W_, slabs, M, N, K, lda, ldc, splits,   \
                                                  stream);                                       \
  return rs4_launch<0, 8, 5, 1, BM>(C_, A_, W_, slabs, M, N, K, lda, ldc, splits, stream);
    if (bm64) { LMX_RS4_E(64) }
    LMX_RS4_E(128)
#undef LMX_RS4_E
  }
  const int shape = cfg & 3, bm128 = (cfg >> 2) & 1, bm64 = (cfg >> 3) & 1;
  const int nt = (cfg >> 5) & 1, rm = (cfg >> 6) & 1;
  const int rot = (cfg >> 7) & 1 ? 5 : 0;     // bit 7: K order rotated per column tile
  const int bm = bm64 ? 64 : bm128 ? 128 : 256;
  // shape 1 (D 8 / NA 5) needs 256+ VGPRs: the compiler spills, and a spill
  // of an inline-asm load destination before its data lands is silent
  // corruption (cdna guide §5.7 item 1) -- not built
  if (shape == 3 || shape == 1) return -1;
  if (splits > 1 && epi != 2 && splits != 2 && splits != 4 && splits != 8 && splits != 16)
    return -1;
  const int U = shape == 2 ? 2 : 3;
  const int nk64 = (K / splits) / RS_BK;
  if (nk64 < U || nk64 % U != 0) return -1;
  if (epi != 0 && epi != 2 && epi != 3) return -1;
  if (rm && (ldw < K || ldw % 8 != 0 || 32L * ldw * 2 > (1L << 31))) return -1;
  if ((splits > 1 || epi == 2) && slabs == nullptr) return -2;
  const int tiles = ((M + bm - 1) / bm) * (N / RS_BN);
  if (splits > 1 && epi != 2 && (tickets == nullptr || tiles > n_tickets)) return -3;
  auto C_ = (bf16_t*)C;
  auto A_ = (const bf16_t*)A;
  auto W_ = (const bf16_t*)W;
#define LMX_RS_E(D, NA, NT, RM, BM)                                                             \
  if (epi == 3) return rs_launch<3, D, NA, NT, RM, BM>(C_, A_, W_, slabs, tickets, M, N, K, lda, \
                                                       ldw, ldc, splits, rot, stream);               \
  if (epi == 2) return rs_launch<2, D, NA, NT, RM, BM>(C_, A_, W_, slabs, tickets, M, N, K, lda, \
                                                       ldw, ldc, splits, rot, stream);               \
  return rs_launch<0, D, NA, NT, RM, BM>(C_, A_, W_, slabs, tickets, M, N, K, lda, ldw, ldc,     \
                                         splits, rot, stream);
  // all-rows tiles (BM 256) are built for the partials epilogue only: the
  // bf16 and SwiGLU epilogues spill there (a spilled ring register is silent
  // corruption; build.py audits every instantiation) and no table entry uses them
#define LMX_RS_B(D, NA, NT, RM)                 \
  if (bm == 64) { LMX_RS_E(D, NA, NT, RM, 64) } \
  if (bm == 128) { LMX_RS_E(D, NA, NT, RM, 128) } \
  if (epi != 2) return -1;                      \
  return rs_launch<2, D, NA, NT, RM, 256>(C_, A_, W_, slabs, tickets, M, N, K, lda, ldw, ldc, \
                                          splits, rot, stream);
#define LMX_RS(D, NA)                                  \
  if (nt && rm) { LMX_RS_B(D, NA, 1, 1) }              \
  if (nt) { LMX_RS_B(D, NA, 1, 0) }                    \
  if (rm) { LMX_RS_B(D, NA, 0, 1) }                    \
  LMX_RS_B(D, NA, 0, 0)
  switch (shape) {
    case 2: { LMX_RS(4, 3) }
    default: { LMX_RS(6, 4) }
  }
#undef LMX_RS
#undef LMX_RS_B
#undef LMX_RS_E
}

}  // namespace lmx
