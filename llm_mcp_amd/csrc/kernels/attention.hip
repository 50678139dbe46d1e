// K3 + K4: paged attention for gfx950 on 16x16x32 bf16 MFMA.
//
// One building block serves both phases.  A wave owns 16 "columns"; a column
// is one (query token, query head) pair of a single sequence / kv head.  For a
// 32-token KV page it computes
//     S^T[16 keys x 16 cols] = K[keys x 128] . Q^T[128 x cols]    (2 tiles)
//     O^T[128 x 16 cols]    += V^T[128 x 32 keys] . P^T[32 keys x cols]
// with the *column on the MFMA lane* (C/D map col = lane&15), so the online
// softmax statistics of a column live in the same lanes as that column's
// output accumulator: the rescale needs no cross-lane traffic, and the P
// accumulator feeds the PV MFMA as its B operand with no LDS round trip (the
// k index of the PV product is permuted so that B element j of lane group g is
// key 4g+j (j<4) or 16+4g+j-4 (j>=4), exactly where S^T left it; the V^T
// operand is read with the same permutation as two 8-byte loads from the
// key-quad V page [BS/4][D][4], see rope_cache.hip for the cache layout).
//
//   decode  (K4): columns = the G query heads of one token (G = Hq/Hkv <= 16);
//                 the 4 waves split the page range, combined through LDS, and
//                 long contexts are split over workgroups (split-K) with a
//                 separate reduce kernel.
//   prefill (K3): columns = (16/G queries) x (G heads): the K/V page read is
//                 shared by all heads of the kv group; each wave walks its own
//                 causal key range; varlen batches via a host-built tile list.
#include <algorithm>
#include <climits>
#include <type_traits>
#include <utility>

#include "common.h"

namespace lmx {

constexpr int BS = 32;   // KV page (block) size in tokens
constexpr float LOG2E = 1.4426950408889634f;

// max / sum over the 4 lanes c, c+16, c+32, c+48 (one MFMA column's 4 row
// groups) with v_permlane16_swap / v_permlane32_swap: VALU lane exchanges
// instead of two ds_bpermute round trips through the LDS unit on the softmax's
// serial chain.  permlane16_swap(x, x) yields {rows 0,0,2,2 ; rows 1,1,3,3} of
// x (16-lane rows), so op(first, second) is the xor-16 reduction; the 32-lane
// form does the same across halves.
// v_max_f32 as one instruction (fmaxf on values hipcc cannot prove canonical
// -- MFMA results, lane swaps -- gets a canonicalising v_max per operand)
__device__ __forceinline__ float max2f(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// v_max3_f32 as one instruction (the same canonicalisation otherwise doubles
// the row-max VALU of the softmax)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ float col4_max(float x) {
  const unsigned u = __float_as_uint(x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = max2f(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const unsigned v = __float_as_uint(x);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return max2f(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float col4_sum(float x) {
  const unsigned u = __float_as_uint(x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const unsigned v = __float_as_uint(x);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <int HD>
struct PageState {
  float m;                // running max (log2 domain) of this lane's column
  float l;                // running denominator
  f32x4_t acc[HD / 16];   // O^T: row d = 16i + 4g + r, col = lane&15
};

template <int HD>
__device__ __forceinline__ void state_init(PageState<HD>& st) {
  st.m = -INFINITY;
  st.l = 0.f;
#pragma unroll
  for (int i = 0; i < HD / 16; ++i) st.acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
}

// Process one KV page for the 16 columns of this wave.
//  key_lo/key_hi: absolute key positions of this page; a key is visible to the
//  lane's column iff key_pos <= lim (lim = causal limit of the column, already
//  clipped to ctx-1).
// K/V page loads; NTL: non-temporal (the decode step reads each page once per
// layer, with the whole model streamed between two reads of it)
template <bool NTL>
__device__ __forceinline__ bf16x8_t kv_frag16B(const bf16_t* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(p));
  else return load_frag16B(p);
}

template <bool NTL>
__device__ __forceinline__ bf16x8_t kv_frag_2x8B(const bf16_t* p0, const bf16_t* p1) {
  if constexpr (NTL) {
    const bf16x4_t a = __builtin_nontemporal_load(reinterpret_cast<const bf16x4_t*>(p0));
    const bf16x4_t b = __builtin_nontemporal_load(reinterpret_cast<const bf16x4_t*>(p1));
    return bf16x8_t{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  } else {
    return load_frag_2x8B(p0, p1);
  }
}

template <int HD, bool NTL = false>
__device__ __forceinline__ void process_page(PageState<HD>& st, const bf16x8_t (&qf)[HD / 32],
                                             const bf16_t* __restrict__ kpage,
                                             const bf16_t* __restrict__ vpage, int page_pos0,
                                             int lim, float scale_log2) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  f32x4_t s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  constexpr int KS = HD / 32, NT = HD / 16;
  bf16x8_t ka[KS], kb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    ka[s] = kv_frag16B<NTL>(kpage + c * HD + 32 * s + 8 * g);
    kb[s] = kv_frag16B<NTL>(kpage + (16 + c) * HD + 32 * s + 8 * g);
  }
  // V^T fragments (issued early so they overlap the QK MFMAs and softmax)
  bf16x8_t vf[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
    vf[i] = kv_frag_2x8B<NTL>(vpage + vq_off(16 * i + c, 4 * g, HD),
                              vpage + vq_off(16 * i + c, 16 + 4 * g, HD));
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    s0 = mfma16(ka[s], qf[s], s0);
    s1 = mfma16(kb[s], qf[s], s1);
  }
  float x[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k0 = page_pos0 + 4 * g + r, k1 = k0 + 16;
    x[r] = (k0 <= lim) ? s0[r] * scale_log2 : -INFINITY;
    x[4 + r] = (k1 <= lim) ? s1[r] * scale_log2 : -INFINITY;
  }
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) mx = fmaxf(mx, x[j]);
  mx = col4_max(mx);        // VALU lane swaps: no LDS traffic in the page loop
  const float m_new = fmaxf(st.m, mx);
  // a column may see no visible key in this page (causal tail): keep its state
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  const float alpha = fast_exp2(st.m - m_use);
  float p[8], rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { p[j] = fast_exp2(x[j] - m_use); rs += p[j]; }
  rs = col4_sum(rs);
  st.l = st.l * alpha + rs;
  st.m = m_new;
  bf16x8_t pf;
#pragma unroll
  for (int j = 0; j < 8; ++j) pf[j] = (short)f2bf(p[j]);
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    st.acc[i] *= alpha;
    st.acc[i] = mfma16(vf[i], pf, st.acc[i]);
  }
}

// Split form of process_page for the pipelined decode loop: the page's K and
// V^T fragments are loaded into registers one page ahead of their use.
template <int HD>
struct PageFrags {
  bf16x8_t ka[HD / 32], kb[HD / 32], vf[HD / 16];
};

template <int HD>
__device__ __forceinline__ void load_page(PageFrags<HD>& f, const bf16_t* __restrict__ kpage,
                                          const bf16_t* __restrict__ vpage) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < HD / 32; ++s) {
    f.ka[s] = load_frag16B(kpage + c * HD + 32 * s + 8 * g);
    f.kb[s] = load_frag16B(kpage + (16 + c) * HD + 32 * s + 8 * g);
  }
#pragma unroll
  for (int i = 0; i < HD / 16; ++i)
    f.vf[i] = load_frag_2x8B(vpage + vq_off(16 * i + c, 4 * g, HD),
                             vpage + vq_off(16 * i + c, 16 + 4 * g, HD));
}

template <int HD>
__device__ __forceinline__ void compute_page(PageState<HD>& st, const bf16x8_t (&qf)[HD / 32],
                                             const PageFrags<HD>& f, int page_pos0, int lim,
                                             float scale_log2);

// ---- rolling register ring with hand-counted waits (decode MODE 9) --------
// A page's K and V^T fragments are issued as inline-asm loads from a
// wave-uniform SGPR page base + the lane's offset + an immediate, so hipcc
// neither counts them nor drains them with its own vmcnt(0) at the loop top
// (why the compiler-scheduled pipelines, modes 1 and 7, never kept the next
// page in flight: profiles/r4_decode_attention_pmc.md).  Rolling ring, one
// page of registers: the next page's K loads issue as soon as this page's QK
// MFMAs have read K, its V loads as soon as PV has read V, so every wave keeps
// 8-16 KB in flight through the whole loop.  Waits are counted in issue order
// (K(j) is followed by V(j): vmcnt(VOPS); V(j) by K(j + 1): vmcnt(KOPS)), the
// discipline of K14's weight ring (rsgemm.hip).
template <int HD>
struct RingK { bf16x8_t a[HD / 32], b[HD / 32]; };   // key rows c / 16 + c
template <int HD>
struct RingV { bf16x4_t lo[HD / 16], hi[HD / 16]; }; // V^T keys 4g.. / 16 + 4g..
template <int HD>
constexpr int ring_kops() { return 2 * (HD / 32); }
template <int HD>
constexpr int ring_vops() { return 2 * (HD / 16); }

template <int IMM>
__device__ __forceinline__ void ring_ld16(bf16x8_t& r, const void* sbase, unsigned voff) {
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3"
               : "=v"(r) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}
template <int IMM>
__device__ __forceinline__ void ring_ld8(bf16x4_t& r, const void* sbase, unsigned voff) {
  asm volatile("global_load_dwordx2 %0, %1, %2 offset:%3"
               : "=v"(r) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}

// lane offsets (bytes) inside a K page [BS][HD] and a key-quad V page
// [BS/4][HD][4]: K rows c and 16 + c (+ 64 s by immediate); V^T lo = keys
// 4g.., hi = keys 16 + 4g.. of d = 16 i + c (+ 128 i by immediate)
struct RingOffs { unsigned ka, kb, vlo, vhi; };
template <int HD>
__device__ __forceinline__ RingOffs ring_offs() {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  RingOffs o;
  o.ka = (unsigned)(c * HD * 2 + 16 * g);
  o.kb = o.ka + 16 * HD * 2;
  o.vlo = (unsigned)(g * HD * 8 + 8 * c);
  o.vhi = o.vlo + 4 * HD * 8;
  return o;
}

template <int HD, int... I>
__device__ __forceinline__ void ring_issue_k(RingK<HD>& f, const void* kp, const RingOffs& o,
                                             std::integer_sequence<int, I...>) {
  (ring_ld16<64 * I>(f.a[I], kp, o.ka), ...);
  (ring_ld16<64 * I>(f.b[I], kp, o.kb), ...);
}
template <int HD, int... I>
__device__ __forceinline__ void ring_issue_v(RingV<HD>& f, const void* vp, const RingOffs& o,
                                             std::integer_sequence<int, I...>) {
  (ring_ld8<128 * I>(f.lo[I], vp, o.vlo), ...);
  (ring_ld8<128 * I>(f.hi[I], vp, o.vhi), ...);
}

// wait until at most CNT vector-memory ops are outstanding; the fragments are
// in/out operands so nothing reads them before the wait
template <int CNT, int HD>
__device__ __forceinline__ void ring_wait_k(RingK<HD>& f) {
  if constexpr (HD == 128)
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.a[2]), "+v"(f.a[3]), "+v"(f.b[0]),
                   "+v"(f.b[1]), "+v"(f.b[2]), "+v"(f.b[3])
                 : "n"(CNT) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%4)"
                 : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.b[0]), "+v"(f.b[1]) : "n"(CNT) : "memory");
}
template <int CNT, int HD>
__device__ __forceinline__ void ring_wait_v(RingV<HD>& f) {
  if constexpr (HD == 128)
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(f.lo[0]), "+v"(f.lo[1]), "+v"(f.lo[2]), "+v"(f.lo[3]), "+v"(f.lo[4]),
                   "+v"(f.lo[5]), "+v"(f.lo[6]), "+v"(f.lo[7]), "+v"(f.hi[0]), "+v"(f.hi[1]),
                   "+v"(f.hi[2]), "+v"(f.hi[3]), "+v"(f.hi[4]), "+v"(f.hi[5]), "+v"(f.hi[6]),
                   "+v"(f.hi[7])
                 : "n"(CNT) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(f.lo[0]), "+v"(f.lo[1]), "+v"(f.lo[2]), "+v"(f.lo[3]), "+v"(f.hi[0]),
                   "+v"(f.hi[1]), "+v"(f.hi[2]), "+v"(f.hi[3])
                 : "n"(CNT) : "memory");
}

template <int CNT>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// the ring refill overwrites registers MFMAs just read; hipcc pads no hazard
// for an asm instruction (rsgemm.hip rs_mfma_war_pad)
__device__ __forceinline__ void ring_war_pad() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
}

__device__ __forceinline__ f32x4_t mfma16k16(bf16x4_t a, bf16x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// S^T of one page from the K slot
template <int HD>
__device__ __forceinline__ void ring_qk(const RingK<HD>& k, const bf16x8_t (&qf)[HD / 32],
                                        f32x4_t& s0, f32x4_t& s1) {
  s0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s1 = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < HD / 32; ++s) {
    s0 = mfma16(k.a[s], qf[s], s0);
    s1 = mfma16(k.b[s], qf[s], s1);
  }
}

// masked, scaled scores of one page.  The empty asm pins their computation
// (VALU reads of the QK MFMA results, which wait for the MFMAs to finish)
// before the K slot refill that follows in program order.
template <int HD>
__device__ __forceinline__ void ring_scores(f32x4_t s0, f32x4_t s1, int page_pos0, int lim,
                                            float scale_log2, float (&x)[8]) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int k0 = page_pos0 + 4 * g + k, k1 = k0 + 16;
    x[k] = (k0 <= lim) ? s0[k] * scale_log2 : -INFINITY;
    x[4 + k] = (k1 <= lim) ? s1[k] * scale_log2 : -INFINITY;
  }
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                    "+v"(x[6]), "+v"(x[7]));
}

// online softmax + PV from the V slot.  The V^T halves stay in their own
// 2-VGPR load destinations (a 4-VGPR reassembly would be copies of registers
// whose data may not have landed), so PV runs as two 16x16x16 MFMAs per 16-row
// d block: keys 4g.. against P's first four values, 16 + 4g.. the last four.
template <int HD>
__device__ __forceinline__ void ring_pv(PageState<HD>& st, const RingV<HD>& v,
                                        const float (&x)[8]) {
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) mx = fmaxf(mx, x[j]);
  mx = col4_max(mx);
  const float m_new = fmaxf(st.m, mx);
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  const float alpha = fast_exp2(st.m - m_use);
  float p[8], rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { p[j] = fast_exp2(x[j] - m_use); rs += p[j]; }
  rs = col4_sum(rs);
  st.l = st.l * alpha + rs;
  st.m = m_new;
  bf16x4_t plo, phi;
#pragma unroll
  for (int j = 0; j < 4; ++j) { plo[j] = (short)f2bf(p[j]); phi[j] = (short)f2bf(p[4 + j]); }
#pragma unroll
  for (int i = 0; i < HD / 16; ++i) {
    st.acc[i] *= alpha;
    st.acc[i] = mfma16k16(v.lo[i], plo, st.acc[i]);
    st.acc[i] = mfma16k16(v.hi[i], phi, st.acc[i]);
  }
}

template <int HD>
__device__ __forceinline__ void compute_page(PageState<HD>& st, const bf16x8_t (&qf)[HD / 32],
                                             const PageFrags<HD>& f, int page_pos0, int lim,
                                             float scale_log2) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  f32x4_t s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < HD / 32; ++s) {
    s0 = mfma16(f.ka[s], qf[s], s0);
    s1 = mfma16(f.kb[s], qf[s], s1);
  }
  float x[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k0 = page_pos0 + 4 * g + r, k1 = k0 + 16;
    x[r] = (k0 <= lim) ? s0[r] * scale_log2 : -INFINITY;
    x[4 + r] = (k1 <= lim) ? s1[r] * scale_log2 : -INFINITY;
  }
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) mx = fmaxf(mx, x[j]);
  mx = col4_max(mx);        // VALU lane swaps: no LDS traffic in the page loop
  const float m_new = fmaxf(st.m, mx);
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  const float alpha = fast_exp2(st.m - m_use);
  float p[8], rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { p[j] = fast_exp2(x[j] - m_use); rs += p[j]; }
  rs = col4_sum(rs);
  st.l = st.l * alpha + rs;
  st.m = m_new;
  bf16x8_t pf;
#pragma unroll
  for (int j = 0; j < 8; ++j) pf[j] = (short)f2bf(p[j]);
#pragma unroll
  for (int i = 0; i < HD / 16; ++i) {
    st.acc[i] *= alpha;
    st.acc[i] = mfma16(f.vf[i], pf, st.acc[i]);
  }
}

// ---------------------------------------------------------------- decode ----
// Optional fused K2 + K5 for decode rows (cos_sin == nullptr: off).  The row's
// q / k / v are the unrotated QKV projection output (q at the row start, k at
// Hq*HD, v at (Hq+Hkv)*HD); positions[b] is the token's rotary position,
// slots[b] its cache slot (-1: padding row, nothing written).
struct RopeIn {
  const int* positions;
  const float* cos_sin;   // [max_pos][HD]: cos | sin (rope_cache.hip)
  const int* slots;
};

// q fragments of one lane (column c = head, 8 elements per s-block at
// 32s + 8g) rotated in registers: element e < HD/2 pairs with e + HD/2, which
// sits in block s + KS/2 of the same lane.  Same fp32 expression and bf16
// rounding as rope_cache_kernel.
template <int HD>
__device__ __forceinline__ void rope_q_frags(bf16x8_t (&qf)[HD / 32], const float* __restrict__ cs,
                                             int g) {
  constexpr int KS = HD / 32, half = HD / 2;
#pragma unroll
  for (int s = 0; s < KS / 2; ++s) {
    const int e = 32 * s + 8 * g;
    const float4 c0 = *reinterpret_cast<const float4*>(cs + e);
    const float4 c1 = *reinterpret_cast<const float4*>(cs + e + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(cs + half + e);
    const float4 s1 = *reinterpret_cast<const float4*>(cs + half + e + 4);
    const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = bf2f((uint16_t)qf[s][j]), b = bf2f((uint16_t)qf[s + KS / 2][j]);
      qf[s][j] = (short)f2bf(a * cc[j] - b * ss[j]);
      qf[s + KS / 2][j] = (short)f2bf(b * cc[j] + a * ss[j]);
    }
  }
}

// The new token's k (rotated) and v of kv head kvh into its cache slot, by ONE
// wave: lanes [0, HD/8) rotate 4 pairs of k each, lanes [16, 16 + HD/4) move
// 4 v elements each into the key-quad page.  No wait here: the caller (the
// wave that later reads the page holding the slot) retires the stores with
// s_waitcnt vmcnt(0) before that read, so the other waves never wait on it.
template <int HD>
__device__ __forceinline__ void rope_write_kv(const bf16_t* __restrict__ krow,
                                              const bf16_t* __restrict__ vrow,
                                              const float* __restrict__ cs, int slot, int kvh,
                                              int Hkv, bf16_t* __restrict__ k_cache,
                                              bf16_t* __restrict__ v_cache) {
  constexpr int half = HD / 2;
  const int lane = threadIdx.x & 63;
  if (slot < 0) return;
  const long blk = slot / BS, off = slot % BS;
  if (lane < HD / 8) {
    const int i = 4 * lane;
    const bf16x4_t x1 = *reinterpret_cast<const bf16x4_t*>(krow + i);
    const bf16x4_t x2 = *reinterpret_cast<const bf16x4_t*>(krow + half + i);
    const float4 c = *reinterpret_cast<const float4*>(cs + i);
    const float4 sn = *reinterpret_cast<const float4*>(cs + half + i);
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
    bf16x4_t o1, o2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = bf2f((uint16_t)x1[j]), b = bf2f((uint16_t)x2[j]);
      o1[j] = (short)f2bf(a * cc[j] - b * ss[j]);
      o2[j] = (short)f2bf(b * cc[j] + a * ss[j]);
    }
    bf16_t* kp = k_cache + ((blk * Hkv + kvh) * BS + off) * HD;
    *reinterpret_cast<bf16x4_t*>(kp + i) = o1;
    *reinterpret_cast<bf16x4_t*>(kp + half + i) = o2;
  } else if (lane >= 16 && lane < 16 + HD / 4) {
    const int d = 4 * (lane - 16);
    const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(vrow + d);
    bf16_t* vp = v_cache + (blk * Hkv + kvh) * (BS * HD) + vq_off(d, off, HD);
#pragma unroll
    for (int j = 0; j < 4; ++j) vp[4 * j] = (bf16_t)v[j];
  }
}

// Partition length used for a sequence: the requested split-K granule, grown
// (in 128-token steps) when the context would need more than max_parts
// partitions, so the grid baked into a captured graph always covers it.
__device__ __forceinline__ int effective_part(int ctx, int part_tokens, int max_parts) {
  int need = (ctx + max_parts - 1) / max_parts;
  need = (need + 127) & ~127;
  return need > part_tokens ? need : part_tokens;
}

// One (partition, kv head, sequence) segment of the decode attention, by one
// 256-thread workgroup.
// MODE 0: one page at a time (load, then compute); MODE 1: the next page's
// block id and K/V fragments are loaded before the current page is computed
// (two pages in flight per wave); MODE 2: loads only (diagnostic ceiling);
// MODE 3: loads only, every instruction one contiguous 1 KB (diagnostic);
// MODE 5: MODE 0 with non-temporal K/V loads; MODE 6: MODE 0 with a
// block-table load per page.  MODE 0 / 5 read the segment's block ids once
// into a VGPR (lane i: page pg0 + i) and take them by readlane, so a page's
// K/V loads do not wait on its block-table load.
template <int HD>
struct DecodeSmem {
  float ml[4][16][2];
  float o[4][16][HD + 4];
};

template <int HD, int MODE>
__device__ __forceinline__ void decode_segment(
    DecodeSmem<HD>& sm, int p, int kvh, int b, const bf16_t* __restrict__ q, long q_stride,
    const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ context_lens,
    bf16_t* __restrict__ out, long out_stride, float* __restrict__ part_o,
    float* __restrict__ part_ml, int Hq, int Hkv, float scale, int part_tokens, int max_parts,
    const RopeIn rp) {
  float (&sm_ml)[4][16][2] = sm.ml;
  float (&sm_o)[4][16][HD + 4] = sm.o;
  const int ctx = context_lens[b];
  part_tokens = effective_part(ctx, part_tokens, max_parts);
  const int nparts = (ctx + part_tokens - 1) / part_tokens;
  if (p >= nparts) return;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // wave-uniform in the compiler's view too: page indices, block ids and the
  // page-loop control stay scalar (s_load / s_cbranch, no exec masking)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t0 = p * part_tokens, t1 = min(t0 + part_tokens, ctx);
  constexpr bool kOnePage = MODE == 0 || MODE == 5 || MODE == 6;
  constexpr bool kRing = MODE == 9;

  bf16x8_t qf[HD / 32];
  const bf16_t* qrow = q + (long)b * q_stride + (long)(kvh * G + c) * HD;
#pragma unroll
  for (int s = 0; s < HD / 32; ++s)
    qf[s] = (c < G) ? load_frag16B(qrow + 32 * s + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  const int pg0 = t0 / BS, pg1 = (t1 + BS - 1) / BS;
  // fused rotary + cache write of this step's token: every wave rotates its q
  // fragments; the wave that will read the last page (the one holding
  // position ctx-1, in the last partition) writes the new k / v first and
  // retires those stores just before it loads that page
  bool writer = false;
  const float* cs = nullptr;
  if (rp.cos_sin) {
    cs = rp.cos_sin + (long)rp.positions[b] * HD;
    // the one-page-at-a-time loops rotate q under their first page's loads
    if constexpr (!kOnePage) rope_q_frags<HD>(qf, cs, g);
    writer = p == nparts - 1 && wave == (pg1 - 1 - pg0) % 4;
    if (writer) {
      const bf16_t* krow = q + (long)b * q_stride + (long)(Hq + kvh) * HD;
      rope_write_kv<HD>(krow, krow + (long)Hkv * HD, cs, rp.slots[b], kvh, Hkv,
                        const_cast<bf16_t*>(k_cache), const_cast<bf16_t*>(v_cache));
      // the ring retires the stores by count just before it issues the page
      // that holds the slot
      if constexpr (!kOnePage && !kRing) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }

  PageState<HD> st;
  state_init(st);
  const float scale_log2 = scale * LOG2E;
  const int* bt = block_tables + (long)b * bt_stride;
  if constexpr (kRing) {
    // pages of this wave: j-th = pg0 + wave + 4 j.  Block ids by readlane from
    // one VGPR holding the wave's ids (lane j: its j-th page, 8192 tokens of
    // context); its compiler-counted load is consumed before the first ring
    // load issues (a later one would make hipcc drain the ring)
    const int wpg = pg0 + wave + 4 * lane;
    const int btv = wpg < pg1 ? bt[wpg] : 0;
    auto blk_of = [&](int j) -> long {
      if (j < 64) return __builtin_amdgcn_readlane(btv, j);
      return bt[pg0 + wave + 4 * j];
    };
    const int npg = pg1 - pg0;
    const int nw = npg > wave ? (npg - wave + 3) / 4 : 0;
    const RingOffs ro = ring_offs<HD>();
    auto page_k = [&](int j) -> const void* {
      return k_cache + (blk_of(j) * Hkv + kvh) * (BS * HD);
    };
    auto page_v = [&](int j) -> const void* {
      return v_cache + (blk_of(j) * Hkv + kvh) * (BS * HD);
    };
    constexpr int KOPS = ring_kops<HD>(), VOPS = ring_vops<HD>();
    // Every compiler-counted load used below is consumed before the first
    // ring load issues (hipcc would wait for it with vmcnt(0) inside the loop).
#pragma unroll
    for (int s = 0; s < HD / 32; ++s) asm volatile("" : "+v"(qf[s]));
    const int lim = t1 - 1;
    auto pos_of = [&](int j) { return (pg0 + wave + 4 * j) * BS; };
    // The writer's last page (j = nw - 1) holds the slot: before its K loads
    // issue, every op but the V loads of the page before it retires (the
    // stores are older than every ring load).
    RingK<HD> rk;
    RingV<HD> rv;
    f32x4_t s0, s1;
    float x[8];
    if (nw > 0) {
      if (writer && nw == 1) vm_wait<0>();
      ring_issue_k<HD>(rk, page_k(0), ro, std::make_integer_sequence<int, HD / 32>{});
      ring_issue_v<HD>(rv, page_v(0), ro, std::make_integer_sequence<int, HD / 16>{});
    }
    // steady state: one exit, the same waits every iteration (no branch merges
    // two asm-defined copies of a slot; hipcc would place that phi's copies
    // before the wait)
    int j = 0;
    for (; j + 1 < nw; ++j) {
      ring_wait_k<VOPS>(rk);
      ring_qk<HD>(rk, qf, s0, s1);
      ring_scores<HD>(s0, s1, pos_of(j), lim, scale_log2, x);
      ring_war_pad();
      if (writer && j + 1 == nw - 1) vm_wait<VOPS>();
      ring_issue_k<HD>(rk, page_k(j + 1), ro, std::make_integer_sequence<int, HD / 32>{});
      ring_wait_v<KOPS>(rv);
      ring_pv<HD>(st, rv, x);
      ring_war_pad();
      ring_issue_v<HD>(rv, page_v(j + 1), ro, std::make_integer_sequence<int, HD / 16>{});
    }
    if (nw > 0) {
      ring_wait_k<VOPS>(rk);
      ring_qk<HD>(rk, qf, s0, s1);
      ring_scores<HD>(s0, s1, pos_of(j), lim, scale_log2, x);
      ring_wait_v<0>(rv);
      ring_pv<HD>(st, rv, x);
    }
  } else if constexpr (kOnePage) {
    int btv = 0;
    if constexpr (MODE != 6) btv = pg0 + lane < pg1 ? bt[pg0 + lane] : 0;
    auto blk_of = [&](int pg) -> long {
      if constexpr (MODE != 6) {
        if (pg - pg0 < 64) return __builtin_amdgcn_readlane(btv, pg - pg0);
      }
      return bt[pg];
    };
    int pg = pg0 + wave;
    if (cs) {
      if (pg < pg1 && !(writer && pg == pg1 - 1)) {
        // first page: its K/V fragments are in flight while q rotates (the
        // rotation's cos/sin round trip no longer serialises the segment)
        const long blk = blk_of(pg);
        PageFrags<HD> f;
        load_page(f, k_cache + (blk * Hkv + kvh) * (BS * HD),
                  v_cache + (blk * Hkv + kvh) * (BS * HD));
        rope_q_frags<HD>(qf, cs, g);
        compute_page(st, qf, f, pg * BS, t1 - 1, scale_log2);
        pg += 4;
      } else {
        rope_q_frags<HD>(qf, cs, g);
      }
    }
    for (; pg < pg1; pg += 4) {
      if (writer && pg == pg1 - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long blk = blk_of(pg);
      const bf16_t* kp = k_cache + (blk * Hkv + kvh) * (BS * HD);
      const bf16_t* vp = v_cache + (blk * Hkv + kvh) * (BS * HD);
      process_page<HD, MODE == 5>(st, qf, kp, vp, pg * BS, t1 - 1, scale_log2);
    }
  } else {
    int pg = pg0 + wave;
    PageFrags<HD> cur;
    if (pg < pg1) {
      const long blk = bt[pg];
      load_page(cur, k_cache + (blk * Hkv + kvh) * (BS * HD),
                v_cache + (blk * Hkv + kvh) * (BS * HD));
    }
    for (; pg < pg1; pg += 4) {
      PageFrags<HD> nxt;
      const bool more = pg + 4 < pg1;
      if (more) {
        const long blk = bt[pg + 4];
        load_page(nxt, k_cache + (blk * Hkv + kvh) * (BS * HD),
                  v_cache + (blk * Hkv + kvh) * (BS * HD));
      }
      if constexpr (MODE == 1) {
        compute_page(st, qf, cur, pg * BS, t1 - 1, scale_log2);
      } else if constexpr (MODE == 3) {
        // probe: the same bytes as whole 1-KB contiguous pieces per instruction
        const long blk = bt[pg];
        const bf16_t* kp = k_cache + (blk * Hkv + kvh) * (BS * HD);
        const bf16_t* vp = v_cache + (blk * Hkv + kvh) * (BS * HD);
#pragma unroll
        for (int s2 = 0; s2 < HD / 32; ++s2) {
          cur.ka[s2] = load_frag16B(kp + (2 * s2) * 512 + lane * 8);
          cur.kb[s2] = load_frag16B(kp + (2 * s2 + 1) * 512 + lane * 8);
        }
#pragma unroll
        for (int i = 0; i < HD / 16; ++i) cur.vf[i] = load_frag16B(vp + i * 512 + lane * 8);
#pragma unroll
        for (int s2 = 0; s2 < HD / 32; ++s2) asm volatile("" ::"v"(cur.ka[s2]), "v"(cur.kb[s2]));
#pragma unroll
        for (int i = 0; i < HD / 16; ++i) asm volatile("" ::"v"(cur.vf[i]));
      } else {
#pragma unroll
        for (int s2 = 0; s2 < HD / 32; ++s2) asm volatile("" ::"v"(cur.ka[s2]), "v"(cur.kb[s2]));
#pragma unroll
        for (int i = 0; i < HD / 16; ++i) asm volatile("" ::"v"(cur.vf[i]));
      }
      if (more) cur = nxt;
    }
  }
  // combine the 4 waves
  if (g == 0) { sm_ml[wave][c][0] = st.m; sm_ml[wave][c][1] = st.l; }
#pragma unroll
  for (int i = 0; i < HD / 16; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm_o[wave][c][16 * i + 4 * g + r] = st.acc[i][r];
  __syncthreads();
  for (int e = threadIdx.x; e < G * HD; e += blockDim.x) {
    const int h = e / HD, d = e % HD;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm_ml[w][h][0]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float mw = sm_ml[w][h][0];
      const float f = (mw == -INFINITY) ? 0.f : fast_exp2(mw - M);
      L += sm_ml[w][h][1] * f;
      O += sm_o[w][h][d] * f;
    }
    const int head = kvh * G + h;
    if (nparts == 1) {
      out[(long)b * out_stride + (long)head * HD + d] = f2bf(O / L);
    } else {
      const long idx = ((long)b * Hq + head) * max_parts + p;
      part_o[idx * HD + d] = O;
      if (d == 0) { part_ml[idx * 2] = M; part_ml[idx * 2 + 1] = L; }
    }
  }
}


// grid (max_parts, Hkv, B), block 256: one workgroup per segment.  order
// (optional): sequence of each grid z-slice, longest context first, so the
// workgroups dispatched last are the short ones (profiles/r2_decode_attention.md)
template <int HD, int MODE>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    const bf16_t* __restrict__ q, long q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, const int* __restrict__ order,
    bf16_t* __restrict__ out, long out_stride,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, int Hkv, float scale,
    int part_tokens, int max_parts, RopeIn rp) {
  __shared__ DecodeSmem<HD> sm;
  decode_segment<HD, MODE>(sm, blockIdx.x, blockIdx.y, order ? order[blockIdx.z] : blockIdx.z, q,
                           q_stride, k_cache, v_cache, block_tables, bt_stride, context_lens,
                           out, out_stride, part_o, part_ml, Hq, Hkv, scale, part_tokens,
                           max_parts, rp);
}

// Persistent form (one partition per sequence): a fixed grid of about the
// resident workgroup count walks the (sequence, kv head) segments in
// longest-first order with a grid stride, so no workgroup launches ragged
// rounds behind the first and the per-workgroup start-up is paid once per
// resident slot.
template <int HD, int MODE, int OCC = 3>
__global__ void __launch_bounds__(256, OCC) paged_decode_persist_kernel(
    const bf16_t* __restrict__ q, long q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, const int* __restrict__ order,
    bf16_t* __restrict__ out, long out_stride, int B, int Hq, int Hkv, float scale,
    int part_tokens, RopeIn rp) {
  __shared__ DecodeSmem<HD> sm;
  const int nseg = B * Hkv;
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int r = seg / Hkv, kvh = seg - r * Hkv;
    decode_segment<HD, MODE>(sm, 0, kvh, order ? order[r] : r, q, q_stride, k_cache, v_cache,
                          block_tables, bt_stride, context_lens, out, out_stride, nullptr,
                          nullptr, Hq, Hkv, scale, part_tokens, 1, rp);
    __syncthreads();            // the segment's LDS combine is read before the next reuses it
  }
}

// grid (Hq, B), block HD (one thread per d)
template <int HD>
__global__ void __launch_bounds__(128) paged_decode_reduce_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_ml,
    const int* __restrict__ context_lens, bf16_t* __restrict__ out, long out_stride, int Hq,
    int part_tokens, int max_parts) {
  const int head = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int ctx = context_lens[b];
  part_tokens = effective_part(ctx, part_tokens, max_parts);
  const int nparts = (ctx + part_tokens - 1) / part_tokens;
  if (nparts <= 1) return;
  const long base = ((long)b * Hq + head) * max_parts;
  float M = -INFINITY;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, part_ml[(base + p) * 2]);
  float L = 0.f, O = 0.f;
  for (int p = 0; p < nparts; ++p) {
    const float f = fast_exp2(part_ml[(base + p) * 2] - M);
    L += part_ml[(base + p) * 2 + 1] * f;
    O += part_o[(base + p) * HD + d] * f;
  }
  out[(long)b * out_stride + (long)head * HD + d] = f2bf(O / L);
}

// loop form (probe / A-B knob): 0 default -- the persistent grid when every
// sequence is one partition, else one workgroup per segment; 1 pipelined
// pages; 2, 3 load-only diagnostics; 4 one workgroup per segment always; 5 the
// default forms with non-temporal K/V loads
static int g_decode_mode = 0;
void set_decode_mode(int mode) { g_decode_mode = mode; }

// resident 256-thread decode workgroups: occ per CU (3: 168 VGPRs incl. AGPRs)
static int decode_resident_wgs(int occ = 3) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    cus = n;
  }
  return occ * cus;
}

int paged_decode(const void* q, long q_stride, const void* k_cache, const void* v_cache,
                 const int* block_tables, int bt_stride, const int* context_lens,
                 const int* order, void* out,
                 long out_stride, float* part_o, float* part_ml, int B, int Hq, int Hkv, int D,
                 int block_size, float scale, int part_tokens, int max_parts,
                 const int* rope_positions, const float* cos_sin, const int* slots,
                 hipStream_t stream) {
  if (B <= 0) return 0;
  if (cos_sin && (!rope_positions || !slots)) return -5;
  const RopeIn rp{rope_positions, cos_sin, slots};
  if ((D != 128 && D != 64) || block_size != BS) return -1;
  if (Hq % Hkv != 0 || Hq / Hkv > 16) return -2;
  if (part_tokens % (4 * BS) != 0) return -3;
  if (max_parts > 1 && (!part_o || !part_ml)) return -4;
#define LMX_DEC_K(HDV, MODE)                                                                  \
  paged_decode_kernel<HDV, MODE><<<dim3(max_parts, Hkv, B), dim3(256), 0, stream>>>(          \
      (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
      bt_stride, context_lens, order, (bf16_t*)out, out_stride, part_o, part_ml, Hq, Hkv,     \
      scale, part_tokens, max_parts, rp);
#define LMX_DEC_P(HDV, MODE)                                                                  \
  paged_decode_persist_kernel<HDV, MODE><<<dim3(std::min(B * Hkv, decode_resident_wgs())), dim3(256), \
                                      0, stream>>>(                                           \
      (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
      bt_stride, context_lens, order, (bf16_t*)out, out_stride, B, Hq, Hkv, scale, part_tokens, \
      rp);
#define LMX_DEC_R(HDV, OCC)                                                                   \
  paged_decode_persist_kernel<HDV, 9, OCC>                                                    \
      <<<dim3(std::min(B * Hkv, decode_resident_wgs(OCC))), dim3(256), 0, stream>>>(          \
      (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
      bt_stride, context_lens, order, (bf16_t*)out, out_stride, B, Hq, Hkv, scale, part_tokens, \
      rp);
  // mode 0 with no more segments than CUs (a TP rank's single kv head, e.g.
  // 256 rows x 1 kv head): one workgroup per segment, the grid form -- the
  // persistent form walks one segment per workgroup there anyway and measured
  // 22.2 vs 19.6 us (profiles/r5_proxy70.md)
  const int mode = (g_decode_mode == 0 && max_parts == 1 && B * Hkv <= decode_resident_wgs(1))
                       ? 4 : g_decode_mode;
#define LMX_DEC(HDV)                                                                          \
  if (mode == 9 && max_parts == 1) { LMX_DEC_R(HDV, 2) }                                      \
  else if (mode == 10 && max_parts == 1) { LMX_DEC_R(HDV, 3) }                       \
  else if ((mode == 9 || mode == 10)) { LMX_DEC_K(HDV, 9) }                 \
  else if (mode == 0 && max_parts == 1) { LMX_DEC_P(HDV, 0) }                        \
  else if (mode == 5 && max_parts == 1) { LMX_DEC_P(HDV, 5) }                        \
  else if (mode == 6 && max_parts == 1) { LMX_DEC_P(HDV, 6) }                        \
  else if (mode == 6) { LMX_DEC_K(HDV, 6) }                                          \
  else if (mode == 5) { LMX_DEC_K(HDV, 5) }                                          \
  else if (mode == 1) { LMX_DEC_K(HDV, 1) }                                          \
  else if (mode == 2) { LMX_DEC_K(HDV, 2) }                                          \
  else if (mode == 3) { LMX_DEC_K(HDV, 3) }                                          \
  else { LMX_DEC_K(HDV, 0) }                                                                  \
  if (max_parts > 1)                                                                          \
    paged_decode_reduce_kernel<HDV><<<dim3(Hq, B), dim3(HDV), 0, stream>>>(                   \
        part_o, part_ml, context_lens, (bf16_t*)out, out_stride, Hq, part_tokens, max_parts);
  if (D == 128) { LMX_DEC(128) } else { LMX_DEC(64) }
#undef LMX_DEC
#undef LMX_DEC_K
#undef LMX_DEC_P
#undef LMX_DEC_R
  return (int)hipGetLastError();
}

// --------------------------------------------------------------- prefill ----
// Prefill / encoder attention (K3): flash-style, K/V tiles shared through LDS.
//
//   grid (num_tiles, Hkv), block 256 = 4 waves; tiles[t] = {seq, q_start}.
//   A workgroup serves PQ = 4 * NG * (16/G) queries x G heads of one
//   (seq, kv head): each wave owns NG groups of 16 "columns" (query, head)
//   and keeps the S^T / O^T formulation of the decode kernel (softmax
//   statistics and O accumulators on the same lane, P fed straight from the
//   S accumulators as the PV B-operand via the permuted-k order).
//   Per iteration one 64-key tile (two 32-token pages) of K and V is moved
//   HBM -> LDS by global_load_lds (16 B per lane, no VGPR hop) into a double
//   buffer; the next tile's DMA is issued before the current tile's MFMAs.
//   The K image is [key][d] with its 16-B chunks XOR-swizzled by the key row
//   and the V image [d][key] with its 8-B units swizzled by d/4, both applied
//   on the global source address (the DMA writes lane-linear), so the
//   fragment reads are bank-conflict free.
//
//  q:  [T_total][Hq][D] rows at q_stride (tokens of seq s start at cu_q[s])
//  context_lens[s] = total keys of seq s (cached prefix + this chunk)
//  causal: query i of the chunk sits at absolute position ctx - qlen + i.
constexpr int PF_TK = 64;    // keys per LDS tile (two pages)
// column groups per wave: 4 at D = 64 (twice the MFMA work per K/V byte read
// from LDS; the registers fit at 2 waves / SIMD), 2 at D = 128.  Must match
// ops.prefill_q_per_tile.
template <int HD>
constexpr int pf_groups() { return HD == 64 ? 4 : 2; }

template <int HD>
__device__ __forceinline__ int kswz(int r) {
  return HD == 128 ? (r & 15) : ((r >> 1) & 7);
}

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void pf_glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds, 16, 0, 0);
}

// LDS V image: 16-B chunk slot of (quad q, d pair p) is p ^ pf_vswz(q), so
// the four key quads a ds_read_b64 lane group touches land 32 banks apart
__device__ __forceinline__ int pf_vswz(int q) { return (q & 3) * 8; }

// V^T fragment (keys 4g..4g+3 and 16+4g..16+4g+3 of row d) from the LDS page image
template <int HD>
__device__ __forceinline__ bf16x8_t pf_vfrag(const bf16_t* vpg, int d, int g) {
  const int q0 = g, q1 = 4 + g;
  const bf16_t* p0 = vpg + ((q0 * (HD / 2) + ((d >> 1) ^ pf_vswz(q0))) * 8 + (d & 1) * 4);
  const bf16_t* p1 = vpg + ((q1 * (HD / 2) + ((d >> 1) ^ pf_vswz(q1))) * 8 + (d & 1) * 4);
  return load_frag_2x8B(p0, p1);
}

// DMA one 32-token page of K and of V into the LDS tile slot `pslot`
// (PW waves: 64 PW x 8 elements per instruction).
template <int HD, int PW>
__device__ __forceinline__ void pf_stage_page(bf16_t* k_lds, bf16_t* v_lds,
                                              const bf16_t* __restrict__ kp,
                                              const bf16_t* __restrict__ vp) {
  const int tid = threadIdx.x, wave = tid >> 6;
  constexpr int PAGE = BS * HD;            // elements per page
  constexpr int PER = 512 * PW;            // elements per instruction of the workgroup
  static_assert(PAGE % PER == 0, "a page is whole DMA instructions");
#pragma unroll
  for (int j = 0; j < PAGE / PER; ++j) {
    const int off = j * PER + tid * 8;
    // K: row = key, 16-B chunk position swizzled by the row
    const int kr = off / HD, kpos = (off % HD) / 8;
    pf_glds16(kp + kr * HD + 8 * (kpos ^ kswz<HD>(kr)), k_lds + j * PER + wave * 512);
    // V: key-quad page [BS/4][HD][4]; LDS chunk (quad q, slot pp) holds the
    // global chunk d = 2p, 2p+1 with p = pp ^ vswz(q) (conflict-free 8-B
    // fragment reads, pf_vfrag)
    const int ch = off / 8, q = ch / (HD / 2), pp = ch % (HD / 2);
    pf_glds16(vp + ((long)q * HD + 2 * (pp ^ pf_vswz(q))) * 4, v_lds + j * PER + wave * 512);
  }
}

template <int CNT>
__device__ __forceinline__ void pf_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}

// NST: LDS ring slots of 64-key K/V tiles.  NST = 2: the next tile's DMA is in
// flight while the current tile computes, drained (vmcnt 0) at the next
// barrier.  NST = 3: two tiles in flight across a raw s_barrier with a counted
// vmcnt (cdna guide §5 "Pipelining across barriers").
// PW: waves per workgroup.  4 (two workgroups per CU) or 8 (one workgroup per
// CU, same waves per SIMD and registers per wave): 8 waves serve twice the
// queries from one K/V tile, so the tiles a (sequence, kv head) streams from
// L2 / HBM into LDS are moved half as often -- the short causal walks of a
// GQA prefill chunk (32 queries per 4-wave workgroup at G = 4) are bound by
// that tile latency, not by the MFMAs.
template <int HD, int NST, int PW = 4, int PF_NG = pf_groups<HD>()>
__global__ void __launch_bounds__(64 * PW, 8 / PW) paged_prefill_kernel(
    const bf16_t* __restrict__ q, long q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ context_lens,
    const int* __restrict__ tiles, bf16_t* __restrict__ out, long out_stride, int Hq, int Hkv,
    float scale, int causal, float rescale_thr, int xcd, const int* __restrict__ rope_pos,
    const float* __restrict__ rope_cs) {
  extern __shared__ __attribute__((aligned(16))) char pf_smem[];
  constexpr int PAGE = BS * HD;
  // buffer b: K pages at b*4*PAGE + {0, PAGE}, V pages at b*4*PAGE + 2*PAGE + {0, PAGE}
  bf16_t* const lds = reinterpret_cast<bf16_t*>(pf_smem);
  constexpr int KS = HD / 32, NT = HD / 16;

  // XCD-aware order: the workgroups of one (kv head, sequence) -- its query
  // tiles, which all stream the same K/V pages -- are consecutive logical ids
  // and xcd_remap puts consecutive ids on one XCD, so the pages are read from
  // HBM into that XCD's L2 once instead of once per XCD (hardware hands
  // linear workgroup b to XCD b % 8)
  const int nwg = gridDim.x * gridDim.y;
  const int lin0 = blockIdx.x + blockIdx.y * gridDim.x;
  const int lin = xcd ? xcd_remap(lin0, nwg) : lin0;
  // xcd 2: the tile list walked backwards -- the host lists a sequence's query
  // tiles in ascending order, so causal chunks then start their longest
  // key walks first and the short ones fill the tail
  const int tile = xcd == 2 ? (int)gridDim.x - 1 - lin % (int)gridDim.x : lin % (int)gridDim.x;
  const int kvh = lin / gridDim.x;
  const int seq = tiles[2 * tile], q_start = tiles[2 * tile + 1];
  // queries per 16-lane column group; with G not dividing 16 (e.g. Qwen2.5's
  // 7) the last 16 - QG*G lanes of a group are idle
  const int G = Hq / Hkv, QG = 16 / G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int qbeg = cu_q[seq], qlen = cu_q[seq + 1] - qbeg;
  const int ctx = context_lens[seq];
  const int wg_q1 = min(q_start + PW * PF_NG * QG, qlen);  // one past the WG's last query
  const int wg_lim = causal ? (ctx - qlen + wg_q1 - 1) : (ctx - 1);
  const int ntiles = wg_lim / PF_TK + 1;
  const int last_page = (ctx - 1) / BS;
  const int* bt = block_tables + (long)seq * bt_stride;

  // this lane's columns
  int lim[PF_NG];
  bool valid[PF_NG];
  int qi[PF_NG];
  bf16x8_t qf[PF_NG][KS];
#pragma unroll
  for (int n = 0; n < PF_NG; ++n) {
    qi[n] = q_start + (wave * PF_NG + n) * QG + c / G;
    valid[n] = c < QG * G && qi[n] < qlen;
    lim[n] = valid[n] ? (causal ? (ctx - qlen + qi[n]) : (ctx - 1)) : -1;
  }
  auto stage = [&](int t, int buf) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int pg = min(2 * t + pp, last_page);
      const long blk = bt[pg];
      const bf16_t* kp = k_cache + (blk * Hkv + kvh) * PAGE;
      const bf16_t* vp = v_cache + (blk * Hkv + kvh) * PAGE;
      bf16_t* base = lds + buf * 4 * PAGE;
      pf_stage_page<HD, PW>(base + pp * PAGE, base + 2 * PAGE + pp * PAGE, kp, vp);
    }
  };
  // LDS-DMA instructions per thread per tile (2 pages x K and V)
  constexpr int LPS = 4 * (PAGE / (512 * PW));

  // Q fragments through LDS (one image row per column: [wave][n][c][HD]) by
  // LDS-DMA, not plain loads: an ordinary global load whose result the tile
  // loop consumes makes hipcc drain the whole DMA ring (vmcnt 0) before the
  // first MFMA of EVERY tile (guide §5 item 4b).  The image borrows the first
  // QSL ring slots; K/V tile t lives in slot (t + QSL) % NST, so the first
  // NST - QSL tiles are staged into the other slots while Q is still in
  // flight (the Q and tile-0 latencies overlap instead of adding up at the
  // start of every workgroup: ~5 tiles per workgroup on a 546-token causal
  // chunk).
  constexpr int QROWS = PW * PF_NG * 16, QCH = HD / 8;  // rows, 16-B chunks per row
  constexpr int QSL = (QROWS * HD + 4 * PAGE - 1) / (4 * PAGE);
  constexpr int EARLY = NST - QSL;                       // tiles staged under the Q load
  static_assert(QSL <= NST, "Q image fits the ring");
  {
#pragma unroll
    for (int j = 0; j < QROWS * QCH / (64 * PW); ++j) {
      const int e = j * 64 * PW + threadIdx.x, row = e / QCH, ch = e % QCH;
      const int rw = row / (PF_NG * 16), rn = (row / 16) % PF_NG, rc = row % 16;
      const int rq = q_start + (rw * PF_NG + rn) * QG + rc / G;
      const bool ok = rc < QG * G && rq < qlen;
      const bf16_t* src = q + (long)(qbeg + (ok ? rq : 0)) * q_stride +
                          (long)(kvh * G + (ok ? rc % G : 0)) * HD + 8 * ch;
      pf_glds16(src, lds + j * 512 * PW + wave * 512);
    }
#pragma unroll
    for (int p = 0; p < EARLY && p < NST - 1; ++p)
      if (p < ntiles) stage(p, (p + QSL) % NST);
    // Q landed: only the early tiles' DMA (issued after it) may remain
    if constexpr (EARLY >= 2) {
      if (ntiles >= 2) pf_vmwait<2 * LPS>(); else pf_vmwait<LPS>();
    } else if constexpr (EARLY == 1) {
      pf_vmwait<LPS>();
    } else {
      pf_vmwait<0>();
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int n = 0; n < PF_NG; ++n) {
      const bf16_t* qrow = lds + ((wave * PF_NG + n) * 16 + c) * HD;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        qf[n][s] = valid[n] ? load_frag16B(qrow + 32 * s + 8 * g)
                            : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();     // every wave holds its Q before the ring reuses the slots
    // fused rotary embedding of q (rope_cs != nullptr): the rope/cache kernel
    // then leaves q untouched and skips its read-modify-write of the q rows
    // (3/4 of that kernel's traffic at G = 4); same fp32 expression and bf16
    // rounding as the cache kernel (rope_q_frags, shared with decode)
    if (rope_cs) {
#pragma unroll
      for (int n = 0; n < PF_NG; ++n)
        if (valid[n]) rope_q_frags<HD>(qf[n], rope_cs + (long)rope_pos[qbeg + qi[n]] * HD, g);
    }
  }
  // smallest column limit of the wave: tiles below it need no mask
  int wave_lo = INT_MAX;
#pragma unroll
  for (int n = 0; n < PF_NG; ++n) wave_lo = min(wave_lo, valid[n] ? lim[n] : INT_MAX);
  wave_lo = min(wave_lo, __shfl_xor(wave_lo, 1, 64));
  wave_lo = min(wave_lo, __shfl_xor(wave_lo, 2, 64));
  wave_lo = min(wave_lo, __shfl_xor(wave_lo, 4, 64));
  wave_lo = min(wave_lo, __shfl_xor(wave_lo, 8, 64));
  const bool wave_idle = q_start + wave * PF_NG * QG >= qlen;   // wave-uniform

  float m[PF_NG], l[PF_NG];
  f32x4_t acc[PF_NG][NT];
#pragma unroll
  for (int n = 0; n < PF_NG; ++n) {
    m[n] = -INFINITY;
    l[n] = 0.f;
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[n][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const float scale_log2 = scale * LOG2E;

#pragma unroll
  for (int p = EARLY; p < NST - 1; ++p)    // the rest of the prologue, into the Q slots
    if (p < ntiles) stage(p, (p + QSL) % NST);
  for (int t = 0; t < ntiles; ++t) {
    const int buf = (t + QSL) % NST;
    // tile t landed once at most the tiles issued after it remain in flight
    if (t + NST - 2 < ntiles) pf_vmwait<(NST - 2) * LPS>(); else pf_vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();    // raw: a __syncthreads fence would drain the ring
    // refill the slot every wave finished reading at t - 1
    if (t + NST - 1 < ntiles) stage(t + NST - 1, (t + NST - 1 + QSL) % NST);
    if (wave_idle) continue;
    const bf16_t* kt = lds + buf * 4 * PAGE;
    const bf16_t* vt = kt + 2 * PAGE;
    const int key0 = t * PF_TK;
    // One 64-key tile, software-pipelined over the wave's column groups so the
    // softmax VALU of group n-1 issues between the S MFMAs of group n, and the
    // softmax of the last group between the PV MFMAs of group 0 (the MFMA and
    // VALU pipes of a SIMD run concurrently; in the plain S -> softmax -> PV
    // order a wave idles one while it feeds the other):
    //   S(0) | S(1) + sm(0) | ... | PV(0) + sm(NG-1) | PV(1) ... PV(NG-1)
    // K fragments are read once and kept for every group, V fragments too.
    // The softmax is branch-free inside a region (the lazy rescale decision
    // is a wave-uniform select; the O^T rescale of group n -- rare -- runs
    // between regions, before PV(n)); the causal mask is a tile-level variant.
    auto tile_body = [&](auto mask_tag) {
      constexpr bool MASK = decltype(mask_tag)::value;
      f32x4_t s[PF_NG][4];
      bf16x8_t pf[PF_NG][2];
      bool need[PF_NG];
      float alpha[PF_NG];
      bf16x8_t kf[4][KS];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int row = (kb & 1) * 16 + c;               // key row inside its page
        const bf16_t* krow = kt + (kb >> 1) * PAGE + row * HD;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          kf[kb][ks] = load_frag16B(krow + 8 * ((ks * 4 + g) ^ kswz<HD>(row)));
      }
      const f32x4_t z4 = {0.f, 0.f, 0.f, 0.f};
      auto s_mma = [&](int n) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            s[n][kb] = mfma16(kf[kb][ks], qf[n][ks], ks == 0 ? z4 : s[n][kb]);
      };
      typedef float f32x2_t __attribute__((ext_vector_type(2)));
      auto softmax = [&](int n) {
        f32x2_t x[8];                                    // x[2 kb + h] = keys 16 kb + 4 g + 2 h + {0, 1}
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int h = 0; h < 2; ++h) x[2 * kb + h] = f32x2_t{s[n][kb][2 * h], s[n][kb][2 * h + 1]};
        if constexpr (MASK) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = key0 + kb * 16 + 4 * g + r;
              x[2 * kb + (r >> 1)][r & 1] = key <= lim[n] ? x[2 * kb + (r >> 1)][r & 1] : -INFINITY;
            }
        }
        // 16 values: a max3 tree (8 instructions, depth 3)
        const float t0 = max3f(x[0].x, x[0].y, x[1].x), t1 = max3f(x[1].y, x[2].x, x[2].y);
        const float t2 = max3f(x[3].x, x[3].y, x[4].x), t3 = max3f(x[4].y, x[5].x, x[5].y);
        const float t4 = max3f(x[6].x, x[6].y, x[7].x);
        float mx = max3f(max3f(t0, t1, t2), max3f(t3, t4, x[7].y), -INFINITY);
        mx = col4_max(mx);
        const float mx2 = mx * scale_log2;               // -inf stays -inf (scale > 0)
        // lazy rescale (guide T13): the running max m (log2 units) is raised
        // only when a tile's max exceeds it by more than rescale_thr; until then
        // p = 2^(x - m) <= 2^thr.  The wave rescales together (exact alpha per
        // column, 1 where it did not grow).
        const bool nd = __ballot(mx2 > m[n] + rescale_thr) != 0;
        const float m_new = nd ? max2f(m[n], mx2) : m[n];
        const float al = (nd && m_new != -INFINITY) ? fast_exp2(m[n] - m_new) : 1.f;
        l[n] *= al;
        m[n] = m_new;
        need[n] = nd;
        alpha[n] = al;
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
        const f32x2_t sc2 = {scale_log2, scale_log2}, nm2 = {-m_use, -m_use};
        f32x2_t rs2 = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          f32x2_t y = x[j] * sc2 + nm2;
          y.x = fast_exp2(y.x);
          y.y = fast_exp2(y.y);
          x[j] = y;
          rs2 += y;
        }
        l[n] += col4_sum(rs2.x + rs2.y);
        // page p: keys 4g+r (block 2p) then 16+4g+r (block 2p+1) -> permuted-k B operand
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t w = pack_bf16x2(x[4 * pp + j].x, x[4 * pp + j].y);
            pf[n][pp][2 * j] = (short)(w & 0xffff);
            pf[n][pp][2 * j + 1] = (short)(w >> 16);
          }
      };
      auto rescale = [&](int n) {
        // a real (wave-uniform) branch: the lazy rescale is rare, and hipcc
        // otherwise may speculate it into an unconditional acc *= alpha
        if (need[n]) {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int i = 0; i < NT; ++i) acc[n][i] *= alpha[n];
        }
      };
      // interleave hint for one region: MFMAs spread through the VALU stream
      auto interleave = [&](int nmfma) {
        for (int i = 0; i < nmfma; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // 5 VALU
        }
      };
      s_mma(0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 1; n < PF_NG; ++n) {
        s_mma(n);
        softmax(n - 1);
        interleave(4 * KS);
        __builtin_amdgcn_sched_barrier(0);
        rescale(n - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      // V^T fragments of both pages (kept for every group)
      bf16x8_t vf[2][NT];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int i = 0; i < NT; ++i) vf[pp][i] = pf_vfrag<HD>(vt + pp * PAGE, 16 * i + c, g);
      auto pv = [&](int n) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int i = 0; i < NT; ++i) acc[n][i] = mfma16(vf[pp][i], pf[n][pp], acc[n][i]);
      };
      pv(0);
      softmax(PF_NG - 1);
      interleave(2 * NT);
      __builtin_amdgcn_sched_barrier(0);
      rescale(PF_NG - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 1; n < PF_NG; ++n) pv(n);
    };
    const bool need_mask = key0 + PF_TK - 1 > wave_lo;
    if (need_mask) tile_body(std::true_type{}); else tile_body(std::false_type{});
  }
  // Epilogue: O^T through LDS, so every output row leaves as whole 16-B pieces
  // (8 global_store_dwordx4 per lane instead of 16 dwordx2 at a 32-B stride;
  // per-lane row-stride stores are issue-bound, guide T21).  Each wave stages
  // its PF_NG x 16 columns into its own [column][16-B chunk] image, chunk index
  // XOR the column's low bits (2-way conflicts on the 8-B writes, none on the
  // 16-B reads), after a barrier that retires every wave's reads of the last
  // K/V tile (the ring has no DMA in flight after the last tile).
  constexpr int OCOLS = PF_NG * 16, CH = HD / 8, ROWB = HD * 2;
  static_assert(PW * OCOLS * ROWB <= NST * 4 * PAGE * 2, "O image fits the ring");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  char* const oimg = pf_smem + wave * OCOLS * ROWB;
#pragma unroll
  for (int n = 0; n < PF_NG; ++n) {
    const float inv = l[n] > 0.f ? 1.f / l[n] : 0.f;
    const int col = n * 16 + c;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      bf16x4_t o4;
#pragma unroll
      for (int r = 0; r < 4; ++r) o4[r] = (short)f2bf(acc[n][i][r] * inv);
      const int chunk = 2 * i + (g >> 1);                 // d = 16 i + 4 g
      *reinterpret_cast<bf16x4_t*>(oimg + col * ROWB + 16 * (chunk ^ (col & (CH - 1))) +
                                   8 * (g & 1)) = o4;
    }
  }
#pragma unroll
  for (int k = 0; k < OCOLS * CH / 64; ++k) {
    const int e = k * 64 + lane, col = e / CH, j = e % CH;
    const bf16x8_t v =
        *reinterpret_cast<const bf16x8_t*>(oimg + col * ROWB + 16 * (j ^ (col & (CH - 1))));
    const int n = col / 16, cc = col % 16;
    const int qq = q_start + (wave * PF_NG + n) * QG + cc / G;
    if (cc < QG * G && qq < qlen)
      *reinterpret_cast<bf16x8_t*>(out + (long)(qbeg + qq) * out_stride +
                                   (long)(kvh * G + cc % G) * HD + 8 * j) = v;
  }
}

// lazy-rescale threshold of the prefill softmax, log2 units (0: rescale
// whenever a column's max grows -- the test knob of guide §5.4 rule 26)
static float g_prefill_rescale_thr = 8.f;
void set_prefill_rescale_thr(float thr) { g_prefill_rescale_thr = thr; }
// LDS ring slots of the prefill kernel (0: default per head dim; 2 or 3: A/B knob)
static int g_prefill_stages = 0;
void set_prefill_stages(int n) { g_prefill_stages = (n == 2 || n == 3) ? n : 0; }
// prefill workgroup order: 2 (default) XCD-aware with the tile list walked backwards, 1
// XCD-aware, 0 hardware order (A/B knob)
static int g_prefill_xcd = 2;
void set_prefill_xcd(int on) { g_prefill_xcd = on < 0 ? 0 : (on > 2 ? 2 : on); }

// q_per_tile: the tile list's queries per workgroup (ops.prefill_q_per_tile);
// it selects the workgroup width PW = q_per_tile / (column groups x 16/G):
// 4 or 8 waves (8 only at head dim 128)
// rope_pos / rope_cs (both or neither): rotate q in the kernel (q rows of qkv
// unrotated; positions per row, cos_sin [max_pos][D] as rope_cache.hip)
int paged_prefill(const void* q, long q_stride, const void* k_cache, const void* v_cache,
                  const int* block_tables, int bt_stride, const int* cu_q,
                  const int* context_lens, const int* tiles, int num_tiles, void* out,
                  long out_stride, int Hq, int Hkv, int D, int block_size, float scale,
                  int causal, int q_per_tile, const int* rope_pos, const float* rope_cs,
                  hipStream_t stream) {
  if ((rope_pos == nullptr) != (rope_cs == nullptr)) return -4;
  if (num_tiles <= 0) return 0;
  if ((D != 128 && D != 64) || block_size != BS) return -1;
  if (Hq % Hkv != 0 || Hq / Hkv > 16) return -2;
  const int per_wave = (D == 128 ? pf_groups<128>() : pf_groups<64>()) * (16 / (Hq / Hkv));
  const int pw = q_per_tile / per_wave;
  if (q_per_tile % per_wave != 0 || (pw != 4 && pw != 8) || (pw == 8 && D != 128)) return -3;
#define LMX_PRE(HDV, NSTV, PWV)                                                               \
  {                                                                                           \
    constexpr int smem = NSTV * 4 * BS * HDV * 2;                                             \
    static bool attr = false;                                                                 \
    if (smem > 65536 && !attr) {                                                              \
      (void)hipFuncSetAttribute((const void*)paged_prefill_kernel<HDV, NSTV, PWV>,            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, smem);            \
      attr = true;                                                                            \
    }                                                                                         \
    paged_prefill_kernel<HDV, NSTV, PWV><<<dim3(num_tiles, Hkv), dim3(64 * PWV), smem,        \
                                           stream>>>(                                         \
        (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache,           \
        block_tables, bt_stride, cu_q, context_lens, tiles, (bf16_t*)out, out_stride, Hq, Hkv, \
        scale, causal, g_prefill_rescale_thr, g_prefill_xcd, rope_pos, rope_cs);              \
  }
  // 2 slots by default: 3 measured equal at D = 64 and 1.55x slower at D = 128
  // with 4-wave workgroups (96 KB of LDS leaves one workgroup per CU) --
  // tools/prefill_attn_probe.py; the 8-wave form is one workgroup per CU anyway
  const int nst = g_prefill_stages ? g_prefill_stages : 2;
  if (D == 128) {
    if (pw == 8) {
      if (nst == 3) LMX_PRE(128, 3, 8) else LMX_PRE(128, 2, 8)
    } else {
      if (nst == 3) LMX_PRE(128, 3, 4) else LMX_PRE(128, 2, 4)
    }
  } else {
    if (nst == 3) LMX_PRE(64, 3, 4) else LMX_PRE(64, 2, 4)
  }
#undef LMX_PRE
  return (int)hipGetLastError();
}

}  // namespace lmx
