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
// d-major V page, see rope_cache.hip for the cache layout).
//
//   decode  (K4): columns = the G query heads of one token (G = Hq/Hkv <= 16);
//                 the 4 waves split the page range, combined through LDS, and
//                 long contexts are split over workgroups (split-K) with a
//                 separate reduce kernel.
//   prefill (K3): columns = (16/G queries) x (G heads): the K/V page read is
//                 shared by all heads of the kv group; each wave walks its own
//                 causal key range; varlen batches via a host-built tile list.
#include "common.h"

namespace lmx {

constexpr int BS = 32;   // KV page (block) size in tokens
constexpr float LOG2E = 1.4426950408889634f;

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
template <int HD>
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
    ka[s] = load_frag16B(kpage + c * HD + 32 * s + 8 * g);
    kb[s] = load_frag16B(kpage + (16 + c) * HD + 32 * s + 8 * g);
  }
  // V^T fragments (issued early so they overlap the QK MFMAs and softmax)
  bf16x8_t vf[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const bf16_t* vr = vpage + (16 * i + c) * BS;
    vf[i] = load_frag_2x8B(vr + 4 * g, vr + 16 + 4 * g);
  }
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
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float m_new = fmaxf(st.m, mx);
  // a column may see no visible key in this page (causal tail): keep its state
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  const float alpha = exp2f(st.m - m_use);
  float p[8], rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { p[j] = exp2f(x[j] - m_use); rs += p[j]; }
  rs += __shfl_xor(rs, 16, 64);
  rs += __shfl_xor(rs, 32, 64);
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

// ---------------------------------------------------------------- decode ----
// Partition length used for a sequence: the requested split-K granule, grown
// (in 128-token steps) when the context would need more than max_parts
// partitions, so the grid baked into a captured graph always covers it.
__device__ __forceinline__ int effective_part(int ctx, int part_tokens, int max_parts) {
  int need = (ctx + max_parts - 1) / max_parts;
  need = (need + 127) & ~127;
  return need > part_tokens ? need : part_tokens;
}

// grid (max_parts, Hkv, B), block 256.
template <int HD>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    const bf16_t* __restrict__ q, long q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, bf16_t* __restrict__ out, long out_stride,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, int Hkv, float scale,
    int part_tokens, int max_parts) {
  __shared__ float sm_ml[4][16][2];
  __shared__ float sm_o[4][16][HD + 4];
  const int p = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int ctx = context_lens[b];
  part_tokens = effective_part(ctx, part_tokens, max_parts);
  const int nparts = (ctx + part_tokens - 1) / part_tokens;
  if (p >= nparts) return;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int t0 = p * part_tokens, t1 = min(t0 + part_tokens, ctx);

  bf16x8_t qf[HD / 32];
  const bf16_t* qrow = q + (long)b * q_stride + (long)(kvh * G + c) * HD;
#pragma unroll
  for (int s = 0; s < HD / 32; ++s)
    qf[s] = (c < G) ? load_frag16B(qrow + 32 * s + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};

  PageState<HD> st;
  state_init(st);
  const float scale_log2 = scale * LOG2E;
  const int pg0 = t0 / BS, pg1 = (t1 + BS - 1) / BS;
  const int* bt = block_tables + (long)b * bt_stride;
  for (int pg = pg0 + wave; pg < pg1; pg += 4) {
    const long blk = bt[pg];
    const bf16_t* kp = k_cache + (blk * Hkv + kvh) * (BS * HD);
    const bf16_t* vp = v_cache + (blk * Hkv + kvh) * (BS * HD);
    process_page(st, qf, kp, vp, pg * BS, t1 - 1, scale_log2);
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
      const float f = (mw == -INFINITY) ? 0.f : exp2f(mw - M);
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
    const float f = exp2f(part_ml[(base + p) * 2] - M);
    L += part_ml[(base + p) * 2 + 1] * f;
    O += part_o[(base + p) * HD + d] * f;
  }
  out[(long)b * out_stride + (long)head * HD + d] = f2bf(O / L);
}

int paged_decode(const void* q, long q_stride, const void* k_cache, const void* v_cache,
                 const int* block_tables, int bt_stride, const int* context_lens, void* out,
                 long out_stride, float* part_o, float* part_ml, int B, int Hq, int Hkv, int D,
                 int block_size, float scale, int part_tokens, int max_parts,
                 hipStream_t stream) {
  if (B <= 0) return 0;
  if ((D != 128 && D != 64) || block_size != BS) return -1;
  if (Hq % Hkv != 0 || Hq / Hkv > 16) return -2;
  if (part_tokens % (4 * BS) != 0) return -3;
  if (max_parts > 1 && (!part_o || !part_ml)) return -4;
#define LMX_DEC(HDV)                                                                          \
  paged_decode_kernel<HDV><<<dim3(max_parts, Hkv, B), dim3(256), 0, stream>>>(                \
      (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
      bt_stride, context_lens, (bf16_t*)out, out_stride, part_o, part_ml, Hq, Hkv, scale,      \
      part_tokens, max_parts);                                                                \
  if (max_parts > 1)                                                                          \
    paged_decode_reduce_kernel<HDV><<<dim3(Hq, B), dim3(HDV), 0, stream>>>(                   \
        part_o, part_ml, context_lens, (bf16_t*)out, out_stride, Hq, part_tokens, max_parts);
  if (D == 128) { LMX_DEC(128) } else { LMX_DEC(64) }
#undef LMX_DEC
  return (int)hipGetLastError();
}

// --------------------------------------------------------------- prefill ----
// tiles[t] = {seq, q_start}; a workgroup serves 4 waves x (16/G) queries of
// one (seq, kv head).  grid (num_tiles, Hkv), block 256.
//  q:  [T_total][Hq][D] rows at q_stride (tokens of seq s start at cu_q[s])
//  context_lens[s] = total keys of seq s (cached prefix + this chunk)
//  causal: query i of the chunk sits at absolute position ctx - qlen + i.
template <int HD>
__global__ void __launch_bounds__(256) paged_prefill_kernel(
    const bf16_t* __restrict__ q, long q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ context_lens,
    const int* __restrict__ tiles, bf16_t* __restrict__ out, long out_stride, int Hq, int Hkv,
    float scale, int causal) {
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int seq = tiles[2 * tile], q_start = tiles[2 * tile + 1];
  const int G = Hq / Hkv, QPW = 16 / G;  // queries per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int qbeg = cu_q[seq], qlen = cu_q[seq + 1] - qbeg;
  const int ctx = context_lens[seq];
  const int qi = q_start + wave * QPW + c / G;  // query index inside the chunk
  const int head = kvh * G + (c % G);
  const bool valid = (c < QPW * G) && (qi < qlen);
  const int lim = causal ? (ctx - qlen + qi) : (ctx - 1);
  // the wave's key range: up to its last valid query's limit
  const int qi_last = min(q_start + wave * QPW + QPW - 1, qlen - 1);
  if (q_start + wave * QPW >= qlen) return;  // whole wave idle (no barriers below)
  const int wave_lim = causal ? (ctx - qlen + qi_last) : (ctx - 1);

  bf16x8_t qf[HD / 32];
  const bf16_t* qrow = q + (long)(qbeg + (valid ? qi : 0)) * q_stride + (long)head * HD;
#pragma unroll
  for (int s = 0; s < HD / 32; ++s)
    qf[s] = valid ? load_frag16B(qrow + 32 * s + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};

  PageState<HD> st;
  state_init(st);
  const float scale_log2 = scale * LOG2E;
  const int* bt = block_tables + (long)seq * bt_stride;
  const int npg = wave_lim / BS + 1;
  const int my_lim = valid ? lim : -1;
  for (int pg = 0; pg < npg; ++pg) {
    const long blk = bt[pg];
    const bf16_t* kp = k_cache + (blk * Hkv + kvh) * (BS * HD);
    const bf16_t* vp = v_cache + (blk * Hkv + kvh) * (BS * HD);
    process_page(st, qf, kp, vp, pg * BS, my_lim, scale_log2);
  }
  if (!valid) return;
  const float inv = st.l > 0.f ? 1.f / st.l : 0.f;
  bf16_t* orow = out + (long)(qbeg + qi) * out_stride + (long)head * HD;
#pragma unroll
  for (int i = 0; i < HD / 16; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) orow[16 * i + 4 * g + r] = f2bf(st.acc[i][r] * inv);
}

int paged_prefill(const void* q, long q_stride, const void* k_cache, const void* v_cache,
                  const int* block_tables, int bt_stride, const int* cu_q,
                  const int* context_lens, const int* tiles, int num_tiles, void* out,
                  long out_stride, int Hq, int Hkv, int D, int block_size, float scale,
                  int causal, hipStream_t stream) {
  if (num_tiles <= 0) return 0;
  if ((D != 128 && D != 64) || block_size != BS) return -1;
  if (Hq % Hkv != 0 || 16 % (Hq / Hkv) != 0) return -2;
#define LMX_PRE(HDV)                                                                          \
  paged_prefill_kernel<HDV><<<dim3(num_tiles, Hkv), dim3(256), 0, stream>>>(                  \
      (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
      bt_stride, cu_q, context_lens, tiles, (bf16_t*)out, out_stride, Hq, Hkv, scale, causal);
  if (D == 128) { LMX_PRE(128) } else { LMX_PRE(64) }
#undef LMX_PRE
  return (int)hipGetLastError();
}

}  // namespace lmx
