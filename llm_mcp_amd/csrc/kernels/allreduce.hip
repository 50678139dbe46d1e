// X1/X2: tensor-parallel all-reduce over peer memory (xGMI), bf16 sum with
// fp32 accumulation, for the decode-sized messages of a TP group.
//
// Why not only RCCL: a ring moves 2(W-1)/W * S bytes through ONE xGMI link per
// direction and pays 2(W-1) latency hops; decode all-reduces (T x d x 2 B =
// 16 KB ... 4 MB at d = 8192) are latency-bound.  MI355X peers are fully
// connected (7 links per GPU), so here every rank reads its peers' buffers
// directly, all links at once:
//   * one-shot (small S): every rank reads all W inputs and sums;
//     one hop, W-1 x S bytes per rank spread over W-1 links;
//   * two-shot (larger S): reduce-scatter (rank r sums shard r from all peers)
//     then all-gather (read every other reduced shard from its owner);
//     2 (W-1)/W x S bytes per rank, still all links in parallel.
// Buffers: each rank owns one hipExtMallocWithFlags(hipDeviceMallocUncached)
// region mapped into every peer by hipIpcOpenMemHandle.  Uncached (MTYPE UC)
// memory makes a peer's stores visible once they complete, so a publish is
// "stores; s_waitcnt vmcnt(0); barrier; flag store" with no L2 write-back.
// Layout of a region (bytes):
//   [0, 256)           control: epoch (u32), arrival ticket (u32), error (u32)
//   [256, 256 + 12 KB) flags[3 phases][128 blocks][8 ranks] (u32 epochs)
//   [16 KB, ...)       2 parities x {input copy (slot_bytes), result (slot_bytes)}
// Epochs live on the device (read at kernel start, advanced by the last block
// to finish) so a captured hipGraph replays correctly.  Consecutive calls
// alternate the data parity; a rank can only reach call e + 2 after every
// peer has signalled in call e + 1, i.e. after the peers' call-e kernels (and
// their reads of parity e) completed, so no trailing barrier is needed.
// Every wait is bounded (spin_max polls): a missing peer sets the error word
// and the kernel still exits, so the grid always drains.
// The same regions also carry the decode step's logits all-gather (mode 2/3
// of the kernel), so a TP group's captured decode graph holds no RCCL
// collective at all.
#include <cstring>

#include "common.h"

namespace lmx {

constexpr int AR_MAX_W = 8, AR_MAX_BLOCKS = 128, AR_THREADS = 512;
constexpr long AR_CTL = 0, AR_FLAGS = 256, AR_DATA = 16384;

struct ArPeers {
  char* p[AR_MAX_W];
};

__device__ __forceinline__ uint32_t* ar_flags(char* base, int phase) {
  return reinterpret_cast<uint32_t*>(base + AR_FLAGS) + phase * AR_MAX_BLOCKS * AR_MAX_W;
}

// block-level rendezvous of block b across the W ranks
template <int W>
__device__ __forceinline__ void ar_barrier(const ArPeers& peers, int rank, int phase, int b,
                                           uint32_t e, int spin_max) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this thread's slot stores landed
  __syncthreads();
  const int t = threadIdx.x;
  if (t < W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(ar_flags(peers.p[t], phase) + b * AR_MAX_W + rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = ar_flags(peers.p[rank], phase) + b * AR_MAX_W + t;
    int it = 0;
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++it > spin_max) {
        __hip_atomic_store(reinterpret_cast<uint32_t*>(peers.p[rank] + AR_CTL) + 2, 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// rendezvous of a group of ``cs`` blocks [g0, g0 + cs): block b signals its
// own flag (to every rank, or only to this rank when ``local``), then waits
// until every block of the group has signalled on every rank (local: on
// this rank) -- the fused norm's column-split blocks of one row group
template <int W>
__device__ __forceinline__ void ar_group_barrier(const ArPeers& peers, int rank, int phase, int b,
                                                 int g0, int cs, bool local, uint32_t e,
                                                 int spin_max) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x, nr = local ? 1 : W;
  if (t < nr) {
    const int q = local ? rank : t;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(ar_flags(peers.p[q], phase) + b * AR_MAX_W + rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (t < nr * cs) {
    const int q = local ? rank : t % W, blk = g0 + t / nr;
    const uint32_t* f = ar_flags(peers.p[rank], phase) + blk * AR_MAX_W + q;
    int it = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++it > spin_max) {
        __hip_atomic_store(reinterpret_cast<uint32_t*>(peers.p[rank] + AR_CTL) + 2, 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__device__ __forceinline__ void add8(float (&acc)[8], const u16x8& v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += bf2f(v.v[j]);
}

__device__ __forceinline__ u16x8 pack8(const float (&acc)[8]) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = f2bf(acc[j]);
  return o;
}

template <int W>
__global__ void __launch_bounds__(AR_THREADS) allreduce_kernel(
    u16x8* out, const u16x8* inp, long n8, int rank, ArPeers peers,
    long slot_bytes, int two_shot, int spin_max) {
  char* own = peers.p[rank];
  uint32_t* ctl = reinterpret_cast<uint32_t*>(own + AR_CTL);
  const uint32_t e = ctl[0] + 1u;
  const long par_off = AR_DATA + (long)(e & 1u) * 2 * slot_bytes;
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  auto in_slot = [&](int q) { return reinterpret_cast<u16x8*>(peers.p[q] + par_off); };
  auto res_slot = [&](int q) { return reinterpret_cast<u16x8*>(peers.p[q] + par_off + slot_bytes); };

  if (two_shot >= 2) {
    // all-gather (X3, the vocab-parallel logits of a decode step): every rank
    // publishes its n8-chunk input in its own slot; mode 2: every rank reads
    // all W chunks into out[q * n8 + i]; mode 3: only rank 0 reads (the
    // others only publish -- a gather to the sampling leader).  Same parity
    // / epoch protocol as the reductions: a rank reaches call e + 2 only
    // after every peer signalled in call e + 1, i.e. after the readers'
    // call-e kernels completed.
    const long per = (n8 + nb - 1) / nb, lo = b * per, hi = min(n8, lo + per);
    u16x8* mine = in_slot(rank);
    for (long i = lo + t; i < hi; i += AR_THREADS) mine[i] = inp[i];
    ar_barrier<W>(peers, rank, 0, b, e, spin_max);
    if (two_shot == 2 || rank == 0) {
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const u16x8* src = q == rank ? inp : in_slot(q);
        for (long i = lo + t; i < hi; i += AR_THREADS) out[q * n8 + i] = src[i];
      }
    }
  } else if (!two_shot) {
    const long per = (n8 + nb - 1) / nb, lo = b * per, hi = min(n8, lo + per);
    u16x8* mine = in_slot(rank);
    for (long i = lo + t; i < hi; i += AR_THREADS) mine[i] = inp[i];
    ar_barrier<W>(peers, rank, 0, b, e, spin_max);
    for (long i = lo + t; i < hi; i += AR_THREADS) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) add8(acc, in_slot(q)[i]);   // rank order: same sum everywhere
      out[i] = pack8(acc);
    }
  } else {
    const long s = n8 / W;                        // shard length (host: n8 % W == 0)
    const long per = (s + nb - 1) / nb, lo = b * per, hi = min(s, lo + per);
    u16x8* mine = in_slot(rank);
#pragma unroll
    for (int q = 0; q < W; ++q)
      for (long i = lo + t; i < hi; i += AR_THREADS) mine[q * s + i] = inp[q * s + i];
    ar_barrier<W>(peers, rank, 0, b, e, spin_max);
    u16x8* res = res_slot(rank);
    for (long i = lo + t; i < hi; i += AR_THREADS) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) add8(acc, in_slot(q)[rank * s + i]);
      const u16x8 o = pack8(acc);
      res[rank * s + i] = o;
      out[rank * s + i] = o;
    }
    ar_barrier<W>(peers, rank, 1, b, e, spin_max);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      if (q == rank) continue;
      const u16x8* src = res_slot(q);
      for (long i = lo + t; i < hi; i += AR_THREADS) out[q * s + i] = src[q * s + i];
    }
  }
  // the last block to finish advances the epoch for the next call
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == (uint32_t)(nb - 1)) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------- all-reduce + residual + RMSNorm --
// One TP sub-layer tail in one kernel: o = sum over ranks of the row-parallel
// projection's bf16 partial (rank order, fp32, rounded to bf16 -- exactly what
// allreduce_kernel returns), residual += o (bf16, as rmsnorm_kernel keeps the
// hidden state), h = rmsnorm(residual) * w.  Replaces the GEMM -> all-reduce ->
// residual-add RMSNorm triple's last two launches and the o round trip
// between them; the residual stream is bitwise what they produce, h up to the
// summation order of the row's sum of squares.
//
// Grid: row groups x ``cs`` column chunks.  Block b = (row group b / cs, chunk
// b % cs) moves and sums only its chunk of each row, so a decode step's few
// rows per rank (T / W at two-shot: 32 at 256 rows and W = 8) still spread
// over up to 128 CUs instead of one CU per row.  The chunks of a row meet
// through per-chunk partial sums of squares kept beside the data:
//   one-shot: block (g, c) publishes chunk c of its rows, meets block (g, c)
//     of every rank, sums every rank's copy, writes residual chunk c and its
//     partial; a LOCAL rendezvous of the row group's cs blocks then makes the
//     row's partials visible, and each block norms its chunk;
//   two-shot: rows are sharded by rank (S = ceil(T / W) rows each); the owner's
//     block (g, c) sums chunk c of its shard rows into its result slot with the
//     partial sum of squares of residual + o beside it (the residual is the
//     same on every rank); after a rendezvous over the row group's cs blocks on
//     every rank, each block reads chunk c and the cs partials of every row from
//     its owner and norms it.  Every rank sums the same partials in the same
//     order, so h is the same on every rank.
template <int VPT>
__device__ __forceinline__ void ar_load_chunk(float (&o)[VPT][8], const u16x8* __restrict__ src,
                                              int dc) {
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * AR_THREADS;
    if (c < dc) {
      const u16x8 v = src[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[k][j] = bf2f(v.v[j]);
    }
  }
}

// residual chunk += bf16(o) (written back), returns the block's sum of squares
template <int VPT>
__device__ __forceinline__ float ar_residual_chunk(u16x8* __restrict__ res, const float (&o)[VPT][8],
                                                   int dc, bool write, float* scratch) {
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * AR_THREADS;
    if (c < dc) {
      const u16x8 r = res[c];
      u16x8 hb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hb.v[j] = f2bf(bf2f(f2bf(o[k][j])) + bf2f(r.v[j]));
        const float v = bf2f(hb.v[j]);
        ss += v * v;
      }
      if (write) res[c] = hb;
    }
  }
  return block_sum(ss, scratch);
}

// h chunk = residual chunk (already updated) * inv * w
template <int VPT>
__device__ __forceinline__ void ar_scale_chunk(u16x8* __restrict__ h, const u16x8* __restrict__ res,
                                               const u16x8* __restrict__ w, float inv, int dc) {
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * AR_THREADS;
    if (c < dc) {
      const u16x8 r = res[c], wv = w[c];
      u16x8 y;
#pragma unroll
      for (int j = 0; j < 8; ++j) y.v[j] = f2bf(bf2f(r.v[j]) * inv * bf2f(wv.v[j]));
      h[c] = y;
    }
  }
}

template <int W, int VPT>
__global__ void __launch_bounds__(AR_THREADS) allreduce_norm_kernel(
    u16x8* __restrict__ h_out, u16x8* __restrict__ residual, const u16x8* __restrict__ inp,
    const u16x8* __restrict__ w, int T, int d8, float eps, int rank, ArPeers peers,
    long slot_bytes, int two_shot, int cs, int spin_max) {
  __shared__ float scratch[16];
  char* own = peers.p[rank];
  uint32_t* ctl = reinterpret_cast<uint32_t*>(own + AR_CTL);
  const uint32_t e = ctl[0] + 1u;
  const long par_off = AR_DATA + (long)(e & 1u) * 2 * slot_bytes;
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  const int nr = nb / cs, rg = b / cs, ch = b % cs, g0 = rg * cs;
  const int dc = d8 / cs, c0 = ch * dc;               // this block's 16-B columns
  const long ss_off = (long)T * d8 * 16;              // partials [T][cs] after the rows
  auto in_slot = [&](int q) { return reinterpret_cast<u16x8*>(peers.p[q] + par_off); };
  auto res_base = [&](int q) { return peers.p[q] + par_off + slot_bytes; };
  auto partials = [&](int q, int row) {
    return reinterpret_cast<float*>(res_base(q) + ss_off) + (long)row * cs;
  };
  auto publish = [&](int row) {
    u16x8* dst = in_slot(rank) + (long)row * d8 + c0;
    const u16x8* src = inp + (long)row * d8 + c0;
    for (int c = t; c < dc; c += AR_THREADS) dst[c] = src[c];
  };
  // fp32 rank-order sum of every rank's copy of this block's chunk of a row
  auto row_sum = [&](int row, float (&o)[VPT][8]) {
#pragma unroll
    for (int k = 0; k < VPT; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[k][j] = 0.f;
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const u16x8* src = in_slot(q) + (long)row * d8 + c0;
#pragma unroll
      for (int k = 0; k < VPT; ++k) {
        const int c = t + k * AR_THREADS;
        if (c < dc) {
          const u16x8 v = src[c];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[k][j] += bf2f(v.v[j]);
        }
      }
    }
  };
  // the row's inverse RMS from the cs partials a rank left beside its rows
  auto row_inv = [&](int q, int row) {
    const float* pp = partials(q, row);
    float ss = 0.f;
    for (int c = 0; c < cs; ++c) ss += pp[c];
    return rsqrtf(ss / (float)(d8 * 8) + eps);
  };
  float o[VPT][8];
  if (!two_shot) {
    for (int row = rg; row < T; row += nr) publish(row);
    ar_group_barrier<W>(peers, rank, 0, b, b, 1, false, e, spin_max);
    for (int row = rg; row < T; row += nr) {
      row_sum(row, o);
      const float ss = ar_residual_chunk<VPT>(residual + (long)row * d8 + c0, o, dc, true,
                                              scratch);
      if (t == 0) partials(rank, row)[ch] = ss;
    }
    ar_group_barrier<W>(peers, rank, 2, b, g0, cs, true, e, spin_max);
    for (int row = rg; row < T; row += nr)
      ar_scale_chunk<VPT>(h_out + (long)row * d8 + c0, residual + (long)row * d8 + c0, w + c0,
                          row_inv(rank, row), dc);
  } else {
    const int S = (T + W - 1) / W;
#pragma unroll
    for (int q = 0; q < W; ++q)
      for (int i = rg; i < S && q * S + i < T; i += nr) publish(q * S + i);
    ar_group_barrier<W>(peers, rank, 0, b, b, 1, false, e, spin_max);
    for (int i = rg; i < S && rank * S + i < T; i += nr) {
      const int row = rank * S + i;
      row_sum(row, o);
      u16x8* dst = reinterpret_cast<u16x8*>(res_base(rank)) + (long)row * d8 + c0;
#pragma unroll
      for (int k = 0; k < VPT; ++k) {
        const int c = t + k * AR_THREADS;
        if (c < dc) {
          u16x8 y;
#pragma unroll
          for (int j = 0; j < 8; ++j) y.v[j] = f2bf(o[k][j]);
          dst[c] = y;
        }
      }
      // the partial of residual + o, as every rank will form it (not written here)
      const float ss = ar_residual_chunk<VPT>(residual + (long)row * d8 + c0, o, dc, false,
                                              scratch);
      if (t == 0) partials(rank, row)[ch] = ss;
    }
    ar_group_barrier<W>(peers, rank, 1, b, g0, cs, false, e, spin_max);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      for (int i = rg; i < S && q * S + i < T; i += nr) {
        const int row = q * S + i;
        ar_load_chunk<VPT>(o, reinterpret_cast<const u16x8*>(res_base(q)) + (long)row * d8 + c0,
                           dc);
        u16x8* res_row = residual + (long)row * d8 + c0;
        // o is bf16 already: f2bf(o) inside is exact
        (void)ar_residual_chunk<VPT>(res_row, o, dc, true, scratch);
        ar_scale_chunk<VPT>(h_out + (long)row * d8 + c0, res_row, w + c0, row_inv(q, row), dc);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == (uint32_t)(nb - 1)) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ----------------------------------------------------------------- host ----
long ar_region_bytes(long slot_bytes) { return AR_DATA + 4 * slot_bytes; }

int ar_alloc(void** ptr, long slot_bytes) {
  const size_t n = (size_t)ar_region_bytes(slot_bytes);
  hipError_t e = hipExtMallocWithFlags(ptr, n, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, n);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

int ar_free(void* ptr) { return (int)hipFree(ptr); }

int ar_ipc_handle(void* ptr, void* handle_out /* 64 B */) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int ar_ipc_open(void** ptr, const void* handle /* 64 B */) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int ar_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int ar_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// error word of this rank's region (device -> host read, synchronous)
int ar_error(void* own, int clear) {
  uint32_t v = 0;
  hipError_t e = hipMemcpy(&v, (char*)own + AR_CTL + 8, 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return -(int)e;
  if (clear && v) {
    const uint32_t z = 0;
    e = hipMemcpy((char*)own + AR_CTL + 8, &z, 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) return -(int)e;
  }
  return (int)v;
}

// the error word copied into pinned host memory on the stream (no sync): a
// step's host code reads the copy a later step left there
int ar_error_async(void* own, void* host, hipStream_t stream) {
  return (int)hipMemcpyAsync(host, (char*)own + AR_CTL + 8, 4, hipMemcpyDeviceToHost, stream);
}

int allreduce(void* out, const void* inp, long nbytes, int rank, int world,
              const unsigned long long* peer_ptrs, long slot_bytes, int two_shot, int blocks,
              int spin_max, hipStream_t stream) {
  if (nbytes <= 0) return 0;
  if (world < 2 || world > AR_MAX_W || rank < 0 || rank >= world) return -1;
  if (nbytes % 16 != 0 || nbytes > slot_bytes) return -2;
  const long n8 = nbytes / 16;
  if (two_shot == 1 && n8 % world != 0) return -3;
  if (two_shot < 0 || two_shot > 3) return -7;
  if (blocks < 1 || blocks > AR_MAX_BLOCKS) return -4;
  if (((uintptr_t)out | (uintptr_t)inp) % 16 != 0) return -5;
  ArPeers p;
  for (int q = 0; q < AR_MAX_W; ++q) p.p[q] = q < world ? (char*)peer_ptrs[q] : nullptr;
  for (int q = 0; q < world; ++q)
    if (!p.p[q]) return -6;
#define LMX_AR(WV)                                                                             \
  allreduce_kernel<WV><<<dim3(blocks), dim3(AR_THREADS), 0, stream>>>(                         \
      (u16x8*)out, (const u16x8*)inp, n8, rank, p, slot_bytes, two_shot, spin_max);
  switch (world) {
    case 2: LMX_AR(2) break;
    case 3: LMX_AR(3) break;
    case 4: LMX_AR(4) break;
    case 5: LMX_AR(5) break;
    case 6: LMX_AR(6) break;
    case 7: LMX_AR(7) break;
    default: LMX_AR(8) break;
  }
#undef LMX_AR
  return (int)hipGetLastError();
}

// fused all-reduce + residual add + RMSNorm of [T, cols] bf16 rows: ``groups``
// row groups x ``cs`` column chunks (cs divides cols / 8)
int allreduce_norm(void* h_out, void* residual, const void* inp, const void* w, int T, int cols,
                   float eps, int rank, int world, const unsigned long long* peer_ptrs,
                   long slot_bytes, int two_shot, int groups, int cs, int spin_max,
                   hipStream_t stream) {
  if (T <= 0) return 0;
  if (world < 2 || world > AR_MAX_W || rank < 0 || rank >= world) return -1;
  if (cols % 8 != 0 || cs < 1 || (cols / 8) % cs != 0 || cols / 8 / cs > AR_THREADS * 4)
    return -2;
  if ((long)T * cols * 2 + (long)T * cs * 4 > slot_bytes) return -2;
  if (groups < 1 || groups * cs > AR_MAX_BLOCKS) return -4;
  if (((uintptr_t)h_out | (uintptr_t)residual | (uintptr_t)inp | (uintptr_t)w) % 16 != 0)
    return -5;
  if (two_shot < 0 || two_shot > 1) return -7;
  ArPeers p;
  for (int q = 0; q < AR_MAX_W; ++q) p.p[q] = q < world ? (char*)peer_ptrs[q] : nullptr;
  for (int q = 0; q < world; ++q)
    if (!p.p[q]) return -6;
  const int d8 = cols / 8;
  const int vpt = (d8 / cs + AR_THREADS - 1) / AR_THREADS;
#define LMX_ARN(WV, VV)                                                                        \
  allreduce_norm_kernel<WV, VV><<<dim3(groups * cs), dim3(AR_THREADS), 0, stream>>>(           \
      (u16x8*)h_out, (u16x8*)residual, (const u16x8*)inp, (const u16x8*)w, T, d8, eps, rank, p,  \
      slot_bytes, two_shot, cs, spin_max);
#define LMX_ARN_W(WV)                 \
  if (vpt <= 1) { LMX_ARN(WV, 1) }    \
  else if (vpt <= 2) { LMX_ARN(WV, 2) } \
  else { LMX_ARN(WV, 4) }
  switch (world) {
    case 2: LMX_ARN_W(2) break;
    case 4: LMX_ARN_W(4) break;
    case 8: LMX_ARN_W(8) break;
    default: return -1;
  }
#undef LMX_ARN_W
#undef LMX_ARN
  return (int)hipGetLastError();
}

}  // namespace lmx
