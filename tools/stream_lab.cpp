// Read-stream lab: what rate does a plain load stream reach on MI355X when it
// reads whole pages picked from a table (the paged KV cache's pattern) instead
// of one linear run?  Standalone (no torch): hipcc --offload-arch=gfx950 -O3.
//
//   stream_lab PAGE_KB PATTERN INFLIGHT WGS_PER_CU
//     PATTERN 0: pages in address order (linear stream)
//             1: pages in random order over a 4 GB buffer
//             2: random pages, each wave reads a page as 16 rows x 64 B per
//                instruction (the decode kernel's K fragment shape)
//             3: the decode-attention pattern: a "page" is an 8 KB K page AND an
//                8 KB V page from two random places; K as the 16 rows x 64 B
//                fragments, V as the kernel's 8-B key-quad fragment loads
//                (16 dwordx2 per lane instead of 8 dwordx4)
//             4: as 3 with V read as 8 dwordx4 (1 KB contiguous per instruction)
//     INFLIGHT: pages per wave in flight (1 or 2)
// Every launch reads 768 MB; launches rotate over disjoint page sets so the
// 256 MB Infinity Cache holds nothing a launch reads.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// one wave reads page p: NL loads of 1 KB (16 B per lane)
template <int NL, int FRAG>
__device__ __forceinline__ void load_page(u32x4 (&r)[NL], const char* base, int lane) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    long off;
    if (FRAG) {   // 16 rows x 64 B: row = lane & 15 (256-B rows), 16-B chunk = lane >> 4
      const int blk = i;                 // 1 KB block of the page: rows 16*(blk/4).., 64-B col (blk%4)
      off = (long)(16 * (blk / 4) + (lane & 15)) * 256 + 64 * (blk % 4) + 16 * (lane >> 4);
    } else {
      off = (long)i * 1024 + lane * 16;
    }
    r[i] = *reinterpret_cast<const u32x4*>(base + off);
  }
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// pattern 3 / 4: one 8 KB K page (16 rows x 64 B fragments) + one 8 KB V page
template <int V16>
__global__ void __launch_bounds__(256) kv_stream(const char* __restrict__ buf,
                                                 const int* __restrict__ pages, int npairs,
                                                 unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  unsigned acc = 0;
  for (int p = wave; p < npairs; p += nwaves) {
    const char* kp = buf + (long)pages[2 * p] * 8192;
    const char* vp = buf + (long)pages[2 * p + 1] * 8192;
    u32x4 k[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      k[s] = *reinterpret_cast<const u32x4*>(kp + c * 256 + 64 * s + 16 * g);
      k[4 + s] = *reinterpret_cast<const u32x4*>(kp + (16 + c) * 256 + 64 * s + 16 * g);
    }
    if constexpr (V16) {
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u32x4*>(vp + i * 1024 + lane * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= v[i].x ^ v[i].w;
    } else {
      u32x2 v[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[i] = *reinterpret_cast<const u32x2*>(vp + g * 1024 + 128 * i + 8 * c);
        v[8 + i] = *reinterpret_cast<const u32x2*>(vp + (4 + g) * 1024 + 128 * i + 8 * c);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= v[i].x ^ v[i].y;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) acc ^= k[s].x ^ k[s].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int NL, int FRAG, int INFL>
__global__ void __launch_bounds__(256) page_stream(const char* __restrict__ buf,
                                                   const int* __restrict__ pages, int npages,
                                                   unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  unsigned acc = 0;
  constexpr long PB = NL * 1024L;
  if constexpr (INFL == 1) {
    for (int p = wave; p < npages; p += nwaves) {
      u32x4 r[NL];
      load_page<NL, FRAG>(r, buf + pages[p] * PB, lane);
#pragma unroll
      for (int i = 0; i < NL; ++i) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
    }
  } else {
    // two pages per wave in flight: straight-line pairs
    for (int p = wave; p < npages; p += 2 * nwaves) {
      u32x4 a[NL], b[NL];
      const bool two = p + nwaves < npages;
      load_page<NL, FRAG>(a, buf + pages[p] * PB, lane);
      if (two) load_page<NL, FRAG>(b, buf + pages[p + nwaves] * PB, lane);
#pragma unroll
      for (int i = 0; i < NL; ++i) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
      if (two) {
#pragma unroll
        for (int i = 0; i < NL; ++i) acc ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int NL, int FRAG, int INFL>
static float run(const char* buf, const int* pages, int npages, int wgs, unsigned* sink,
                 int rot, const std::vector<const int*>& tables) {
  hipEvent_t s, e;
  CHECK(hipEventCreate(&s));
  CHECK(hipEventCreate(&e));
  page_stream<NL, FRAG, INFL><<<wgs, 256>>>(buf, tables[0], npages, sink);
  CHECK(hipDeviceSynchronize());
  const int iters = 30;
  CHECK(hipEventRecord(s));
  for (int i = 0; i < iters; ++i)
    page_stream<NL, FRAG, INFL><<<wgs, 256>>>(buf, tables[i % rot], npages, sink);
  CHECK(hipEventRecord(e));
  CHECK(hipEventSynchronize(e));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, s, e));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    printf("usage: stream_lab PAGE_KB PATTERN INFLIGHT WGS_PER_CU\n");
    return 2;
  }
  const int page_kb = atoi(argv[1]), pattern = atoi(argv[2]), infl = atoi(argv[3]);
  const int wpc = atoi(argv[4]);
  const long total = 4L << 30;             // 4 GB buffer
  const long read = 768L << 20;            // bytes per launch
  const long pb = page_kb * 1024L;
  const long nbuf_pages = total / pb;
  const int npages = (int)(read / pb);
  const int rot = (int)std::min<long>(5, nbuf_pages / npages);
  char* buf;
  unsigned* sink;
  CHECK(hipMalloc(&buf, total));
  CHECK(hipMemset(buf, 1, total));
  CHECK(hipMalloc(&sink, 64));
  std::vector<int> perm(nbuf_pages);
  for (long i = 0; i < nbuf_pages; ++i) perm[i] = (int)i;
  std::mt19937 rng(1);
  if (pattern != 0) std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<const int*> tables;
  for (int r = 0; r < rot; ++r) {
    int* d;
    CHECK(hipMalloc(&d, npages * sizeof(int)));
    CHECK(hipMemcpy(d, perm.data() + (long)r * npages, npages * sizeof(int),
                    hipMemcpyHostToDevice));
    tables.push_back(d);
  }
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int wgs = wpc * cus;
  const int frag = pattern == 2;
  float us = -1;
  if (pattern >= 3) {
    if (page_kb != 8) { printf("patterns 3/4 use 8 KB pages\n"); return 2; }
    const int npairs = npages / 2;
    hipEvent_t s0, e0;
    CHECK(hipEventCreate(&s0));
    CHECK(hipEventCreate(&e0));
    auto launch = [&](const int* t) {
      if (pattern == 4) kv_stream<1><<<wgs, 256>>>(buf, t, npairs, sink);
      else kv_stream<0><<<wgs, 256>>>(buf, t, npairs, sink);
    };
    launch(tables[0]);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(s0));
    for (int i = 0; i < 30; ++i) launch(tables[i % rot]);
    CHECK(hipEventRecord(e0));
    CHECK(hipEventSynchronize(e0));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, s0, e0));
    us = ms * 1000.f / 30;
    printf("page  8 KB pattern %d (%s) wgs/CU %d: %7.1f us  %5.2f TB/s\n", pattern,
           pattern == 3 ? "K frag + V 8-B frag pages" : "K frag + V 1-KB rows", wpc, us,
           read / us / 1e6);
    return 0;
  }
#define RUN(NL)                                                                           \
  if (frag && infl == 2) us = run<NL, 1, 2>(buf, nullptr, npages, wgs, sink, rot, tables); \
  else if (frag) us = run<NL, 1, 1>(buf, nullptr, npages, wgs, sink, rot, tables);         \
  else if (infl == 2) us = run<NL, 0, 2>(buf, nullptr, npages, wgs, sink, rot, tables);    \
  else us = run<NL, 0, 1>(buf, nullptr, npages, wgs, sink, rot, tables);
  switch (page_kb) {
    case 2: { RUN(2) break; }
    case 4: { RUN(4) break; }
    case 8: { RUN(8) break; }
    case 16: { RUN(16) break; }
    default: printf("page_kb in 2/4/8/16\n"); return 2;
  }
  printf("page %2d KB pattern %d (%s) inflight %d wgs/CU %d: %7.1f us  %5.2f TB/s\n", page_kb,
         pattern, pattern == 0 ? "linear" : pattern == 1 ? "random" : "random, 16x64B frag",
         infl, wpc, us, read / us / 1e6);
  return 0;
}
