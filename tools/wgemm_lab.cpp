// Standalone lab for the K12 weight-streaming GEMM (tools/lab_kernels/wgemm.hip):
// no torch, so a run on a fresh GPU box starts in seconds.  For one decode
// projection shape it checks each configuration against a plain fp32
// reference on a sample of rows, then times it on COLD weights (the weight
// operand rotates over copies > 512 MB, so every call streams it from HBM as
// in a decode step), and times a plain streaming read of the same bytes as
// the achievable-HBM yardstick.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLMX_WGEMM_LAB
//          -I llm_mcp_amd/csrc/kernels -I tools/lab_kernels tools/wgemm_lab.cpp -o tools/labbin/wgemm_lab
// run:   wgemm_lab <N> <K> <M> <epi> <cfg:splits>[,...] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "wgemm.hip"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__global__ void fill_kernel(bf16_t* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = f2bf(((float)(h & 0xffffff) / 16777216.f * 2.f - 1.f) * scale);
  }
}

// reference for the sampled rows: one thread per (row, column)
__global__ void ref_kernel(float* out, const bf16_t* A, const bf16_t* W, const int* rows, int nrows,
                           int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, ri = blockIdx.y;
  if (n >= N || ri >= nrows) return;
  const bf16_t* a = A + (long)rows[ri] * K;
  const bf16_t* w = W + (long)n * K;
  float s = 0.f;
  for (int k = 0; k < K; k += 8) {
    const u16x8 av = *reinterpret_cast<const u16x8*>(a + k);
    const u16x8 wv = *reinterpret_cast<const u16x8*>(w + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(av.v[j]) * bf2f(wv.v[j]);
  }
  out[(long)ri * N + n] = s;
}

__global__ void slab_sum_kernel(bf16_t* C, const float* slabs, int S, int M, int N) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += slabs[(long)k * M * N + i];
  C[i] = f2bf(s);
}

__global__ void stream_kernel(const f32x4_t* p, long n, float* sink) {
  f32x4_t acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += __builtin_nontemporal_load(p + i);
  if (acc[0] == 1234.5f) sink[0] = acc[1];
}

// W-stream probe: one 256-thread workgroup per CU (as K12), each wave streams
// its own contiguous share with plain 16-B vector loads, R loads in flight per
// lane (software-pipelined register ring): can register staging beat the
// LDS-DMA ring's 5.1-5.4 TB/s?
template <int R>
__global__ void __launch_bounds__(256, 1) wstream_kernel(const f32x4_t* __restrict__ p, long vecs_per_wave,
                                                       float* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f32x4_t* q = p + ((long)blockIdx.x * 4 + wave) * vecs_per_wave + lane;
  f32x4_t r[R], acc = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < R; ++j) r[j] = __builtin_nontemporal_load(q + 64 * j);
  const long n = vecs_per_wave / 64;
  for (long i = R; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      acc += r[j];
      r[j] = __builtin_nontemporal_load(q + 64 * (i + j));
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc += r[j];
  if (acc[0] == 1234.5f) sink[0] = acc[1];
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s N K M epi cfg:splits[,...] [iters]\n", argv[0]);
    return 1;
  }
  const int N = std::atoi(argv[1]), K = std::atoi(argv[2]), M = std::atoi(argv[3]);
  const int epi = std::atoi(argv[4]);
  const int iters = argc > 6 ? std::atoi(argv[6]) : 30;
  const long wbytes = (long)N * K * 2;
  const int copies = (int)std::max<long>(2, (512l << 20) / wbytes + 1);
  std::printf("shape N=%d K=%d M=%d epi=%d: W %.1f MB x %d copies\n", N, K, M, epi, wbytes / 1e6,
              copies);
  bf16_t *A, *Wall, *Wpk, *C;
  float *slabs, *ref;
  unsigned* cnt;
  int* rows_d;
  CK(hipMalloc(&A, (long)M * K * 2));
  CK(hipMalloc(&Wall, wbytes * copies));
  CK(hipMalloc(&Wpk, wbytes * copies));
  int packed_for = -1;
  CK(hipMalloc(&C, (long)M * N * 2));
  const long slab_elems = (long)32 * M * N + (long)256 * 256 * 256;   // S <= 32 partial planes
  CK(hipMalloc(&slabs, slab_elems * 4));
  CK(hipMalloc(&cnt, 65536 * 4));
  CK(hipMemset(cnt, 0, 65536 * 4));
  fill_kernel<<<1024, 256>>>(A, (long)M * K, 17u, 1.f);
  for (int c = 0; c < copies; ++c)
    fill_kernel<<<4096, 256>>>(Wall + (long)c * N * K, (long)N * K, 99u, 0.05f);  // same data
  std::vector<int> rows;
  for (int r : {0, 1, 15, 16, 17, 31, 47, 100, 127, 128, 129, 144, 200, 239, 255})
    if (r < M) rows.push_back(r);
  if (M - 1 > 0 && rows.back() != M - 1) rows.push_back(M - 1);
  const int nr = (int)rows.size();
  CK(hipMalloc(&rows_d, nr * 4));
  CK(hipMemcpy(rows_d, rows.data(), nr * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&ref, (long)nr * N * 4));
  ref_kernel<<<dim3((N + 255) / 256, nr), 256>>>(ref, A, Wall, rows_d, nr, N, K);
  CK(hipDeviceSynchronize());
  std::vector<float> href((long)nr * N);
  CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));
  const int ncol = epi == 3 ? N / 2 : N;
  std::vector<uint16_t> hc((long)M * ncol);
  float* sink;
  CK(hipMalloc(&sink, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  // HBM yardstick: nontemporal 16-B streaming read of one W copy per call
  {
    auto run = [&](int i) {
      stream_kernel<<<4096, 256>>>((const f32x4_t*)(Wall + (long)(i % copies) * N * K), wbytes / 16,
                                   sink);
    };
    for (int i = 0; i < 3; ++i) run(i);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) run(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    std::printf("  stream-read W: %.2f us  %.2f TB/s\n", us, wbytes / us / 1e6);
  }

  {
    const long vpw = wbytes / 16 / 1024;     // 256 workgroups x 4 waves
    auto runR = [&](auto kern, int R) {
      auto run = [&](int i) {
        kern<<<256, 256>>>((const f32x4_t*)(Wall + (long)(i % copies) * N * K), vpw, sink);
      };
      for (int i = 0; i < 3; ++i) run(i);
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) run(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      std::printf("  wstream R=%-2d (1 WG/CU, 4 waves): %.2f us  %.2f TB/s\n", R, us,
                  vpw * 16.0 * 1024 / us / 1e6);
    };
    if (std::getenv("LMX_LAB_WSTREAM")) {
      runR(wstream_kernel<4>, 4);
      runR(wstream_kernel<8>, 8);
      runR(wstream_kernel<16>, 16);
      runR(wstream_kernel<24>, 24);
    }
  }

  char* list = argv[5];
  for (char* tok = std::strtok(list, ","); tok; tok = std::strtok(nullptr, ",")) {
    int cfg = 0, S = 1;
    std::sscanf(tok, "%i:%d", &cfg, &S);
    if ((cfg & 0x800) && packed_for != (cfg & 0x81f)) {
      for (int c = 0; c < copies; ++c)
        if (lmx::wgemm_rs_pack(Wpk + (long)c * N * K, Wall + (long)c * N * K, N, K, K, cfg & 31,
                               nullptr)) {
          std::printf("  rs pack failed for cfg %#x\n", cfg);
          break;
        }
      CK(hipDeviceSynchronize());
      packed_for = cfg & 0x81f;
    }
    if (!(cfg & 0x800) && (cfg & 128) && packed_for != (cfg & 1055)) {
      for (int c = 0; c < copies; ++c)
        if (lmx::wgemm_pack(Wpk + (long)c * N * K, Wall + (long)c * N * K, N, K, K, cfg, nullptr)) {
          std::printf("  pack failed for cfg %#x\n", cfg);
          break;
        }
      CK(hipDeviceSynchronize());
      packed_for = cfg & 1055;
    }
    bf16_t* Wsrc = (cfg & (128 | 0x800)) ? Wpk : Wall;
    auto launch = [&](int i) {
      if (cfg & 0x800)
        return lmx::wgemm_rs(C, A, Wsrc + (long)(i % copies) * N * K, slabs, cnt, 65536, M, N, K,
                             K, ncol, cfg & 63, S, epi, nullptr);
      return lmx::wgemm(C, A, Wsrc + (long)(i % copies) * N * K, slabs, cnt, 65536, M, N, K, K, K,
                        ncol, cfg, S, epi, nullptr);
    };
    int rc = launch(0);
    if (rc != 0) {
      std::printf("  cfg %#x S=%d: launch rc %d\n", cfg, S, rc);
      continue;
    }
    CK(hipDeviceSynchronize());
    double maxerr = 0, maxref = 0;
    if (!(cfg & 64) || (cfg & 0x800)) {
      if (epi == 2) {
        slab_sum_kernel<<<(int)(((long)M * N + 255) / 256), 256>>>(C, slabs, S, M, N);
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
      for (int ri = 0; ri < nr; ++ri) {
        const int m = rows[ri];
        for (int c = 0; c < ncol; ++c) {
          float want;
          if (epi == 3) {
            const int b = c / 4, r = c % 4;
            const float g = href[(long)ri * N + 8 * b + r], u = href[(long)ri * N + 8 * b + 4 + r];
            want = g / (1.f + std::exp(-g)) * u;
          } else {
            want = href[(long)ri * N + c];
          }
          uint32_t bits = (uint32_t)hc[(long)m * ncol + c] << 16;
          float got;
          std::memcpy(&got, &bits, 4);
          maxerr = std::max(maxerr, (double)std::fabs(got - want));
          maxref = std::max(maxref, (double)std::fabs(want));
        }
      }
    }
    for (int i = 1; i < 3; ++i) launch(i);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double tf = 2.0 * M * N * (double)K / us / 1e6;
    std::printf("  cfg %#4x S=%-2d %8.2f us  %5.2f TB/s W  %6.1f TF  maxerr %.3g (|ref| %.3g)%s\n",
                cfg, S, us, wbytes / us / 1e6, tf, maxerr, maxref,
                (!(cfg & 64) && maxerr > 0.02 * maxref + 1e-3) ? "  MISMATCH" : "");
  }
  return 0;
}
