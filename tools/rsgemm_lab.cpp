// Standalone lab for the K14 register-streamed decode GEMM
// (llm_mcp_amd/csrc/kernels/rsgemm.hip) against K11 (dgemm.hip) on one decode
// projection shape: no torch, so a run on a fresh GPU box starts in seconds.
// Every configuration is first checked against a plain fp32 reference on a
// sample of rows, then timed on COLD weights (the weight operand rotates over
// copies > 512 MB, so each call streams it from HBM as in a decode step);
// a plain streaming read of the same bytes is the achievable-HBM yardstick.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I llm_mcp_amd/csrc/kernels
//          tools/rsgemm_lab.cpp -o tools/labbin/rsgemm_lab
// run:   rsgemm_lab <N> <K> <M> <epi> <spec>[,<spec>...] [iters]
//        spec  rs:<cfg>:<splits>   K14 (cfg bits: 0-1 ring shape, 5 nt, 6 row-major W)
//              dg:<cfg>:<splits>   K11 (epi 2 = partials)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dgemm.hip"
#include "rsgemm.hip"

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

__global__ void fill_kernel(bf16_t* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = f2bf(((float)(h & 0xffffff) / 16777216.f * 2.f - 1.f) * scale);
  }
}

__global__ void ref_kernel(float* out, const bf16_t* A, const bf16_t* W, const int* rows, int nrows,
                           int N, int K, long lda) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, ri = blockIdx.y;
  if (n >= N || ri >= nrows) return;
  const bf16_t* a = A + (long)rows[ri] * lda;
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

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s N K M epi spec[,spec...] [iters]\n", argv[0]);
    return 1;
  }
  const int N = std::atoi(argv[1]), K = std::atoi(argv[2]), M = std::atoi(argv[3]);
  const int epi = std::atoi(argv[4]);
  const int iters = argc > 6 ? std::atoi(argv[6]) : 30;
  const long wbytes = (long)N * K * 2;
  // LAB_COPIES: weight copies the calls rotate over (default: > 512 MB, so every
  // call streams cold weights from HBM; 1 = the same copy every call: warm in L2 /
  // the 256 MB Infinity Cache as far as it fits)
  const char* ce = std::getenv("LAB_COPIES");
  const int copies = ce ? std::max(1, std::atoi(ce))
                        : (int)std::max<long>(2, (512l << 20) / wbytes + 1);
  // LAB_LDA_PAD: elements of padding per activation row (the row stride the
  // kernels see), to move rows off a common L2 channel
  const char* pe = std::getenv("LAB_LDA_PAD");
  const long lda = K + (pe ? std::atol(pe) : 0);
  std::printf("shape N=%d K=%d M=%d epi=%d: W %.1f MB x %d copies, lda %ld\n", N, K, M, epi,
              wbytes / 1e6, copies, lda);
  bf16_t *A, *Wall, *Wpk, *C;
  float *slabs, *ref, *sink;
  unsigned* cnt;
  int* rows_d;
  CK(hipMalloc(&A, (long)M * lda * 2));
  CK(hipMalloc(&Wall, wbytes * copies));
  CK(hipMalloc(&Wpk, wbytes * copies));
  CK(hipMalloc(&C, (long)M * N * 2));
  const long slab_elems = (long)32 * M * N;
  CK(hipMalloc(&slabs, slab_elems * 4));
  CK(hipMalloc(&cnt, 65536 * 4));
  CK(hipMemset(cnt, 0, 65536 * 4));
  CK(hipMalloc(&sink, 16));
  fill_kernel<<<1024, 256>>>(A, (long)M * lda, 17u, 1.f);
  for (int c = 0; c < copies; ++c)
    fill_kernel<<<4096, 256>>>(Wall + (long)c * N * K, (long)N * K, 99u, 0.05f);  // same data
  for (int c = 0; c < copies; ++c)
    if (lmx::rsgemm_pack(Wpk + (long)c * N * K, Wall + (long)c * N * K, N, K, K, nullptr)) {
      std::printf("rsgemm_pack failed\n");
      return 3;
    }
  std::vector<int> rows;
  for (int r : {0, 1, 15, 16, 17, 31, 47, 100, 127, 128, 129, 144, 200, 239, 255})
    if (r < M) rows.push_back(r);
  if (M - 1 > 0 && rows.back() != M - 1) rows.push_back(M - 1);
  const int nr = (int)rows.size();
  CK(hipMalloc(&rows_d, nr * 4));
  CK(hipMemcpy(rows_d, rows.data(), nr * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&ref, (long)nr * N * 4));
  ref_kernel<<<dim3((N + 255) / 256, nr), 256>>>(ref, A, Wall, rows_d, nr, N, K, lda);
  CK(hipDeviceSynchronize());
  std::vector<float> href((long)nr * N);
  CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));
  const int ncol = epi == 3 ? N / 2 : N;
  std::vector<uint16_t> hc((long)M * ncol);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_it = [&](auto&& run) {
    for (int i = 0; i < 3; ++i) run(i);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) run(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / iters;
  };
  {
    const double us = time_it([&](int i) {
      stream_kernel<<<4096, 256>>>((const f32x4_t*)(Wall + (long)(i % copies) * N * K),
                                   wbytes / 16, sink);
    });
    std::printf("  stream-read W: %.2f us  %.2f TB/s\n", us, wbytes / us / 1e6);
  }

  char* list = argv[5];
  for (char* tok = std::strtok(list, ","); tok; tok = std::strtok(nullptr, ",")) {
    char kind[8] = {0};
    int cfg = 0, S = 1;
    if (std::sscanf(tok, "%2[a-z]:%i:%d", kind, &cfg, &S) < 2) continue;
    const bool rs = std::strcmp(kind, "rs") == 0;
    auto launch = [&](int i) {
      if (rs)
        return lmx::rsgemm(C, A, ((cfg & 64) ? Wall : Wpk) + (long)(i % copies) * N * K, slabs,
                           cnt, 65536, M, N, K, lda, K, ncol, cfg, S, epi, nullptr);
      return lmx::dgemm(C, A, Wall + (long)(i % copies) * N * K, slabs, cnt, 65536, M, N, K, lda, K,
                        ncol, cfg, S, epi, nullptr);
    };
    int rc = launch(0);
    if (rc != 0) {
      std::printf("  %s cfg %#x S=%d: launch rc %d\n", kind, cfg, S, rc);
      continue;
    }
    CK(hipDeviceSynchronize());
    if (epi == 2) {
      slab_sum_kernel<<<(int)(((long)M * N + 255) / 256), 256>>>(C, slabs, S, M, N);
      CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (int ri = 0; ri < nr; ++ri) {
      const int m = rows[ri];
      for (int c = 0; c < ncol; ++c) {
        float want;
        if (epi == 3) {     // SwiGLU over [16 gate | 16 up] rows
          const int b = c / 16, r = c % 16;
          const float g = href[(long)ri * N + 32 * b + r], u = href[(long)ri * N + 32 * b + 16 + r];
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
    const double us = time_it(launch);
    const double tf = 2.0 * M * N * (double)K / us / 1e6;
    std::printf("  %s cfg %#4x S=%-2d %8.2f us  %5.2f TB/s W  %6.1f TF  maxerr %.3g (|ref| %.3g)%s\n",
                kind, cfg, S, us, wbytes / us / 1e6, tf, maxerr, maxref,
                maxerr > 0.02 * maxref + 1e-3 ? "  MISMATCH" : "");
  }
  return 0;
}
