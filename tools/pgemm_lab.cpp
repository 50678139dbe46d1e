// Standalone lab for the K13 design points (variants 0-3 of
// tools/lab_kernels/pgemm_lab.hip; 2 is the kernel the extension ships):
// no torch, so a run on a fresh GPU box starts in seconds.  For one shape it
// checks each variant against a plain fp32 reference on a sample of rows,
// then times it (warm operands, 20 calls).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I llm_mcp_amd/csrc/kernels
//          -I tools/lab_kernels tools/pgemm_lab.cpp -o tools/labbin/pgemm_lab
// run:   pgemm_lab <M> <N> <K> <act 0|2> <variant>[,<variant>...] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pgemm_lab.hip"

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
                           int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, ri = blockIdx.y;
  if (n >= N || ri >= nrows) return;
  const bf16_t* a = A + (long)rows[ri] * K;
  const bf16_t* w = W + (long)n * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(a[k]) * bf2f(w[k]);
  out[(long)ri * N + n] = s;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s M N K act variant[,variant...] [iters]\n", argv[0]);
    return 1;
  }
  const int M = std::atoi(argv[1]), N = std::atoi(argv[2]), K = std::atoi(argv[3]);
  const int act = std::atoi(argv[4]);
  const int iters = argc > 6 ? std::atoi(argv[6]) : 20;
  if (M <= 0 || N % 256 || K % 64 || K < 192 || (act != 0 && act != 2)) {
    std::fprintf(stderr, "unsupported shape\n");
    return 1;
  }
  bf16_t *A, *W, *C;
  float* ref;
  int* rows_d;
  CK(hipMalloc(&A, (long)M * K * 2));
  CK(hipMalloc(&W, (long)N * K * 2));
  CK(hipMalloc(&C, (long)M * N * 2));
  fill_kernel<<<1024, 256>>>(A, (long)M * K, 17u, 1.f);
  fill_kernel<<<1024, 256>>>(W, (long)N * K, 99u, 1.f / std::sqrt((float)K));
  std::vector<int> rows;
  for (int r : {0, 1, 127, 128, 255, 256, 1000, 4095, 8191, 16383, 32767})
    if (r < M) rows.push_back(r);
  if (rows.back() != M - 1) rows.push_back(M - 1);
  const int nr = (int)rows.size();
  CK(hipMalloc(&rows_d, nr * 4));
  CK(hipMemcpy(rows_d, rows.data(), nr * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&ref, (long)nr * N * 4));
  ref_kernel<<<dim3(N / 256, nr), 256>>>(ref, A, W, rows_d, nr, N, K);
  CK(hipDeviceSynchronize());
  std::vector<float> href((long)nr * N);
  CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint16_t> hc((long)M * N);
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const long tiles = (long)((M + 255) / 256) * (N / 256);
  const int grid = (int)std::min<long>(cus, tiles);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("shape M=%d N=%d K=%d act=%d grid=%d\n", M, N, K, act, grid);
  for (char* tok = std::strtok(argv[5], ","); tok; tok = std::strtok(nullptr, ",")) {
    const int variant = std::atoi(tok);
    auto launch = [&] { return lmx::pgemm_lab(C, A, W, M, N, K, act, grid, variant, nullptr); };
    if (int rc = launch()) {
      std::printf("  variant %d: launch rc %d\n", variant, rc);
      continue;
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (int ri = 0; ri < nr; ++ri)
      for (int c = 0; c < N; ++c) {
        float want = href[(long)ri * N + c];
        if (act == 2) want = want / (1.f + std::exp(-want));
        uint32_t bits = (uint32_t)hc[(long)rows[ri] * N + c] << 16;
        float got;
        std::memcpy(&got, &bits, 4);
        maxerr = std::max(maxerr, (double)std::fabs(got - want));
        maxref = std::max(maxref, (double)std::fabs(want));
      }
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    std::printf("  variant %d: %9.2f us  %7.1f TF  maxerr %.3g (|ref| %.3g)%s\n", variant, us,
                2.0 * M * N * (double)K / us / 1e6, maxerr, maxref,
                maxerr > 0.02 * maxref + 2e-2 ? "  MISMATCH" : "");
  }
  return 0;
}
