// pybind11 entry points of the HIP kernel library (_lmx_kernels).
//
// The Python side (llm_mcp_amd/ops/kernels.py) validates shapes, dtypes,
// contiguity and device placement of torch tensors on the host and passes raw
// device pointers plus the current HIP stream; nothing here allocates or
// synchronises, so every launch is hipGraph-capturable.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <string>
#include <vector>
#include <stdexcept>
#include <string>

namespace lmx {
int rmsnorm(void*, void*, const void*, const void*, int, int, long, long, float, hipStream_t);
int layernorm(void*, const void*, const void*, const void*, const void*, int, int, float,
              hipStream_t);
int rope_cache(void*, long, const int*, const float*, int, int, int, int, const int*, void*, void*,
               int, int, int, const void*, const void*, float, int, hipStream_t);
int kv_write(const void*, const void*, long, const int*, int, int, int, void*, void*, int,
             hipStream_t);
void set_decode_mode(int);
void set_slab_norm_threads(int);
void set_prefill_rescale_thr(float);
void set_prefill_stages(int);
void set_prefill_xcd(int);
int paged_decode(const void*, long, const void*, const void*, const int*, int, const int*,
                 const int*, void*,
                 long, float*, float*, int, int, int, int, int, float, int, int, const int*,
                 const float*, const int*, hipStream_t);
int paged_prefill(const void*, long, const void*, const void*, const int*, int, const int*,
                  const int*, const int*, int, void*, long, int, int, int, int, float, int, int,
                  const int*, const float*, hipStream_t);
int sample(const void*, int, long, int, int, const float*, const int*, const float*,
           const uint64_t*, const int*, int*, float*, int, hipStream_t);
int glu(void*, const void*, long, int, int, int, hipStream_t);
int apply_penalties(void*, long, int, int, const int*, const int*, const float*, const int*, int,
                    int, hipStream_t);
int race_sample_phase(int, int, int, const void*, int, long, int, int, int, int, const float*,
                      const int*, const float*, const uint64_t*, const int*, const float*, int,
                      float*, float*, int*, float*, hipStream_t);
int embed_gather(void*, const void*, const int*, int, int, int, int, hipStream_t);
int ids_from_prev(int*, const int*, const int*, int, hipStream_t);
int mean_pool_l2(float*, float*, const void*, const int*, int, int, int, int, int, hipStream_t);
int bias_act(void*, const void*, long, int, int, hipStream_t);
int gemm_splitk(void*, const void*, const void*, float*, int*, int, int, int, long, long, long,
                int, hipStream_t);
int gemm_nt(void*, const void*, const void*, const void*, const void*, int, int, int, long, long,
            long, int, hipStream_t);
int dgemm(void*, const void*, const void*, float*, unsigned*, int, int, int, int, long, long, long,
          int, int, int, hipStream_t);
int dgemm_num_configs();
int rsgemm(void*, const void*, const void*, float*, unsigned*, int, int, int, int, long, long, long,
           int, int, int, hipStream_t);
int rsgemm_pack(void*, const void*, int, int, long, hipStream_t);
int rmsnorm_slabs(void*, void*, const float*, int, long, const void*, int, int, long, float,
                  hipStream_t);
int dgemm_config(int, int*, int*);
int dgemm_sk_pieces(int, int, int, int, int);
int pgemm(void*, const void*, const void*, const void*, int, int, int, long, long, long, int, int,
          int, int, float*, hipStream_t);
int row_scale(float*, const float*, int, const void*, long, int, int, float, hipStream_t);
int pgemm_sk(void*, const void*, const void*, void*, void*, int, int, int, int, long, long, long,
             int, int, int, hipStream_t);
long ar_region_bytes(long);
int ar_alloc(void**, long);
int ar_free(void*);
int ar_ipc_handle(void*, void*);
int ar_ipc_open(void**, const void*);
int ar_ipc_close(void*);
int ar_ipc_handle_size();
int ar_error(void*, int);
int ar_error_async(void*, void*, hipStream_t);
int allreduce_norm(void*, void*, const void*, const void*, int, int, float, int, int,
                   const unsigned long long*, long, int, int, int, int, hipStream_t);
int allreduce(void*, const void*, long, int, int, const unsigned long long*, long, int, int, int,
              hipStream_t);
}  // namespace lmx

namespace py = pybind11;
typedef unsigned long long uptr;

template <typename T>
static T* P(uptr p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uptr s) { return reinterpret_cast<hipStream_t>(s); }

static void check(int rc, const char* what) {
  if (rc != 0) {
    const char* es = rc > 0 ? hipGetErrorString((hipError_t)rc) : "invalid arguments";
    throw std::runtime_error(std::string("lmx kernel ") + what + " failed (" + std::to_string(rc) +
                             "): " + es);
  }
}

PYBIND11_MODULE(_lmx_kernels, m) {
  m.doc() = "llm_mcp_amd gfx950 HIP kernels";
  m.def("rmsnorm", [](uptr out, uptr residual, uptr x, uptr w, int rows, int cols, long in_stride,
                      long out_stride, float eps, uptr stream) {
    check(lmx::rmsnorm(P<void>(out), P<void>(residual), P<void>(x), P<void>(w), rows, cols,
                       in_stride, out_stride, eps, S(stream)),
          "rmsnorm");
  });
  m.def("layernorm", [](uptr out, uptr x, uptr residual, uptr w, uptr b, int rows, int cols,
                        float eps, uptr stream) {
    check(lmx::layernorm(P<void>(out), P<void>(x), P<void>(residual), P<void>(w), P<void>(b), rows,
                         cols, eps, S(stream)),
          "layernorm");
  });
  m.def("rope_cache", [](uptr qkv, long qkv_stride, uptr positions, uptr cos_sin, int T, int Hq,
                         int Hkv, int D, uptr slots, uptr kc, uptr vc, int BS, int rot_k,
                         int tile_from, uptr q_norm, uptr k_norm, float eps, int skip_q,
                         uptr stream) {
    check(lmx::rope_cache(P<void>(qkv), qkv_stride, P<int>(positions), P<float>(cos_sin), T, Hq, Hkv,
                          D, P<int>(slots), P<void>(kc), P<void>(vc), BS, rot_k, tile_from,
                          P<void>(q_norm), P<void>(k_norm), eps, skip_q, S(stream)),
          "rope_cache");
  });
  m.def("kv_write", [](uptr k, uptr v, long stride, uptr slots, int T, int Hkv, int D, uptr kc,
                       uptr vc, int BS, uptr stream) {
    check(lmx::kv_write(P<void>(k), P<void>(v), stride, P<int>(slots), T, Hkv, D, P<void>(kc),
                        P<void>(vc), BS, S(stream)),
          "kv_write");
  });
  m.def("paged_decode", [](uptr q, long q_stride, uptr kc, uptr vc, uptr bt, int bt_stride,
                           uptr ctx, uptr order, uptr out, long out_stride, uptr part_o,
                           uptr part_ml, int B, int Hq, int Hkv, int D, int BS, float scale,
                           int part_tokens, int max_parts, uptr positions, uptr cos_sin,
                           uptr slots, uptr stream) {
    check(lmx::paged_decode(P<void>(q), q_stride, P<void>(kc), P<void>(vc), P<int>(bt), bt_stride,
                            P<int>(ctx), P<int>(order), P<void>(out), out_stride, P<float>(part_o),
                            P<float>(part_ml), B, Hq, Hkv, D, BS, scale, part_tokens, max_parts,
                            P<int>(positions), P<float>(cos_sin), P<int>(slots), S(stream)),
          "paged_decode");
  });
  m.def("set_slab_norm_threads", [](int t) { lmx::set_slab_norm_threads(t); },
        "probe knob: workgroup size cap of the slab RMSNorm (default 512)");
  m.def("set_decode_mode", [](int mode) { lmx::set_decode_mode(mode); },
        "paged decode loop: 0 one page at a time, 1 next page prefetched, 2 loads only (probe)");
  m.def("set_prefill_rescale_thr", [](float thr) { lmx::set_prefill_rescale_thr(thr); },
        "prefill softmax: raise the running max only past this many log2 units (0: always)");
  m.def("set_prefill_stages", [](int n) { lmx::set_prefill_stages(n); },
        "prefill attention LDS ring slots: 0 default per head dim, 2 or 3");
  m.def("set_prefill_xcd", [](int on) { lmx::set_prefill_xcd(on); },
        "prefill attention workgroup order: 2 XCD-aware, tile list reversed (default), 1 XCD-aware, 0 hardware order");
  m.def("paged_prefill", [](uptr q, long q_stride, uptr kc, uptr vc, uptr bt, int bt_stride,
                            uptr cu_q, uptr ctx, uptr tiles, int num_tiles, uptr out,
                            long out_stride, int Hq, int Hkv, int D, int BS, float scale,
                            int causal, int q_per_tile, uptr rope_pos, uptr rope_cs,
                            uptr stream) {
    check(lmx::paged_prefill(P<void>(q), q_stride, P<void>(kc), P<void>(vc), P<int>(bt),
                             bt_stride, P<int>(cu_q), P<int>(ctx), P<int>(tiles), num_tiles,
                             P<void>(out), out_stride, Hq, Hkv, D, BS, scale, causal, q_per_tile,
                             P<int>(rope_pos), P<float>(rope_cs), S(stream)),
          "paged_prefill");
  });
  m.def("sample", [](uptr logits, int is_bf16, long stride, int B, int V, uptr temp, uptr topk,
                     uptr topp, uptr seeds, uptr offsets, uptr out_tok, uptr out_lp,
                     int max_rounds, uptr stream) {
    check(lmx::sample(P<void>(logits), is_bf16, stride, B, V, P<float>(temp), P<int>(topk),
                      P<float>(topp), P<uint64_t>(seeds), P<int>(offsets), P<int>(out_tok),
                      P<float>(out_lp), max_rounds, S(stream)),
          "sample");
  });
  m.def("glu", [](uptr out, uptr x, long rows, int I, int act, int block, uptr stream) {
    check(lmx::glu(P<void>(out), P<void>(x), rows, I, act, block, S(stream)), "glu");
  });
  m.def("ids_from_prev", [](uptr ids, uptr src, uptr prev, int n, uptr stream) {
    check(lmx::ids_from_prev(P<int>(ids), P<int>(src), P<int>(prev), n, S(stream)),
          "ids_from_prev");
  });
  m.def("embed_gather", [](uptr out, uptr table, uptr ids, int T, int d, int vs, int vr,
                           uptr stream) {
    check(lmx::embed_gather(P<void>(out), P<void>(table), P<int>(ids), T, d, vs, vr, S(stream)),
          "embed_gather");
  });
  m.def("mean_pool_l2", [](uptr out, uptr acc, uptr h, uptr cu, int nseq, int T, int d, int dims,
                           int norm, uptr stream) {
    check(lmx::mean_pool_l2(P<float>(out), P<float>(acc), P<void>(h), P<int>(cu), nseq, T, d, dims,
                            norm, S(stream)),
          "mean_pool_l2");
  });
  m.def("bias_act", [](uptr x, uptr bias, long rows, int n, int act, uptr stream) {
    check(lmx::bias_act(P<void>(x), P<void>(bias), rows, n, act, S(stream)), "bias_act");
  });
  m.def("gemm_splitk", [](uptr C, uptr A, uptr W, uptr slabs, uptr tickets, int M, int N, int K,
                          long lda, long ldw, long ldc, int splits, uptr stream) {
    check(lmx::gemm_splitk(P<void>(C), P<void>(A), P<void>(W), P<float>(slabs), P<int>(tickets), M,
                           N, K, lda, ldw, ldc, splits, S(stream)),
          "gemm_splitk");
  });
  m.def("dgemm", [](uptr C, uptr A, uptr W, uptr slabs, uptr tickets, int n_tickets, int M, int N,
                    int K, long lda, long ldw, long ldc, int cfg, int splits, int epi,
                    uptr stream) {
    check(lmx::dgemm(P<void>(C), P<void>(A), P<void>(W), P<float>(slabs), P<unsigned>(tickets),
                     n_tickets, M, N, K, lda, ldw, ldc, cfg, splits, epi, S(stream)),
          "dgemm");
  });
  m.def("rmsnorm_slabs", [](uptr out, uptr residual, uptr slabs, int nsl, long slab_stride,
                            uptr w, int rows, int cols, long out_stride, float eps, uptr stream) {
    check(lmx::rmsnorm_slabs(P<void>(out), P<void>(residual), P<float>(slabs), nsl, slab_stride,
                             P<void>(w), rows, cols, out_stride, eps, S(stream)),
          "rmsnorm_slabs");
  });
  m.def("dgemm_sk_pieces", [](int M, int N, int K, int cfg, int groups) {
    return lmx::dgemm_sk_pieces(M, N, K, cfg, groups);
  });
  m.def("dgemm_configs", []() {
    std::vector<std::pair<int, int>> out;
    for (int i = 0; i < lmx::dgemm_num_configs(); ++i) {
      int bm = 0, bn = 0;
      lmx::dgemm_config(i, &bm, &bn);
      out.emplace_back(bm, bn);
    }
    return out;
  });
  // ---- K14 register-streamed decode GEMM (rsgemm.hip) ----
  m.def("rsgemm", [](uptr C, uptr A, uptr Wp, uptr slabs, uptr tickets, int n_tickets, int M, int N,
                     int K, long lda, long ldw, long ldc, int cfg, int splits, int epi,
                     uptr stream) {
    check(lmx::rsgemm(P<void>(C), P<void>(A), P<void>(Wp), P<float>(slabs), P<unsigned>(tickets),
                      n_tickets, M, N, K, lda, ldw, ldc, cfg, splits, epi, S(stream)),
          "rsgemm");
  });
  m.def("rsgemm_pack", [](uptr out, uptr W, int N, int K, long ldw, uptr stream) {
    check(lmx::rsgemm_pack(P<void>(out), P<void>(W), N, K, ldw, S(stream)), "rsgemm_pack");
  });
  // ---- K13 large-M GEMM (pgemm.hip) ----
  m.def("pgemm", [](uptr C, uptr A, uptr W, uptr bias, int M, int N, int K, long lda, long ldw,
                    long ldc, int act, int grid, int res, int wpacked, uptr nrm, uptr stream) {
    check(lmx::pgemm(P<void>(C), P<void>(A), P<void>(W), P<void>(bias), M, N, K, lda, ldw, ldc,
                     act, grid, res, wpacked, P<float>(nrm), S(stream)),
          "pgemm");
  });
  m.def("row_scale", [](uptr s, uptr part, int np, uptr x, long x_stride, int M, int cols,
                        float eps, uptr stream) {
    check(lmx::row_scale(P<float>(s), P<float>(part), np, P<void>(x), x_stride, M, cols, eps,
                         S(stream)),
          "row_scale");
  }, "RMSNorm row scales rsqrt(mean(x^2) + eps): from fp32 partials [M][P] or bf16 rows x");
  m.def("pgemm_sk", [](uptr C, uptr A, uptr W, uptr slabs, uptr cnt, int n_cnt, int M, int N,
                       int K, long lda, long ldw, long ldc, int act, int splits, int epi,
                       uptr stream) {
    check(lmx::pgemm_sk(P<void>(C), P<void>(A), P<void>(W), P<void>(slabs), P<void>(cnt), n_cnt,
                        M, N, K, lda, ldw, ldc, act, splits, epi, S(stream)),
          "pgemm_sk");
  });
  // ---- peer-memory all-reduce (allreduce.hip) ----
  m.def("ar_region_bytes", [](long slot) { return lmx::ar_region_bytes(slot); });
  m.def("ar_alloc", [](long slot) {
    void* p = nullptr;
    check(lmx::ar_alloc(&p, slot), "ar_alloc");
    return (uptr)p;
  });
  m.def("ar_free", [](uptr p) { check(lmx::ar_free(P<void>(p)), "ar_free"); });
  m.def("ar_ipc_handle", [](uptr p) {
    std::string h((size_t)lmx::ar_ipc_handle_size(), '\0');
    check(lmx::ar_ipc_handle(P<void>(p), h.data()), "ar_ipc_handle");
    return py::bytes(h);
  });
  m.def("ar_ipc_open", [](py::bytes handle) {
    std::string h = handle;
    if ((int)h.size() != lmx::ar_ipc_handle_size())
      throw std::runtime_error("ar_ipc_open: bad handle size");
    void* p = nullptr;
    check(lmx::ar_ipc_open(&p, h.data()), "ar_ipc_open");
    return (uptr)p;
  });
  m.def("ar_ipc_close", [](uptr p) { check(lmx::ar_ipc_close(P<void>(p)), "ar_ipc_close"); });
  m.def("ar_error", [](uptr own, int clear) {
    const int v = lmx::ar_error(P<void>(own), clear);
    if (v < 0) check(-v, "ar_error");
    return v;
  });
  m.def("allreduce_norm", [](uptr h_out, uptr residual, uptr inp, uptr w, int T, int cols,
                             float eps, int rank, int world, std::vector<unsigned long long> peers,
                             long slot_bytes, int two_shot, int groups, int cs, int spin_max,
                             uptr stream) {
    if ((int)peers.size() < world) throw std::runtime_error("allreduce_norm: peers < world");
    check(lmx::allreduce_norm(P<void>(h_out), P<void>(residual), P<void>(inp), P<void>(w), T,
                              cols, eps, rank, world, peers.data(), slot_bytes, two_shot, groups,
                              cs, spin_max, S(stream)),
          "allreduce_norm");
  });
  m.def("ar_error_async", [](uptr own, uptr host, uptr stream) {
    check(lmx::ar_error_async(P<void>(own), P<void>(host), S(stream)), "ar_error_async");
  });
  m.def("allreduce", [](uptr out, uptr inp, long nbytes, int rank, int world,
                        std::vector<unsigned long long> peers, long slot_bytes, int two_shot,
                        int blocks, int spin_max, uptr stream) {
    if ((int)peers.size() < world) throw std::runtime_error("allreduce: peers < world");
    check(lmx::allreduce(P<void>(out), P<void>(inp), nbytes, rank, world, peers.data(), slot_bytes,
                         two_shot, blocks, spin_max, S(stream)),
          "allreduce");
  });
  m.def("apply_penalties", [](uptr logits, long ld, int B, int V, uptr win, uptr ngen, uptr pen,
                              uptr on, int W, int v0, uptr stream) {
    check(lmx::apply_penalties(P<void>(logits), ld, B, V, P<const int>(win), P<const int>(ngen),
                               P<const float>(pen), P<const int>(on), W, v0, S(stream)),
          "apply_penalties");
  });
  m.def("race_sample_phase", [](int phase, int round, int max_rounds, uptr logits, int is_bf16,
                                long stride, int B, int Vs, int v0, int V, uptr temp, uptr topk,
                                uptr topp, uptr seeds, uptr offsets, uptr gath, int W, uptr rec,
                                uptr st, uptr out_tok, uptr out_lp, uptr stream) {
    check(lmx::race_sample_phase(phase, round, max_rounds, P<void>(logits), is_bf16, stride, B, Vs,
                                 v0, V, P<float>(temp), P<int>(topk), P<float>(topp),
                                 P<uint64_t>(seeds), P<int>(offsets), P<float>(gath), W,
                                 P<float>(rec), P<float>(st), P<int>(out_tok), P<float>(out_lp),
                                 S(stream)),
          "race_sample_phase");
  });
  m.def("gemm_nt", [](uptr C, uptr A, uptr W, uptr bias, uptr residual, int M, int N, int K,
                      long lda, long ldw, long ldc, int act, uptr stream) {
    check(lmx::gemm_nt(P<void>(C), P<void>(A), P<void>(W), P<void>(bias), P<void>(residual), M, N,
                       K, lda, ldw, ldc, act, S(stream)),
          "gemm_nt");
  });
}
