// Probe: does hipBLASLt's per-call split-K / workgroup-mapping override
// (hipblaslt_ext::GemmTuning) beat the best plain solution on the decode
// projection GEMMs?  For each shape: every listed solution with its built-in
// split (short timing), then the fastest candidates again with splitK in
// {2,3,4,6,8} and wgm in {0,8}.  Prints one JSON line per shape.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 lt_splitk_probe.cpp -lhipblaslt -o lt_splitk_probe
// run (GPU): ./lt_splitk_probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto _e = (x); if (_e != 0) { std::fprintf(stderr, "%s:%d err %d\n", __FILE__, __LINE__, int(_e)); std::exit(1); } } while (0)

struct Shape { const char* name; int64_t M, N, K; };

int main() {
  const Shape shapes[] = {
      {"8b_qkv", 1024, 6144, 4096},   {"8b_o", 1024, 4096, 4096},
      {"8b_gate_up", 1024, 28672, 4096}, {"8b_down", 1024, 4096, 14336},
      {"8b_lm_head", 1024, 128256, 4096},
      {"70b_qkv", 256, 10240, 8192},  {"70b_o", 256, 8192, 8192},
      {"70b_gate_up", 256, 57344, 8192}, {"70b_down", 256, 8192, 28672},
  };
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  const size_t ws_bytes = size_t(128) << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, HIPBLAS_OP_T, HIPBLAS_OP_N,
                                HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all));
  for (const Shape& s : shapes) {
    const int64_t M = s.M, N = s.N, K = s.K;
    void *w, *x, *y;
    CK(hipMalloc(&w, N * K * 2));
    CK(hipMalloc(&x, M * K * 2));
    CK(hipMalloc(&y, M * N * 2));
    CK(hipMemset(w, 0x3c, N * K * 2));  // 0x3c3c bf16 ~ 0.0115
    CK(hipMemset(x, 0x3c, M * K * 2));
    hipblasLtMatmulDesc_t desc;
    hipblasLtMatrixLayout_t la, lb, lc;
    const hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)));
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, N, M, N));
    const float alpha = 1.f, beta = 0.f;
    hipblaslt_ext::Gemm g(h, desc, &alpha, w, la, x, lb, &beta, y, lc, y, lc);
    auto time_it = [&](hipblasLtMatmulAlgo_t& algo, hipblaslt_ext::GemmTuning& t, int iters) -> float {
      size_t need = 0;
      if (g.isAlgoSupported(algo, t, need) != HIPBLAS_STATUS_SUCCESS || need > ws_bytes) return -1.f;
      if (g.initialize(algo, t, ws, false, st) != HIPBLAS_STATUS_SUCCESS) return -1.f;
      if (g.run(st) != HIPBLAS_STATUS_SUCCESS) return -1.f;
      for (int i = 0; i < 2; ++i) g.run(st);
      hipEventRecord(e0, st);
      for (int i = 0; i < iters; ++i) g.run(st);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      return 1000.f * ms / iters;
    };
    // warm the clocks
    {
      hipblaslt_ext::GemmTuning t;
      for (int i = 0; i < 3 && i < (int)all.size(); ++i) time_it(all[i].algo, t, 20);
    }
    std::vector<std::pair<float, size_t>> plain;
    for (size_t i = 0; i < all.size(); ++i) {
      hipblaslt_ext::GemmTuning t;
      float us = time_it(all[i].algo, t, 4);
      if (us > 0.f) plain.emplace_back(us, i);
    }
    std::sort(plain.begin(), plain.end());
    float best_plain = 1e30f, best = 1e30f;
    int best_plain_idx = -1, best_idx = -1, best_sk = 0, best_wgm = 0;
    const int cand = std::min<int>(10, (int)plain.size());
    for (int c = 0; c < cand; ++c) {
      size_t i = plain[c].second;
      for (int sk : {0, 2, 3, 4, 6, 8}) {
        for (int wgm : {0, 8}) {
          hipblaslt_ext::GemmTuning t;
          t.setSplitK(sk);
          t.setWgm(wgm);
          float us = time_it(all[i].algo, t, 20);
          if (us <= 0.f) continue;
          int idx = hipblaslt_ext::getIndexFromAlgo(all[i].algo);
          if (sk == 0 && wgm == 0 && us < best_plain) { best_plain = us; best_plain_idx = idx; }
          if (us < best) { best = us; best_idx = idx; best_sk = sk; best_wgm = wgm; }
        }
      }
    }
    const double flop = 2.0 * M * N * K;
    std::printf("{\"shape\": \"%s\", \"M\": %ld, \"N\": %ld, \"K\": %ld, \"solutions\": %zu, "
                "\"best_plain_us\": %.2f, \"best_plain_algo\": %d, \"best_us\": %.2f, \"best_algo\": %d, "
                "\"splitK\": %d, \"wgm\": %d, \"plain_PF\": %.3f, \"best_PF\": %.3f}\n",
                s.name, (long)M, (long)N, (long)K, plain.size(), best_plain, best_plain_idx, best,
                best_idx, best_sk, best_wgm, flop / best_plain / 1e9, flop / best / 1e9);
    std::fflush(stdout);
    hipblasLtMatmulDescDestroy(desc);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipFree(w);
    hipFree(x);
    hipFree(y);
  }
  return 0;
}
