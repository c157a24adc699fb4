// Probe: what operand rate can ONE CU pull into its LDS by LDS-DMA on the decode-GEMM access
// pattern, with no MFMA at all?  (gemm_xd's "~54 GB/s per CU ingest
// ceiling" was measured inside the GEMM, with one 4-wave workgroup per CU.)
//
// Each workgroup streams the operand panels of one output tile exactly as gemm_xd does -
// A (activations) rows [TM tm, +TM), W (weight) rows [TN tn, +TN), 64-deep K tiles of 128-B
// row segments, 8 rows per buffer_load_dwordx4 ... lds - through an S-slot LDS ring (counted
// vmcnt + one barrier per K tile), and the tile order is gemm_xd's: XCD label b % 8 owns a
// contiguous block of the column-major tile order, so the row tiles of a weight panel share
// one L2.  Variables: ring slots S, waves per workgroup, workgroups per CU (grid), tile shape,
// and whether the weights stream from HBM (rotated copies > the 256 MB MALL) or stay
// cache-resident.  Prints one JSON line per configuration: GB/s per CU and chip TB/s.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 ingest_probe.hip -o ingest_probe
// run (GPU): ./ingest_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t _e = (x);                                                       \
    if (_e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(_e)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr;

template <int N>
__device__ __forceinline__ void vmcnt() {
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}

// One workgroup = one tile (TM + TN rows per K tile), W waves, S LDS slots of (TM + TN) x 128 B.
template <int S, int W, int TM, int TN>
__global__ __launch_bounds__(64 * W) void ingest_kernel(const char* __restrict__ A,
                                                       const char* __restrict__ Wt, int K,
                                                       int tiles_m, int tiles_n, int per_xcd) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int ROWS = TM + TN;
  constexpr int PER = ROWS / 8 / W;  // DMA instructions per wave per K tile
  static_assert(ROWS % (8 * W) == 0, "rows per wave");
  const int b = blockIdx.x;
  const int item = (b & 7) * per_xcd + (b >> 3);
  if (item >= tiles_m * tiles_n) return;
  const int tn = item / tiles_m, tm = item - tn * tiles_m;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (size_t)tm * TM * K * 2), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Wt + (size_t)tn * TN * K * 2), (short)0, 0x7FFFFFFF, 0x00020000);
  unsigned voff[PER];
  bool isa[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int r = (PER * 8) * wv + 8 * i + (lane >> 3);
    isa[i] = r < TM;
    voff[i] = (unsigned)((isa[i] ? r : r - TM) * K * 2 + (lane & 7) * 16);
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_ptr)lds + (PER * 8) * wv * 128;
  const int nk = K / 64;
  auto issue = [&](int kt) {
    const unsigned dst = lds0 + (kt % S) * ROWS * 128;
    const unsigned kb = kt * 128;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(dst + i * 1024) : "memory");
      if (isa[i])
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voff[i]), "s"(ra), "s"(kb) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voff[i]), "s"(rw), "s"(kb) : "memory");
    }
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + S - 1 < nk) {
      issue(kt + S - 1);
      vmcnt<(S - 1) * PER>();  // own K tile kt landed
    } else {
      vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();  // everyone's: slot kt % S free for K tile kt + S
    asm volatile("" ::: "memory");
  }
  vmcnt<0>();
}

struct Run {
  const char* name;
  int S, W, TM, TN, wg_per_cu;
};

template <int S, int W, int TM, int TN>
float run_cfg(const char* A, const std::vector<char*>& ws, int K, int M, int N, int reps,
              int* grid_out) {
  const int tiles_m = M / TM, tiles_n = N / TN, tiles = tiles_m * tiles_n;
  const int per_xcd = (tiles + 7) / 8;
  const int lds = S * (TM + TN) * 128;
  CK(hipFuncSetAttribute((const void*)ingest_kernel<S, W, TM, TN>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL((ingest_kernel<S, W, TM, TN>), dim3(8 * per_xcd), dim3(64 * W), lds, 0, A,
                       ws[w % ws.size()], K, tiles_m, tiles_n, per_xcd);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((ingest_kernel<S, W, TM, TN>), dim3(8 * per_xcd), dim3(64 * W), lds, 0, A,
                       ws[r % ws.size()], K, tiles_m, tiles_n, per_xcd);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  *grid_out = 8 * per_xcd;
  return ms * 1e3f / reps;  // us per launch
}

template <int S, int W, int TM, int TN>
void report(const char* tag, const char* A, const std::vector<char*>& ws, int K, int M, int N,
            const char* src) {
  int grid = 0;
  const float us = run_cfg<S, W, TM, TN>(A, ws, K, M, N, 20, &grid);
  const double bytes = (double)grid * (TM + TN) * (double)K * 2;  // per launch, into LDS
  const int cus = 256;
  std::printf(
      "{\"cfg\": \"%s\", \"src\": \"%s\", \"S\": %d, \"waves\": %d, \"tile\": \"%dx%d\", "
      "\"M\": %d, \"N\": %d, \"K\": %d, \"grid\": %d, \"us\": %.1f, \"GBs_per_CU\": %.1f, "
      "\"chip_TBs\": %.2f, \"kib_in_flight_per_wg\": %d}\n",
      tag, src, S, W, TM, TN, M, N, K, grid, us, bytes / us / 1e3 / cus * (grid < cus ? (double)cus / grid : 1.0),
      bytes / us / 1e6, (S - 1) * (TM + TN) * 128 / 1024);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  // argv[1]: "hbm" or "resident" to run one weight source only (PMC passes), both by default
  const std::string only = argc > 1 ? argv[1] : "";
  const int K = 4096;
  const int M = 1024;
  const int N = 4096;  // Llama-3-8B o projection at the headline decode batch
  char* A;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMemset(A, 1, (size_t)M * K * 2));
  // weights: 12 rotated copies of 32 MB = 384 MB (> the 256 MB MALL: streamed from HBM, as
  // inside a decode step) or one copy (cache-resident)
  std::vector<char*> hbm, one;
  for (int i = 0; i < 12; ++i) {
    char* w;
    CK(hipMalloc(&w, (size_t)N * K * 2));
    CK(hipMemset(w, 1, (size_t)N * K * 2));
    hbm.push_back(w);
  }
  one.push_back(hbm[0]);
  for (int pass = 0; pass < 2; ++pass) {
    const auto& ws = pass == 0 ? hbm : one;
    const char* src = pass == 0 ? "hbm" : "resident";
    if (!only.empty() && only != src) continue;
    // gemm_xd 1x4 (128 x 128 tiles): 256 workgroups, 1 per CU
    report<2, 4, 128, 128>("xd128x128", A, ws, K, M, N, src);
    report<3, 4, 128, 128>("xd128x128", A, ws, K, M, N, src);
    report<4, 4, 128, 128>("xd128x128", A, ws, K, M, N, src);
    report<4, 8, 128, 128>("xd128x128", A, ws, K, M, N, src);
    report<4, 16, 128, 128>("xd128x128", A, ws, K, M, N, src);
    // smaller tiles = more workgroups per CU (LDS: 2 x 48 KiB)
    report<3, 4, 128, 64>("xd128x64", A, ws, K, M, N, src);
    report<4, 4, 64, 128>("xd64x128", A, ws, K, M, N, src);
    report<4, 4, 64, 64>("xd64x64", A, ws, K, M, N, src);
    report<8, 4, 64, 64>("xd64x64", A, ws, K, M, N, src);
    // 256 x 256 (gemm_w4 / prefill tile), 2 slots
    report<2, 4, 256, 256>("w4_256x256", A, ws, K, M, N, src);
  }
  return 0;
}
