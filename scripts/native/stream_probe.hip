// Probe: the chip's plain HBM read ceiling, as a function of how many CUs stream
// (the decode attention's 5.2 TB/s had only torch `sum` / `copy_` baselines).
//
// A persistent grid of G workgroups (256 threads) sweeps a 4 GiB bf16 buffer (16x the 256 MB
// Infinity Cache) with 16-B-per-lane loads (`global_load_dwordx4`, default policy or `nt`),
// U loads in flight per lane, each workgroup a contiguous 1/G share in 16 KiB steps, and folds
// the data into one xor per lane (written once, so nothing is dead code).  G sweeps 32 .. 2048;
// at G <= 256 every workgroup lands on its own CU (round-robin over the 8 XCDs; the distinct
// (XCC, SE, CU) ids the workgroups ran on are counted from HW_ID / XCC_ID and printed).
// A second table times the same sweep through the decode attention's access shape: 4 KiB
// chunks (one K or V block of one kv head) at random block order.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 stream_probe.hip -o stream_probe
// run (GPU): ./stream_probe            one JSON line per configuration
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <set>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(_e));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// where the workgroup ran: XCC id (HW_REG_XCC_ID) and SE / SH / CU bits of HW_ID
__device__ __forceinline__ unsigned where_am_i() {
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));     // HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));    // XCC_ID[3:0]
  return (xcc << 16) | ((hw >> 8) & 0xFF);
}

// contiguous sweep: workgroup b reads [b * per, (b + 1) * per) 16-B units, U per lane per step
template <int U, bool NT>
__global__ __launch_bounds__(256) void sweep_kernel(const u32x4* __restrict__ src, long per,
                                                    unsigned* __restrict__ sink,
                                                    unsigned* __restrict__ where) {
  const u32x4* p = src + (long)blockIdx.x * per;
  u32x4 acc = {0u, 0u, 0u, 0u};
  const long step = 256L * U;
  for (long i = threadIdx.x; i + (U - 1) * 256 < per; i += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<NT>(p + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (threadIdx.x == 0) where[blockIdx.x] = where_am_i();
}

// attention-shaped: items of `chunk` 16-B units (a 4 KiB K or V block row set) at the
// offsets of `order` (a random permutation), wave w of the grid takes items w, w + W, ...
// with one item per wave in flight plus the next issued (as the persistent decode kernel)
template <bool NT>
__global__ __launch_bounds__(256) void gather_kernel(const u32x4* __restrict__ src,
                                                     const int* __restrict__ order, int n_items,
                                                     unsigned* __restrict__ sink) {
  constexpr int CH = 256;  // 4 KiB = 256 units = 4 per lane
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  u32x4 acc = {0u, 0u, 0u, 0u};
  int it = blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 cur[4], nxt[4];
  if (it < n_items) {
    const u32x4* p = src + (long)order[it] * CH;
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = ld16<NT>(p + lane + 64 * u);
  }
  for (; it < n_items; it += W) {
    const int nx = it + W;
    if (nx < n_items) {
      const u32x4* p = src + (long)order[nx] * CH;
#pragma unroll
      for (int u = 0; u < 4; ++u) nxt[u] = ld16<NT>(p + lane + 64 * u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= cur[u];
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// the decode attention's exact per-lane addressing: one 16 KiB item = an 8 KiB K block
// ([32 tok][128 D]: instruction s of lanes (t, g) reads token t's dims 32 s + 8 g .. + 8, for
// tokens 0-15 and 16-31) and an 8 KiB V block (8 groups x [128 D][4 tok]: 8-B loads of 16
// rows per group), registers only; DEPTH items in flight per wave (1 = the kernel today: the
// next item's loads issued while the current one is consumed)
struct KV16 {
  u32x4 k[8];
  unsigned long long v[16];
};

template <int DEPTH>
__global__ __launch_bounds__(256, 2) void attnkv_kernel(const u32x4* __restrict__ src,
                                                        const int* __restrict__ order,
                                                        int n_items, unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int W = gridDim.x * 4;
  unsigned acc = 0;
  auto load = [&](KV16& r, int it) {
    const char* kb = reinterpret_cast<const char*>(src) + (long)order[it] * 16384;
    const char* vb = kb + 8192;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      r.k[s] = *reinterpret_cast<const u32x4*>(kb + t * 256 + 64 * s + 16 * g);
      r.k[4 + s] = *reinterpret_cast<const u32x4*>(kb + (16 + t) * 256 + 64 * s + 16 * g);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r.v[i] = *reinterpret_cast<const unsigned long long*>(vb + g * 1024 + (16 * i + t) * 8);
      r.v[8 + i] = *reinterpret_cast<const unsigned long long*>(vb + (4 + g) * 1024 + (16 * i + t) * 8);
    }
  };
  auto fold = [&](const KV16& r) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= r.k[j].x ^ r.k[j].w;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= (unsigned)r.v[j];
  };
  KV16 buf[DEPTH + 1];
  int it = blockIdx.x * 4 + (threadIdx.x >> 6);
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (it + d * W < n_items) load(buf[d], it + d * W);
  for (; it < n_items; it += W) {
    const int nx = it + DEPTH * W;
    if (nx < n_items) load(buf[DEPTH], nx);
    fold(buf[0]);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) buf[d] = buf[d + 1];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int DEPTH>
void attnkv(const u32x4* buf, const int* order, int n_items, unsigned* sink, int G) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((attnkv_kernel<DEPTH>), dim3(G), dim3(256), 0, 0, buf, order, n_items, sink);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((attnkv_kernel<DEPTH>), dim3(G), dim3(256), 0, 0, buf, order, n_items, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double tbs = (double)n_items * 16384 * reps / (ms * 1e-3) / 1e12;
  std::printf("{\"probe\": \"attn_kv_addressing\", \"items_in_flight_per_wave\": %d, \"wgs\": %d, "
              "\"TBs\": %.3f}\n", DEPTH, G, tbs);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int U, bool NT>
void sweep(const u32x4* buf, long n16, unsigned* sink, unsigned* where, int G) {
  const long per = (n16 / G) / (256L * U) * (256L * U);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((sweep_kernel<U, NT>), dim3(G), dim3(256), 0, 0, buf, per, sink, where);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((sweep_kernel<U, NT>), dim3(G), dim3(256), 0, 0, buf, per, sink, where);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned> w(G);
  CK(hipMemcpy(w.data(), where, G * sizeof(unsigned), hipMemcpyDeviceToHost));
  const std::set<unsigned> cus(w.begin(), w.end());
  const double bytes = (double)per * G * 16;
  const double tbs = bytes * reps / (ms * 1e-3) / 1e12;
  std::printf("{\"probe\": \"sweep\", \"nt\": %d, \"loads_in_flight_per_lane\": %d, \"wgs\": %d, "
              "\"distinct_cus\": %zu, \"TBs\": %.3f, \"GBs_per_wg\": %.1f}\n",
              (int)NT, U, G, cus.size(), tbs, tbs * 1e3 / G);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <bool NT>
void gather(const u32x4* buf, const int* order, int n_items, unsigned* sink, int G) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((gather_kernel<NT>), dim3(G), dim3(256), 0, 0, buf, order, n_items, sink);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gather_kernel<NT>), dim3(G), dim3(256), 0, 0, buf, order, n_items, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)n_items * 4096;
  const double tbs = bytes * reps / (ms * 1e-3) / 1e12;
  std::printf("{\"probe\": \"gather4k\", \"nt\": %d, \"wgs\": %d, \"TBs\": %.3f, "
              "\"GBs_per_wg\": %.1f}\n", (int)NT, G, tbs, tbs * 1e3 / G);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const long bytes = 4L << 30;
  const long n16 = bytes / 16;
  u32x4* buf;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0x5a, bytes));
  unsigned *sink, *where;
  CK(hipMalloc(&sink, 4096 * 256 * sizeof(unsigned)));
  CK(hipMalloc(&where, 4096 * sizeof(unsigned)));
  const int grids[] = {32, 64, 96, 128, 160, 192, 256, 512, 1024, 2048};
  for (int G : grids) sweep<4, false>(buf, n16, sink, where, G);
  for (int G : grids) sweep<8, false>(buf, n16, sink, where, G);
  for (int G : grids) sweep<8, true>(buf, n16, sink, where, G);
  for (int G : {256, 512, 1024}) sweep<16, false>(buf, n16, sink, where, G);
  // attention-shaped gather: every 4 KiB chunk of 4 GiB once, random order
  const int n_items = (int)(bytes / 4096);
  std::vector<int> order(n_items);
  std::iota(order.begin(), order.end(), 0);
  std::shuffle(order.begin(), order.end(), std::mt19937(1));
  int* d_order;
  CK(hipMalloc(&d_order, n_items * sizeof(int)));
  CK(hipMemcpy(d_order, order.data(), n_items * sizeof(int), hipMemcpyHostToDevice));
  for (int G : {64, 96, 128, 192, 256, 384, 512, 1024}) gather<false>(buf, d_order, n_items, sink, G);
  for (int G : {128, 256, 512}) gather<true>(buf, d_order, n_items, sink, G);
  CK(hipFree(d_order));
  // the attention's K / V addressing over random 16 KiB items (K block + V block)
  const int n_kv = (int)(bytes / 16384);
  std::vector<int> ord16(n_kv);
  std::iota(ord16.begin(), ord16.end(), 0);
  std::shuffle(ord16.begin(), ord16.end(), std::mt19937(2));
  CK(hipMalloc(&d_order, n_kv * sizeof(int)));
  CK(hipMemcpy(d_order, ord16.data(), n_kv * sizeof(int), hipMemcpyHostToDevice));
  for (int G : {256, 512}) attnkv<1>(buf, d_order, n_kv, sink, G);
  for (int G : {256, 512}) attnkv<2>(buf, d_order, n_kv, sink, G);
  CK(hipFree(d_order));
  CK(hipFree(buf));
  CK(hipFree(sink));
  CK(hipFree(where));
  return 0;
}
